// In-tree default plugins that every reference profile implicitly enables
// (vendor/k8s.io/kubernetes/pkg/scheduler/apis/config/v1beta2/default_plugins.go:34-106):
// PrioritySort, NodeUnschedulable, NodeName, NodePorts, NodeResourcesFit,
// NodeResourcesBalancedAllocation, TaintToleration, NodeAffinity, DefaultBinder.
// DefaultPreemption lives in preemption.cc.
#include <algorithm>
#include <cmath>

#include "framework/plugin.h"
#include "scheduler/cache.h"

namespace xsched {
namespace {

// ---------------------------------------------------------- PrioritySort ----
class PrioritySort : public Plugin {
 public:
  PrioritySort() : Plugin("PrioritySort", kQueueSort) {}
  bool less(const QueuedPodInfo& a, const QueuedPodInfo& b) const override {
    if (a.pod->priority != b.pod->priority) return a.pod->priority > b.pod->priority;
    if (a.timestamp_us != b.timestamp_us) return a.timestamp_us < b.timestamp_us;
    return a.enqueue_seq < b.enqueue_seq;
  }
};

// ----------------------------------------------------- NodeUnschedulable ----
class NodeUnschedulable : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  NodeUnschedulable() : Plugin("NodeUnschedulable", kFilter) {}
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    if (!ni.node) return Status::unresolvable("node not found");
    if (!ni.node->unschedulable) return {};
    Taint t{"node.kubernetes.io/unschedulable", "", "NoSchedule"};
    for (const auto& tol : p.tolerations)
      if (tol.tolerates(t)) return {};
    return XS_FIXED_STATUS(Code::UnschedulableAndUnresolvable, "node(s) were unschedulable");
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Node", kAdd | kUpdateNodeTaint, ""}};
  }
};

// -------------------------------------------------------------- NodeName ----
class NodeName : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  NodeName() : Plugin("NodeName", kFilter) {}
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    if (p.node_name.empty() || p.node_name == ni.name()) return {};
    return XS_FIXED_STATUS(Code::UnschedulableAndUnresolvable, "node(s) didn't match the requested node name");
  }
  std::vector<ClusterEvent> events_to_register() const override { return {{"Node", kAdd, ""}}; }
};

// ------------------------------------------------------------- NodePorts ----
class NodePorts : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  NodePorts() : Plugin("NodePorts", kPreFilter | kFilter) {}
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    for (const auto& port : p.host_ports) {
      for (const auto& [ip, proto, hp] : ni.used_ports) {
        if (hp != port.host_port || proto != port.protocol) continue;
        if (ip == "0.0.0.0" || port.host_ip == "0.0.0.0" || ip == port.host_ip)
          return XS_FIXED_STATUS(Code::Unschedulable, "node(s) didn't have free ports for the requested pod ports");
      }
    }
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"Node", kAdd, ""}};
  }
};

// ------------------------------------------------------ NodeResourcesFit ----
// Scoring strategies per NodeResourcesFitArgs.scoringStrategy (1.23):
// LeastAllocated (default), MostAllocated, RequestedToCapacityRatio.
struct ResourceWeight {
  int id;
  int64_t weight;
};

std::vector<ResourceWeight> parse_weights(const Json& arr, std::vector<ResourceWeight> dflt) {
  if (!arr.is_array() || arr.size() == 0) return dflt;
  std::vector<ResourceWeight> out;
  for (const auto& r : arr.items())
    out.push_back(ResourceWeight{res_id(r["name"].as_string()), std::max<int64_t>(1, r["weight"].as_int(1))});
  return out;
}

class NodeResourcesFit : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  explicit NodeResourcesFit(const Json& args) : Plugin("NodeResourcesFit", kPreFilter | kFilter | kScore) {
    for (const auto& r : args["ignoredResources"].items()) ignored_.push_back(res_id(r.as_string()));
    for (const auto& g : args["ignoredResourceGroups"].items()) ignored_groups_.push_back(g.as_string());
    const Json& ss = args["scoringStrategy"];
    strategy_ = ss["type"].str_or("LeastAllocated");
    weights_ = parse_weights(ss["resources"], {{kCPU, 1}, {kMemory, 1}});
    for (const auto& pt : ss["requestedToCapacityRatio"]["shape"].items())
      shape_.emplace_back(pt["utilization"].as_int(), pt["score"].as_int());
    unresolvable_beyond_allocatable_ = args["unresolvableBeyondAllocatable"].as_bool(false);
  }

  bool ignored(int id) const {
    if (std::find(ignored_.begin(), ignored_.end(), id) != ignored_.end()) return true;
    if (!ignored_groups_.empty()) {
      std::string n = ResourceRegistry::get().name(id);
      auto slash = n.find('/');
      if (slash != std::string::npos) {
        std::string prefix = n.substr(0, slash);
        for (const auto& g : ignored_groups_)
          if (g == prefix) return true;
      }
    }
    return false;
  }

  static constexpr uint64_t kBeyondAllocatable = 1ull << 63;  // above every resource id
  static_assert(kMaxRes < 63);
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    // Failures are encoded as a resource bitmask (bit kPods = "Too many
    // pods") and their Status is built once per distinct mask per thread.
    uint64_t fail = 0;
    if (ni.num_pods() + 1 > ni.allocatable.get(kPods) && ni.allocatable.has(kPods)) fail |= 1ull << kPods;
    const Res& req = p.request();
    for (uint64_t m = req.mask; m; m &= m - 1) {
      int i = __builtin_ctzll(m);
      if (i == kPods) continue;
      int64_t want = req.v[i];
      if (want == 0) continue;
      if (i > kPods && ignored(i)) continue;
      int64_t free = ni.allocatable.get(i) - ni.requested.get(i);
      if (want > free) {
        fail |= 1ull << i;
        // More than the node has at all: evicting pods cannot help. Opt-in
        // (unresolvableBeyondAllocatable), the verdict is then unresolvable
        // and preemption skips the node, as newer upstream does; k8s 1.23,
        // the reference's version, always says Unschedulable.
        if (unresolvable_beyond_allocatable_ && want > ni.allocatable.get(i)) fail |= kBeyondAllocatable;
      }
    }
    if (!fail) return {};
    thread_local std::unordered_map<uint64_t, Status> memo;
    auto it = memo.find(fail);
    if (it != memo.end()) return it->second;
    std::vector<std::string> reasons;
    if (fail & (1ull << kPods)) reasons.push_back("Too many pods");
    for (uint64_t m = fail & ~((1ull << kPods) | kBeyondAllocatable); m; m &= m - 1)
      reasons.push_back("Insufficient " + ResourceRegistry::get().name(__builtin_ctzll(m)));
    Code code = (fail & kBeyondAllocatable) ? Code::UnschedulableAndUnresolvable : Code::Unschedulable;
    return memo.emplace(fail, Status::interned(code, std::move(reasons))).first->second;
  }

  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    int64_t num = 0, den = 0;
    for (const auto& w : weights_) {
      int64_t alloc = ni.allocatable.get(w.id);
      int64_t req = (w.id == kCPU || w.id == kMemory) ? ni.nonzero_requested.get(w.id) + p.nonzero_request().get(w.id)
                                                       : ni.requested.get(w.id) + p.request().get(w.id);
      int64_t s = 0;
      if (strategy_ == "MostAllocated") {
        s = (alloc == 0 || req > alloc) ? 0 : req * kMaxNodeScore / alloc;
      } else if (strategy_ == "RequestedToCapacityRatio") {
        s = shape_score(alloc == 0 ? 100 : std::min<int64_t>(100, req * 100 / alloc));
      } else {
        s = (alloc == 0 || req > alloc) ? 0 : (alloc - req) * kMaxNodeScore / alloc;
      }
      num += s * w.weight;
      den += w.weight;
    }
    return {den ? num / den : 0, {}};
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"Node", kAdd | kUpdateNodeAllocatable, ""}};
  }

 private:
  int64_t shape_score(int64_t util) const {
    if (shape_.empty()) return 0;
    if (util <= shape_.front().first) return shape_.front().second * kMaxNodeScore / 10;
    for (size_t i = 1; i < shape_.size(); ++i) {
      if (util <= shape_[i].first) {
        auto [x0, y0] = shape_[i - 1];
        auto [x1, y1] = shape_[i];
        int64_t y = y0 + (y1 - y0) * (util - x0) / std::max<int64_t>(1, x1 - x0);
        return y * kMaxNodeScore / 10;
      }
    }
    return shape_.back().second * kMaxNodeScore / 10;
  }
  std::vector<int> ignored_;
  std::vector<std::string> ignored_groups_;
  bool unresolvable_beyond_allocatable_ = false;
  std::string strategy_;
  std::vector<ResourceWeight> weights_;
  std::vector<std::pair<int64_t, int64_t>> shape_;
};

// ------------------------------------------ NodeResourcesBalancedAllocation ----
class BalancedAllocation : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  explicit BalancedAllocation(const Json& args) : Plugin("NodeResourcesBalancedAllocation", kScore) {
    weights_ = parse_weights(args["resources"], {{kCPU, 1}, {kMemory, 1}});
  }
  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    double fr[kMaxRes];  // one fraction per weighted resource (no allocation per node)
    size_t n = 0;
    for (const auto& w : weights_) {
      int64_t alloc = ni.allocatable.get(w.id);
      if (alloc == 0) continue;
      int64_t req = (w.id == kCPU || w.id == kMemory) ? ni.nonzero_requested.get(w.id) + p.nonzero_request().get(w.id)
                                                       : ni.requested.get(w.id) + p.request().get(w.id);
      double f = static_cast<double>(req) / static_cast<double>(alloc);
      if (f >= 1) return {0, {}};  // over-committed
      if (n < static_cast<size_t>(kMaxRes)) fr[n++] = f;
    }
    if (n < 2) return {kMaxNodeScore, {}};
    double mean = 0;
    for (size_t i = 0; i < n; ++i) mean += fr[i];
    mean /= static_cast<double>(n);
    double var = 0;
    for (size_t i = 0; i < n; ++i) var += (fr[i] - mean) * (fr[i] - mean);
    double sd = n == 2 ? std::fabs(fr[0] - fr[1]) / 2 : std::sqrt(var / static_cast<double>(n));
    return {static_cast<int64_t>((1 - sd) * kMaxNodeScore), {}};
  }

 private:
  std::vector<ResourceWeight> weights_;
};

// ------------------------------------------------------- TaintToleration ----
class TaintToleration : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  TaintToleration() : Plugin("TaintToleration", kFilter | kPreScore | kScore) {}
  // Raw score counts untolerated PreferNoSchedule taints: with none in the
  // cluster it is 0 everywhere and the reversed normalization is flat.
  bool score_all_zero(const Pod&, const Snapshot& s) const override { return s.nodes_with_prefer_no_schedule == 0; }
  int64_t score_skip_value() const override { return kMaxNodeScore; }  // reversed normalize of all-zero
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    if (!ni.node) return Status::error("invalid nodeInfo");
    for (const auto& t : ni.node->taints) {
      if (t.effect != "NoSchedule" && t.effect != "NoExecute") continue;
      bool ok = false;
      for (const auto& tol : p.tolerations)
        if (tol.tolerates(t)) {
          ok = true;
          break;
        }
      if (!ok) return Status::unresolvable("node(s) had taint {" + t.key + ": " + t.value + "}, that the pod didn't tolerate");
    }
    return {};
  }
  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    int64_t n = 0;
    for (const auto& t : ni.node->taints) {
      if (t.effect != "PreferNoSchedule") continue;
      bool ok = false;
      for (const auto& tol : p.tolerations)
        if ((tol.effect.empty() || tol.effect == "PreferNoSchedule") && tol.tolerates(t)) ok = true;
      if (!ok) ++n;
    }
    return {n, {}};
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState&, const Pod&, std::vector<NodeScore>& s) override {
    default_normalize_score(kMaxNodeScore, true, s);
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override { return {{"Node", kAdd | kUpdateNodeTaint, ""}}; }
};

// ---------------------------------------------------------- NodeAffinity ----
bool term_matches(const NodeSelectorTerm& t, const Node& n) { return node_selector_term_matches(t, n); }

class NodeAffinity : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_all_zero(const Pod& p, const Snapshot&) const override { return p.preferred_node_terms.empty(); }
  explicit NodeAffinity(const Json& args) : Plugin("NodeAffinity", kPreFilter | kFilter | kPreScore | kScore) {
    if (const Json* aa = args.get("addedAffinity")) {
      if (const Json* req = aa->path({"requiredDuringSchedulingIgnoredDuringExecution", "nodeSelectorTerms"})) {
        has_added_ = true;
        Json fake = Json::object();
        Json spec = Json::object();
        Json aff = Json::object();
        Json na = Json::object();
        Json r = Json::object();
        r.set("nodeSelectorTerms", *req);
        na.set("requiredDuringSchedulingIgnoredDuringExecution", r);
        aff.set("nodeAffinity", na);
        spec.set("affinity", aff);
        fake.set("spec", spec);
        added_ = Pod::from_json(fake)->required_node_terms;
      }
    }
  }
  static bool required_matches(const Pod& p, const Node& n) { return pod_matches_node_selector_and_affinity(p, n); }
  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    if (!ni.node) return Status::error("node not found");
    if (has_added_) {
      bool ok = false;
      for (const auto& t : added_)
        if (term_matches(t, *ni.node)) ok = true;
      if (!ok)
        return XS_FIXED_STATUS(Code::UnschedulableAndUnresolvable,
                               "node(s) didn't match scheduler-enforced node affinity");
    }
    if (!required_matches(p, *ni.node))
      return XS_FIXED_STATUS(Code::UnschedulableAndUnresolvable, "node(s) didn't match Pod's node affinity/selector");
    return {};
  }
  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    int64_t s = 0;
    for (const auto& t : p.preferred_node_terms)
      if (t.weight != 0 && term_matches(t.pref, *ni.node)) s += t.weight;
    return {s, {}};
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState&, const Pod&, std::vector<NodeScore>& s) override {
    default_normalize_score(kMaxNodeScore, false, s);
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override { return {{"Node", kAdd | kUpdateNodeLabel, ""}}; }

 private:
  bool has_added_ = false;
  std::vector<NodeSelectorTerm> added_;
};

// --------------------------------------------------------- DefaultBinder ----
class DefaultBinder : public Plugin {
 public:
  explicit DefaultBinder(Handle& h) : Plugin("DefaultBinder", kBind), h_(h) {}
  Status bind(CycleState&, const PodPtr& p, const std::string& node) override {
    try {
      h_.client->bind(*p, node, Json::object());
    } catch (const std::exception& e) {
      return Status::error(e.what());
    }
    return {};
  }

 private:
  Handle& h_;
};

PluginRegistrar r1("PrioritySort", [](const Json&, Handle&) { return std::make_shared<PrioritySort>(); });
PluginRegistrar r2("NodeUnschedulable", [](const Json&, Handle&) { return std::make_shared<NodeUnschedulable>(); });
PluginRegistrar r3("NodeName", [](const Json&, Handle&) { return std::make_shared<NodeName>(); });
PluginRegistrar r4("NodePorts", [](const Json&, Handle&) { return std::make_shared<NodePorts>(); });
PluginRegistrar r5("NodeResourcesFit", [](const Json& a, Handle&) { return std::make_shared<NodeResourcesFit>(a); });
PluginRegistrar r6("NodeResourcesBalancedAllocation",
                   [](const Json& a, Handle&) { return std::make_shared<BalancedAllocation>(a); });
PluginRegistrar r7("TaintToleration", [](const Json&, Handle&) { return std::make_shared<TaintToleration>(); });
PluginRegistrar r8("NodeAffinity", [](const Json& a, Handle&) { return std::make_shared<NodeAffinity>(a); });
PluginRegistrar r9("DefaultBinder", [](const Json&, Handle& h) { return std::make_shared<DefaultBinder>(h); });

}  // namespace

void link_intree_plugins() {}

}  // namespace xsched
