// Trimaran load-aware scoring: TargetLoadPacking and
// LoadVariationRiskBalancing, fed by load-watcher WatcherMetrics.
//
// Reference: pkg/trimaran/{handler.go, targetloadpacking/targetloadpacking.go:
// 181-294, loadvariationriskbalancing/{loadvariationriskbalancing.go:91-130,
// analysis.go:48-161, collector.go}} and the load-watcher wire types
// (vendor/github.com/paypal/load-watcher/pkg/watcher/watcher.go:63-101).
//
// Metrics transport (MI355X-native): the control plane (Python telemetry
// provider: rocm-smi / amd-smi / sysfs, or an external load-watcher service)
// publishes the WatcherMetrics document as a `loadwatchermetrics` object in
// the API store; the plugins watch that kind, so Score never does I/O and a
// refresh is one informer event. GPU metric types ("GPU" utilization %,
// "GPUMemory" %, and from amd-smi "GPUMemoryBandwidth" = HBM controller
// activity % and "XGMI" = xGMI traffic % of link capacity) extend the
// CPU/Memory set:
//  * TargetLoadPacking arg `resourceType: GPU` packs on live MI355X busy %
//    (capacity = amd.com/gpu, a pod's predicted use = its GPU limit);
//    `resourceType: GPUMemoryBandwidth` packs on HBM bandwidth the same way
//    (a GPU pod is predicted to drive its GPUs' HBM);
//  * LoadVariationRiskBalancing adds risk dimensions for GPU busy and HBM
//    bandwidth when the pod requests GPUs, and for xGMI when it is also a
//    PodGroup member (gang ranks all-reduce over xGMI); score = min over the
//    valid dimensions.
// Fixed: the pod-assign cache drops fully-stale node entries (the reference's
// cleanupCache keeps them when every entry is stale, handler.go:114-138).
#include <array>
#include <cmath>
#include <cstdlib>
#include <map>
#include <shared_mutex>
#include <unordered_map>

#include "framework/plugin.h"
#include "store/store.h"

namespace xsched {
namespace {

constexpr int64_t kReportingIntervalS = 60;   // metricsAgentReportingIntervalSeconds
constexpr int64_t kCacheCleanupUs = 5LL * 60 * 1000000;

// Metric types / operators are interned at parse time so Score compares
// integers, not strings, per node.
enum MType : uint8_t { kTCPU, kTMemory, kTGPU, kTGPUMemory, kTGPUMemoryBandwidth, kTXGMI, kTOther };
enum MOp : uint8_t { kOpAVG, kOpSTD, kOpLatest, kOpEmpty, kOpOther };
MType mtype(const std::string& s) {
  if (s == "CPU") return kTCPU;
  if (s == "Memory") return kTMemory;
  if (s == "GPU") return kTGPU;
  if (s == "GPUMemory") return kTGPUMemory;
  if (s == "GPUMemoryBandwidth") return kTGPUMemoryBandwidth;
  if (s == "XGMI") return kTXGMI;
  return kTOther;
}
MOp mop(const std::string& s) {
  if (s == "AVG") return kOpAVG;
  if (s == "STD") return kOpSTD;
  if (s == "Latest") return kOpLatest;
  if (s.empty()) return kOpEmpty;
  return kOpOther;
}
struct Metric {
  MType type = kTOther;
  MOp op = kOpOther;
  double value = 0;
};
struct WatcherMetrics {
  bool present = false;
  int64_t window_end = 0;
  std::unordered_map<std::string, std::vector<Metric>> nodes;
  std::unordered_map<std::string, int64_t> node_end;  // per-node window end (merged views)
  int64_t end_for(const std::string& node) const {
    auto it = node_end.find(node);
    return it == node_end.end() ? window_end : it->second;
  }
};

WatcherMetrics parse_metrics(const Json& j) {
  WatcherMetrics m;
  const Json* data = j.get("data");
  if (!data) return m;
  const Json* nmm = data->get("NodeMetricsMap");
  if (!nmm) nmm = data->get("nodeMetricsMap");
  if (!nmm || !nmm->is_object()) return m;
  m.present = true;
  m.window_end = j["window"]["end"].as_int(0);
  for (const auto& [node, nm] : nmm->members()) {
    auto& vec = m.nodes[node];
    for (const auto& x : nm["metrics"].items())
      vec.push_back(Metric{mtype(x["type"].as_string()), mop(x["operator"].as_string()), x["value"].as_double()});
  }
  return m;
}

// Shared state of one Trimaran plugin instance: latest metrics + the
// recently-bound pod cache.
class TrimaranBase : public Plugin {
 public:
  TrimaranBase(std::string name, Handle& h) : Plugin(std::move(name), kScore), h_(h) {}

  std::vector<std::string> watched_kinds() const override { return {"loadwatchermetrics", "pods"}; }

  void on_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr& old) override {
    EventType t = static_cast<EventType>(type);
    if (kind == "loadwatchermetrics") {
      // Several documents may coexist: one cluster-wide document (a
      // load-watcher service) and/or one per node (our node agents publish
      // their own window). The view is their union; for a node present in
      // several, the freshest window wins.
      const std::string& name = (*obj)["metadata"]["name"].as_string();
      std::unique_lock<std::shared_mutex> g(mu_);
      if (t == EventType::Deleted)
        sources_.erase(name);
      else
        sources_[name] = std::make_shared<const WatcherMetrics>(parse_metrics(*obj));
      auto merged = std::make_shared<WatcherMetrics>();
      for (const auto& [src, wm] : sources_) {
        if (!wm->present) continue;
        merged->present = true;
        merged->window_end = std::max(merged->window_end, wm->window_end);
        for (const auto& [node, vec] : wm->nodes) {
          auto it = merged->node_end.find(node);
          if (it != merged->node_end.end() && it->second >= wm->window_end) continue;
          merged->nodes[node] = vec;
          merged->node_end[node] = wm->window_end;
        }
      }
      metrics_ = std::move(merged);
      return;
    }
    // Pod-assign cache over assigned pods (handler.go:68-101).
    auto np = Pod::from_json(*obj, *h_.gpu_names);
    if (np->node_name.empty()) return;
    Shard& sh = shard(np->node_name);
    std::unique_lock<std::shared_mutex> g(sh.mu);
    auto& assigned_ = sh.assigned;
    if (t == EventType::Deleted) {
      auto it = assigned_.find(np->node_name);
      if (it == assigned_.end()) return;
      auto& v = it->second;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].second->uid() == np->uid()) {
          v.erase(v.begin() + static_cast<long>(i));
          break;
        }
      return;
    }
    std::string old_node;
    if (old) old_node = (*old)["spec"]["nodeName"].as_string();
    if (!np->node_name.empty() && np->node_name != old_node)
      assigned_[np->node_name].emplace_back(wall_now_us() / 1000000, np);
  }

  void start() override {
    timer_ = h_.timers->every(kCacheCleanupUs, [this] { cleanup(); });
  }

  // Unit-test hook for handler_test.go:12 TestHandlerCacheCleanup:
  // "podAssignCache" seeds args.node's entries (args.entries: [{name,
  // ageSeconds (null = the zero time)}]), applies an OnUpdate that assigns
  // the pod args.update to that node, runs cleanupCache and returns the
  // node's remaining pod names in order.
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    if (what != "podAssignCache") return Plugin::debug_call(what, s, p, args);
    const std::string node = args["node"].as_string();
    const int64_t now = wall_now_us() / 1000000;
    auto make = [&](const std::string& name, const std::string& on) {
      auto q = std::make_shared<Pod>();
      q->meta.ns = "default";
      q->meta.name = name;
      q->meta.uid = name;
      q->node_name = on;
      return q;
    };
    {
      Shard& sh = shard(node);
      std::unique_lock<std::shared_mutex> g(sh.mu);
      auto& v = sh.assigned[node];
      v.clear();
      for (const auto& e : args["entries"].items())
        v.emplace_back(e["ageSeconds"].is_null() ? 0 : now - e["ageSeconds"].as_int(), make(e["name"].as_string(), node));
    }
    if (args["update"].is_string()) {
      Json oldp = Json::object(), newp = Json::object();
      for (Json* o : {&oldp, &newp}) {
        Json md = Json::object();
        md.set("name", Json(args["update"].as_string()));
        md.set("namespace", Json("default"));
        md.set("uid", Json(args["update"].as_string()));
        o->set("metadata", std::move(md));
      }
      Json spec = Json::object();
      spec.set("nodeName", Json(node));
      newp.set("spec", std::move(spec));
      on_object_event("pods", static_cast<int>(EventType::Modified), std::make_shared<Json>(std::move(newp)),
                      std::make_shared<Json>(std::move(oldp)));
    }
    cleanup();
    Json out = Json::object(), names = Json::array();
    const Shard& sh = shard(node);
    std::shared_lock<std::shared_mutex> g(sh.mu);
    if (auto it = sh.assigned.find(node); it != sh.assigned.end())
      for (const auto& e : it->second) names.push_back(Json(e.second->name()));
    out.set("pods", std::move(names));
    return out;
  }
  void stop() override {
    if (timer_) h_.timers->cancel(timer_);
  }

  void cleanup() {
    int64_t now = wall_now_us() / 1000000;
    for (auto& sh : shards_) {
      std::unique_lock<std::shared_mutex> g(sh.mu);
      for (auto it = sh.assigned.begin(); it != sh.assigned.end();) {
        auto& v = it->second;
        size_t idx = 0;
        while (idx < v.size() && v[idx].first + kReportingIntervalS <= now) ++idx;
        v.erase(v.begin(), v.begin() + static_cast<long>(idx));
        it = v.empty() ? sh.assigned.erase(it) : std::next(it);
      }
    }
  }

 protected:
  std::shared_ptr<const WatcherMetrics> metrics() const {
    std::shared_lock<std::shared_mutex> g(mu_);
    return metrics_;
  }
  // The metrics document of this scheduling cycle: fetched once per cycle
  // and kept in CycleState, so the node-parallel Score takes no plugin lock
  // and no shared_ptr refcount per node.
  struct MetricsView : StateData {
    std::shared_ptr<const WatcherMetrics> m;
    std::shared_ptr<StateData> clone() const override { return std::make_shared<MetricsView>(*this); }
  };
  const WatcherMetrics& cycle_metrics(CycleState& s) const {
    if (auto* v = s.read_as<MetricsView>(view_key_)) return *v->m;
    std::lock_guard<std::mutex> g(view_mu_);
    if (auto* v = dynamic_cast<MetricsView*>(s.read_raw(view_key_))) return *v->m;
    auto v = std::make_shared<MetricsView>();
    v->m = metrics();
    const WatcherMetrics* out = v->m.get();
    s.write(view_key_, std::move(v));
    return *out;
  }
  // Pods bound to `node` after the metrics window (or within one reporting
  // interval of its end) are not reflected in the metrics yet. The cache is
  // sharded by node so parallel Score workers rarely share a lock.
  template <typename F>
  void for_missing(const std::string& node, int64_t window_end, F&& f) const {
    const Shard& sh = shard(node);
    std::shared_lock<std::shared_mutex> g(sh.mu);
    auto it = sh.assigned.find(node);
    if (it == sh.assigned.end()) return;
    for (const auto& [ts, pod] : it->second)
      if (ts > window_end || (ts <= window_end && window_end - ts < kReportingIntervalS)) f(*pod);
  }

  struct Shard {
    mutable std::shared_mutex mu;
    std::unordered_map<std::string, std::vector<std::pair<int64_t, PodPtr>>> assigned;
  };
  static constexpr size_t kShards = 32;
  Shard& shard(const std::string& node) { return shards_[std::hash<std::string>{}(node) % kShards]; }
  const Shard& shard(const std::string& node) const { return shards_[std::hash<std::string>{}(node) % kShards]; }

  Handle& h_;
  mutable std::shared_mutex mu_;
  mutable std::mutex view_mu_;
  std::string view_key_ = name_ + "/metrics-view";
  std::shared_ptr<const WatcherMetrics> metrics_ = std::make_shared<WatcherMetrics>();
  std::map<std::string, std::shared_ptr<const WatcherMetrics>> sources_;
  std::array<Shard, kShards> shards_;
  uint64_t timer_ = 0;
};

// --------------------------------------------------------- TargetLoadPacking ----
class TargetLoadPacking : public TrimaranBase {
 public:
  TargetLoadPacking(const Json& args, Handle& h) : TrimaranBase("TargetLoadPacking", h) {
    target_ = static_cast<double>(args["targetUtilization"].as_int(40));
    if (target_ <= 0) target_ = 40;
    const Json& mult = args["defaultRequestsMultiplier"];
    multiplier_ = mult.is_string() ? std::strtod(mult.as_string().c_str(), nullptr) : mult.as_double(1.5);
    if (multiplier_ <= 0) multiplier_ = 1.5;
    const Json& dr = args["defaultRequests"]["cpu"];
    default_milli_ = dr.is_string() ? Quantity::parse(dr.as_string()).milli_value() : 1000;
    const std::string rt = args["resourceType"].str_or("CPU");
    gpu_mode_ = rt == "GPU" || rt == "GPUMemoryBandwidth";
    want_ = rt == "GPU" ? kTGPU : rt == "GPUMemoryBandwidth" ? kTGPUMemoryBandwidth : kTCPU;
  }

  // PredictUtilisation (targetloadpacking.go:286-294).
  int64_t predict(const Container& c) const {
    if (gpu_mode_) {
      int gid = h_.gpu_names->gpu_id();
      return c.limits.has(gid) ? c.limits.get(gid) * 1000 : 0;  // milli-GPUs
    }
    if (c.limits.has(kCPU)) return c.limits.get(kCPU);
    if (c.requests.has(kCPU)) return static_cast<int64_t>(std::llround(static_cast<double>(c.requests.get(kCPU)) * multiplier_));
    return default_milli_;
  }
  int64_t pod_usage(const Pod& p) const {
    int64_t u = 0;
    for (const auto& c : p.containers) u += predict(c);
    if (!gpu_mode_) u += p.overhead().get(kCPU);
    return u;
  }

  std::pair<int64_t, Status> score(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    const WatcherMetrics* m = &cycle_metrics(s);
    if (!m->present) return {kMinNodeScore, {}};
    auto it = m->nodes.find(ni.name());
    if (it == m->nodes.end()) return {kMinNodeScore, {}};
    const MType want = want_;
    double util = 0;
    bool found = false;
    for (const auto& x : it->second)
      if (x.type == want && (x.op == kOpAVG || x.op == kOpLatest)) {
        util = x.value;
        found = true;
      }
    if (!found) return {kMinNodeScore, {}};
    double cap = gpu_mode_ ? static_cast<double>(ni.node->capacity.get(h_.gpu_names->gpu_id()) * 1000)
                           : static_cast<double>(ni.node->capacity.get(kCPU));
    double used = util / 100.0 * cap;
    int64_t missing = 0;
    for_missing(ni.name(), m->end_for(ni.name()), [&](const Pod& q) { missing += pod_usage(q); });
    double pred = 0;
    if (cap != 0) pred = 100.0 * (used + static_cast<double>(pod_usage(p)) + static_cast<double>(missing)) / cap;
    if (pred > target_) {
      if (pred > 100) return {kMinNodeScore, {}};
      return {static_cast<int64_t>(std::llround(target_ * (100 - pred) / (100 - target_))), {}};
    }
    return {static_cast<int64_t>(std::llround((100 - target_) * pred / target_ + target_)), {}};
  }

 private:
  double target_ = 40, multiplier_ = 1.5;
  int64_t default_milli_ = 1000;
  bool gpu_mode_ = false;
  MType want_ = kTCPU;
};

// ------------------------------------------------ LoadVariationRiskBalancing ----
struct ResourceStats {
  double used_avg = 0, used_std = 0, req = 0, capacity = 0;
  // computeScore (analysis.go:48-78)
  double score(double margin, double sensitivity) {
    if (capacity <= 0) return 0;
    req = std::max(req, 0.0);
    used_avg = std::max(std::min(used_avg, capacity), 0.0);
    used_std = std::max(std::min(used_std, capacity), 0.0);
    double mu = std::max(std::min((used_avg + req) / capacity, 1.0), 0.0);
    double sigma = std::max(std::min(used_std / capacity, 1.0), 0.0);
    if (sensitivity >= 0) sigma = std::pow(sigma, 1.0 / sensitivity);
    sigma = std::max(std::min(sigma * margin, 1.0), 0.0);
    return (1.0 - (mu + sigma) / 2.0) * kMaxNodeScore;
  }
};

bool resource_data(const std::vector<Metric>& ms, MType type, double* avg, double* sd) {
  bool valid = false, avg_found = false;
  *avg = *sd = 0;
  for (const auto& x : ms) {
    if (x.type != type) continue;
    if (x.op == kOpAVG) {
      *avg = x.value;
      avg_found = true;
    } else if (x.op == kOpSTD) {
      *sd = x.value;
    } else if ((x.op == kOpEmpty || x.op == kOpLatest) && !avg_found) {
      *avg = x.value;
    }
    valid = true;
  }
  return valid;
}

class LoadVariationRiskBalancing : public TrimaranBase {
 public:
  LoadVariationRiskBalancing(const Json& args, Handle& h) : TrimaranBase("LoadVariationRiskBalancing", h) {
    margin_ = args["safeVarianceMargin"].as_double(1.0);
    sensitivity_ = args["safeVarianceSensitivity"].as_double(1.0);
    if (margin_ < 0) margin_ = 1.0;
    if (sensitivity_ < 0) sensitivity_ = 1.0;
  }

  std::pair<int64_t, Status> score(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    const WatcherMetrics* m = &cycle_metrics(s);
    if (!m->present) return {kMinNodeScore, {}};
    auto it = m->nodes.find(ni.name());
    if (it == m->nodes.end()) return {kMinNodeScore, {}};
    int64_t req_cpu = 0, req_mem = 0;
    requested(p, &req_cpu, &req_mem);
    constexpr int kDims = 5;  // cpu, memory, GPU busy, HBM bandwidth, xGMI
    double scores[kDims];
    bool valid[kDims] = {false, false, false, false, false};
    double avg, sd;
    ResourceStats rs;
    if (create_stats(it->second, *ni.node, req_cpu, req_mem, kTCPU, &rs)) {
      scores[0] = rs.score(margin_, sensitivity_);
      valid[0] = true;
    }
    if (create_stats(it->second, *ni.node, req_cpu, req_mem, kTMemory, &rs)) {
      scores[1] = rs.score(margin_, sensitivity_);
      valid[1] = true;
    }
    // GPU dimensions: capacity = the node's GPUs, the pod's request = its
    // GPUs (a GPU pod can drive its devices' engines, HBM and links fully).
    int gid = h_.gpu_names->gpu_id();
    auto gpu_dim = [&](MType type, int slot) {
      if (!resource_data(it->second, type, &avg, &sd)) return;
      ResourceStats rs;
      rs.capacity = static_cast<double>(ni.node->allocatable.get(gid));
      rs.req = static_cast<double>(p.limit_sum().get(gid));
      rs.used_avg = avg * rs.capacity / 100;
      rs.used_std = sd * rs.capacity / 100;
      scores[slot] = rs.score(margin_, sensitivity_);
      valid[slot] = true;
    };
    if (p.limit_sum().get(gid) > 0) {
      gpu_dim(kTGPU, 2);
      gpu_dim(kTGPUMemoryBandwidth, 3);
      if (!p.pod_group.empty()) gpu_dim(kTXGMI, 4);
    }
    int n_valid = 0;
    for (int i = 0; i < kDims; ++i) n_valid += int(valid[i]);
    double total = 0;
    if (n_valid >= 2) {
      total = 1e300;
      for (int i = 0; i < kDims; ++i)
        if (valid[i]) total = std::min(total, scores[i]);
    } else {
      for (int i = 0; i < kDims; ++i)
        if (valid[i]) total = std::max(total, scores[i]);
    }
    return {static_cast<int64_t>(std::llround(total)), {}};
  }

  // getResourceRequested (analysis.go:134-161): Σ containers, max with each
  // init container (cpu/memory), plus the pod overhead.
  static void requested(const Pod& p, int64_t* cpu, int64_t* mem) {
    *cpu = *mem = 0;
    for (const auto& c : p.containers) {
      *cpu += c.requests.get(kCPU);
      *mem += c.requests.get(kMemory);
    }
    for (const auto& c : p.init_containers) {
      *cpu = std::max(*cpu, c.requests.get(kCPU));
      *mem = std::max(*mem, c.requests.get(kMemory));
    }
    *cpu += p.overhead().get(kCPU);
    *mem += p.overhead().get(kMemory);
  }
  // createResourceStats (analysis.go:81-110): usage statistics of one
  // resource in the resource's units (milli-CPU, MiB).
  static bool create_stats(const std::vector<Metric>& ms, const Node& node, int64_t req_cpu, int64_t req_mem,
                           MType type, ResourceStats* rs) {
    double avg, sd;
    if (!resource_data(ms, type, &avg, &sd)) return false;
    *rs = ResourceStats{};
    if (type == kTCPU) {
      rs->capacity = static_cast<double>(node.allocatable.get(kCPU));
      rs->req = static_cast<double>(req_cpu);
    } else {
      const double mega = 1.0 / 1024.0 / 1024.0;
      rs->capacity = static_cast<double>(node.allocatable.get(kMemory)) * mega;
      rs->req = static_cast<double>(req_mem) * mega;
    }
    rs->used_avg = avg * rs->capacity / 100;
    rs->used_std = sd * rs->capacity / 100;
    return true;
  }

  // Unit-test hooks for the reference's analysis_test.go tables:
  // "computeScore" (TestComputeScore :74), "createResourceStats"
  // (Test_createResourceStats :212; args.metrics, args.resource, the node
  // named by args.node), "getResourceRequested" (TestGetResourceRequested).
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    Json out = Json::object();
    if (what == "computeScore") {
      ResourceStats rs;
      rs.capacity = args["capacity"].as_double(0);
      rs.req = args["req"].as_double(0);
      rs.used_avg = args["usedAvg"].as_double(0);
      rs.used_std = args["usedStdev"].as_double(0);
      out.set("score", Json(rs.score(args["margin"].as_double(1), args["sensitivity"].as_double(1))));
      return out;
    }
    if (what == "getResourceRequested" || what == "createResourceStats") {
      int64_t cpu = 0, mem = 0;
      requested(*p, &cpu, &mem);
      if (what == "getResourceRequested") {
        out.set("milliCPU", Json(cpu));
        out.set("memory", Json(mem));
        return out;
      }
      std::vector<Metric> ms;
      for (const auto& x : args["metrics"].items())
        ms.push_back(Metric{mtype(x["type"].as_string()), mop(x["operator"].as_string()), x["value"].as_double()});
      NodeInfoPtr ni = h_.snapshot ? h_.snapshot->get(args["node"].as_string()) : nullptr;
      if (!ni || !ni->node) throw std::runtime_error("createResourceStats: no node " + args["node"].str_or(""));
      ResourceStats rs;
      const bool ok = create_stats(ms, *ni->node, cpu, mem, args["resource"].as_string() == "cpu" ? kTCPU : kTMemory,
                                   &rs);
      out.set("valid", Json(ok));
      if (ok) {
        out.set("capacity", Json(rs.capacity));
        out.set("req", Json(rs.req));
        out.set("usedAvg", Json(rs.used_avg));
        out.set("usedStdev", Json(rs.used_std));
      }
      return out;
    }
    return TrimaranBase::debug_call(what, s, p, args);
  }

 private:
  double margin_ = 1.0, sensitivity_ = 1.0;
};

PluginRegistrar r1("TargetLoadPacking", [](const Json& a, Handle& h) { return std::make_shared<TargetLoadPacking>(a, h); });
PluginRegistrar r2("LoadVariationRiskBalancing",
                   [](const Json& a, Handle& h) { return std::make_shared<LoadVariationRiskBalancing>(a, h); });

}  // namespace

void link_trimaran_plugins() {}

}  // namespace xsched
