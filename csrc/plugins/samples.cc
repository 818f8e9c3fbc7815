// NodeResourcesAllocatable, PodState and QOSSort.
//
// Reference: pkg/noderesources/{allocatable.go:61-171,resource_allocation.go}
// (score = Σ w·(Least ? -allocatable : +allocatable) / Σw, min-max
// normalised; all-equal -> MinNodeScore), pkg/podstate/pod_state.go:59-97
// (#terminating - #nominated, min-max normalised) and pkg/qos/queue_sort.go:
// 43-58 (priority, then Guaranteed > Burstable > BestEffort).
#include <climits>

#include "framework/plugin.h"
#include "scheduler/queue.h"

namespace xsched {
namespace {

void min_max_normalize(std::vector<NodeScore>& scores) {
  int64_t hi = LLONG_MIN + 1, lo = LLONG_MAX;
  for (const auto& s : scores) {
    hi = std::max(hi, s.score);
    lo = std::min(lo, s.score);
  }
  int64_t old_range = hi - lo, new_range = kMaxNodeScore - kMinNodeScore;
  for (auto& s : scores) s.score = old_range == 0 ? kMinNodeScore : (s.score - lo) * new_range / old_range + kMinNodeScore;
}

class NodeResourcesAllocatable : public Plugin {
 public:
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  explicit NodeResourcesAllocatable(const Json& args) : Plugin("NodeResourcesAllocatable", kScore) {
    most_ = args["mode"].str_or("Least") == "Most";
    for (const auto& r : args["resources"].items()) {
      const int64_t w = r["weight"].as_int(1);
      // NewAllocatable (allocatable.go:80-118)
      if (w <= 0)
        throw std::runtime_error("resource Weight of " + r["name"].as_string() + " should be a positive value, got " +
                                 std::to_string(w));
      weights_.emplace_back(res_id(r["name"].as_string()), w);
    }
    if (weights_.empty()) weights_ = {{kCPU, 1 << 20}, {kMemory, 1}};
  }
  std::pair<int64_t, Status> score(CycleState&, const Pod&, const NodeInfo& ni) override {
    __int128 num = 0;
    int64_t wsum = 0;
    for (auto [id, w] : weights_) {
      int64_t cap = ni.allocatable.get(id);
      num += static_cast<__int128>(most_ ? cap : -cap) * w;
      wsum += w;
    }
    return {wsum ? static_cast<int64_t>(num / wsum) : 0, {}};
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState&, const Pod&, std::vector<NodeScore>& s) override {
    min_max_normalize(s);
    return {};
  }

 private:
  bool most_ = false;
  std::vector<std::pair<int, int64_t>> weights_;
};

class PodState : public Plugin {
 public:
  explicit PodState(Handle& h) : Plugin("PodState", kScore), h_(h) {}
  std::pair<int64_t, Status> score(CycleState&, const Pod&, const NodeInfo& ni) override {
    int64_t nominated = h_.nominator && !h_.nominator->empty()
                            ? static_cast<int64_t>(h_.nominator->nominated_pods_for_node(ni.name()).size())
                            : 0;
    int64_t terminating = 0;
    for (const auto& p : ni.pods) terminating += p->terminating() ? 1 : 0;
    return {terminating - nominated, {}};
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState&, const Pod&, std::vector<NodeScore>& s) override {
    min_max_normalize(s);
    return {};
  }

 private:
  Handle& h_;
};

class QOSSort : public Plugin {
 public:
  QOSSort() : Plugin("QOSSort", kQueueSort) {}
  static bool comp_qos(QoS a, QoS b) {
    if (a == QoS::Guaranteed) return true;
    if (a == QoS::Burstable) return b != QoS::Guaranteed;
    return b == QoS::BestEffort;
  }
  bool less(const QueuedPodInfo& a, const QueuedPodInfo& b) const override {
    int32_t p1 = a.pod->priority, p2 = b.pod->priority;
    return p1 > p2 || (p1 == p2 && comp_qos(a.pod->qos, b.pod->qos));
  }
};

PluginRegistrar r1("NodeResourcesAllocatable",
                   [](const Json& a, Handle&) { return std::make_shared<NodeResourcesAllocatable>(a); });
PluginRegistrar r2("PodState", [](const Json&, Handle& h) { return std::make_shared<PodState>(h); });
PluginRegistrar r3("QOSSort", [](const Json&, Handle&) { return std::make_shared<QOSSort>(); });

}  // namespace

void link_noderesources_plugin() {}
void link_sample_plugins() {}

}  // namespace xsched
