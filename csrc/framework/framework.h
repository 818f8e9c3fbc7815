// Per-profile framework runtime: runs the enabled plugins of each extension
// point in configured order.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/framework/runtime/
// framework.go (RunPreFilterPlugins, RunFilterPluginsWithNominatedPods,
// RunScorePlugins with weights + NormalizeScore, Reserve/Unreserve (reverse),
// Permit with the 15-minute cap :46, PreBind/Bind/PostBind).
#pragma once

#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "framework/plugin.h"
#include "framework/waiting_pods.h"

namespace xsched {

struct ProfileConfig {
  std::string scheduler_name = kDefaultSchedulerName;
  std::map<uint32_t, std::vector<std::string>> enabled;  // ext point -> plugin names (ordered)
  std::map<std::string, int64_t> score_weights;
  std::map<std::string, Json> plugin_args;
  int percentage_of_nodes_to_score = 0;
  bool run_all_filters = false;
  static ProfileConfig from_json(const Json& j);
};

// One pod template's equivalence cache over the snapshot's node positions,
// kept as columns (structure of arrays): a lookup reads a node version and a
// value from dense arrays instead of a per-node record of a few hundred bytes,
// so a scan over a window of nodes touches one cache line per 8 nodes and
// column. Filter verdicts and raw (pre-normalization) Score values are valid
// while the node's generation matches the one recorded with them.
struct EqTable {
  size_t n = 0;   // snapshot positions
  size_t ns = 0;  // scorers (raw columns)
  std::vector<int64_t> filter_gen;
  std::vector<Status> filter;
  // The verdict with the node's nominated pods added, for the set of them
  // whose signature is nom_sig (Framework::nominated_signature).
  std::vector<int64_t> nom_gen;
  std::vector<uint64_t> nom_sig;
  std::vector<Status> nom_filter;
  // Score, per node version score_gen[pos]: raw[k * n + pos] for the scorers
  // k in cols[pos] (bit k), and plain_sum, the weighted sum of the "plain"
  // scorers in plain_mask[pos] (node-local, no normalization).
  std::vector<int64_t> score_gen;
  std::vector<uint64_t> cols;
  std::vector<uint64_t> plain_mask;
  std::vector<int64_t> plain_sum;
  std::vector<int64_t> raw;

  void reset(size_t nodes) {
    n = nodes;
    ns = 0;
    filter_gen.assign(n, -1);
    filter.assign(n, Status());
    nom_gen.assign(n, -1);
    nom_sig.assign(n, 0);
    nom_filter.assign(n, Status());
    score_gen.assign(n, -1);
    cols.assign(n, 0);
    plain_mask.assign(n, 0);
    plain_sum.assign(n, 0);
    raw.clear();
  }
  // Sizes the raw columns for `scorers` (every score entry invalid on change).
  void ensure_scorers(size_t scorers) {
    if (ns == scorers && raw.size() == ns * n) return;
    ns = scorers;
    raw.assign(ns * n, 0);
    score_gen.assign(n, -1);
  }
  int64_t& raw_at(size_t k, size_t pos) { return raw[k * n + pos]; }
};
struct EqScoreCache {
  std::vector<char> local;    // per scorer: raw score is node-local for this pod
  EqTable* table = nullptr;      // the template's table (nullptr: uncached)
  const int* pos = nullptr;      // the nodes' snapshot positions, in run_score order
  size_t npos = 0;               // entries in pos
  const int64_t* gen = nullptr;  // node versions by snapshot position (Snapshot::gen)
};

class Framework {
 public:
  Framework(const ProfileConfig& cfg, Handle handle);
  ~Framework();

  const std::string& profile_name() const { return cfg_.scheduler_name; }
  const ProfileConfig& config() const { return cfg_; }
  Handle& handle() { return handle_; }
  PluginPtr plugin(const std::string& name) const;
  const std::vector<PluginPtr>& all_plugins() const { return all_; }
  bool has(uint32_t point) const;

  bool less(const QueuedPodInfo& a, const QueuedPodInfo& b) const;

  Status run_pre_filter(CycleState& s, const Pod& p);
  Status run_pre_filter_add_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_add, const NodeInfo& ni);
  Status run_pre_filter_remove_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_remove, const NodeInfo& ni);
  // Whether adding or removing `other` changes any PreFilter extension's
  // state for `to_schedule` (Plugin::pre_filter_extension_affects).
  // `except` (optional): a plugin name whose extensions are not asked.
  bool pre_filter_extensions_affected(const CycleState& s, const Pod& to_schedule, const Pod& other,
                                      const std::string* except = nullptr) const;
  Status run_filter(CycleState& s, const Pod& p, const NodeInfo& ni);
  Status run_filter_with_nominated_pods(CycleState& s, const Pod& p, const NodeInfo& ni);
  // Hash of the nominated pods on `ni` that run_filter_with_nominated_pods
  // would add for `p` (priority >= p's, not p itself), 0 if none. `cacheable`
  // turns false when one of them reacts with a PreFilter extension.
  uint64_t nominated_signature(const CycleState& s, const Pod& p, const NodeInfo& ni, bool* cacheable) const;
  // The same over the node's nominated list when the caller already has it.
  uint64_t nominated_signature(const CycleState& s, const Pod& p, const std::vector<PodPtr>* list,
                               bool* cacheable) const;
  // The same on a NodeInfo the caller owns (a preemption dry run's scratch):
  // nominated pods are added to it and removed again, no copy is made.
  Status run_filter_with_nominated_pods_inplace(CycleState& s, const Pod& p, NodeInfo& ni);
  std::pair<PostFilterResult, Status> run_post_filter(CycleState& s, const Pod& p, const NodeStatusMap& m);
  Status run_pre_score(CycleState& s, const Pod& p, const NodeList& nodes);
  // Weighted sum of all score plugins per node (same order as `nodes`).
  // `breakdown` (optional) receives ("Plugin*weight", normalized scores).
  // Only scores are filled on the scheduling path; `total[i].name` is set
  // when a breakdown is requested (explain), since callers index `nodes`.
  using ScoreBreakdown = std::vector<std::pair<std::string, std::vector<int64_t>>>;
  Status run_score(CycleState& s, const Pod& p, const NodeList& nodes, std::vector<NodeScore>& total,
                   ScoreBreakdown* breakdown = nullptr, EqScoreCache* eq = nullptr);
  // Equivalence cache: every Filter plugin node-local for `p`?
  bool filters_node_local(const Pod& p, const Snapshot& s) const;
  // Per scorer (scorer order): raw Score node-local for `p`? Empty if none is.
  std::vector<char> local_scorers(const Pod& p, const Snapshot& s) const;
  void local_scorers(const Pod& p, const Snapshot& s, std::vector<char>& out) const;  // into a reused buffer
  Status run_reserve(CycleState& s, const PodPtr& p, const std::string& node);
  void run_unreserve(CycleState& s, const PodPtr& p, const std::string& node);
  // Returns Success, an unschedulable/error status, or Wait (then `on_done`
  // fires exactly once when the pod is allowed/rejected/timed out).
  Status run_permit(CycleState& s, const PodPtr& p, const std::string& node, std::function<void(const Status&)> on_done);
  Status run_pre_bind(CycleState& s, const PodPtr& p, const std::string& node);
  Status run_bind(CycleState& s, const PodPtr& p, const std::string& node);
  void run_post_bind(CycleState& s, const PodPtr& p, const std::string& node);

  std::vector<ClusterEvent> events_for(const std::string& plugin) const;
  std::vector<std::string> watched_kinds() const;
  void dispatch_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr& old);
  // Resources were released on some node (Plugin::capacity_freed); any thread.
  void notify_capacity_freed();
  void start();
  void stop();

  static constexpr int64_t kMaxPermitTimeoutUs = 15LL * 60 * 1000000;  // framework.go:46

 private:
  Status filter_with_nominated(CycleState& s, const Pod& p, const NodeInfo& ni, NodeInfo* inplace);
  ParallelSite score_site_;  // inline-vs-parallel cost model of Score
  void record(const char* point, const Status& st, int64_t start_us, CycleState& s);
  ProfileConfig cfg_;
  Handle handle_;
  std::vector<PluginPtr> all_;
  std::map<std::string, PluginPtr> by_name_;
  std::map<uint32_t, std::vector<PluginPtr>> chain_;
  std::vector<std::pair<PluginPtr, int64_t>> scorers_;
  std::unordered_map<std::string, std::vector<PluginPtr>> kind_watchers_;
  std::vector<PluginPtr> capacity_watchers_;
  PluginPtr queue_sort_;
};

}  // namespace xsched
