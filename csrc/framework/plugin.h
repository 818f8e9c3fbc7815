// Plugin API: one base class with a default (no-op) method per extension
// point plus a bitmask declaring which points the plugin extends.
//
// Maps 1:1 to the reference's framework interfaces (vendor/k8s.io/kubernetes/
// pkg/scheduler/framework/interface.go): QueueSort, PreFilter(+Extensions),
// Filter, PostFilter, PreScore, Score(+NormalizeScore), Reserve/Unreserve,
// Permit, PreBind, Bind, PostBind and EnqueueExtensions. Score receives the
// NodeInfo directly instead of a node name + snapshot lookup.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common/clock.h"
#include "common/json.h"
#include "common/parallel.h"
#include "framework/types.h"

// A Filter verdict with a fixed message, built once per call site for the
// life of the process (Status::immortal): returning it costs a plain copy.
#define XS_FIXED_STATUS(code, msg)                                 \
  ([]() -> const ::xsched::Status& {                               \
    static const ::xsched::Status fixed_status = ::xsched::Status::immortal(code, msg); \
    return fixed_status;                                          \
  }())

namespace xsched {

class Framework;
class SchedulerCache;
class Informers;
class WaitingPods;
class Nominator;
class Metrics;
class GangPlacement;

enum ExtPoint : uint32_t {
  kQueueSort = 1u << 0,
  kPreFilter = 1u << 1,
  kFilter = 1u << 2,
  kPostFilter = 1u << 3,
  kPreScore = 1u << 4,
  kScore = 1u << 5,
  kReserve = 1u << 6,
  kPermit = 1u << 7,
  kPreBind = 1u << 8,
  kBind = 1u << 9,
  kPostBind = 1u << 10,
};
const char* ext_point_name(uint32_t p);
uint32_t ext_point_from_name(const std::string& n);  // "filter" -> kFilter (0 if unknown)

// Writes that plugins/scheduler issue against the API server.
class ApiClient {
 public:
  virtual ~ApiClient() = default;
  virtual void bind(const Pod& pod, const std::string& node, const Json& annotations) = 0;
  virtual void delete_pod(const Pod& pod) = 0;
  virtual void patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) = 0;
  virtual void record_event(const std::string& kind, const std::string& ns, const std::string& name,
                            const std::string& type, const std::string& reason, const std::string& msg) {}
};

// Everything a plugin can reach (framework.Handle).
class Extender;  // scheduler/extender.h

struct Handle {
  Framework* framework = nullptr;
  SchedulerCache* cache = nullptr;
  Informers* informers = nullptr;
  ApiClient* client = nullptr;
  WaitingPods* waiting_pods = nullptr;
  Parallelizer* parallelizer = nullptr;
  Nominator* nominator = nullptr;
  std::shared_ptr<Clock> clock;
  TimerService* timers = nullptr;
  Metrics* metrics = nullptr;
  const Snapshot* snapshot = nullptr;  // the scheduling cycle's snapshot
  const GpuNames* gpu_names = &default_gpu_names();  // the scheduler's (types.h)
  // Moves these pods (when queued as unschedulable or backing off) to the
  // active queue; callable from any thread (e.g. a plugin's timer).
  std::function<void(const std::vector<PodPtr>&)> activate;
  // Parks these pods out of the scheduling queues until activate()
  // (SchedulingQueue::deactivate); callable from any thread.
  std::function<void(const std::vector<PodPtr>&)> deactivate;
  // Coscheduling denied `member`'s group (`why`: postfilter | unreserve |
  // minresources); the scheduler keeps a diagnostic record. Optional.
  std::function<void(const Pod& member, const char* why)> gang_denied;
  // Coscheduling parked `member`'s group (transient GPU shortage). Optional.
  std::function<void(const Pod& member)> gang_parked;
  // xGMI gang co-location state of this profile (scheduler/gang_placement.h):
  // NodeResourceTopologyMatch sets its mode and plans each rank's node set;
  // Coscheduling's gate asks it in Required mode.
  GangPlacement* gangs = nullptr;
  // The first rank of `member`'s gang was planned: could one node take the
  // whole gang at that moment (the gang record's `hostable`)? Optional.
  std::function<void(const Pod& member, bool hostable)> gang_planned;
  // Bracket a long wait inside a binding-cycle extension point (PreBind):
  // the binder pool adds a worker for the duration, so waiting pods cannot
  // starve the bindings of unrelated pods. Optional.
  std::function<void()> blocking_begin, blocking_end;
  // HTTP extenders of the configuration (preemption's callExtenders) and the
  // informer store's objects they are sent.
  const std::vector<std::shared_ptr<Extender>>* extenders = nullptr;
  std::function<JsonPtr(const std::string& kind, const std::string& ns, const std::string& name)> lookup;
};

class Plugin {
 public:
  explicit Plugin(std::string name, uint32_t points)
      : name_(std::move(name)), name_ptr_(&Status::intern_plugin(name_)), points_(points) {}
  virtual ~Plugin() = default;
  const std::string& name() const { return name_; }
  const std::string* name_ptr() const { return name_ptr_; }  // interned
  uint32_t points() const { return points_; }

  // QueueSort
  virtual bool less(const QueuedPodInfo& a, const QueuedPodInfo& b) const { return false; }
  // PreFilter (+ extensions used by preemption dry-runs)
  virtual Status pre_filter(CycleState& s, const Pod& p) { return {}; }
  virtual bool has_pre_filter_extensions() const { return false; }
  virtual Status add_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_add, const NodeInfo& ni) {
    return {};
  }
  virtual Status remove_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_remove, const NodeInfo& ni) {
    return {};
  }
  // False when AddPod/RemovePod of `other` leaves this plugin's PreFilter
  // state for `to_schedule` unchanged. The framework then skips the call, and
  // when no plugin is affected it evaluates nominated pods and preemption
  // dry runs against the cycle's own state instead of a deep clone of it.
  // Must only read `s`.
  virtual bool pre_filter_extension_affects(const CycleState& s, const Pod& to_schedule, const Pod& other) const {
    return true;
  }
  // Filter
  virtual Status filter(CycleState& s, const Pod& p, const NodeInfo& ni) { return {}; }
  // True when this plugin's Filter passes every node for p (e.g. a volume
  // plugin and a pod without volumes): the framework then skips the call for
  // the whole cycle (the PreFilterResult "Skip" of later upstream).
  virtual bool skip_filter(const Pod& p) const { return false; }
  // PostFilter
  virtual std::pair<PostFilterResult, Status> post_filter(CycleState& s, const Pod& p, const NodeStatusMap& m) {
    return {PostFilterResult{}, Status(Code::Unschedulable)};
  }
  // PreScore / Score
  virtual Status pre_score(CycleState& s, const Pod& p, const NodeList& nodes) { return {}; }
  virtual std::pair<int64_t, Status> score(CycleState& s, const Pod& p, const NodeInfo& ni) { return {0, {}}; }
  // Raw scores of every node whose `skip` entry is 0 (skip may be null) into
  // out[i].score, on the calling thread. `pos` (may be null) holds each
  // node's snapshot position. The default calls score() per node; plugins
  // with per-cycle state override it to read that state once.
  virtual Status score_many(CycleState& s, const Pod& p, const NodeList& nodes, const char* skip,
                            std::vector<NodeScore>& out, const int* pos = nullptr) {
    for (size_t i = 0; i < nodes.size(); ++i) {
      if (skip && skip[i]) continue;
      auto [sc, st] = score(s, p, *nodes[i]);
      if (!st.is_success()) return st;
      out[i].score = sc;
    }
    return {};
  }
  virtual bool has_normalize_score() const { return false; }
  virtual Status normalize_score(CycleState& s, const Pod& p, std::vector<NodeScore>& scores) { return {}; }
  // Reserve
  virtual Status reserve(CycleState& s, const PodPtr& p, const std::string& node) { return {}; }
  virtual void unreserve(CycleState& s, const PodPtr& p, const std::string& node) {}
  // Permit: (status, timeout_us) — Wait requests a timeout.
  virtual std::pair<Status, int64_t> permit(CycleState& s, const PodPtr& p, const std::string& node) {
    return {Status(), 0};
  }
  // Binding cycle
  virtual Status pre_bind(CycleState& s, const PodPtr& p, const std::string& node) { return {}; }
  virtual Status bind(CycleState& s, const PodPtr& p, const std::string& node) { return Status(Code::Skip); }
  virtual void post_bind(CycleState& s, const PodPtr& p, const std::string& node) {}
  // Equivalence-cache contract (scheduler.cc eq-cache). True when this
  // plugin's Filter verdict / raw Score for `p` on a node is a function of the
  // pod's template (Pod::template_hash) and that NodeInfo's content (its
  // generation) alone, for the snapshot's node epoch. Plugins that read
  // cluster-wide, time-varying or cross-pod state for this pod return false.
  virtual bool filter_node_local(const Pod& p, const Snapshot& s) const { return false; }
  virtual bool score_node_local(const Pod& p, const Snapshot& s) const { return false; }
  // True when this plugin's raw Score is 0 on every node for this pod (e.g.
  // NodeAffinity without preferred terms). The framework then skips the
  // plugin's Score and NormalizeScore for the cycle: its normalized output is
  // the same on every node, so node ranking and selectHost are unchanged.
  // Not applied when a per-plugin breakdown is requested (explain).
  virtual bool score_all_zero(const Pod& p, const Snapshot& s) const { return false; }
  // The normalized score every node gets when the raw scores are all 0: 0 for
  // min-max/plain normalizers, kMaxNodeScore for reversed ones
  // (TaintToleration's DefaultNormalizeScore(reverse), PodTopologySpread). A
  // skipped plugin still adds this x weight to every total, so hot-path
  // totals equal explain() totals.
  virtual int64_t score_skip_value() const { return 0; }
  // NormalizeScore reads NodeScore::name (not just scores). The framework's
  // reused score rows carry names only for plugins that ask for them.
  virtual bool normalize_uses_names() const { return false; }
  // EnqueueExtensions
  virtual std::vector<ClusterEvent> events_to_register() const { return {}; }
  // Informer hooks (plugins that maintain their own state from watch events,
  // e.g. CapacityScheduling's ElasticQuota infos, Trimaran's pod-assign cache).
  virtual void on_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr& old) {}
  virtual std::vector<std::string> watched_kinds() const { return {}; }
  // Resources were released somewhere in the cluster: an assigned or assumed
  // pod left a node, or a node joined or grew. Delivered (from informer and
  // binder threads, so it must be cheap and thread-safe) to plugins whose
  // wants_capacity_events() is true, e.g. Coscheduling re-probing parked gangs.
  virtual bool wants_capacity_events() const { return false; }
  virtual void capacity_freed() {}
  // Periodic work registered at start (metrics refresh, cache cleanup).
  virtual void start() {}
  virtual void stop() {}
  // Unit-test hook for plugin internals that are not an extension point
  // (Scheduler::plugin_call; e.g. Coscheduling "checkClusterResource",
  // CapacityScheduling "dryRunPreemption"). Returns {"error": ...} when unknown.
  virtual Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) {
    Json out = Json::object();
    out.set("error", Json(name() + " has no debug call " + what));
    return out;
  }

 protected:
  std::string name_;
  const std::string* name_ptr_;
  uint32_t points_;
};
using PluginPtr = std::shared_ptr<Plugin>;

using PluginFactory = std::function<PluginPtr(const Json& args, Handle& handle)>;

class Registry {
 public:
  static Registry& global();
  void add(const std::string& name, PluginFactory f);
  bool has(const std::string& name) const { return factories_.count(name) > 0; }
  PluginPtr make(const std::string& name, const Json& args, Handle& h) const;
  std::vector<std::string> names() const;

 private:
  std::unordered_map<std::string, PluginFactory> factories_;
};

// Static registration helper: XSCHED_REGISTER_PLUGIN(Name, factory).
struct PluginRegistrar {
  PluginRegistrar(const std::string& name, PluginFactory f) { Registry::global().add(name, std::move(f)); }
};
void register_builtin_plugins();  // force-link all plugin translation units

// DefaultNormalizeScore (vendor/.../plugins/helper/normalize_score.go:26-54).
void default_normalize_score(int64_t max_priority, bool reverse, std::vector<NodeScore>& scores);

}  // namespace xsched
