// The scheduler: informer ingestion, the serialized scheduling cycle and the
// asynchronous binding cycle.
//
// Reference call stacks: SURVEY.md §3.1-3.3, i.e. vendor/k8s.io/kubernetes/
// pkg/scheduler/scheduler.go:425-638 (scheduleOne), generic_scheduler.go:93-426
// (findNodesThatFitPod / prioritizeNodes / selectHost, numFeasibleNodesToFind
// with the 100-node minimum :47), eventhandlers.go (informer → cache/queue).
//
// Threads: one informer thread (store watch → informers/cache/queue), one
// scheduling thread, a binding executor pool (Permit waits are continuations,
// not blocked threads), the timer service, and the Filter/Score parallelizer.
#pragma once

#include "common/adaptive_mutex.h"

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common/clock.h"
#include "common/parallel.h"
#include "framework/framework.h"
#include "scheduler/cache.h"
#include "scheduler/extender.h"
#include "scheduler/gang_placement.h"
#include "scheduler/informers.h"
#include "scheduler/metrics.h"
#include "scheduler/queue.h"
#include "scheduler/trace.h"
#include "store/store.h"

namespace xsched {

// ApiClient backed by the in-process ObjectStore.
class StoreClient : public ApiClient {
 public:
  explicit StoreClient(std::shared_ptr<ObjectStore> s) : store_(std::move(s)) {}
  void bind(const Pod& pod, const std::string& node, const Json& annotations) override;
  void delete_pod(const Pod& pod) override;
  void patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) override;
  void record_event(const std::string& kind, const std::string& ns, const std::string& name, const std::string& type,
                    const std::string& reason, const std::string& msg) override;
  bool events_enabled = false;

 private:
  std::shared_ptr<ObjectStore> store_;
  // client-go's EventCorrelator aggregation: the same (object, reason,
  // message) within kAggregateUs bumps count/lastTimestamp of the existing
  // Event instead of creating another (a pod failing for the same reason on
  // every retry is one Event with a count, as upstream).
  static constexpr int64_t kAggregateUs = 600LL * 1000000;
  struct Recent {
    std::string ns, name;  // the Event object
    int64_t count = 0, last_us = 0;
  };
  std::mutex events_mu_;
  std::unordered_map<std::string, Recent> recent_;
  size_t recent_sweep_at_ = 4096;
};

// Bounded worker pool for binding cycles.
class Executor {
 public:
  explicit Executor(int threads);
  ~Executor();
  void submit(std::function<void()> fn);
  // While a Batch is alive, submit() calls from its thread to this executor
  // are collected and handed over under one lock with one wake-up when it
  // ends (a gang's Allows fire k binding cycles from one Permit call).
  class Batch {
   public:
    explicit Batch(Executor& e);
    ~Batch();
    Batch(const Batch&) = delete;
    Batch& operator=(const Batch&) = delete;

   private:
    friend class Executor;
    Executor& e_;
    Batch* prev_;
    std::vector<std::function<void()>> fns_;
  };
  void stop();
  size_t pending() const;
  // A task about to block for a long time (VolumeBinding's PreBind waiting
  // for the PV controller) brackets the wait with these, so blocked tasks
  // never take the pool's last runnable workers (BlockingScope below).
  void enter_blocking();
  void exit_blocking();
  size_t threads() const;

 private:
  // A worker that finishes a task spins briefly on `queued_` before it
  // sleeps, and submit() skips the futex wake while a spinning worker can
  // take the task: under load the scheduling thread hands bindings over
  // without a syscall.
  static constexpr int64_t kSpinNs = 30'000;  // XSCHED_BIND_SPIN_NS overrides (A/B runs)
  static constexpr int kMaxSpinners = 2;
  int64_t spin_ns_ = kSpinNs;
  bool try_pop(std::function<void()>& fn);  // under mu_
  void spawn_locked();
  static constexpr size_t kMaxThreads = 1024;
  int base_ = 1;
  int blocked_ = 0;  // under mu_
  mutable AdaptiveMutex mu_;
  std::condition_variable_any cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> threads_;
  bool stop_ = false;
  std::atomic<int> busy_{0};
  std::atomic<int> queued_{0};
  std::atomic<int> spinners_{0};
  int waiters_ = 0;  // workers in cv_.wait (under mu_)
  int wakes_ = 0;    // notifications sent and not yet consumed by a waking worker (under mu_)
};

struct SchedulerOptions {
  int parallelism = 16;
  int parallel_inline_below = 128;  // node count under which Filter/Score run on the scheduling thread
  int bind_workers = 16;
  int percentage_of_nodes_to_score = 0;
  int64_t pod_initial_backoff_us = 1'000'000;
  int64_t pod_max_backoff_us = 10'000'000;
  int64_t assumed_pod_ttl_us = 15LL * 60 * 1'000'000;
  double metrics_sample_rate = 0.1;  // fraction of cycles with per-extension-point metrics
  bool status_updates = true;        // PodScheduled=False condition patches on failure
  bool events = true;                // FailedScheduling / Preempted events (in-process StoreClient)
  bool equivalence_cache = true;     // reuse node-local Filter/Score results across a pod template
  // Gang ranks share the first rank's node window (find_nodes_that_fit) and a
  // template's last Filter scan is updated instead of repeated (EqEntry::scan).
  // Defaults: on, unless XSCHED_GANG_WINDOW / XSCHED_SCAN_MEMO is "0" (A/B runs).
  bool gang_window = true;
  bool scan_memo = true;
  // Testing: every scan the memo answers is repeated in full and compared
  // (Stats::scan_memo_mismatches).
  bool scan_memo_verify = false;
  bool trace = false;
  uint64_t seed = 0;
  // Debugging: on the first fit error, write the cache and queue (the cache
  // debugger's dump) and the failing pod's diagnosis to this file.
  std::string dump_on_fit_error;
  // Gang-denial records also list every bound pod from the store (the
  // "stale_cache" cause); off by default: it costs O(pods) per denial.
  bool gang_denial_census = false;
  static SchedulerOptions from_json(const Json& j);
};

struct GangRecord {
  std::string pg;  // ns/name
  int size = 0;
  int bound = 0;
  int64_t first_enqueue_us = 0;
  int64_t admit_us = 0;   // last member allowed at Permit
  int64_t bound_us = 0;   // last member bound
  // Placement: distinct nodes the bound members landed on (hashes of their
  // names), and whether one node could take the whole gang when its first
  // rank was planned (-1: not planned, e.g. no GPU ranks or co-location off).
  std::vector<uint64_t> nodes;
  int hostable = -1;
};

// One Coscheduling group denial with the GPU census at that moment
// (Scheduler::note_gang_denied). store_* are -1 without an in-process store.
struct GangDenial {
  std::string pg, why, cause;
  int64_t t_us = 0;
  int min_member = 0, assigned = 0;
  int64_t need_gpus = 0;  // whole GPUs per member
  int cache_free = 0, cache_max_node_free = 0, assumed_held = 0;
  int store_free = -1, store_max_node_free = -1;
  int waiting_at_permit = 0, in_binding = 0;  // assumed pods by stage
};

class Scheduler {
 public:
  // config JSON: {"profiles":[...ProfileConfig...], "options":{...}}
  Scheduler(std::shared_ptr<ObjectStore> store, const Json& config, std::shared_ptr<Clock> clock = nullptr,
            std::shared_ptr<ApiClient> client = nullptr);
  ~Scheduler();

  void start();  // informer + scheduling threads
  void stop();
  // Synchronously drain pending watch events (tests / deterministic drivers).
  size_t sync_informers(int timeout_ms = 0);
  // Run exactly one scheduling cycle on the calling thread (tests). Returns
  // false when the queue was empty within timeout.
  bool schedule_one(int timeout_ms = 0);
  // Wait until no pod is in activeQ/backoff, no binding is in flight and no
  // pod waits at Permit, or timeout. Returns true when idle.
  bool wait_idle(int timeout_ms);
  // Dry-run one scheduling cycle for `pod` (no assume/bind): filter verdicts
  // per node, per-plugin normalized scores and the host that would be chosen.
  Json explain(const Json& pod);
  // Cache debugger (upstream internal/cache/debugger, SIGUSR2 in
  // kube-scheduler): the cache against the listers and the store's Nodes,
  // and a dump of cache, queue and waiting pods.
  Json check_cache() const;
  Json dump_cache() const;
  // Score micro-benchmark (the reference's BenchmarkTargetLoadPackingPlugin,
  // pkg/trimaran/targetloadpacking/targetloadpacking_test.go:267-360):
  // PreScore + node-parallel Score + NormalizeScore of `pod` over every node
  // of the snapshot, `iterations` times. Returns the mean microseconds per
  // pass (and the node count / a checksum of the totals in `out`).
  double score_benchmark(const Json& pod, int iterations, Json* out = nullptr);
  // Plugin unit-test harness (the reference's per-plugin *_test.go tables):
  // runs one extension point of one plugin of the first profile for
  // args["pod"] against the current cache snapshot, on the calling thread,
  // with a fresh CycleState. `point`: less | preFilter | postFilter | permit |
  // reserve | unreserve | postBind, or a plugin debug call (args["runPreFilter"]
  // runs the profile's PreFilter plugins first). Returns {"code", "message", ...}.
  Json plugin_call(const std::string& plugin, const std::string& point, const Json& args);

  SchedulingQueue& queue() { return *queue_; }
  SchedulerCache& cache() { return *cache_; }
  Informers& informers() { return *informers_; }
  Metrics& metrics() { return *metrics_; }
  Tracer& tracer() { return tracer_; }
  TimerService& timers() { return *timers_; }
  Framework* framework_for(const std::string& scheduler_name);
  const std::vector<std::unique_ptr<Framework>>& frameworks() const { return frameworks_; }
  std::shared_ptr<Clock> clock() const { return clock_; }
  std::shared_ptr<ObjectStore> store() const { return store_; }

  struct Stats {
    uint64_t attempts = 0, scheduled = 0, unschedulable = 0, errors = 0, bound = 0, bind_failures = 0;
    uint64_t preemption_attempts = 0;
    uint64_t eq_filter_hits = 0, eq_filter_misses = 0;  // equivalence-cache Filter lookups
    uint64_t scan_memo_served = 0, scan_memo_mismatches = 0;  // EqEntry::scan answers (and failed checks)
  };
  Stats stats() const;
  // Blocks (without the Python lock, from the bindings) until `target`
  // pods have been bound in total / the cache holds no pod; false on timeout.
  bool wait_bound(uint64_t target, int64_t timeout_us) const;
  bool wait_cache_empty(int64_t timeout_us) const;
  std::vector<GangRecord> gang_records(bool clear = false);
  // Group denials since the last clear (the first kMaxGangDenials with
  // their census; `total` counts all of them).
  std::vector<GangDenial> gang_denials(bool clear = false, uint64_t* total = nullptr);
  // Groups Coscheduling parked (transient GPU shortage) since the last clear.
  uint64_t gang_parks(bool clear = false);
  size_t inflight_bindings() const { return inflight_.load(); }
  size_t bind_threads() const { return binder_ ? binder_->threads() : 0; }
  // Pods waiting at Permit (every profile) and binding cycles queued for the
  // binders (the open-loop driver's timeline).
  size_t permit_waiting() const {
    size_t n = 0;
    for (const auto& w : waiting_) n += w->size();
    return n;
  }
  size_t bind_backlog() const { return binder_ ? binder_->pending() : 0; }
  // Seconds since the scheduling loop last ticked (it ticks at least every
  // 100 ms while running; /healthz uses this). 0 before start().
  double loop_age_seconds() const;

 private:
  struct ScheduleResult {
    std::string host;
    int evaluated = 0, feasible = 0;
  };
  struct Diagnosis {
    NodeStatusMap node_to_status;
    std::set<std::string> unschedulable_plugins;
  };
  // Equivalence cache for one (profile, pod template): a slot per snapshot
  // node position, valid for one node epoch (node set / Node objects).
  struct EqEntry {
    uint64_t epoch = 0;
    EqTable table;
    // The last serial Filter scan of this template (find_nodes_that_fit):
    // per scan offset from `start`, the node version it saw and its verdict.
    struct ScanMemo {
      bool valid = false;
      int start = 0, n = 0, to_find = 0, processed = 0;
      uint64_t epoch = 0;
      std::vector<int64_t> gens;
      std::vector<char> ok;
    } scan;
  };
  EqEntry* eq_entry(Framework& fw, const Pod& p);
  void release_retired();
  std::mutex retired_spare_mu_;
  std::vector<std::vector<NodeInfoPtr>> retired_spare_;  // emptied retired batches, capacity kept
  std::vector<Status> fail_buf_;  // find_nodes_that_fit scratch (scheduling thread)
  std::vector<char> nom_mark_;    // nodes with nominated pods, per snapshot position (refresh_nom_mark)
  std::vector<const std::vector<PodPtr>*> nom_list_;  // ... and their lists in the view (valid for the cycle)
  std::vector<std::string> nom_changed_;
  const NominatedMap* nom_src_ = nullptr;  // the view nom_mark_ describes
  uint64_t nom_epoch_ = UINT64_MAX;
  bool nom_mark_valid_ = false;
  void refresh_nom_mark(const NominatedMap* view);
  std::vector<const Status*> fail_ptr_;
  static constexpr size_t kInformerWindow = 64;
  size_t informer_window_ = kInformerWindow;  // XSCHED_INFORMER_WINDOW overrides (A/B runs)
  ParallelSite filter_site_;  // inline-vs-parallel cost model of Filter
  // Per-profile metric cells of the scheduling cycle, cached per metrics
  // epoch (scheduling thread / sched_mu_ only).
  struct CycleMetrics {
    uint64_t epoch = ~0ULL;
    Histogram* algo = nullptr;
    Histogram* e2e = nullptr;
    Histogram* attempt[3] = {};  // scheduled, unschedulable, error
    Counter* attempts[3] = {};
  };
  std::unordered_map<const Framework*, CycleMetrics> cycle_metrics_;
  CycleMetrics& cycle_metrics(const Framework& fw);
  // Binding-cycle histograms shared by the binder threads: looked up once
  // per metrics epoch (under bind_metrics_mu_), then read lock-free. Cells
  // are never freed (Metrics::reset retires them), so a stale pointer read
  // across a reset only loses that observation.
  struct BindMetrics {
    std::atomic<uint64_t> epoch{~0ULL};
    std::atomic<Histogram*> binding{nullptr}, attempts{nullptr};
    std::atomic<Histogram*> permit_wait[2] = {nullptr, nullptr};  // Success, Unschedulable
    std::atomic<Histogram*> pod_duration[8] = {};                  // attempts=1..8
  };
  BindMetrics bind_metrics_;
  std::mutex bind_metrics_mu_;
  BindMetrics& bind_metrics();

  void informer_loop();
  void handle_event(const WatchEvent& ev);
  void handle_pod_event(const WatchEvent& ev);
  // A run of pod Deleted events (a DeleteCollection, a wave torn down):
  // lister and cache updated under one lock each, one cluster event.
  void handle_pod_deletes(const WatchEvent* evs, size_t n);
  PodPtr deleted_pod(const WatchEvent& ev);
  void forget_unassigned_pod(const Pod& p);
  // Resources were released (pod deleted or forgotten, node added or grown):
  // tells the plugins that asked (Plugin::capacity_freed).
  void capacity_freed();
  void report_informer_error(const WatchEvent& ev, const char* what);
  void handle_parsed_pod_event(const WatchEvent& ev, const PodPtr& np, PodPtr old);
  PodPtr bound_copy_of_assumed(const WatchEvent& ev);
  // A status-only Modified event (WatchEvent::status_only) of the version the
  // lister holds: that Pod copied with the new status fields, no parse.
  PodPtr status_copy_of_listed(const WatchEvent& ev);
  // bound_copy_of_assumed, else status_copy_of_listed (nullptr: parse).
  PodPtr copy_for_modified(const WatchEvent& ev) {
    PodPtr p = bound_copy_of_assumed(ev);
    return p ? p : status_copy_of_listed(ev);
  }
  void apply_pod_update(const WatchEvent& ev, const PodPtr& np, PodPtr old);
  void handle_node_event(const WatchEvent& ev);
  void scheduling_loop();
  void schedule_cycle(const QueuedPodInfoPtr& qpi);
  // `feasible_pos` (optional) receives each feasible node's snapshot position.
  Status find_nodes_that_fit(Framework& fw, CycleState& s, const Pod& p, Diagnosis& d, NodeList& feasible,
                             EqEntry* eq = nullptr, bool full_diagnosis = false, std::vector<int>* feasible_pos = nullptr);
  int num_feasible_nodes_to_find(Framework& fw, int n) const;
  // Filter over a PreFilter node set given as a short position list (the
  // nodes hosting a gang): only those nodes are evaluated; the others get
  // the set's `excluded` verdict in the diagnosis.
  Status filter_listed(Framework& fw, CycleState& s, const Pod& p, Diagnosis& d, NodeList& feasible, EqEntry* eq,
                       const NodeRestriction& rs, std::vector<int>* feasible_pos, bool ext);
  // findNodesThatPassExtenders: interested filter extenders narrow
  // `feasible` (and `pos`) in order; their failures join the diagnosis.
  Status run_extender_filters(const Pod& p, NodeList& feasible, std::vector<int>* pos, Diagnosis& d);
  // Extender priorities x weight x (MaxNodeScore / MaxExtenderPriority)
  // added to the plugin totals; errors are ignored as upstream does.
  void add_extender_scores(const Pod& p, const NodeList& feasible, std::vector<NodeScore>& scores,
                           Json* breakdown = nullptr);
  bool extenders_interested(const Pod& p) const;
  Json pod_object(const Pod& p) const;  // the informer store's Pod (what extenders receive)
  // Index of the highest total (reservoir-sampled among ties).
  size_t select_host(const std::vector<NodeScore>& scores);
  // Cycle scratch reused across cycles (scheduling thread only).
  NodeList feasible_buf_;
  std::vector<const NodeInfo*> found_buf_;
  std::vector<int> found_pos_buf_;
  std::vector<int> feasible_pos_buf_;
  std::vector<NodeScore> scores_buf_;
  EqScoreCache esc_buf_;
  // Everything the binding cycle of one assumed pod needs, in one heap
  // object: the Permit continuation and the binder task capture only this
  // pointer (fits std::function's inline buffer, no per-closure allocation).
  struct BindTask {
    Scheduler* self = nullptr;
    Framework* fw = nullptr;
    CycleStatePtr state;
    QueuedPodInfoPtr qpi;
    PodPtr assumed;
    std::string host;
    int64_t cycle = 0;
    int64_t permit_start_us = 0;
    std::shared_ptr<PodsToActivate> to_activate;
    Histogram* e2e = nullptr;  // scheduler_e2e_scheduling_duration_seconds{profile}
    Status permit_status;      // set by the Permit waiter before the task is queued
    // The task owns itself until its binding cycle starts, so the Permit
    // callback and the binder queue hold a raw pointer: a one-pointer capture
    // is stored inside std::function, without a heap block per pod.
    std::shared_ptr<BindTask> keep;
  };
  static void run_bind_task(BindTask* t);
  void binding_cycle(const BindTask& t, const Status& permit_status);
  void handle_failure(Framework& fw, const QueuedPodInfoPtr& qpi, const Status& st, const std::string& reason,
                      const std::string& nominated, int64_t cycle, const std::set<std::string>& plugins);
  void note_gang_enqueue(const Pod& p, int64_t t);
  void note_gang_event(const Pod& p, bool bound);
  void note_gang_planned(const Pod& p, bool hostable);
  void note_gang_denied(const Pod& p, const char* why);
  bool responsible_for(const Pod& p) const;

  std::shared_ptr<ObjectStore> store_;
  std::shared_ptr<Clock> clock_;
  SchedulerOptions opts_;
  std::unique_ptr<TimerService> timers_;
  std::unique_ptr<Parallelizer> parallelizer_;
  // Informer windows parse their pods' JSON on a few helpers ("xs-parse").
  std::unique_ptr<Parallelizer> parse_pool_;
  ParallelSite parse_site_;
  std::unique_ptr<Metrics> metrics_;
  std::unique_ptr<SchedulerCache> cache_;
  std::unique_ptr<Informers> informers_;
  std::unique_ptr<Nominator> nominator_;
  std::unique_ptr<SchedulingQueue> queue_;
  std::shared_ptr<ApiClient> client_;
  ExtenderList extenders_;
  std::shared_ptr<const GpuNames> gpu_names_;  // from the profiles' FlexGPU args
  std::vector<std::unique_ptr<WaitingPods>> waiting_;
  std::vector<std::unique_ptr<GangPlacement>> gang_placements_;  // one per profile (Handle::gangs)
  std::vector<std::unique_ptr<Framework>> frameworks_;
  std::unordered_map<std::string, Framework*> by_name_;
  std::unique_ptr<Executor> binder_;
  // FailedScheduling events: one FIFO worker, off the scheduling loop.
  std::unique_ptr<Executor> status_writer_;
  Snapshot snapshot_;
  Tracer tracer_;
  WatcherPtr watcher_;
  std::vector<std::string> plugin_kinds_;

  std::thread informer_thread_, sched_thread_;
  std::atomic<bool> running_{false};
  std::mutex sched_mu_;  // serializes scheduling cycles (loop vs schedule_one)
  std::atomic<int> inflight_{0};
  std::atomic<int> in_cycle_{0};
  std::atomic<int64_t> loop_tick_us_{0};  // RealClock time of the last loop iteration
  int next_start_node_ = 0;
  // Node window shared by consecutive members of one gang and template
  // (find_nodes_that_fit; scheduling thread only).
  uint64_t window_gang_ = 0, window_tmpl_ = 0;
  int window_start_ = 0, window_n_ = -1;
  std::mt19937_64 rng_;
  std::vector<uint64_t> timer_ids_;
  std::unordered_map<Framework*, std::unordered_map<uint64_t, std::unique_ptr<EqEntry>>> eq_;  // scheduling thread only

  mutable std::mutex stats_mu_;  // gang records and denials, condition memo
  // Stats counters: relaxed atomics, bumped by the scheduling, binding and
  // informer threads without a shared lock.
  struct Counters {
    std::atomic<uint64_t> attempts{0}, scheduled{0}, unschedulable{0}, errors{0}, bound{0}, bind_failures{0};
    std::atomic<uint64_t> preemption_attempts{0}, eq_filter_hits{0}, eq_filter_misses{0};
    std::atomic<uint64_t> scan_memo_served{0}, scan_memo_mismatches{0};
  } cnt_;
  std::atomic<uint64_t> bound_total_{0};  // bound pods, released for wait_bound (cnt_.bound counts the same)
  std::atomic<bool> fit_error_dumped_{false};  // dump_on_fit_error written
  std::unordered_map<std::string, GangRecord> gangs_;  // open groups
  // Completed gangs until a caller collects them: a deque, so the push on a
  // binding thread (under stats_mu_) never moves the records already there
  // (a benchmark collects ~10^5 of them at once).
  std::deque<GangRecord> gang_done_;
  std::unordered_map<int, Histogram*> gang_hist_;  // xsched_gang_admit_seconds{size} (under stats_mu_)
  uint64_t gang_hist_epoch_ = ~0ULL;
  static constexpr size_t kMaxGangDenials = 256;
  std::vector<GangDenial> gang_denials_;
  uint64_t gang_denials_total_ = 0;
  std::atomic<uint64_t> gang_parks_total_{0};
};

}  // namespace xsched
