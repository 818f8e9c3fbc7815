// Scheduler cache: NodeInfos with assumed pods, incremental snapshots.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/internal/cache/cache.go
// (AssumePod :350, FinishBinding, ForgetPod, AddPod confirming an assumed pod,
// UpdateSnapshot with generation tracking) and the 15-minute assumed-pod TTL
// (vendor/.../scheduler.go:62).
//
// Differences by design:
//  * dirty-node tracking instead of a generation-ordered linked list: a
//    snapshot refresh clones exactly the NodeInfos touched since the last one;
//  * per-PodGroup assigned counters (O(1) instead of Coscheduling's
//    O(nodes x pods) CalculateAssignedPods scan, core.go:301-318);
//  * assumed-pod updates (FlexGPU's GPU index) are copy-on-write so Filter
//    workers reading an older snapshot never race with Reserve/Unreserve.
#pragma once

#include "common/adaptive_mutex.h"

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "common/clock.h"
#include "common/json.h"
#include "framework/types.h"

namespace xsched {

class SchedulerCache {
 public:
  SchedulerCache(std::shared_ptr<Clock> clock, int64_t assumed_ttl_us);
  // The owning scheduler's GPU names (re-deriving a mutated pod's GPU
  // assignment); must outlive the cache.
  void set_gpu_names(const GpuNames* gn) { gpu_names_ = gn; }

  void add_node(const NodePtr& n);
  void update_node(const NodePtr& n);
  void remove_node(const std::string& name);
  void set_nrt(const std::string& node, const NRTPtr& nrt);  // nullptr clears

  void add_pod(const PodPtr& p);  // assigned pod observed by the informer
  void update_pod(const PodPtr& old_pod, const PodPtr& new_pod);
  void remove_pod(const Pod& p);
  void remove_pods(const std::vector<PodPtr>& ps);  // one lock for a run of deletions

  // p->node_name must be set. Called by the scheduling thread between cycles
  // (Scheduler holds sched_mu_): the node's NodeInfo is updated in place even
  // while the scheduler's own Snapshot shares it — no Filter/Score worker is
  // running and no other thread reads snapshot NodeInfos — which saves a
  // NodeInfo copy per scheduled pod (and its release on a binder thread).
  // Every other writer (informer, binder) still copies on write.
  Status assume_pod(const PodPtr& p);
  void finish_binding(const Pod& p);
  void forget_pod(const Pod& p);
  bool is_assumed(const std::string& uid) const;
  PodPtr get_pod(const std::string& uid) const;
  // Copy-on-write mutation of a cached (assumed or bound) pod; re-accounts
  // the pod on its node. Returns the new object (nullptr if not cached).
  PodPtr mutate_pod(const std::string& uid, const std::function<void(Pod&)>& fn);
  // In-place annotation of a pod assumed in the current scheduling cycle
  // (FlexGPU Reserve, scheduling thread): no other thread holds that object yet, so there is no
  // copy, and since `fn` may only change annotations, only the node's GPU
  // ledger is re-accounted (Pod::recompute_gpu_assignment). Falls back to
  // mutate_pod for pods that are not (or no longer) assumed.
  // `fn` edits the assumed pod's annotations in place; with `recompute` the
  // GPU assignment is then re-derived from them (false: fn set it).
  PodPtr annotate_assumed_pod(const std::string& uid, const std::function<void(Pod&)>& fn, bool recompute = true);

  // Returns the number of NodeInfo versions refreshed (shared, not cloned:
  // the cache copies on write); replaced versions go to `s.retired`; `lock_wait_us` (optional)
  // receives the time spent waiting for the cache lock (trace diagnostics).
  // `check_assumed` (optional): also reports, under the same lock, whether
  // that pod uid is assumed (the cycle's skipPodSchedule check).
  int update_snapshot(Snapshot& s, int64_t* lock_wait_us = nullptr, const std::string* check_assumed = nullptr,
                      bool* is_assumed = nullptr);
  void cleanup_expired_assumed_pods();

  // Pods of a PodGroup that are assumed or bound, keyed by Pod::pg_key (a
  // 64-bit hash of "ns/name", as NodeInfo::pg_count).
  int assigned_in_group(uint64_t pg_key) const;
  // Nodes hosting assumed or bound pods of the group (by Pod::pg_key).
  std::vector<std::string> nodes_of_group(uint64_t pg_key) const;
  // Both of the above under one lock, into `hosts` (resized; its strings'
  // buffers are reused, so a caller's thread_local vector allocates nothing
  // in steady state). Returns the assigned count.
  int group_placement(uint64_t pg_key, std::vector<std::string>& hosts) const;
  int assigned_in_group(const std::string& pg_full_name) const { return assigned_in_group(pg_key_of(pg_full_name)); }
  // Cache debugger (upstream internal/cache/debugger): compares the cache
  // with the listers' view — `assigned` pods (nodeName set) and Node names —
  // and re-derives every NodeInfo's accounting and the PodGroup counts from
  // the pods. Returns {"clean": bool, "missing_pods", "redundant_pods",
  // "wrong_node", "missing_nodes", "redundant_nodes", "accounting",
  // "group_counts", "assumed"}. Transient differences are expected while
  // events are in flight.
  Json check(const std::vector<PodPtr>& assigned, const std::vector<std::string>& nodes) const;
  // Per node: pods, requested resources and GPU availability (upstream
  // CacheDumper), plus assumed pods.
  Json dump() const;
  size_t node_count() const;
  size_t pod_count() const;
  size_t assumed_count() const;
  NodeInfoPtr node_info_copy(const std::string& name) const;
  // Whole-GPU (SPX) census per node for gang-denial diagnostics: SPX GPUs,
  // free ones, and those held by assumed (not yet bound) pods.
  struct GpuCensusRow {
    std::string node;
    int spx = 0, free_whole = 0, assumed_whole = 0;
  };
  std::vector<GpuCensusRow> gpu_census() const;
  std::vector<std::string> node_names() const;

 private:
  struct PodState {
    PodPtr pod;
    int64_t deadline_us = 0;
    bool binding_finished = false;
  };
  // Bind confirmation of an assumed pod whose informer object accounts the
  // same on its node: records it without touching the NodeInfo (no copy, no
  // generation bump). False when the node must be re-accounted.
  bool confirm_assumed_locked(std::unordered_map<std::string, PodState>::iterator it, const PodPtr& p);
  NodeInfoPtr& info_for(const std::string& node);  // creates a ghost entry
  NodeInfo& writable(NodeInfoPtr& slot);            // copy-on-write before mutating
  bool in_place_ = false;  // assume/annotate on the scheduling thread (under mu_)
  void add_pod_locked(const PodPtr& p);
  void remove_pod_locked(const PodPtr& p);
  void record_delta(const PodPtr& p, const NodeInfo& ni, int d);
  void mark_dirty(const std::string& node);
  void group_delta(const Pod& p, int d);
  void set_node_locked(const NodePtr& n);
  // Cluster-wide Node-derived counts, adjusted per Node change (old -> new)
  // instead of rescanning every node on each snapshot refresh.
  void account_node(const Node* old_node, const Node* new_node);

  std::shared_ptr<Clock> clock_;
  int64_t ttl_us_;
  const GpuNames* gpu_names_ = &default_gpu_names();
  mutable AdaptiveMutex mu_;
  std::unordered_map<std::string, NodeInfoPtr> nodes_;
  std::vector<std::string> order_;  // node names with a Node object, insertion order
  std::unordered_map<std::string, PodState> pod_states_;
  std::atomic<size_t> pod_count_{0};  // pod_states_.size(), readable without mu_
  std::unordered_set<std::string> assumed_;
  // Written under mu_ + group_mu_, read under group_mu_ only: Permit and
  // PreScore read a gang's count without waiting behind NodeInfo copies.
  mutable AdaptiveMutex group_mu_;
  std::unordered_map<uint64_t, int> group_assigned_;
  // PodGroup key -> (node, members on it): where a gang's assumed or bound
  // members sit (XGMIGangAffinity's co-location test without a per-node look).
  std::unordered_map<uint64_t, std::vector<std::pair<std::string, int>>> group_nodes_;
  std::unordered_set<std::string> dirty_;
  bool structure_changed_ = true;
  int64_t generation_ = 0;
  uint64_t node_epoch_ = 1;
  int64_t prefer_nodes_ = 0;
  std::map<int32_t, int64_t> prio_count_;  // pods on nodes per priority (Snapshot::min_pod_priority)
  int64_t foreign_hostnames_ = 0;  // nodes whose hostname label is not their name
  uint64_t topology_epoch_ = 1;     // Snapshot::topology_epoch
  std::vector<PodDelta> pending_deltas_;  // since the last snapshot refresh
  uint64_t delta_seq_ = 0;
  bool track_deltas_ = false;  // once a plugin asked (Snapshot::deltas_wanted)
  // Copied on write while a snapshot still shares it.
  std::shared_ptr<std::unordered_map<std::string, int64_t>> image_spread_ =
      std::make_shared<std::unordered_map<std::string, int64_t>>();
};

}  // namespace xsched
