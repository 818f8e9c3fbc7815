// Scheduling queue: activeQ (heap ordered by the profile's QueueSort),
// podBackoffQ (heap by backoff expiry), unschedulableQ, and the nominator.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/internal/queue/
// scheduling_queue.go (backoff 1s..10s and 60s unschedulable flush,
// :53-66; moveRequestCycle; Activate; MoveAllToActiveOrBackoffQueue with the
// clusterEventMap filter from plugins' EventsToRegister).
#pragma once

#include "common/adaptive_mutex.h"

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "common/clock.h"
#include "framework/types.h"

namespace xsched {

// Binary heap keyed by pod uid with O(log n) update/delete.
class PodHeap {
 public:
  using Less = std::function<bool(const QueuedPodInfo&, const QueuedPodInfo&)>;
  // `tag` (non-zero) is written into Pod::heap_tag of the objects this heap
  // holds, so a caller holding the same object can test membership without
  // a uid lookup (holds()).
  explicit PodHeap(Less less, uint8_t tag = 0) : less_(std::move(less)), tag_(tag) {}
  void set_less(Less l) { less_ = std::move(l); }
  void push(const QueuedPodInfoPtr& p);  // add or update
  QueuedPodInfoPtr pop();
  const QueuedPodInfoPtr& top() const { return v_.front(); }
  QueuedPodInfoPtr get(const std::string& uid) const;
  bool erase(const std::string& uid);
  bool contains(const std::string& uid) const { return pos_.count(uid) > 0; }
  // True when this very Pod object is in the heap (false does not rule out
  // another object of the same pod: use contains() for that).
  bool holds(const Pod& p) const { return tag_ != 0 && p.heap_tag.v == tag_; }
  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  std::vector<QueuedPodInfoPtr> items() const { return v_; }

 private:
  void up(size_t i);
  void down(size_t i);
  void swap_at(size_t a, size_t b);
  Less less_;
  uint8_t tag_ = 0;
  std::vector<QueuedPodInfoPtr> v_;
  std::unordered_map<std::string, QueuedPodInfo*> pos_;  // uid -> entry (index lives in the entry)
};

// Pods nominated onto nodes by preemption (PodNominator).
class Nominator {
 public:
  void add(const PodPtr& p, const std::string& node);  // node "" = use p->nominated_node_name
  void remove(const Pod& p);
  void update(const PodPtr& old_p, const PodPtr& new_p);
  std::vector<PodPtr> nominated_pods_for_node(const std::string& node) const;
  // Every nominated pod with its node, under the lock (callers needing all of
  // them: one pass over the nominations instead of a lookup per node).
  void for_each(const std::function<void(const std::string& node, const PodPtr& p)>& fn) const;
  // Every node's nominated pods for the cycle about to start. Single
  // consumer: the scheduling thread, between cycles. The view is a mirror
  // that the changes since the last call are applied to (O(changes), not a
  // copy of the map); the previous cycle's Filter workers are done with it.
  // `changed` (optional) receives the nodes whose entries this call updated.
  std::shared_ptr<const NominatedMap> view(std::vector<std::string>* changed = nullptr) const;
  std::string nominated_node(const std::string& uid) const;
  size_t size() const;
  bool empty() const { return count_.load(std::memory_order_relaxed) == 0; }  // lock-free fast path

 private:
  std::atomic<size_t> count_{0};
  mutable std::mutex mu_;
  NominatedMap by_node_;
  std::unordered_map<std::string, std::string> node_of_;
  struct Change {
    std::string node;
    PodPtr pod;
    bool add;
  };
  void log_remove(const std::string& node, const PodPtr& p) { log_.push_back(Change{node, p, false}); }
  // Nothing nominated: start an empty mirror (a cycle may still hold the old
  // one) and drop the log, which would otherwise grow while no cycle asks.
  void reset_mirror() {
    log_.clear();
    if (!mirror_->empty()) mirror_ = std::make_shared<NominatedMap>();
  }
  mutable std::vector<Change> log_;  // since the last view()
  mutable std::shared_ptr<NominatedMap> mirror_ = std::make_shared<NominatedMap>();
};

struct QueueOptions {
  int64_t initial_backoff_us = 1'000'000;
  int64_t max_backoff_us = 10'000'000;
  int64_t unschedulable_timeout_us = 60'000'000;
};

class SchedulingQueue {
 public:
  SchedulingQueue(PodHeap::Less less, std::shared_ptr<Clock> clock, QueueOptions opts, Nominator* nominator);

  // clusterEventMap: event -> plugin names interested in it.
  void set_cluster_event_map(std::vector<std::pair<ClusterEvent, std::set<std::string>>> m);

  void add(const PodPtr& p);
  // Moves the pods to activeQ. A pod that is in flight (popped, in its
  // scheduling or binding cycle) is marked instead, and
  // add_unschedulable_if_not_present sends a marked pod to activeQ when that
  // cycle fails: the request is not lost. (The reference drops it,
  // scheduling_queue.go:307-337; its moveRequestCycle covers only cluster
  // events, :376-400,629.)
  void activate(const std::vector<PodPtr>& pods);
  // Parks the pods: moved out of activeQ / backoffQ / unschedulableQ into a
  // holding area that no cluster event and no backoff flush touches; only
  // activate() (or the unschedulable leftover flush) brings them back. A pod
  // in flight is marked and parks when its cycle fails. Coscheduling parks a
  // gang's unplaced members this way while the gang waits for GPUs, so
  // neither each member's own failed cycle nor every PodGroup creation in the
  // cluster (its registered event) churns them.
  void deactivate(const std::vector<PodPtr>& pods);
  // Returns false if the pod is already queued (active/backoff).
  bool add_unschedulable_if_not_present(const QueuedPodInfoPtr& p, int64_t pod_scheduling_cycle);
  size_t pending_activations() const;  // in-flight pods carrying an activation mark
  size_t in_flight() const;
  int64_t scheduling_cycle() const;
  // Blocks until a pod is available or the queue is closed (nullptr).
  QueuedPodInfoPtr pop(int timeout_ms = -1);
  void update(const PodPtr& old_p, const PodPtr& new_p);
  void remove(const Pod& p);
  void assigned_pod_added(const Pod& p);
  void assigned_pod_updated(const Pod& p);
  void move_all_to_active_or_backoff(const ClusterEvent& ev);
  void flush_backoff_completed();
  void flush_unschedulable_leftover();
  void close();

  struct Counts {
    size_t active = 0, backoff = 0, unschedulable = 0, parked = 0;
  };
  Counts counts() const;
  std::vector<QueuedPodInfoPtr> pending_pods() const;
  bool has_pod(const std::string& uid) const;

 private:
  QueuedPodInfoPtr new_info(const PodPtr& p) const;
  bool backing_off(const QueuedPodInfo& p) const;
  int64_t backoff_expiry(const QueuedPodInfo& p) const;
  bool matches_event(const QueuedPodInfo& p, const ClusterEvent& ev) const;
  void move_locked(const std::vector<QueuedPodInfoPtr>& pods, const ClusterEvent& ev);
  static bool affinity_term_matches(const Pod& waiting, const Pod& assigned);

  std::shared_ptr<Clock> clock_;
  QueueOptions opts_;
  Nominator* nominator_;
  // Taken by the scheduling thread per pop and by the informer per event
  // batch, each time briefly: a spinning mutex (common/adaptive_mutex.h).
  mutable AdaptiveMutex mu_;
  std::condition_variable_any cv_;
  PodHeap active_;
  PodHeap backoff_;
  std::unordered_map<std::string, QueuedPodInfoPtr> unschedulable_;
  std::unordered_map<std::string, QueuedPodInfoPtr> parked_;  // deactivate()
  // Popped pods -> what to do when their cycle fails: kNoMark, kActivate
  // (activated while in flight) or kPark (deactivated while in flight). An
  // entry lives until the pod re-enters a queue, is removed, or shows up
  // assigned (every pod ends in one of those), so the map is bounded by the
  // pods that exist.
  enum : uint8_t { kNoMark = 0, kActivate = 1, kPark = 2 };
  std::unordered_map<std::string, uint8_t> in_flight_;
  std::vector<std::pair<ClusterEvent, std::set<std::string>>> event_map_;
  int64_t scheduling_cycle_ = 0;
  int64_t move_request_cycle_ = -1;
  int64_t seq_ = 0;
  bool closed_ = false;
};

}  // namespace xsched
