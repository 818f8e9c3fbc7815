// Pods parked at Permit, with per-plugin timeouts.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/framework/runtime/
// waiting_pods_map.go:83-165 (one goroutine blocks per waiting pod in
// WaitOnPermit). Here a waiting pod is a continuation: whoever resolves it
// (Allow by the last plugin, Reject, or the timer service on timeout) runs the
// registered callback exactly once, so a thousand parked gang members cost
// no threads.
#pragma once

#include "common/adaptive_mutex.h"

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

#include "common/clock.h"
#include "framework/types.h"

namespace xsched {

class WaitingPods;

class WaitingPod : public std::enable_shared_from_this<WaitingPod> {
 public:
  using Done = std::function<void(const Status&)>;
  WaitingPod(PodPtr pod, std::string node, WaitingPods* owner) : pod_(std::move(pod)), node_(std::move(node)), owner_(owner) {}

  const PodPtr& pod() const { return pod_; }
  const std::string& node() const { return node_; }
  std::vector<std::string> pending_plugins() const;
  // Returns true when this call resolved the pod.
  bool allow(const std::string& plugin);
  bool reject(const std::string& plugin, const std::string& msg);
  int64_t created_us() const { return created_us_; }

 private:
  friend class WaitingPods;
  void resolve(const Status& st);  // called without mu_ held

  PodPtr pod_;
  std::string node_;
  WaitingPods* owner_;
  mutable AdaptiveMutex mu_;
  std::map<std::string, uint64_t> pending_;  // plugin -> timer id
  bool done_ = false;
  Done on_done_;
  int64_t created_us_ = 0;
};
using WaitingPodPtr = std::shared_ptr<WaitingPod>;

class WaitingPods {
 public:
  explicit WaitingPods(TimerService* timers) : timers_(timers) {}
  // Registers a waiting pod with plugin->timeout_us; on_done fires once.
  WaitingPodPtr add(const PodPtr& pod, const std::string& node, const std::map<std::string, int64_t>& timeouts,
                    WaitingPod::Done on_done);
  WaitingPodPtr get(const std::string& uid) const;
  void iterate(const std::function<void(const WaitingPodPtr&)>& fn) const;
  // Waiting pods whose Pod::pg_key is `pg_key` (callers still compare the
  // group name: the key is a 64-bit hash). O(group), not O(all waiting).
  void iterate_group(uint64_t pg_key, const std::function<void(const WaitingPodPtr&)>& fn) const;
  size_t size() const;
  // Reject every waiting pod (shutdown).
  void reject_all(const std::string& msg);

 private:
  friend class WaitingPod;
  void remove(const std::string& uid);
  TimerService* timers_;
  mutable AdaptiveMutex mu_;
  std::unordered_map<std::string, WaitingPodPtr> pods_;
  std::unordered_map<uint64_t, std::vector<WaitingPodPtr>> by_group_;
};

}  // namespace xsched
