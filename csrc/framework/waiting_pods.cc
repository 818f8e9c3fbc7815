#include "framework/waiting_pods.h"

#include <vector>

namespace xsched {

std::vector<std::string> WaitingPod::pending_plugins() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  std::vector<std::string> out;
  for (const auto& kv : pending_) out.push_back(kv.first);
  return out;
}

bool WaitingPod::allow(const std::string& plugin) {
  std::vector<uint64_t> cancel;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    if (done_) return false;
    auto it = pending_.find(plugin);
    if (it != pending_.end()) {
      cancel.push_back(it->second);
      pending_.erase(it);
    }
    if (!pending_.empty()) {
      for (uint64_t id : cancel) owner_->timers_->cancel(id);
      return false;
    }
    done_ = true;
  }
  for (uint64_t id : cancel) owner_->timers_->cancel(id);
  resolve(Status());
  return true;
}

bool WaitingPod::reject(const std::string& plugin, const std::string& msg) {
  std::vector<uint64_t> cancel;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    if (done_) return false;
    done_ = true;
    for (const auto& kv : pending_) cancel.push_back(kv.second);
    pending_.clear();
  }
  for (uint64_t id : cancel) owner_->timers_->cancel(id);
  resolve(Status(Code::Unschedulable, msg).with_plugin(plugin));
  return true;
}

void WaitingPod::resolve(const Status& st) {
  owner_->remove(pod_->uid());
  Done cb;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    cb = std::move(on_done_);
  }
  if (cb) cb(st);
}

WaitingPodPtr WaitingPods::add(const PodPtr& pod, const std::string& node, const std::map<std::string, int64_t>& timeouts,
                               WaitingPod::Done on_done) {
  auto wp = std::make_shared<WaitingPod>(pod, node, this);
  wp->on_done_ = std::move(on_done);
  wp->created_us_ = timers_->clock().now_us();
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    pods_[pod->uid()] = wp;
    if (pod->pg_key) by_group_[pod->pg_key].push_back(wp);
  }
  // Arm timers after registration so a zero timeout cannot fire before the
  // pod is visible to IterateOverWaitingPods.
  std::lock_guard<AdaptiveMutex> g(wp->mu_);
  for (const auto& kv : timeouts) {
    std::string plugin = kv.first;
    std::weak_ptr<WaitingPod> weak = wp;
    uint64_t id = timers_->schedule_after(kv.second, [weak, plugin] {
      if (auto p = weak.lock())
        p->reject(plugin, "rejected due to timeout after waiting at permit");
    });
    wp->pending_[plugin] = id;
  }
  return wp;
}

WaitingPodPtr WaitingPods::get(const std::string& uid) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pods_.find(uid);
  return it == pods_.end() ? nullptr : it->second;
}

void WaitingPods::iterate(const std::function<void(const WaitingPodPtr&)>& fn) const {
  std::vector<WaitingPodPtr> snap;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    snap.reserve(pods_.size());
    for (const auto& kv : pods_) snap.push_back(kv.second);
  }
  for (const auto& wp : snap) fn(wp);
}

void WaitingPods::iterate_group(uint64_t pg_key, const std::function<void(const WaitingPodPtr&)>& fn) const {
  std::vector<WaitingPodPtr> snap;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    auto it = by_group_.find(pg_key);
    if (it == by_group_.end()) return;
    snap = it->second;
  }
  for (const auto& wp : snap) fn(wp);
}

size_t WaitingPods::size() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return pods_.size();
}

void WaitingPods::remove(const std::string& uid) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pods_.find(uid);
  if (it == pods_.end()) return;
  if (uint64_t key = it->second->pod()->pg_key) {
    auto git = by_group_.find(key);
    if (git != by_group_.end()) {
      auto& v = git->second;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == it->second) {
          v[i] = std::move(v.back());
          v.pop_back();
          break;
        }
      if (v.empty()) by_group_.erase(git);
    }
  }
  pods_.erase(it);
}

void WaitingPods::reject_all(const std::string& msg) {
  iterate([&](const WaitingPodPtr& wp) { wp->reject("", msg); });
}

}  // namespace xsched
