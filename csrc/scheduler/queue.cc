#include "scheduler/queue.h"

#include <algorithm>
#include <chrono>

namespace xsched {

// ---------------------------------------------------------------- PodHeap ----
void PodHeap::swap_at(size_t a, size_t b) {
  std::swap(v_[a], v_[b]);
  v_[a]->heap_index = a;
  v_[b]->heap_index = b;
}

void PodHeap::up(size_t i) {
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!less_(*v_[i], *v_[p])) break;
    swap_at(i, p);
    i = p;
  }
}

void PodHeap::down(size_t i) {
  size_t n = v_.size();
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && less_(*v_[l], *v_[m])) m = l;
    if (r < n && less_(*v_[r], *v_[m])) m = r;
    if (m == i) return;
    swap_at(i, m);
    i = m;
  }
}

void PodHeap::push(const QueuedPodInfoPtr& p) {
  auto it = pos_.find(p->pod->uid());
  if (it != pos_.end()) {
    size_t i = it->second->heap_index;
    if (tag_) v_[i]->pod->heap_tag.v = 0;
    v_[i] = p;
    if (tag_) p->pod->heap_tag.v = tag_;
    p->heap_index = i;
    it->second = p.get();
    up(i);
    down(p->heap_index);
    return;
  }
  v_.push_back(p);
  if (tag_) p->pod->heap_tag.v = tag_;
  p->heap_index = v_.size() - 1;
  pos_.emplace(p->pod->uid(), p.get());
  up(v_.size() - 1);
}

QueuedPodInfoPtr PodHeap::pop() {
  if (v_.empty()) return nullptr;
  QueuedPodInfoPtr top = v_.front();
  if (tag_) top->pod->heap_tag.v = 0;
  swap_at(0, v_.size() - 1);
  v_.pop_back();
  pos_.erase(top->pod->uid());
  if (!v_.empty()) down(0);
  return top;
}

QueuedPodInfoPtr PodHeap::get(const std::string& uid) const {
  auto it = pos_.find(uid);
  return it == pos_.end() ? nullptr : v_[it->second->heap_index];
}

bool PodHeap::erase(const std::string& uid) {
  auto it = pos_.find(uid);
  if (it == pos_.end()) return false;
  size_t i = it->second->heap_index;
  if (tag_) v_[i]->pod->heap_tag.v = 0;
  size_t last = v_.size() - 1;
  if (i != last) swap_at(i, last);
  v_.pop_back();
  pos_.erase(it);
  if (i < v_.size()) {
    up(i);
    down(i);
  }
  return true;
}

// -------------------------------------------------------------- Nominator ----
void Nominator::add(const PodPtr& p, const std::string& node) {
  std::string n = node.empty() ? p->nominated_node_name : node;
  std::lock_guard<std::mutex> g(mu_);
  // Always remove first (AddNominatedPod semantics).
  auto it = node_of_.find(p->uid());
  if (it != node_of_.end()) {
    auto& vec = by_node_[it->second];
    vec.erase(std::remove_if(vec.begin(), vec.end(), [&](const PodPtr& x) { return x->uid() == p->uid(); }), vec.end());
    if (vec.empty()) by_node_.erase(it->second);
    log_remove(it->second, p);
    node_of_.erase(it);
  }
  if (!n.empty()) {
    node_of_[p->uid()] = n;
    by_node_[n].push_back(p);
    log_.push_back(Change{n, p, true});
  }
  count_.store(node_of_.size(), std::memory_order_relaxed);
  if (node_of_.empty()) reset_mirror();
}

void Nominator::remove(const Pod& p) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = node_of_.find(p.uid());
  if (it == node_of_.end()) return;
  auto& vec = by_node_[it->second];
  PodPtr gone;
  for (const auto& x : vec)
    if (x->uid() == p.uid()) gone = x;
  vec.erase(std::remove_if(vec.begin(), vec.end(), [&](const PodPtr& x) { return x->uid() == p.uid(); }), vec.end());
  if (vec.empty()) by_node_.erase(it->second);
  if (gone) log_remove(it->second, gone);
  node_of_.erase(it);
  count_.store(node_of_.size(), std::memory_order_relaxed);
  if (node_of_.empty()) reset_mirror();
}

void Nominator::update(const PodPtr& old_p, const PodPtr& new_p) {
  // UpdateNominatedPod: when neither version carries a nominated node, keep
  // the in-memory one (the scheduler may have nominated it before the API
  // reflected it).
  std::string node;
  if (old_p->nominated_node_name.empty() && new_p->nominated_node_name.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = node_of_.find(old_p->uid());
    if (it != node_of_.end()) node = it->second;
  }
  add(new_p, node);
}

std::vector<PodPtr> Nominator::nominated_pods_for_node(const std::string& node) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_node_.find(node);
  return it == by_node_.end() ? std::vector<PodPtr>{} : it->second;
}

void Nominator::for_each(const std::function<void(const std::string&, const PodPtr&)>& fn) const {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& [node, pods] : by_node_)
    for (const auto& p : pods) fn(node, p);
}

std::shared_ptr<const NominatedMap> Nominator::view(std::vector<std::string>* changed) const {
  std::lock_guard<std::mutex> g(mu_);
  NominatedMap& m = *mirror_;
  for (auto& c : log_) {
    if (changed) changed->push_back(c.node);
    if (c.add) {
      m[c.node].push_back(std::move(c.pod));
      continue;
    }
    auto it = m.find(c.node);
    if (it == m.end()) continue;
    auto& vec = it->second;
    const std::string& uid = c.pod->uid();
    vec.erase(std::remove_if(vec.begin(), vec.end(), [&](const PodPtr& x) { return x->uid() == uid; }), vec.end());
    if (vec.empty()) m.erase(it);
  }
  log_.clear();
  return mirror_;
}

std::string Nominator::nominated_node(const std::string& uid) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = node_of_.find(uid);
  return it == node_of_.end() ? std::string() : it->second;
}

size_t Nominator::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return node_of_.size();
}

// -------------------------------------------------------- SchedulingQueue ----
SchedulingQueue::SchedulingQueue(PodHeap::Less less, std::shared_ptr<Clock> clock, QueueOptions opts,
                                 Nominator* nominator)
    : clock_(std::move(clock)),
      opts_(opts),
      nominator_(nominator),
      active_(std::move(less), /*tag=*/1),
      backoff_([this](const QueuedPodInfo& a, const QueuedPodInfo& b) { return backoff_expiry(a) < backoff_expiry(b); }) {}

void SchedulingQueue::set_cluster_event_map(std::vector<std::pair<ClusterEvent, std::set<std::string>>> m) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  event_map_ = std::move(m);
}

QueuedPodInfoPtr SchedulingQueue::new_info(const PodPtr& p) const {
  auto q = std::make_shared<QueuedPodInfo>();
  q->pod = p;
  q->timestamp_us = clock_->now_us();
  q->initial_attempt_us = q->timestamp_us;
  q->initial_attempt_wall = wall_now_us();
  return q;
}

int64_t SchedulingQueue::backoff_expiry(const QueuedPodInfo& p) const {
  int64_t d = opts_.initial_backoff_us;
  for (int i = 1; i < p.attempts; ++i) {
    d *= 2;
    if (d > opts_.max_backoff_us) {
      d = opts_.max_backoff_us;
      break;
    }
  }
  if (d > opts_.max_backoff_us) d = opts_.max_backoff_us;
  return p.timestamp_us + d;
}

bool SchedulingQueue::backing_off(const QueuedPodInfo& p) const { return backoff_expiry(p) > clock_->now_us(); }

void SchedulingQueue::add(const PodPtr& p) {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    auto q = new_info(p);
    q->enqueue_seq = ++seq_;
    unschedulable_.erase(p->uid());
    parked_.erase(p->uid());
    backoff_.erase(p->uid());
    in_flight_.erase(p->uid());
    active_.push(q);
  }
  nominator_->add(p, "");
  cv_.notify_one();
}

void SchedulingQueue::activate(const std::vector<PodPtr>& pods) {
  bool moved = false;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    for (const auto& pod : pods) {
      if (active_.holds(*pod)) continue;  // already active: no uid lookups
      const std::string& uid = pod->uid();
      if (active_.contains(uid)) continue;
      QueuedPodInfoPtr q;
      auto it = unschedulable_.find(uid);
      if (it != unschedulable_.end()) {
        q = it->second;
        unschedulable_.erase(it);
      } else if (auto pk = parked_.find(uid); pk != parked_.end()) {
        q = pk->second;
        parked_.erase(pk);
      } else if ((q = backoff_.get(uid))) {
        backoff_.erase(uid);
      }
      if (!q) {  // in flight: remember the request for when its cycle fails
        auto f = in_flight_.find(uid);
        if (f != in_flight_.end()) f->second = kActivate;
        continue;
      }
      active_.push(q);
      moved = true;
    }
  }
  if (moved) cv_.notify_all();
}

void SchedulingQueue::deactivate(const std::vector<PodPtr>& pods) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  for (const auto& pod : pods) {
    const std::string& uid = pod->uid();
    QueuedPodInfoPtr q;
    if ((q = active_.get(uid))) {
      active_.erase(uid);
    } else if ((q = backoff_.get(uid))) {
      backoff_.erase(uid);
    } else if (auto it = unschedulable_.find(uid); it != unschedulable_.end()) {
      q = it->second;
      unschedulable_.erase(it);
    }
    if (q) {
      q->timestamp_us = clock_->now_us();
      parked_[uid] = std::move(q);
      continue;
    }
    // In flight: parked when its cycle fails, unless an activation came in
    // meanwhile (a probe sent for capacity released during the cycle): that
    // is newer than the park and must not be lost (the pod then gets one
    // more attempt and parks again if the capacity is not there).
    if (auto f = in_flight_.find(uid); f != in_flight_.end() && f->second != kActivate) f->second = kPark;
  }
}

bool SchedulingQueue::add_unschedulable_if_not_present(const QueuedPodInfoPtr& p, int64_t pod_cycle) {
  bool activated = false;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    const std::string& uid = p->pod->uid();
    if (unschedulable_.count(uid) || parked_.count(uid) || active_.contains(uid) || backoff_.contains(uid))
      return false;
    p->timestamp_us = clock_->now_us();
    uint8_t mark = kNoMark;
    if (auto f = in_flight_.find(uid); f != in_flight_.end()) {
      mark = f->second;
      in_flight_.erase(f);
    }
    if (mark == kActivate) {
      active_.push(p);  // activated while in flight; Activate skips backoff
      activated = true;
    } else if (mark == kPark) {
      parked_[uid] = p;
    } else if (move_request_cycle_ >= pod_cycle) {
      backoff_.push(p);
    } else {
      unschedulable_[uid] = p;
    }
  }
  nominator_->add(p->pod, "");
  if (activated) cv_.notify_all();
  return true;
}

size_t SchedulingQueue::pending_activations() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  size_t n = 0;
  for (const auto& kv : in_flight_) n += kv.second == kActivate;
  return n;
}

size_t SchedulingQueue::in_flight() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return in_flight_.size();
}

int64_t SchedulingQueue::scheduling_cycle() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return scheduling_cycle_;
}

QueuedPodInfoPtr SchedulingQueue::pop(int timeout_ms) {
  std::unique_lock<AdaptiveMutex> lk(mu_);
  auto ready = [&] { return closed_ || !active_.empty(); };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
    return nullptr;
  if (closed_ && active_.empty()) return nullptr;
  QueuedPodInfoPtr q = active_.pop();
  in_flight_.insert_or_assign(q->pod->uid(), kNoMark);
  q->attempts++;
  scheduling_cycle_++;
  return q;
}

namespace {
bool pod_spec_changed(const Pod& a, const Pod& b) {
  // isPodUpdated: ignore status/resourceVersion-only changes.
  return !(a.request() == b.request() && a.meta.labels == b.meta.labels && a.meta.annotations == b.meta.annotations &&
           a.node_selector == b.node_selector && a.priority == b.priority && a.tolerations.size() == b.tolerations.size());
}
}  // namespace

void SchedulingQueue::update(const PodPtr& old_p, const PodPtr& new_p) {
  bool notify = false;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    const std::string& uid = new_p->uid();
    if (auto q = active_.get(uid)) {
      auto nq = std::make_shared<QueuedPodInfo>(*q);
      nq->pod = new_p;
      active_.push(nq);
      nominator_->update(old_p, new_p);
      return;
    }
    if (auto q = backoff_.get(uid)) {
      auto nq = std::make_shared<QueuedPodInfo>(*q);
      nq->pod = new_p;
      backoff_.push(nq);
      nominator_->update(old_p, new_p);
      return;
    }
    if (auto pk = parked_.find(uid); pk != parked_.end()) {
      auto nq = std::make_shared<QueuedPodInfo>(*pk->second);
      nq->pod = new_p;
      nominator_->update(old_p, new_p);
      if (!pod_spec_changed(*old_p, *new_p)) {
        pk->second = nq;
        return;
      }
      // A parked pod whose spec changed (a user fixed its requests) gets
      // another attempt now, as an unschedulable one does (upstream
      // Update: scheduling_queue.go:436-470), instead of waiting for its
      // gang's next probe or the unschedulable flush.
      parked_.erase(pk);
      if (backing_off(*nq)) {
        backoff_.push(nq);
      } else {
        active_.push(nq);
        notify = true;
      }
      if (notify) cv_.notify_one();
      return;
    }
    auto it = unschedulable_.find(uid);
    if (it != unschedulable_.end()) {
      nominator_->update(old_p, new_p);
      auto nq = std::make_shared<QueuedPodInfo>(*it->second);
      nq->pod = new_p;
      if (pod_spec_changed(*old_p, *new_p)) {
        unschedulable_.erase(it);
        if (backing_off(*nq)) {
          backoff_.push(nq);
        } else {
          active_.push(nq);
          notify = true;
        }
      } else {
        it->second = nq;
      }
    } else {
      // Not queued anywhere: add to activeQ (it may have been in flight).
      in_flight_.erase(uid);
      auto q = new_info(new_p);
      q->enqueue_seq = ++seq_;
      active_.push(q);
      notify = true;
    }
  }
  if (notify) {
    nominator_->add(new_p, "");
    cv_.notify_one();
  }
}

void SchedulingQueue::remove(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  nominator_->remove(p);
  active_.erase(p.uid());
  backoff_.erase(p.uid());
  unschedulable_.erase(p.uid());
  parked_.erase(p.uid());
  in_flight_.erase(p.uid());
}

bool SchedulingQueue::affinity_term_matches(const Pod& waiting, const Pod& assigned) {
  for (const auto& t : waiting.pod_affinity_required) {
    bool ns_ok = t.namespaces.empty() ? assigned.ns() == waiting.ns()
                                      : std::find(t.namespaces.begin(), t.namespaces.end(), assigned.ns()) != t.namespaces.end();
    if (ns_ok && t.selector.matches(assigned.meta.labels)) return true;
  }
  return false;
}

void SchedulingQueue::assigned_pod_added(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  in_flight_.erase(p.uid());  // bound: its cycles are over
  std::vector<QueuedPodInfoPtr> match;
  for (const auto& kv : unschedulable_)
    if (affinity_term_matches(*kv.second->pod, p)) match.push_back(kv.second);
  if (!match.empty()) move_locked(match, ClusterEvent{"Pod", kAdd, "AssignedPodAdd"});
}

void SchedulingQueue::assigned_pod_updated(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  std::vector<QueuedPodInfoPtr> match;
  for (const auto& kv : unschedulable_)
    if (affinity_term_matches(*kv.second->pod, p)) match.push_back(kv.second);
  if (!match.empty()) move_locked(match, ClusterEvent{"Pod", kUpdate, "AssignedPodUpdate"});
}

bool SchedulingQueue::matches_event(const QueuedPodInfo& p, const ClusterEvent& ev) const {
  if (ev.is_wildcard()) return true;
  for (const auto& [e, names] : event_map_) {
    bool ev_match = e.is_wildcard() || (e.resource == ev.resource && (e.action & ev.action) != 0);
    if (!ev_match) continue;
    for (const auto& n : p.unschedulable_plugins)
      if (names.count(n)) return true;
  }
  return false;
}

void SchedulingQueue::move_locked(const std::vector<QueuedPodInfoPtr>& pods, const ClusterEvent& ev) {
  bool activated = false;
  for (const auto& q : pods) {
    if (!matches_event(*q, ev)) continue;
    const std::string& uid = q->pod->uid();
    unschedulable_.erase(uid);
    if (backing_off(*q)) {
      backoff_.push(q);
    } else {
      active_.push(q);
      activated = true;
    }
  }
  move_request_cycle_ = scheduling_cycle_;
  if (activated) cv_.notify_all();
}

void SchedulingQueue::move_all_to_active_or_backoff(const ClusterEvent& ev) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  std::vector<QueuedPodInfoPtr> all;
  all.reserve(unschedulable_.size());
  for (const auto& kv : unschedulable_) all.push_back(kv.second);
  move_locked(all, ev);
}

void SchedulingQueue::flush_backoff_completed() {
  bool moved = false;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    while (!backoff_.empty()) {
      const auto& top = backoff_.top();
      if (backing_off(*top)) break;
      active_.push(backoff_.pop());
      moved = true;
    }
  }
  if (moved) cv_.notify_all();
}

void SchedulingQueue::flush_unschedulable_leftover() {
  std::lock_guard<AdaptiveMutex> g(mu_);
  int64_t now = clock_->now_us();
  std::vector<QueuedPodInfoPtr> stale;
  for (const auto& kv : unschedulable_)
    if (now - kv.second->timestamp_us > opts_.unschedulable_timeout_us) stale.push_back(kv.second);
  // Parked pods too (safety net: their release signal never came).
  for (auto it = parked_.begin(); it != parked_.end();) {
    if (now - it->second->timestamp_us > opts_.unschedulable_timeout_us) {
      unschedulable_[it->first] = it->second;
      stale.push_back(it->second);
      it = parked_.erase(it);
    } else {
      ++it;
    }
  }
  if (!stale.empty()) move_locked(stale, ClusterEvent{"*", kAll, "UnschedulableTimeout"});
}

void SchedulingQueue::close() {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

SchedulingQueue::Counts SchedulingQueue::counts() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return Counts{active_.size(), backoff_.size(), unschedulable_.size(), parked_.size()};
}

std::vector<QueuedPodInfoPtr> SchedulingQueue::pending_pods() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  std::vector<QueuedPodInfoPtr> out = active_.items();
  auto b = backoff_.items();
  out.insert(out.end(), b.begin(), b.end());
  for (const auto& kv : unschedulable_) out.push_back(kv.second);
  for (const auto& kv : parked_) out.push_back(kv.second);
  return out;
}

bool SchedulingQueue::has_pod(const std::string& uid) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return active_.contains(uid) || backoff_.contains(uid) || unschedulable_.count(uid) || parked_.count(uid);
}

}  // namespace xsched
