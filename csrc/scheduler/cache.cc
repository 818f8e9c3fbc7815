#include "scheduler/cache.h"

#include <algorithm>
#include <set>

namespace xsched {

SchedulerCache::SchedulerCache(std::shared_ptr<Clock> clock, int64_t assumed_ttl_us)
    : clock_(std::move(clock)), ttl_us_(assumed_ttl_us) {}

NodeInfoPtr& SchedulerCache::info_for(const std::string& node) {
  auto& ni = nodes_[node];
  if (!ni) ni = std::make_shared<NodeInfo>();
  return ni;
}

// Copy-on-write: snapshot NodeInfos are the cache's own immutable versions
// (update_snapshot shares pointers instead of cloning). A version that a
// snapshot still references is copied before the cache mutates it, so the
// copy happens on the mutating thread (informer, binder, assume) and never
// while the scheduling thread refreshes its snapshot.
NodeInfo& SchedulerCache::writable(NodeInfoPtr& slot) {
  if (!in_place_ && slot.use_count() > 1) slot = slot->clone();
  return *slot;
}

void SchedulerCache::mark_dirty(const std::string& node) {
  dirty_.insert(node);
  auto it = nodes_.find(node);
  if (it != nodes_.end()) writable(it->second).generation = ++generation_;
}

void SchedulerCache::group_delta(const Pod& p, int d) {
  if (!p.pg_key) return;
  std::lock_guard<AdaptiveMutex> g(group_mu_);
  auto it = group_assigned_.try_emplace(p.pg_key, 0).first;
  it->second += d;
  if (it->second <= 0) group_assigned_.erase(it);
  auto& hosts = group_nodes_[p.pg_key];
  auto h = std::find_if(hosts.begin(), hosts.end(), [&](const auto& e) { return e.first == p.node_name; });
  if (h == hosts.end()) {
    if (d > 0) hosts.emplace_back(p.node_name, d);
  } else if ((h->second += d) <= 0) {
    hosts.erase(h);
  }
  if (hosts.empty()) group_nodes_.erase(p.pg_key);
}

int SchedulerCache::group_placement(uint64_t pg_key, std::vector<std::string>& hosts) const {
  std::lock_guard<AdaptiveMutex> g(group_mu_);
  size_t k = 0;
  auto it = group_nodes_.find(pg_key);
  if (it != group_nodes_.end())
    for (const auto& [node, n] : it->second) {
      if (k < hosts.size()) hosts[k].assign(node);  // reuses the string's buffer
      else hosts.push_back(node);
      ++k;
    }
  hosts.resize(k);
  auto a = group_assigned_.find(pg_key);
  return a == group_assigned_.end() ? 0 : a->second;
}

std::vector<std::string> SchedulerCache::nodes_of_group(uint64_t pg_key) const {
  std::lock_guard<AdaptiveMutex> g(group_mu_);
  std::vector<std::string> out;
  auto it = group_nodes_.find(pg_key);
  if (it != group_nodes_.end())
    for (const auto& [node, n] : it->second) out.push_back(node);
  return out;
}

void SchedulerCache::account_node(const Node* old_node, const Node* new_node) {
  prefer_nodes_ += (new_node && new_node->has_prefer_no_schedule) - (old_node && old_node->has_prefer_no_schedule);
  foreign_hostnames_ += (new_node && new_node->foreign_hostname) - (old_node && old_node->foreign_hostname);
  const bool old_imgs = old_node && !old_node->image_sizes.empty();
  const bool new_imgs = new_node && !new_node->image_sizes.empty();
  if (!old_imgs && !new_imgs) return;  // heartbeat-style updates of image-less nodes cost nothing
  if (old_imgs && new_imgs && old_node->image_sizes.size() == new_node->image_sizes.size()) {
    bool same = true;
    for (const auto& kv : new_node->image_sizes)
      if (!old_node->image_sizes.count(kv.first)) {
        same = false;
        break;
      }
    if (same) return;
  }
  if (image_spread_.use_count() > 1) image_spread_ = std::make_shared<std::unordered_map<std::string, int64_t>>(*image_spread_);
  auto& spread = *image_spread_;
  if (old_imgs)
    for (const auto& kv : old_node->image_sizes) {
      auto it = spread.find(kv.first);
      if (it != spread.end() && --it->second <= 0) spread.erase(it);
    }
  if (new_imgs)
    for (const auto& kv : new_node->image_sizes) ++spread[kv.first];
}

void SchedulerCache::set_node_locked(const NodePtr& n) {
  ++node_epoch_;
  auto& ni = info_for(n->name());
  bool was_ghost = ni->node == nullptr;
  if (was_ghost || ni->node->meta.labels != n->meta.labels) ++topology_epoch_;
  account_node(ni->node.get(), n.get());
  writable(ni).set_node(n);
  if (was_ghost) {
    order_.push_back(n->name());
    structure_changed_ = true;
  }
  mark_dirty(n->name());
}

void SchedulerCache::add_node(const NodePtr& n) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  set_node_locked(n);
}

void SchedulerCache::update_node(const NodePtr& n) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  set_node_locked(n);
}

void SchedulerCache::remove_node(const std::string& name) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = nodes_.find(name);
  if (it == nodes_.end()) return;
  ++node_epoch_;
  ++topology_epoch_;
  account_node(it->second->node.get(), nullptr);
  order_.erase(std::remove(order_.begin(), order_.end(), name), order_.end());
  structure_changed_ = true;
  if (it->second->pods.empty()) {
    nodes_.erase(it);
  } else {
    writable(it->second).node = nullptr;  // ghost until its pods are deleted
  }
  dirty_.insert(name);
}

void SchedulerCache::set_nrt(const std::string& node, const NRTPtr& nrt) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = nodes_.find(node);
  if (it == nodes_.end()) {
    if (!nrt) return;
    info_for(node);  // ghost until the Node arrives; keeps the NRT
    it = nodes_.find(node);
  }
  writable(it->second).nrt = nrt;
  mark_dirty(node);
}

// Pods on a ghost node (no Node object) are in no Snapshot and never
// counted, so they need no event either: the Node's arrival bumps the
// topology epoch.
void SchedulerCache::record_delta(const PodPtr& p, const NodeInfo& ni, int d) {
  if (!track_deltas_ || !ni.node) return;
  pending_deltas_.push_back(PodDelta{p, ni.node, d});
  ++delta_seq_;
}

void SchedulerCache::add_pod_locked(const PodPtr& p) {
  auto& ni = info_for(p->node_name);
  writable(ni).add_pod(p);
  ++prio_count_[p->priority];
  group_delta(*p, +1);
  record_delta(p, *ni, +1);
  mark_dirty(p->node_name);
}

void SchedulerCache::remove_pod_locked(const PodPtr& p) {
  auto it = nodes_.find(p->node_name);
  if (it == nodes_.end()) return;
  NodeInfo& ni = writable(it->second);
  if (ni.remove_pod(p->uid())) {
    group_delta(*p, -1);
    record_delta(p, ni, -1);
    auto pit = prio_count_.find(p->priority);
    if (pit != prio_count_.end() && --pit->second <= 0) prio_count_.erase(pit);
  }
  // mark_dirty, with the node already found and writable.
  dirty_.insert(p->node_name);
  ni.generation = ++generation_;
  if (ni.node == nullptr && ni.pods.empty()) nodes_.erase(it);
}

Status SchedulerCache::assume_pod(const PodPtr& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  if (pod_states_.count(p->uid())) return Status::error("pod " + p->key() + " is in the cache, so can't be assumed");
  in_place_ = true;
  add_pod_locked(p);
  in_place_ = false;
  pod_states_[p->uid()] = PodState{p, 0, false};
  pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
  assumed_.insert(p->uid());
  return {};
}

void SchedulerCache::finish_binding(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(p.uid());
  if (it == pod_states_.end() || !assumed_.count(p.uid())) return;
  it->second.binding_finished = true;
  it->second.deadline_us = clock_->now_us() + ttl_us_;
}

void SchedulerCache::forget_pod(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(p.uid());
  if (it == pod_states_.end()) return;
  if (!assumed_.count(p.uid())) return;  // only assumed pods can be forgotten
  PodPtr cur = it->second.pod;
  remove_pod_locked(cur);
  assumed_.erase(p.uid());
  pod_states_.erase(it);
  pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
}

namespace {
// The informer's bound object accounts on its node exactly like the assumed
// copy: same node, spec, labels and GPU placement.
bool same_accounting(const Pod& assumed, const Pod& bound) {
  const GpuAssignment &a = assumed.gpu, &b = bound.gpu;
  return assumed.node_name == bound.node_name && assumed.spec_hash == bound.spec_hash &&
         assumed.meta.labels == bound.meta.labels && assumed.meta.deletion == bound.meta.deletion &&
         assumed.priority == bound.priority && a.kind == b.kind && a.gpus == b.gpus && a.partitions == b.partitions &&
         a.memory == b.memory;
}
}  // namespace

bool SchedulerCache::confirm_assumed_locked(std::unordered_map<std::string, PodState>::iterator it, const PodPtr& p) {
  if (!same_accounting(*it->second.pod, *p)) return false;
  // The node's NodeInfo already holds an equivalent object: leave it (and its
  // generation, so equivalence-cache verdicts for the node stay valid) and
  // only record the informer's object as the pod's current state.
  // Status timestamps the preemption paths read from NodeInfo pods
  // (victim ordering, PreemptionToleration's toleration window).
  it->second.pod->scheduled_at = p->scheduled_at;
  it->second.pod->start_time = p->start_time;
  assumed_.erase(p->uid());
  it->second = PodState{p, 0, false};
  return true;
}

void SchedulerCache::add_pod(const PodPtr& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(p->uid());
  if (it != pod_states_.end()) {
    if (assumed_.count(p->uid())) {
      if (confirm_assumed_locked(it, p)) return;
      // Confirmation of an assumed pod: replace with the informer's object
      // (it carries the bound annotations) on the node it was bound to.
      remove_pod_locked(it->second.pod);
      add_pod_locked(p);
      assumed_.erase(p->uid());
      it->second = PodState{p, 0, false};
    } else {
      remove_pod_locked(it->second.pod);
      add_pod_locked(p);
      it->second.pod = p;
    }
    return;
  }
  add_pod_locked(p);
  pod_states_[p->uid()] = PodState{p, 0, false};
  pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
}

void SchedulerCache::update_pod(const PodPtr& old_pod, const PodPtr& new_pod) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(new_pod->uid());
  if (it == pod_states_.end()) {
    add_pod_locked(new_pod);
    pod_states_[new_pod->uid()] = PodState{new_pod, 0, false};
    pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
    return;
  }
  if (assumed_.count(new_pod->uid())) {
    // An update for an assumed pod means it got bound: confirm it.
    if (confirm_assumed_locked(it, new_pod)) return;
    remove_pod_locked(it->second.pod);
    add_pod_locked(new_pod);
    assumed_.erase(new_pod->uid());
    it->second = PodState{new_pod, 0, false};
    return;
  }
  remove_pod_locked(it->second.pod);
  add_pod_locked(new_pod);
  it->second.pod = new_pod;
}

void SchedulerCache::remove_pod(const Pod& p) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(p.uid());
  if (it == pod_states_.end()) return;
  remove_pod_locked(it->second.pod);
  assumed_.erase(p.uid());
  pod_states_.erase(it);
  pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
}

void SchedulerCache::remove_pods(const std::vector<PodPtr>& ps) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  for (const auto& p : ps) {
    auto it = pod_states_.find(p->uid());
    if (it == pod_states_.end()) continue;
    remove_pod_locked(it->second.pod);
    assumed_.erase(p->uid());
    pod_states_.erase(it);
    pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
  }
}

bool SchedulerCache::is_assumed(const std::string& uid) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return assumed_.count(uid) > 0;
}

PodPtr SchedulerCache::get_pod(const std::string& uid) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(uid);
  return it == pod_states_.end() ? nullptr : it->second.pod;
}

PodPtr SchedulerCache::mutate_pod(const std::string& uid, const std::function<void(Pod&)>& fn) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = pod_states_.find(uid);
  if (it == pod_states_.end()) return nullptr;
  auto fresh = std::make_shared<Pod>(*it->second.pod);
  fn(*fresh);
  fresh->recompute_gpu_assignment(*gpu_names_);
  remove_pod_locked(it->second.pod);
  add_pod_locked(fresh);
  it->second.pod = fresh;
  return fresh;
}

PodPtr SchedulerCache::annotate_assumed_pod(const std::string& uid, const std::function<void(Pod&)>& fn,
                                            bool recompute) {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    auto it = pod_states_.find(uid);
    if (it == pod_states_.end()) return nullptr;
    auto nit = nodes_.find(it->second.pod->node_name);
    if (assumed_.count(uid) && !it->second.binding_finished && nit != nodes_.end()) {
      PodPtr pod = it->second.pod;
      in_place_ = true;  // scheduling thread, same cycle as assume_pod
      NodeInfo& ni = writable(nit->second);
      ni.gpu.apply(pod->gpu, -1);
      fn(*pod);
      if (recompute) pod->recompute_gpu_assignment(*gpu_names_);
      ni.gpu.apply(pod->gpu, +1);
      mark_dirty(pod->node_name);
      in_place_ = false;
      return pod;
    }
  }
  return mutate_pod(uid, fn);
}

namespace {
// Keeps node i's membership in one of the Snapshot's affinity lists in step
// with its current NodeInfo version (swap-remove on leave).
void sync_member(std::vector<NodeInfoPtr>& list, std::vector<int32_t>& pos, std::vector<uint32_t>& idx, size_t i,
                 const NodeInfoPtr& ni, bool want) {
  int32_t p = pos[i];
  if (want) {
    if (p >= 0) {
      if (list[p] != ni) list[p] = ni;
    } else {
      pos[i] = static_cast<int32_t>(list.size());
      list.push_back(ni);
      idx.push_back(static_cast<uint32_t>(i));
    }
  } else if (p >= 0) {
    size_t last = list.size() - 1;
    if (static_cast<size_t>(p) != last) {
      list[p] = std::move(list[last]);
      idx[p] = idx[last];
      pos[idx[p]] = p;
    }
    list.pop_back();
    idx.pop_back();
    pos[i] = -1;
  }
}

void sync_affinity_lists(Snapshot& s, size_t i) {
  const NodeInfoPtr& ni = s.nodes[i];
  sync_member(s.have_pods_with_affinity, s.affinity_pos, s.affinity_idx, i, ni, !ni->pods_with_affinity.empty());
  sync_member(s.have_pods_with_required_anti_affinity, s.anti_pos, s.anti_idx, i, ni,
              !ni->pods_with_required_anti_affinity.empty());
}
}  // namespace

int SchedulerCache::update_snapshot(Snapshot& s, int64_t* lock_wait_us, const std::string* check_assumed,
                                    bool* is_assumed) {
  int64_t t0 = lock_wait_us ? clock_->now_us() : 0;
  std::lock_guard<AdaptiveMutex> g(mu_);
  if (lock_wait_us) *lock_wait_us = clock_->now_us() - t0;
  if (check_assumed && is_assumed) *is_assumed = assumed_.count(*check_assumed) > 0;
  int clones = 0;
  if (structure_changed_) {
    for (auto& ni : s.nodes) s.retired.push_back(std::move(ni));
    s.nodes.clear();
    s.names.clear();
    s.by_name.clear();
    s.index.clear();
    s.nodes.reserve(order_.size());
    s.names.reserve(order_.size());
    for (const auto& name : order_) {
      auto it = nodes_.find(name);
      if (it == nodes_.end() || !it->second->node) continue;
      const NodeInfoPtr& cl = it->second;
      ++clones;
      s.index[name] = s.nodes.size();
      s.nodes.push_back(cl);
      s.names.push_back(name);
      s.by_name[name] = cl;
    }
    structure_changed_ = false;
    s.gen.resize(s.nodes.size());
    s.free_whole.resize(s.nodes.size());
    s.free_xcd.resize(s.nodes.size());
    s.part_mask.resize(s.nodes.size());
    s.reset_gpu_sums();
    for (size_t i = 0; i < s.nodes.size(); ++i) s.set_gpu_summary(i, /*fresh=*/true);
    s.have_pods_with_affinity.clear();
    s.have_pods_with_required_anti_affinity.clear();
    s.affinity_idx.clear();
    s.anti_idx.clear();
    s.affinity_pos.assign(s.nodes.size(), -1);
    s.anti_pos.assign(s.nodes.size(), -1);
    for (size_t i = 0; i < s.nodes.size(); ++i) sync_affinity_lists(s, i);
  } else {
    for (const auto& name : dirty_) {
      auto it = nodes_.find(name);
      if (it == nodes_.end() || !it->second->node) continue;
      auto sit = s.by_name.find(name);
      if (sit == s.by_name.end()) continue;
      const NodeInfoPtr& cl = it->second;
      size_t i = s.index[name];
      // Same pointer: updated in place (assume/Reserve), the Snapshot
      // already sees it; only its list membership may have changed.
      if (sit->second != cl) {
        ++clones;
        s.retired.push_back(s.nodes[i]);
        s.nodes[i] = cl;
        sit->second = cl;
      }
      s.set_gpu_summary(i);
      sync_affinity_lists(s, i);
    }
  }
  dirty_.clear();
  if (s.deltas_wanted && !track_deltas_) {
    // Events were not recorded so far: jump the sequence past the log so
    // no state memoized before now can be replayed.
    track_deltas_ = true;
    delta_seq_ += Snapshot::kMaxDeltas + 1;
  }
  for (auto& d : pending_deltas_) s.deltas.push_back(std::move(d));
  pending_deltas_.clear();
  while (s.deltas.size() > Snapshot::kMaxDeltas) {
    s.retired_deltas.push_back(std::move(s.deltas.front()));
    s.deltas.pop_front();
  }
  s.delta_end = delta_seq_;
  s.topology_epoch = topology_epoch_;
  s.generation = generation_;
  s.nodes_with_prefer_no_schedule = prefer_nodes_;
  s.min_pod_priority = prio_count_.empty() ? INT32_MAX : prio_count_.begin()->first;
  s.hostname_domains_are_nodes = foreign_hostnames_ == 0;
  if (s.image_spread != image_spread_) s.image_spread = image_spread_;
  s.node_epoch = node_epoch_;
  return clones;
}

void SchedulerCache::cleanup_expired_assumed_pods() {
  std::lock_guard<AdaptiveMutex> g(mu_);
  int64_t now = clock_->now_us();
  std::vector<std::string> expired;
  for (const auto& uid : assumed_) {
    auto it = pod_states_.find(uid);
    if (it == pod_states_.end()) continue;
    if (it->second.binding_finished && it->second.deadline_us > 0 && now > it->second.deadline_us)
      expired.push_back(uid);
  }
  for (const auto& uid : expired) {
    auto it = pod_states_.find(uid);
    remove_pod_locked(it->second.pod);
    assumed_.erase(uid);
    pod_states_.erase(it);
    pod_count_.store(pod_states_.size(), std::memory_order_relaxed);
  }
}

int SchedulerCache::assigned_in_group(uint64_t pg_key) const {
  std::lock_guard<AdaptiveMutex> g(group_mu_);
  auto it = group_assigned_.find(pg_key);
  return it == group_assigned_.end() ? 0 : it->second;
}

size_t SchedulerCache::node_count() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return order_.size();
}

size_t SchedulerCache::pod_count() const { return pod_count_.load(std::memory_order_relaxed); }

size_t SchedulerCache::assumed_count() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return assumed_.size();
}

NodeInfoPtr SchedulerCache::node_info_copy(const std::string& name) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = nodes_.find(name);
  return it == nodes_.end() ? nullptr : it->second->clone();
}

std::vector<SchedulerCache::GpuCensusRow> SchedulerCache::gpu_census() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  std::vector<GpuCensusRow> out;
  out.reserve(order_.size());
  std::unordered_map<std::string, size_t> row;
  for (const auto& name : order_) {
    auto it = nodes_.find(name);
    if (it == nodes_.end() || !it->second->node) continue;
    const GpuLedger& L = it->second->gpu;
    GpuCensusRow r;
    r.node = name;
    for (int gi = 0; gi < L.gpu_count; ++gi) r.spx += L.parts[gi] == 1;
    r.free_whole = L.free_gpus();
    row.emplace(name, out.size());
    out.push_back(std::move(r));
  }
  for (const auto& uid : assumed_) {
    auto it = pod_states_.find(uid);
    if (it == pod_states_.end()) continue;
    const Pod& p = *it->second.pod;
    if (p.gpu_demand.kind != GpuDemand::Gpu) continue;
    auto r = row.find(p.node_name);
    if (r != row.end()) out[r->second].assumed_whole += static_cast<int>(p.gpu_demand.amount);
  }
  return out;
}

std::vector<std::string> SchedulerCache::node_names() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return order_;
}

}  // namespace xsched

namespace xsched {

Json SchedulerCache::check(const std::vector<PodPtr>& assigned, const std::vector<std::string>& nodes) const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  Json out = Json::object();
  auto list = [](const std::vector<std::string>& v) {
    Json a = Json::array();
    for (const auto& x : v) a.push_back(Json(x));
    return a;
  };
  // Pods: the listers' assigned pods vs the cache's non-assumed pods.
  std::vector<std::string> missing, redundant, wrong;
  std::unordered_map<std::string, const Pod*> truth;
  for (const auto& p : assigned) truth[p->uid()] = p.get();
  size_t assumed_n = 0;
  for (const auto& [uid, st] : pod_states_) {
    auto it = truth.find(uid);
    if (assumed_.count(uid)) {
      ++assumed_n;  // not bound yet, or bound and not confirmed: either is fine
      if (it != truth.end() && it->second->node_name != st.pod->node_name)
        wrong.push_back(st.pod->key() + ": cache " + st.pod->node_name + ", listers " + it->second->node_name);
      continue;
    }
    if (it == truth.end()) {
      redundant.push_back(st.pod->key());
    } else if (it->second->node_name != st.pod->node_name) {
      wrong.push_back(st.pod->key() + ": cache " + st.pod->node_name + ", listers " + it->second->node_name);
    }
  }
  for (const auto& p : assigned)
    if (!pod_states_.count(p->uid())) missing.push_back(p->key());
  // Nodes.
  std::set<std::string> want(nodes.begin(), nodes.end()), have;
  for (const auto& [name, ni] : nodes_)
    if (ni->node) have.insert(name);
  std::vector<std::string> missing_nodes, redundant_nodes;
  std::set_difference(want.begin(), want.end(), have.begin(), have.end(), std::back_inserter(missing_nodes));
  std::set_difference(have.begin(), have.end(), want.begin(), want.end(), std::back_inserter(redundant_nodes));
  // Accounting: every NodeInfo against one rebuilt from its pods; each pod's
  // NodeInfo is the one of its node.
  Json acct = Json::array();
  for (const auto& [name, ni] : nodes_) {
    std::vector<std::string> bad = ni->verify();
    for (const auto& p : ni->pods)
      if (p->node_name != name) bad.push_back("pod " + p->key() + " names node " + p->node_name);
    if (bad.empty()) continue;
    Json e = Json::object();
    e.set("node", Json(name));
    e.set("fields", list(bad));
    acct.push_back(std::move(e));
  }
  // PodGroup counts: the O(1) counters against a recount of cached pods.
  std::unordered_map<uint64_t, int> recount;
  for (const auto& [uid, st] : pod_states_)
    if (st.pod->pg_key) ++recount[st.pod->pg_key];
  std::vector<std::string> groups;
  {
    std::lock_guard<AdaptiveMutex> gg(group_mu_);
    for (const auto& [k, c] : recount) {
      auto it = group_assigned_.find(k);
      int have_c = it == group_assigned_.end() ? 0 : it->second;
      if (have_c != c)
        groups.push_back(std::to_string(k) + ": counter " + std::to_string(have_c) + ", pods " + std::to_string(c));
    }
    for (const auto& [k, c] : group_assigned_)
      if (c != 0 && !recount.count(k)) groups.push_back(std::to_string(k) + ": counter " + std::to_string(c) + ", pods 0");
  }
  bool clean = missing.empty() && redundant.empty() && wrong.empty() && missing_nodes.empty() &&
               redundant_nodes.empty() && acct.size() == 0 && groups.empty();
  out.set("clean", Json(clean));
  out.set("missing_pods", list(missing));
  out.set("redundant_pods", list(redundant));
  out.set("wrong_node", list(wrong));
  out.set("missing_nodes", list(missing_nodes));
  out.set("redundant_nodes", list(redundant_nodes));
  out.set("accounting", std::move(acct));
  out.set("group_counts", list(groups));
  out.set("assumed", Json(static_cast<int64_t>(assumed_n)));
  return out;
}

Json SchedulerCache::dump() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  Json out = Json::object();
  Json ns = Json::array();
  for (const auto& name : order_) {
    auto it = nodes_.find(name);
    if (it == nodes_.end()) continue;
    const NodeInfo& ni = *it->second;
    Json n = Json::object();
    n.set("name", Json(name));
    Json pods = Json::array();
    for (const auto& p : ni.pods) pods.push_back(Json(p->key() + (assumed_.count(p->uid()) ? " (assumed)" : "")));
    n.set("pods", std::move(pods));
    Json req = Json::object();
    for (uint64_t m = ni.requested.mask; m; m &= m - 1) {
      int id = __builtin_ctzll(m);
      req.set(ResourceRegistry::get().name(id), Json(ni.requested.v[id]));
    }
    n.set("requested", std::move(req));
    if (ni.gpu.gpu_count > 0) {
      Json gj = Json::object();
      gj.set("gpus", Json(ni.gpu.gpu_count));
      gj.set("free_whole", Json(ni.gpu.free_gpus()));
      gj.set("free_xcds", Json(ni.gpu.free_xcds()));
      gj.set("free_memory", Json(ni.gpu.free_memory()));
      n.set("gpu", std::move(gj));
    }
    n.set("generation", Json(ni.generation));
    ns.push_back(std::move(n));
  }
  out.set("nodes", std::move(ns));
  out.set("pods", Json(static_cast<int64_t>(pod_states_.size())));
  out.set("assumed", Json(static_cast<int64_t>(assumed_.size())));
  return out;
}

}  // namespace xsched
