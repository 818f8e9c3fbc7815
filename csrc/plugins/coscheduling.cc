// Coscheduling: PodGroup gang admission.
//
// Reference: pkg/coscheduling/coscheduling.go:42-252 and
// pkg/coscheduling/core/core.go:56-382.
// Semantics kept: QueueSort by priority, PodGroup creation time, ns/name;
// PreFilter denies recently-denied groups (TTL cache), groups with fewer
// labelled pods than minMember and groups whose MinResources do not fit the
// cluster; Permit waits until assigned+1 >= minMember and then Allows every
// waiting sibling; Wait activates siblings; PostFilter/Unreserve reject the
// whole group and deny it for deniedPGExpirationTimeSeconds; PostBind
// patches the PodGroup status when its phase flips.
//
// Differences by design: assigned counts come from the cache's per-group
// counter (O(1)) instead of a scan of every pod on every node; the TTL maps
// are swept by the shared timer service.
//
// Deliberate deviation (arg transientShortage, default "Park";
// docs/ARCHITECTURE.md §4, "Gang parking"): a gang of GPU ranks whose
// remaining members do not fit the GPUs free right now is *parked* instead of
// denied for deniedPGExpirationTimeSeconds:
//  * PreFilter gate: before a member is placed, the GPUs (or XCD partitions)
//    free in the cycle's snapshot, less those still owed to gangs already
//    waiting at Permit and to the oldest parked gang, must cover the group's
//    remaining members; otherwise the group parks (Unschedulable, nothing is
//    assumed, so it holds no GPUs that other gangs wait for);
//  * PostFilter: a member that fails Filter while the gate's arithmetic says
//    the GPUs are short rejects its waiting siblings (releasing their GPUs)
//    and parks the group instead of denying it;
//  * every release of capacity (a pod deleted or forgotten, a node added)
//    sends one probe member of the oldest parked group back to the active
//    queue (skipping backoff); when its gate passes the group un-parks and the
//    next parked group is probed.
// Genuine shortfalls keep the reference's semantics: a group bigger than the
// cluster's GPUs, a failure the GPU count does not explain (affinity,
// fragmentation, CPU/memory) and Permit timeouts are denied for the TTL.
// "Deny" restores the reference's behaviour everywhere.
#include <algorithm>
#include <unordered_set>
#include <array>
#include <deque>
#include <map>
#include <mutex>
#include <unordered_map>

#include <atomic>

#include "framework/plugin.h"
#include "framework/waiting_pods.h"
#include "scheduler/cache.h"
#include "scheduler/gang_placement.h"
#include "scheduler/informers.h"
#include "scheduler/metrics.h"
#include "store/store.h"

namespace xsched {
namespace {

// go-cache style TTL set of PodGroups (core.go:103-104: lastDeniedPG,
// permittedPG), keyed by Pod::pg_key. `has` on an empty set (the common case:
// no group denied) is one atomic load, no lock.
class TTLSet {
 public:
  explicit TTLSet(std::shared_ptr<Clock> c) : clock_(std::move(c)) {}
  void add(uint64_t k, int64_t ttl_us) {
    std::lock_guard<std::mutex> g(mu_);
    m_[k] = clock_->now_us() + ttl_us;
    size_.store(m_.size(), std::memory_order_release);
  }
  bool has(uint64_t k) {
    if (size_.load(std::memory_order_acquire) == 0) return false;
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(k);
    if (it == m_.end()) return false;
    if (clock_->now_us() >= it->second) {
      m_.erase(it);
      size_.store(m_.size(), std::memory_order_release);
      return false;
    }
    return true;
  }
  void erase(uint64_t k) {
    if (size_.load(std::memory_order_acquire) == 0) return;
    std::lock_guard<std::mutex> g(mu_);
    m_.erase(k);
    size_.store(m_.size(), std::memory_order_release);
  }
  void sweep() {
    std::lock_guard<std::mutex> g(mu_);
    int64_t now = clock_->now_us();
    for (auto it = m_.begin(); it != m_.end();) it = now >= it->second ? m_.erase(it) : std::next(it);
    size_.store(m_.size(), std::memory_order_release);
  }

 private:
  std::shared_ptr<Clock> clock_;
  std::mutex mu_;
  std::unordered_map<uint64_t, int64_t> m_;
  std::atomic<size_t> size_{0};
};

class Coscheduling : public Plugin {
 public:
  Coscheduling(const Json& args, Handle& h)
      : Plugin("Coscheduling", kQueueSort | kPreFilter | kPostFilter | kReserve | kPermit | kPostBind),
        h_(h),
        denied_(h.clock),
        permitted_(h.clock) {
    permit_wait_us_ = args["permitWaitingTimeSeconds"].as_int(60) * 1000000;
    denied_ttl_us_ = args["deniedPGExpirationTimeSeconds"].as_int(20) * 1000000;
    const std::string mode = args["transientShortage"].str_or("Park");
    if (mode == "Park") park_ = true;
    else if (mode == "Deny") park_ = false;
    else throw std::runtime_error("Coscheduling transientShortage must be Park or Deny, not " + mode);
  }

  void start() override {
    sweep_id_ = h_.timers->every(3'000'000, [this] {
      denied_.sweep();
      permitted_.sweep();
      sweep_outstanding();
    });
  }
  void stop() override {
    if (sweep_id_) h_.timers->cancel(sweep_id_);
  }

  // ---- QueueSort ----
  // GetCreationTimestamp (core.go:255-265). A PodGroup's creationTimestamp
  // never changes, so once found it is memoized on the queued pod (Less runs
  // O(log n) times per heap operation, under the queue lock).
  MicroTime creation(const QueuedPodInfo& q) const {
    if (q.sort_key_cache != INT64_MIN) return q.sort_key_cache;
    if (!q.pod->pod_group.empty())
      if (auto pg = h_.informers->pod_group_of(*q.pod)) {
        q.sort_key_cache = pg->meta.creation;
        return q.sort_key_cache;
      }
    return q.initial_attempt_wall;
  }
  bool less(const QueuedPodInfo& a, const QueuedPodInfo& b) const override {
    const int32_t pa = a.priority(), pb = b.priority();
    if (pa != pb) return pa > pb;
    MicroTime ta = creation(a), tb = creation(b);
    if (ta == tb) return key_less(*a.pod, *b.pod);
    return ta < tb;
  }
  // "ns/name" < "ns/name" without building the strings (gang members tie on
  // the group timestamp, so this runs on most heap comparisons).
  static bool key_less(const Pod& a, const Pod& b) {
    if (a.ns() == b.ns()) return a.name() < b.name();
    auto at = [](const Pod& p, size_t i) -> unsigned char {
      size_t n = p.ns().size();
      return static_cast<unsigned char>(i < n ? p.ns()[i] : i == n ? '/' : p.name()[i - n - 1]);
    };
    size_t la = a.ns().size() + 1 + a.name().size(), lb = b.ns().size() + 1 + b.name().size();
    for (size_t i = 0, m = std::min(la, lb); i < m; ++i) {
      unsigned char ca = at(a, i), cb = at(b, i);
      if (ca != cb) return ca < cb;
    }
    return la < lb;
  }

  // ---- PreFilter (core.go:149-196) ----
  Status pre_filter(CycleState&, const Pod& p) override {
    if (p.pod_group.empty()) return {};
    auto pg = h_.informers->pod_group_of(p);
    if (!pg) return {};
    if (denied_.has(p.pg_key)) {
      // A parked group that is now denied leaves the parking line (its
      // requeue timer brings the members back after the TTL).
      if (park_) drop_parked(p.pg_key, false);
      return Status::unresolvable("pod with pgName: " + p.pg_full_name() + " last failed in " +
                                  std::to_string(denied_ttl_us_ / 1000000) + "s, deny");
    }
    size_t n = h_.informers->count_pods_in_group_of(p);
    if (static_cast<int64_t>(n) < pg->min_member) {
      // A parked group that lost members (one deleted, the PodGroup kept)
      // cannot pass the gate until new ones arrive: it must not stay at the
      // head of the line, where it would hold back every younger gang. Its
      // members return to the queues and wait for a Pod add, as upstream.
      if (park_) drop_parked(p.pg_key, true);
      return Status::unresolvable("pre-filter pod " + p.name() + " cannot find enough sibling pods, current pods number: " +
                                  std::to_string(n) + ", minMember of group: " + std::to_string(pg->min_member));
    }
    if (park_) {
      Status gs = gang_gate(p, *pg);
      if (!gs.is_success()) return gs;
    }
    if (!pg->has_min_resources) return {};
    if (permitted_.has(p.pg_key)) return {};
    Res need = pg->min_resources;
    need.set(kPods, pg->min_member);
    if (!check_cluster_resource(need, p)) {
      deny(p, "minresources");
      return Status::unresolvable("resource gap for PodGroup " + p.pg_full_name());
    }
    permitted_.add(p.pg_key, wait_time(*pg));
    return {};
  }

  // CheckClusterResource (core.go:322-382): greedily subtract each node's
  // free resources (with this group's own pods counted as free).
  bool check_cluster_resource(Res need, const Pod& member) const {
    if (!h_.snapshot) return false;
    for (const auto& ni : h_.snapshot->nodes) {
      if (!ni->node) continue;
      Res left;
      Res requested = ni->requested;
      int64_t pods = ni->num_pods();
      for (const auto& q : ni->pods)
        if (q->pg_key == member.pg_key && q->pod_group == member.pod_group && q->ns() == member.ns()) {
          requested -= q->request();
          --pods;
        }
      left.set(kPods, ni->allocatable.get(kPods) - pods);
      for (uint64_t m = ni->allocatable.mask; m; m &= m - 1) {
        int i = __builtin_ctzll(m);
        if (i == kPods) continue;
        left.set(i, ni->allocatable.get(i) - requested.get(i));
      }
      bool all_done = true;
      for (uint64_t m = need.mask; m; m &= m - 1) {
        int i = __builtin_ctzll(m);
        if (need.v[i] <= 0) continue;
        need.v[i] -= left.get(i);
        if (need.v[i] > 0) all_done = false;
      }
      if (all_done) return true;
    }
    for (uint64_t m = need.mask; m; m &= m - 1)
      if (need.v[__builtin_ctzll(m)] > 0) return false;
    return true;
  }

  int64_t wait_time(const PodGroup& pg) const {
    if (pg.schedule_timeout_seconds >= 0) return static_cast<int64_t>(pg.schedule_timeout_seconds) * 1000000;
    if (permit_wait_us_ > 0) return permit_wait_us_;
    return 60'000'000;  // util.DefaultWaitTime
  }

  // ---- PostFilter (coscheduling.go:140-176) ----
  std::pair<PostFilterResult, Status> post_filter(CycleState&, const Pod& p, const NodeStatusMap& m) override {
    auto pg = p.pod_group.empty() ? nullptr : h_.informers->pod_group_of(p);
    if (!pg) return {PostFilterResult{}, Status::unschedulable("can not find pod group")};
    // Deliberate deviation: when the cycle failed on this plugin's own
    // PreFilter (siblings not created yet, or group already denied) there is
    // no placement evidence, so the group is not (re-)denied — the reference
    // would deny it and, for the "denied" case, keep refreshing the TTL.
    if (!m.empty() && m.begin()->second.failed_plugin() == name())
      return {PostFilterResult{}, Status(Code::Unschedulable)};
    std::string full = p.pg_full_name();
    int assigned = h_.cache->assigned_in_group(p.pg_key);
    if (assigned >= pg->min_member) return {PostFilterResult{}, Status(Code::Unschedulable)};
    float gap = static_cast<float>(pg->min_member - assigned) / static_cast<float>(std::max(1, pg->min_member));
    if (gap <= 0.1f) return {PostFilterResult{}, Status(Code::Unschedulable)};
    if (park_ && gpu_shortage_explains(p, *pg)) {
      // Transient GPU shortage: release the siblings' GPUs, park the group.
      if (h_.metrics)
        h_.metrics->inc("xsched_coscheduling_gate_waits_total",
                        kind_slot(p.gpu_demand.kind) == 0 ? "cause=\"postfilter\",kind=\"gpu\""
                                                          : "cause=\"postfilter\",kind=\"xcd\"");
      park_rejecting(p, *pg);
      permitted_.erase(p.pg_key);
      return {PostFilterResult{}, XS_FIXED_STATUS(Code::Unschedulable,
                                                  "PodGroup parked: its remaining members need more GPUs than are "
                                                  "free; it retries when GPUs are released")};
    }
    reject_group(p, "optimistic rejection in PostFilter");
    drop_outstanding(p.pg_key);
    deny(p, "postfilter");
    permitted_.erase(p.pg_key);
    return {PostFilterResult{},
            Status::unschedulable("PodGroup " + full + " gets rejected due to Pod " + p.name() +
                                  " is unschedulable even after PostFilter")};
  }

  // Denies p's group for the TTL and, when the TTL runs out, moves its
  // unschedulable members back to the active queue. Without that, a group
  // denied after its last member arrived (e.g. a Permit timeout breaking a
  // gang deadlock at full capacity) waits for the unschedulable-queue flush
  // (60 s): no cluster event is left to requeue it.
  // One requeue timer per group at a time: Unreserve runs once per rejected
  // member, so a gang denial calls deny() k times; later calls only push the
  // pending timer's deadline (it re-arms itself for the remainder).
  void deny(const Pod& p, const char* why) {
    const bool fresh_denial = !denied_.has(p.pg_key);
    denied_.add(p.pg_key, denied_ttl_us_);
    if (fresh_denial && h_.gang_denied) h_.gang_denied(p, why);
    if (!h_.timers || !h_.activate) return;
    const int64_t due = h_.clock->now_us() + denied_ttl_us_ + 1000;
    {
      std::lock_guard<std::mutex> g(requeue_mu_);
      auto [it, fresh] = requeue_due_.try_emplace(p.pg_key, due);
      if (!fresh) {
        it->second = std::max(it->second, due);
        return;
      }
    }
    auto member = std::make_shared<Pod>();
    member->meta.ns = p.ns();
    member->pod_group = p.pod_group;
    member->pg_key = p.pg_key;
    arm_requeue(member, denied_ttl_us_ + 1000);
  }

  void arm_requeue(const std::shared_ptr<Pod>& member, int64_t after_us) {
    h_.timers->schedule_after(after_us, [this, member] {
      {
        std::lock_guard<std::mutex> g(requeue_mu_);
        auto it = requeue_due_.find(member->pg_key);
        if (it == requeue_due_.end()) return;
        int64_t left = it->second - h_.clock->now_us();
        if (left > 0) {  // denied again meanwhile: wait out the newest denial
          arm_requeue(member, left);
          return;
        }
        requeue_due_.erase(it);
      }
      if (denied_.has(member->pg_key)) return;
      std::vector<PodPtr> pods;
      for (auto& q : h_.informers->pods_in_group_of(*member))
        if (q->node_name.empty()) pods.push_back(std::move(q));
      if (!pods.empty()) h_.activate(pods);
    });
  }

  // Rejects every waiting member of p's group (the group index visits only
  // that group's waiting pods; names are still compared, as the key is a hash).
  void reject_group(const Pod& p, const std::string& msg) {
    h_.waiting_pods->iterate_group(p.pg_key, [&](const WaitingPodPtr& wp) {
      const Pod& wpod = *wp->pod();
      if (wpod.ns() == p.ns() && wpod.pod_group == p.pod_group) wp->reject(name(), msg);
    });
  }
  int count_waiting(const Pod& p) {
    int n = 0;
    h_.waiting_pods->iterate_group(p.pg_key, [&](const WaitingPodPtr& wp) {
      const Pod& wpod = *wp->pod();
      n += wpod.ns() == p.ns() && wpod.pod_group == p.pod_group;
    });
    return n;
  }

  // ---- Permit (coscheduling.go:184-216, core.go:199-216) ----
  std::pair<Status, int64_t> permit(CycleState& s, const PodPtr& p, const std::string&) override {
    if (p->pod_group.empty()) return {Status(), 0};
    auto pg = h_.informers->pod_group_of(*p);
    if (!pg) return {Status::unschedulable("PodGroup not found"), 0};
    // The cache already holds this (assumed) pod, so `assigned` includes it:
    // equivalent to the reference's snapshot count + 1.
    int assigned = h_.cache->assigned_in_group(p->pg_key);
    if (assigned < pg->min_member) {
      if (park_) note_outstanding(*p, pg->min_member - assigned);
      // The first waiting member activates its siblings; the next ones of the
      // same gang, arriving in order with more members assigned, would list
      // and re-activate the same pods (O(k^2) per gang of k). A gang that
      // starts over (fewer assigned than last time) activates again.
      if (p->pg_key != act_key_ || assigned <= act_assigned_) activate_siblings(*p, s);
      act_key_ = p->pg_key;
      act_assigned_ = assigned;
      return {Status(Code::Wait), wait_time(*pg)};
    }
    if (park_) drop_outstanding(p->pg_key);
    h_.waiting_pods->iterate_group(p->pg_key, [&](const WaitingPodPtr& wp) {
      const Pod& q = *wp->pod();  // flat group key first: no string build per waiting pod
      if (q.pg_key == p->pg_key && q.pod_group == p->pod_group && q.ns() == p->ns()) wp->allow(name());
    });
    return {Status(), 0};
  }

  void activate_siblings(const Pod& p, CycleState& s) {
    auto* pta = s.read_as<PodsToActivate>(kPodsToActivateKey);
    if (!pta) return;
    auto pods = h_.informers->pods_in_group_of(p);
    std::lock_guard<std::mutex> g(pta->mu);
    for (const auto& q : pods)
      if (q->uid() != p.uid()) pta->pods.push_back(q);
  }

  // ---- Reserve / Unreserve (coscheduling.go:219-237) ----
  Status reserve(CycleState&, const PodPtr&, const std::string&) override { return {}; }
  void unreserve(CycleState&, const PodPtr& p, const std::string&) override {
    if (p->pod_group.empty()) return;
    auto pg = h_.informers->pod_group_of(*p);
    if (!pg) {
      // The group was deleted while this member waited at Permit: nothing to
      // reject or deny, but the GPUs noted as owed to it must not stay owed
      // (they held every later gang's gate shut until the 15-min sweep).
      if (park_) drop_outstanding(p->pg_key);
      return;
    }
    // A sibling rejected because its group parked (PostFilter): no denial.
    if (park_ && consume_parked_reject(p->pg_key, p->uid())) return;
    reject_group(*p, "rejection in Unreserve");
    drop_outstanding(p->pg_key);
    deny(*p, "unreserve");
    permitted_.erase(p->pg_key);
  }

  // ---- PostBind (core.go:220-252) ----
  void post_bind(CycleState&, const PodPtr& p, const std::string&) override {
    if (p->pod_group.empty()) return;
    auto pg = h_.informers->pod_group_of(*p);
    if (!pg) return;
    // Deliberate fix: the reference increments the lister's status.scheduled,
    // which is only written back on a phase change (core.go:220-252), so the
    // count goes stale after the first member (a gang of 4 sticks at
    // Scheduling/1). We take the larger of that and the group's assigned
    // (assumed + bound) pods from the cache.
    int32_t scheduled = std::max<int32_t>(pg->scheduled + 1, h_.cache->assigned_in_group(p->pg_key));
    std::string phase;
    Json status = Json::object();
    if (scheduled >= pg->min_member) {
      phase = "Scheduled";
    } else {
      phase = "Scheduling";
      if (pg->schedule_start_time == 0) status.set("scheduleStartTime", Json(format_rfc3339(wall_now_us())));
    }
    if (phase == pg->phase) return;  // the reference PATCHes only on phase change
    // The gang's members bind concurrently and the PodGroup in the informer
    // lags our own PATCH, so every member would see the old phase and send
    // the same PATCH (8 per 8-rank gang): one PATCH per group and phase.
    if (!note_patched(p->pg_key, pg->meta.uid, phase)) return;
    status.set("phase", Json(phase));
    status.set("scheduled", Json(static_cast<int64_t>(scheduled)));
    Json patch = Json::object();
    patch.set("status", std::move(status));
    try {
      h_.client->patch("podgroups", pg->meta.ns, pg->meta.name, patch);
    } catch (const std::exception&) {
    }
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kAdd, ""}, {"PodGroup", kAdd | kUpdate, ""}};
  }

  // A deleted PodGroup leaves the PATCH memo (its entries would otherwise
  // live out the memo window: 10^5 of them after a few seconds at full
  // rate).
  std::vector<std::string> watched_kinds() const override { return {"podgroups"}; }
  void on_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr&) override {
    if (kind != "podgroups" || static_cast<EventType>(type) != EventType::Deleted || !obj) return;
    const Json& md = (*obj)["metadata"];
    std::string full = md["namespace"].str_or("default");
    full.push_back('/');
    full += md["name"].as_string();
    const uint64_t key = pg_key_of(full);
    {
      PatchShard& sh = patch_shard(key);
      std::lock_guard<std::mutex> g(sh.mu);
      sh.map.erase(key);
    }
    if (park_) forget_group(key, md["uid"].as_string());
  }
  // A deleted group leaves the parking state: GPUs owed to it at Permit, its
  // parked entry (the oldest parked group reserves its need against every
  // younger gang until a probe finds it empty) and its pending rejections,
  // at once rather than at the next probe or sweep (an open-loop overload
  // ends with thousands of gangs deleted mid-admission).
  void forget_group(uint64_t key, const std::string& uid) {
    std::vector<PodPtr> probe;
    {
      std::lock_guard<std::mutex> g(park_mu_);
      // A member of the group may be inside its cycle right now, holding the
      // PodGroup object from before the deletion: its gate must not park the
      // group again after this (it would stay in the line with no event left
      // to remove it). Remembered by uid, so a group recreated under the same
      // name parks as usual.
      if (!uid.empty()) {
        // Expired in insertion order (O(1) amortised: a burst wave deletes
        // thousands of groups per second).
        const int64_t now = h_.clock->now_us();
        while (!deleted_order_.empty() && now - deleted_order_.front().first > kRejectWindowUs) {
          deleted_uids_.erase(deleted_order_.front().second);
          deleted_order_.pop_front();
        }
        if (deleted_uids_.insert(uid).second) deleted_order_.emplace_back(now, uid);
      }
      erase_outstanding_locked(key);
      parked_rejects_.erase(key);
      unpark_locked(key, probe);
    }
    if (!probe.empty()) h_.activate(probe);
  }
  // Removes `key` from the parking line. When it was the head of its kind's
  // line or that kind's outstanding probe, the next group of the kind is
  // probed (appended to `probe`).
  void unpark_locked(uint64_t key, std::vector<PodPtr>& probe) {
    auto pos = parked_pos_.find(key);
    int slot = -1;
    bool head = false;
    if (pos != parked_pos_.end()) {
      slot = pos->second.slot;
      head = oldest_locked(slot) == parked_.find(pos->second);
      parked_.erase(pos->second);
      parked_pos_.erase(pos);
      parked_n_.store(parked_.size(), std::memory_order_release);
    }
    for (int k = 0; k < 2; ++k) {
      const bool was_probe = probe_key_[k] == key;
      if (was_probe) probe_key_[k] = 0;
      if ((was_probe || (head && k == slot)) && !probe_key_[k]) {
        auto more = next_probe_locked(k);
        probe.insert(probe.end(), more.begin(), more.end());
      }
    }
    take_wake_locked(probe);
  }
  // PreFilter found p's group denied or short of members: it leaves the
  // parking line; with `wake` its parked members return to the queues.
  void drop_parked(uint64_t key, bool wake) {
    if (parked_n_.load(std::memory_order_acquire) == 0) return;
    std::vector<PodPtr> probe;
    Pod member;
    bool was = false;
    {
      std::lock_guard<std::mutex> g(park_mu_);
      auto pos = parked_pos_.find(key);
      if (pos == parked_pos_.end()) return;
      member.meta.ns = parked_[pos->second].ns;
      member.pod_group = parked_[pos->second].group;
      member.pg_key = key;
      was = true;
      unpark_locked(key, probe);
    }
    if (was && wake)
      for (auto& q : h_.informers->pods_in_group_of(member))
        if (q->node_name.empty()) probe.push_back(std::move(q));
    if (!probe.empty()) h_.activate(probe);
  }

  // Unit-test hook (core/core_test.go:303 TestCheckClusterResource):
  // args["need"] is a resource list; `p` names the group whose own pods count
  // as free. "deny" puts p's group in the denied cache (core_test.go:42's
  // pre-filled lastDeniedPG).
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    Json out = Json::object();
    if (what == "checkClusterResource") {
      out.set("enough", Json(check_cluster_resource(Res::from_json(args["need"]), *p)));
      return out;
    }
    if (what == "deny") {
      denied_.add(p->pg_key, denied_ttl_us_);
      out.set("denied", Json(true));
      return out;
    }
    if (what == "parking") {  // parked groups (oldest first) and GPUs owed to gangs at Permit
      std::lock_guard<std::mutex> g(park_mu_);
      Json groups = Json::array();
      for (const auto& [k, pk] : parked_) {
        Json e = Json::object();
        e.set("podGroup", Json(pk.ns + "/" + pk.group));
        e.set("kind", Json(pk.kind == GpuDemand::Gpu ? "gpu" : "xcd"));
        e.set("need", Json(pk.need));
        groups.push_back(std::move(e));
      }
      out.set("parked", std::move(groups));
      out.set("outstandingGpus", Json(owed_[0]));
      out.set("outstandingXcdMembers", Json(owed_[1]));
      Json probes = Json::array();
      for (int k = 0; k < 2; ++k)
        if (probe_key_[k]) probes.push_back(Json(k == 0 ? "gpu" : "xcd"));
      out.set("probing", std::move(probes));
      out.set("parksTotal", Json(static_cast<int64_t>(parks_total_)));
      return out;
    }
    return Plugin::debug_call(what, s, p, args);
  }

 private:
  // True the first time (group uid, phase) is seen within kPatchMemoUs. The
  // memo only has to outlive the informer's lag behind our own PATCH (a
  // repeated PATCH is harmless), so entries expire in insertion order from a
  // per-shard queue, O(1) per call: no sweep over the map (an amortized full
  // sweep of 10^5 entries held every binder waiting on one lock for tens of
  // ms in the open-loop runs, profiles/r5k_*). Shards split the lock.
  static constexpr int64_t kPatchMemoUs = 10'000'000;
  static constexpr size_t kPatchShards = 16;
  struct Patched {
    std::string uid, phase;
    int64_t at_us = 0;
  };
  struct PatchShard {
    std::mutex mu;
    std::unordered_map<uint64_t, Patched> map;
    std::deque<std::pair<int64_t, uint64_t>> order;  // (inserted at, key), oldest first
  };
  PatchShard& patch_shard(uint64_t key) { return patch_shards_[(key ^ (key >> 29)) % kPatchShards]; }
  bool note_patched(uint64_t key, const std::string& uid, const std::string& phase) {
    const int64_t now = h_.clock->now_us();
    PatchShard& sh = patch_shard(key);
    std::lock_guard<std::mutex> g(sh.mu);
    while (!sh.order.empty() && now - sh.order.front().first >= kPatchMemoUs) {
      auto it = sh.map.find(sh.order.front().second);
      if (it != sh.map.end() && now - it->second.at_us >= kPatchMemoUs) sh.map.erase(it);
      sh.order.pop_front();
    }
    auto& e = sh.map[key];
    if (e.uid == uid && e.phase == phase && now - e.at_us < kPatchMemoUs) return false;
    e = {uid, phase, now};
    sh.order.emplace_back(now, key);
    return true;
  }
  std::array<PatchShard, kPatchShards> patch_shards_;

  // ---- Gang gate and parking ----
  // Units: whole GPUs for GPU ranks, members for XCD-partition ranks (their
  // footprint depends on the node's partition size).
  static int kind_slot(GpuDemand::Kind k) { return k == GpuDemand::Gpu ? 0 : 1; }
  static bool gated(const GpuDemand& d) {
    return (d.kind == GpuDemand::Gpu || d.kind == GpuDemand::Xcd) && d.amount > 0;
  }
  static int64_t units_for(const GpuDemand& d, int64_t members) {
    return d.kind == GpuDemand::Gpu ? members * d.amount : members;
  }
  // XCDs one member of `amount` XCDs occupies on a GPU with `xpp`-XCD partitions.
  static int64_t footprint(int64_t amount, int64_t xpp) { return (amount + xpp - 1) / xpp * xpp; }
  static int64_t footprint_for_mask(int64_t amount, int mask) {
    int64_t per = 0;
    for (int b = 0; b < 4; ++b)
      if (mask & (1 << b)) {
        const int64_t use = footprint(amount, int64_t{1} << b);
        if (per == 0 || use < per) per = use;
      }
    return per;
  }
  // Free units in the cycle's snapshot (from its running totals: O(1) for GPU
  // ranks, 16 terms for XCD ranks).
  int64_t free_units(const GpuDemand& d) const {
    const Snapshot& s = *h_.snapshot;
    if (d.kind == GpuDemand::Gpu) return s.sum_free_whole / std::max<int64_t>(1, d.amount);
    int64_t members = 0;
    for (int m = 1; m < 16; ++m) {
      const int64_t per = footprint_for_mask(d.amount, m);
      if (per > 0) members += s.sum_free_xcd_by_mask[m] / per;
    }
    return members;
  }
  // Units the whole cluster could give this kind of rank if nothing ran.
  // Partition modes are Node state, so the count is memoized per node epoch.
  int64_t total_units(const GpuDemand& d) {
    const Snapshot& s = *h_.snapshot;
    const uint64_t tag = (static_cast<uint64_t>(d.kind) << 56) ^ static_cast<uint64_t>(d.amount);
    if (total_memo_epoch_ == s.node_epoch && total_memo_nodes_ == s.nodes.size())
      if (auto it = total_memo_.find(tag); it != total_memo_.end()) return it->second;
    if (total_memo_epoch_ != s.node_epoch || total_memo_nodes_ != s.nodes.size()) {
      total_memo_.clear();
      total_memo_epoch_ = s.node_epoch;
      total_memo_nodes_ = s.nodes.size();
    }
    return total_memo_[tag] = count_total_units(d);
  }
  int64_t count_total_units(const GpuDemand& d) const {
    int64_t t = 0;
    for (const auto& ni : h_.snapshot->nodes) {
      const GpuLedger& L = ni->gpu;
      for (int g = 0; g < L.gpu_count; ++g) {
        if (d.kind == GpuDemand::Gpu) {
          t += L.parts[g] == 1;
        } else if (L.xcds_per_part(g) > 0) {
          t += 8 / std::max<int64_t>(1, footprint(d.amount, L.xcds_per_part(g)));
        }
      }
    }
    return d.kind == GpuDemand::Gpu ? t / std::max<int64_t>(1, d.amount) : t;
  }
  struct Parked {
    std::string ns, group;
    GpuDemand::Kind kind = GpuDemand::None;
    int64_t need = 0;  // units for the group's remaining members
  };
  // (kind slot, PodGroup creation, pg_key): each kind's line is a contiguous
  // run of the map, oldest first, so its head is one lower_bound away even
  // with thousands of groups of the other kind parked ahead of it.
  struct ParkKey {
    int slot = 0;
    MicroTime creation = 0;
    uint64_t key = 0;
    bool operator<(const ParkKey& o) const {
      return slot != o.slot ? slot < o.slot : creation != o.creation ? creation < o.creation : key < o.key;
    }
  };
  // Gate verdict for p's group (scheduling thread, snapshot current): pass
  // when the free units, less those owed to other gangs at Permit and to an
  // older parked group of the same kind, cover the remaining members, and
  // (NRT gangColocation: Required) one node can take all of them. Parks the
  // group on failure.
  Status gang_gate(const Pod& p, const PodGroup& pg) {
    const GpuDemand& d = p.gpu_demand;
    if (!gated(d) || !h_.snapshot) return {};
    const int assigned = h_.cache->assigned_in_group(p.pg_key);
    const int64_t remaining = pg.min_member - assigned;
    if (remaining <= 0) return {};
    const int64_t need = units_for(d, remaining);
    const int64_t free = free_units(d);
    const int slot = kind_slot(d.kind);
    // Required co-location: a gang that one idle node could hold waits until
    // one node can take all of its ranks (counting ranks owed to gangs
    // anchored on a node). Only before its first rank is placed: a started
    // gang follows its hosts (NRT PreFilter).
    const bool coloc_ok = assigned > 0 || colocated_now(p, remaining);
    std::vector<PodPtr> probe;
    bool pass;
    bool probe_answer = false;  // p's cycle is the probe its group was sent
    uint64_t probe_seq = 0;     // releases seen when that probe went out
    {
      std::lock_guard<std::mutex> g(park_mu_);
      if (parked_.empty() && owed_[slot] == 0 && free >= need && coloc_ok) return {};  // common case
      int64_t reserved = owed_[slot];
      if (auto o = outstanding_.find(p.pg_key); o != outstanding_.end() && kind_slot(o->second.kind) == slot)
        reserved -= o->second.units;
      const ParkKey me{slot, pg.meta.creation, p.pg_key};
      auto pos = parked_pos_.find(p.pg_key);
      // The oldest parked group of this kind holds a reservation against
      // younger groups that have not started (so big gangs are not starved
      // by a stream of small ones).
      if (assigned == 0) {
        auto head = oldest_locked(slot);
        if (head != parked_.end() && head->first < me) reserved += head->second.need;
      }
      pass = free - reserved >= need && coloc_ok;
      if (p.pg_key == probe_key_[slot]) {  // the probe's answer is in
        probe_key_[slot] = 0;
        probe_answer = true;
        probe_seq = probe_seq_[slot];
      }
      if (pass && pos != parked_pos_.end()) {
        parked_.erase(pos->second);
        parked_pos_.erase(pos);
        parked_n_.store(parked_.size(), std::memory_order_release);
        // Chain: the next parked group of this kind may fit what is left
        // (one release can cover several gangs).
        if (!probe_key_[slot]) probe = next_probe_locked(slot);
      }
      take_wake_locked(probe);
    }
    if (!probe.empty()) h_.activate(probe);
    if (pass) return {};
    // The whole group can never fit: Filter fails and PostFilter denies (reference).
    if (units_for(d, pg.min_member) > total_units(d)) return {};
    if (h_.metrics) {  // which term of the gate held the group back
      int64_t owed_others = 0;
      {
        std::lock_guard<std::mutex> g(park_mu_);
        owed_others = owed_[slot];
        if (auto o = outstanding_.find(p.pg_key); o != outstanding_.end() && kind_slot(o->second.kind) == slot)
          owed_others -= o->second.units;
      }
      const char* cause = !coloc_ok                      ? "colocation"
                          : free < need                  ? "free"
                          : free - owed_others < need    ? "owed"
                                                         : "head";
      h_.metrics->inc("xsched_coscheduling_gate_waits_total",
                      std::string("cause=\"") + cause + (slot == 0 ? "\",kind=\"gpu\"" : "\",kind=\"xcd\""));
    }
    // A group already part-placed releases what its waiting members hold (no
    // hold-and-wait between gangs), as PostFilter's park does.
    if (assigned > 0) park_rejecting(p, pg);
    else if (park(p, pg, d.kind, need)) park_members(p);
    if (probe_answer) {
      // GPUs released after this probe went out skipped their own probe (one
      // was outstanding), yet this cycle may have read a snapshot from before
      // them: with no later release to come, the line would wait forever. So
      // a negative answer is probed again when a release happened meanwhile
      // (after park_members, so the activation wins over the park mark).
      std::vector<PodPtr> again;
      {
        std::lock_guard<std::mutex> g(park_mu_);
        if (release_seq_ != probe_seq && !probe_key_[slot]) again = next_probe_locked(slot);
        take_wake_locked(again);
      }
      if (!again.empty()) h_.activate(again);
    }
    if (!coloc_ok && free >= need)
      return XS_FIXED_STATUS(Code::Unschedulable,
                             "PodGroup parked: no node can host all of its remaining ranks on one xGMI mesh "
                             "(gangColocation: Required); it retries when GPUs are released");
    return XS_FIXED_STATUS(Code::Unschedulable,
                           "PodGroup parked: its remaining members need more GPUs than are free; it retries when "
                           "GPUs are released");
  }
  // NRT gangColocation Required: can one node take `remaining` ranks of p's
  // kind now? True when co-location is not required or the gang is larger
  // than any node (it has to span nodes).
  bool colocated_now(const Pod& p, int64_t remaining) {
    if (!h_.gangs || h_.gangs->mode() != GangPlacement::Mode::Required || !h_.snapshot) return true;
    if (remaining > h_.gangs->node_capacity(*h_.snapshot, p)) return true;
    return h_.gangs->hostable(*h_.snapshot, p, remaining);
  }
  // PostFilter: does the gate's arithmetic (counting this member's own
  // remaining group) explain the Filter failure?
  bool gpu_shortage_explains(const Pod& p, const PodGroup& pg) {
    const GpuDemand& d = p.gpu_demand;
    if (!gated(d) || !h_.snapshot) return false;
    const int assigned = h_.cache->assigned_in_group(p.pg_key);
    const int64_t need_all = units_for(d, pg.min_member);
    if (need_all > total_units(d)) return false;
    const int64_t remaining = std::max<int64_t>(1, pg.min_member - assigned);
    if (assigned == 0 && !colocated_now(p, remaining)) return true;
    int64_t owed_others;
    {
      std::lock_guard<std::mutex> g(park_mu_);
      owed_others = owed_[kind_slot(d.kind)];
      if (auto o = outstanding_.find(p.pg_key); o != outstanding_.end() && kind_slot(o->second.kind) == kind_slot(d.kind))
        owed_others -= o->second.units;
    }
    return free_units(d) - owed_others < units_for(d, remaining);
  }
  // False when the group was deleted meanwhile (forget_group): not parked.
  bool park(const Pod& p, const PodGroup& pg, GpuDemand::Kind kind, int64_t need) {
    std::lock_guard<std::mutex> g(park_mu_);
    if (!deleted_uids_.empty() && deleted_uids_.count(pg.meta.uid)) return false;
    auto pos = parked_pos_.find(p.pg_key);
    if (pos != parked_pos_.end()) {
      parked_[pos->second].need = need;
      return true;
    }
    const ParkKey k{kind_slot(kind), pg.meta.creation, p.pg_key};
    Parked& pk = parked_[k];
    pk.ns = p.ns();
    pk.group = p.pod_group;
    pk.kind = kind;
    pk.need = need;
    parked_pos_[p.pg_key] = k;
    parked_n_.store(parked_.size(), std::memory_order_release);
    ++parks_total_;
    if (h_.metrics) h_.metrics->inc("xsched_coscheduling_parked_total", "");
    if (h_.gang_parked) h_.gang_parked(p);
    return true;
  }
  // PostFilter's park: the waiting siblings are rejected (their Unreserve
  // must not deny the group: exactly those pods are remembered), nothing
  // stays owed, the group parks.
  void park_rejecting(const Pod& p, const PodGroup& pg) {
    std::vector<std::string> uids;
    h_.waiting_pods->iterate_group(p.pg_key, [&](const WaitingPodPtr& wp) {
      const Pod& wpod = *wp->pod();
      if (wpod.ns() == p.ns() && wpod.pod_group == p.pod_group) uids.push_back(wpod.uid());
    });
    {
      std::lock_guard<std::mutex> g(park_mu_);
      if (!uids.empty()) {
        auto& r = parked_rejects_[p.pg_key];
        r.first.insert(r.first.end(), uids.begin(), uids.end());
        r.second = h_.clock->now_us();
      }
      erase_outstanding_locked(p.pg_key);
    }
    if (park(p, pg, p.gpu_demand.kind, units_for(p.gpu_demand, pg.min_member)))
      park_members(p);  // before the rejections, so the rejected siblings park as their cycles fail
    reject_group(p, "PodGroup parked in PostFilter: GPUs are short for its remaining members");
  }
  // The group's unplaced members leave the scheduling queues until a probe
  // un-parks it: one failed cycle per parked gang, not one per member, and no
  // churn from the cluster events the members' plugin registered.
  void park_members(const Pod& p) {
    if (!h_.deactivate) return;
    std::vector<PodPtr> members;
    for (auto& q : h_.informers->pods_in_group_of(p))
      if (q->node_name.empty()) members.push_back(std::move(q));
    if (!members.empty()) h_.deactivate(members);
  }
  // Unreserve of a sibling that park_rejecting rejected: absorbed (no denial).
  // Any other Unreserve of the group (a Permit timeout, a bind failure) is not.
  bool consume_parked_reject(uint64_t key, const std::string& uid) {
    std::lock_guard<std::mutex> g(park_mu_);
    if (!rejects_pending_locked(key)) return false;
    auto it = parked_rejects_.find(key);
    auto& v = it->second.first;
    auto u = std::find(v.begin(), v.end(), uid);
    if (u == v.end()) return false;
    v.erase(u);
    if (v.empty()) parked_rejects_.erase(it);
    return true;
  }
  // Rejections of a just-parked group still to land (a stale list, e.g. a
  // sibling allowed or timed out between the listing and the reject, expires).
  bool rejects_pending_locked(uint64_t key) {
    auto it = parked_rejects_.find(key);
    if (it == parked_rejects_.end()) return false;
    if (h_.clock->now_us() - it->second.second > kRejectWindowUs) {
      parked_rejects_.erase(it);
      return false;
    }
    return true;
  }
  // The oldest parked group of a kind slot (parked_.end() when none).
  std::map<ParkKey, Parked>::iterator oldest_locked(int slot) {
    auto it = parked_.lower_bound(ParkKey{slot, INT64_MIN, 0});
    return it != parked_.end() && it->first.slot == slot ? it : parked_.end();
  }
  // One member of the oldest parked group of this kind whose rejections have
  // all landed (so its own GPUs are back), for the active queue. Groups that
  // can no longer pass the gate (denied, deleted, fewer pods than minMember,
  // nothing left to schedule) leave the line here, so none of them holds the
  // head. Caller holds park_mu_.
  std::vector<PodPtr> next_probe_locked(int slot) {
    std::vector<PodPtr> out;
    for (auto it = oldest_locked(slot); it != parked_.end(); it = oldest_locked(slot)) {
      const uint64_t key = it->first.key;
      if (rejects_pending_locked(key)) return out;  // the last Unreserve probes
      Pod member;
      member.meta.ns = it->second.ns;
      member.pod_group = it->second.group;
      member.pg_key = key;
      auto pg = h_.informers->pod_group_of(member);
      bool viable = pg && !denied_.has(key) &&
                    static_cast<int64_t>(h_.informers->count_pods_in_group_of(member)) >= pg->min_member;
      // A member the cache does not hold (an assumed pod may not show its
      // node in the lister yet): activating one that is binding would lose
      // the probe until kProbeStaleUs.
      if (viable)
        for (auto& q : h_.informers->pods_in_group_of(member))
          if (q->node_name.empty() && !q->terminating() && !h_.cache->get_pod(q->uid())) {
            out.push_back(std::move(q));
            break;
          }
      if (!out.empty()) {
        probe_key_[slot] = key;
        probe_sent_us_[slot] = h_.clock->now_us();
        probe_seq_[slot] = release_seq_;
        return out;
      }
      // Not viable: off the line; its unplaced members go back to the
      // queues (they meet the reason in PreFilter and wait for an event, as
      // upstream) instead of staying out of them.
      parked_pos_.erase(key);
      parked_.erase(it);
      parked_n_.store(parked_.size(), std::memory_order_release);
      if (!viable) {
        for (auto& q : h_.informers->pods_in_group_of(member))
          if (q->node_name.empty()) wake_.push_back(std::move(q));
      }
    }
    return out;
  }
  bool wants_capacity_events() const override { return park_; }
  void capacity_freed() override {
    if (parked_n_.load(std::memory_order_acquire) == 0) return;
    std::vector<PodPtr> probe;
    {
      std::lock_guard<std::mutex> g(park_mu_);
      ++release_seq_;
      // One probe per kind at a time: a probe still queued answers for this
      // release too (its gate reads the snapshot of its own cycle, which
      // includes it). XCD gangs are probed apart from whole-GPU gangs, so a
      // big whole-GPU gang at the head never holds back XCD ranks that fit.
      const int64_t now = h_.clock->now_us();
      for (int k = 0; k < 2; ++k) {
        if (probe_key_[k] && now - probe_sent_us_[k] < kProbeStaleUs) continue;
        if (probe_key_[k] && h_.metrics) h_.metrics->inc("xsched_coscheduling_probes_total", "result=\"stale\"");
        probe_key_[k] = 0;
        auto more = next_probe_locked(k);
        probe.insert(probe.end(), more.begin(), more.end());
      }
      take_wake_locked(probe);
    }
    if (!probe.empty()) h_.activate(probe);
  }
  void take_wake_locked(std::vector<PodPtr>& out) {
    if (wake_.empty()) return;
    out.insert(out.end(), std::make_move_iterator(wake_.begin()), std::make_move_iterator(wake_.end()));
    wake_.clear();
  }
  struct Owed {
    GpuDemand::Kind kind = GpuDemand::None;
    int64_t units = 0;
    int64_t at_us = 0;
  };
  void note_outstanding(const Pod& p, int64_t remaining) {
    if (!gated(p.gpu_demand)) return;
    std::lock_guard<std::mutex> g(park_mu_);
    erase_outstanding_locked(p.pg_key);
    Owed& o = outstanding_[p.pg_key];
    o.kind = p.gpu_demand.kind;
    o.units = units_for(p.gpu_demand, remaining);
    o.at_us = h_.clock->now_us();
    owed_[kind_slot(o.kind)] += o.units;
  }
  void drop_outstanding(uint64_t key) {
    std::lock_guard<std::mutex> g(park_mu_);
    erase_outstanding_locked(key);
  }
  void erase_outstanding_locked(uint64_t key) {
    auto it = outstanding_.find(key);
    if (it == outstanding_.end()) return;
    owed_[kind_slot(it->second.kind)] -= it->second.units;
    outstanding_.erase(it);
  }
  // Safety net: a gang whose Permit wait ended without reaching this plugin
  // (e.g. its PodGroup vanished) stops being owed after the longest wait.
  void sweep_outstanding() {
    std::lock_guard<std::mutex> g(park_mu_);
    const int64_t now = h_.clock->now_us();
    for (auto it = outstanding_.begin(); it != outstanding_.end();) {
      if (now - it->second.at_us > kMaxPermitUs) {
        owed_[kind_slot(it->second.kind)] -= it->second.units;
        it = outstanding_.erase(it);
      } else {
        ++it;
      }
    }
    for (auto it = parked_rejects_.begin(); it != parked_rejects_.end();)
      it = now - it->second.second > kRejectWindowUs ? parked_rejects_.erase(it) : std::next(it);
  }
  // A probe not answered within this long (its pod went elsewhere: bound,
  // deleted, failed before the gate) no longer holds back the next one.
  static constexpr int64_t kProbeStaleUs = 5'000;
  static constexpr int64_t kRejectWindowUs = 1'000'000;
  static constexpr int64_t kMaxPermitUs = 15LL * 60 * 1'000'000;  // framework cap
  bool park_ = true;
  // total_units memo (scheduling thread only).
  std::unordered_map<uint64_t, int64_t> total_memo_;
  uint64_t total_memo_epoch_ = 0;
  size_t total_memo_nodes_ = 0;
  std::mutex park_mu_;
  std::map<ParkKey, Parked> parked_;
  std::unordered_map<uint64_t, ParkKey> parked_pos_;
  std::atomic<size_t> parked_n_{0};
  // pg_key -> (uids of the siblings park_rejecting rejected, when)
  std::unordered_map<uint64_t, std::pair<std::vector<std::string>, int64_t>> parked_rejects_;
  // PodGroups deleted in the last second (forget_group), by uid, and in
  // deletion order for expiry.
  std::unordered_set<std::string> deleted_uids_;
  std::deque<std::pair<int64_t, std::string>> deleted_order_;
  std::vector<PodPtr> wake_;  // members of groups dropped from the line, for the active queue
  std::unordered_map<uint64_t, Owed> outstanding_;
  int64_t owed_[2] = {0, 0};
  uint64_t probe_key_[2] = {0, 0};  // per kind slot: the group whose probe is out
  int64_t probe_sent_us_[2] = {0, 0};
  uint64_t release_seq_ = 0;         // capacity_freed calls (guarded by park_mu_)
  uint64_t probe_seq_[2] = {0, 0};   // release_seq_ when each kind's probe went out
  uint64_t parks_total_ = 0;
  // Permit (scheduling thread only): the gang whose waiting member last
  // activated its siblings, and how many members it had assigned then.
  uint64_t act_key_ = 0;
  int act_assigned_ = 0;

  Handle& h_;
  TTLSet denied_, permitted_;
  std::mutex requeue_mu_;
  std::unordered_map<uint64_t, int64_t> requeue_due_;  // pg_key -> when its pending requeue timer fires
  int64_t permit_wait_us_ = 60'000'000;
  int64_t denied_ttl_us_ = 20'000'000;
  uint64_t sweep_id_ = 0;
};

PluginRegistrar reg("Coscheduling", [](const Json& a, Handle& h) { return std::make_shared<Coscheduling>(a, h); });

}  // namespace

void link_coscheduling_plugin() {}

}  // namespace xsched
