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
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include <atomic>

#include "framework/plugin.h"
#include "framework/waiting_pods.h"
#include "scheduler/cache.h"
#include "scheduler/informers.h"

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
  }

  void start() override {
    sweep_id_ = h_.timers->every(3'000'000, [this] {
      denied_.sweep();
      permitted_.sweep();
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
    if (denied_.has(p.pg_key))
      return Status::unresolvable("pod with pgName: " + p.pg_full_name() + " last failed in " +
                                  std::to_string(denied_ttl_us_ / 1000000) + "s, deny");
    size_t n = h_.informers->count_pods_in_group_of(p);
    if (static_cast<int64_t>(n) < pg->min_member)
      return Status::unresolvable("pre-filter pod " + p.name() + " cannot find enough sibling pods, current pods number: " +
                                  std::to_string(n) + ", minMember of group: " + std::to_string(pg->min_member));
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
    reject_group(p, "optimistic rejection in PostFilter");
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

  // ---- Permit (coscheduling.go:184-216, core.go:199-216) ----
  std::pair<Status, int64_t> permit(CycleState& s, const PodPtr& p, const std::string&) override {
    if (p->pod_group.empty()) return {Status(), 0};
    auto pg = h_.informers->pod_group_of(*p);
    if (!pg) return {Status::unschedulable("PodGroup not found"), 0};
    // The cache already holds this (assumed) pod, so `assigned` includes it:
    // equivalent to the reference's snapshot count + 1.
    int assigned = h_.cache->assigned_in_group(p->pg_key);
    if (assigned < pg->min_member) {
      activate_siblings(*p, s);
      return {Status(Code::Wait), wait_time(*pg)};
    }
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
    if (!pg) return;
    reject_group(*p, "rejection in Unreserve");
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
    return Plugin::debug_call(what, s, p, args);
  }

 private:
  // True the first time (group uid, phase) is seen within kPatchMemoUs.
  static constexpr int64_t kPatchMemoUs = 60'000'000;
  bool note_patched(uint64_t key, const std::string& uid, const std::string& phase) {
    const int64_t now = h_.clock->now_us();
    std::lock_guard<std::mutex> g(patched_mu_);
    auto& e = patched_[key];
    if (e.uid == uid && e.phase == phase && now - e.at_us < kPatchMemoUs) return false;
    e = {uid, phase, now};
    // Amortized expiry: sweep when the memo has doubled since the last sweep
    // (a sweep on every call past a fixed size made each PostBind O(groups)
    // once thousands of distinct groups had bound within the memo window).
    if (patched_.size() > patched_sweep_at_) {
      for (auto it = patched_.begin(); it != patched_.end();)
        it = now - it->second.at_us >= kPatchMemoUs ? patched_.erase(it) : std::next(it);
      patched_sweep_at_ = std::max<size_t>(8192, 2 * patched_.size());
    }
    return true;
  }
  struct Patched {
    std::string uid, phase;
    int64_t at_us = 0;
  };
  std::mutex patched_mu_;
  std::unordered_map<uint64_t, Patched> patched_;
  size_t patched_sweep_at_ = 8192;

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
