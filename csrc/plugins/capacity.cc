// CapacityScheduling: ElasticQuota admission (min guaranteed, max cap) and
// quota-aware preemption.
//
// Reference: pkg/capacityscheduling/capacity_scheduling.go:54-907 and
// elasticquota.go:26-181. Kept semantics:
//  * one quota per namespace, the first one listed wins;
//  * PreFilter snapshots every quota into the CycleState, sums nominated pods
//    (same namespace with priority >= preemptor into both sums, other
//    namespaces whose quota is not over min into the global sum) and rejects
//    when used+inEQ > Max or Σused+global > ΣMin;
//  * cmp2 compares cpu, memory and only the scalar resources present in the
//    request (a scalar missing from the bound counts as 0);
//  * AddPod/RemovePod PreFilter extensions update the snapshot during
//    preemption dry runs; Reserve/Unreserve update the live quota;
//  * PostFilter preempts on every node (offset 0, all candidates) with the
//    quota-aware victim rules of SelectVictimsOnNode.
// Fixed (Appendix C5): the live quota map is only touched under the plugin
// lock (the reference reads it unlocked in PreFilter / addElasticQuota).
#include <algorithm>
#include <array>
#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>

#include "framework/framework.h"
#include "framework/plugin.h"
#include "scheduler/informers.h"
#include "scheduler/preemption.h"
#include "scheduler/queue.h"
#include "store/store.h"

namespace xsched {
namespace {

// cmp2(x1, x2, y): x1 + x2 > y on cpu, memory, or any scalar present in x1.
bool cmp2(const Res& x1, const Res& x2, const Res& y) {
  if (x1.get(kCPU) + x2.get(kCPU) > y.get(kCPU)) return true;
  if (x1.get(kMemory) + x2.get(kMemory) > y.get(kMemory)) return true;
  for (uint64_t m = x1.mask; m; m &= m - 1) {
    int id = __builtin_ctzll(m);
    if (id <= kPods) continue;  // ScalarResources only
    if (x1.v[id] + x2.get(id) > y.get(id)) return true;
  }
  return false;
}
bool cmp(const Res& x, const Res& y) { return cmp2(x, Res{}, y); }

// One namespace's quota as the scheduling cycle sees it.
struct Quota {
  Res min, max, used;
  bool used_over_min_with(const Res& req) const { return cmp2(req, used, min); }
  bool used_over_max_with(const Res& req) const { return cmp2(req, used, max); }
  bool used_over_min() const { return cmp(used, min); }
};

// Live quota of one namespace: the pods counted in `used` (a pod event can
// repeat, so add/delete are idempotent by key) and the immutable Quota last
// published for it (reset on change, rebuilt on the next publish).
struct EQInfo {
  std::string ns;
  std::set<std::string> pods;
  Res min, max, used;
  std::shared_ptr<const Quota> published;
  bool add_pod(const Pod& p) {
    if (!pods.insert(p.key()).second) return false;
    used += p.request();
    published.reset();
    return true;
  }
  bool delete_pod(const Pod& p) {
    if (!pods.erase(p.key())) return false;
    used -= p.request();
    published.reset();
    return true;
  }
};
using EQInfos = std::map<std::string, EQInfo>;

// Every quota at one version of the live state; shared by the cycles that
// run at that version (published when a PreFilter finds the live state
// changed, reusing the Quota of every namespace that did not).
struct QuotaView {
  std::unordered_map<std::string, std::shared_ptr<const Quota>> q;
  Res sum_used, sum_min;
};

// The CycleState's quota snapshot: the shared view plus this cycle's own
// changes (preemption dry runs add and remove pods through the PreFilter
// extensions). The reference deep-copies every ElasticQuotaInfo, including
// each namespace's set of pod keys, into every cycle
// (capacity_scheduling.go:201-211, elasticquota.go Clone).
struct EQSnapshot : StateData {
  std::shared_ptr<const QuotaView> base;
  std::unordered_map<std::string, Res> delta;  // namespace -> change of `used`
  Res delta_sum;
  std::shared_ptr<StateData> clone() const override { return std::make_shared<EQSnapshot>(*this); }

  const Quota* find(const std::string& ns) const {
    auto it = base->q.find(ns);
    return it == base->q.end() ? nullptr : it->second.get();
  }
  bool has(const std::string& ns) const { return find(ns) != nullptr; }
  // The namespace's quota with this cycle's changes applied (requires has(ns)).
  Quota quota(const std::string& ns) const {
    Quota out = *find(ns);
    auto d = delta.find(ns);
    if (d != delta.end()) out.used += d->second;
    return out;
  }
  bool aggregated_used_over_min_with(const Res& req) const {
    Res used = base->sum_used;
    used += delta_sum;
    used += req;
    return cmp(used, base->sum_min);
  }
  const Res* delta_of(const std::string& ns) const {
    auto d = delta.find(ns);
    return d == delta.end() ? nullptr : &d->second;
  }
  // PreFilterExtensions AddPod / RemovePod. The reference only moves pods
  // its quota counts (addPodIfNotPresent / deletePodIfPresent); the live
  // accounting counts assigned pods while they are Running or Pending (it
  // drops one on any other phase), so the same filter applies here: removing
  // an Unknown/Succeeded/Failed victim must not subtract its request again.
  void add(const Pod& p, int sign);
};
struct CSPreFilterState : StateData {
  Res pod_req, nominated_in_eq_with_req, nominated_with_req;
  std::shared_ptr<StateData> clone() const override { return std::make_shared<CSPreFilterState>(*this); }
};

// ---- Guards for the dry-run memo (PreemptionPolicy::guarded_victims) ----
// SelectVictimsOnNode reads cluster-wide state only through the predicates
// below, each on the cycle's quota snapshot plus the changes its own dry run
// made so far on this node (`delta`, a function of the node's pods). While a
// node is dry-run with recording on, every predicate evaluated is logged
// with its arguments and outcome; a remembered result is reused for a later
// preemptor only if each logged predicate, re-evaluated on that cycle's
// snapshot and PreFilter sums, comes out the same.
enum GuardKind : uint8_t { kGHas, kGOverMin, kGOverMinWith, kGOverMaxWith, kGAggOverMinWith };
enum GuardArg : uint8_t { kArgNone, kArgPodReq, kArgInEq, kArgGlobal };
struct EQGuard {
  GuardKind kind;
  GuardArg arg;
  bool out;
  std::string ns;
  Res delta;  // this dry run's change of `used` (per namespace, or summed) when evaluated
};
bool same_guard(const EQGuard& a, const EQGuard& b) {
  return a.kind == b.kind && a.arg == b.arg && a.out == b.out && a.ns == b.ns && a.delta.mask == b.delta.mask &&
         a.delta == b.delta;
}
struct EQGuards : VictimGuards {
  std::vector<EQGuard> v;
  uint64_t hash = 0;
  // Verdict of the last dry run that checked this set (interned sets are
  // shared by every node whose dry run read the same predicates, so a run
  // evaluates each distinct set once). Written only with the same value
  // within a run: the verdict is stored before the run number is published.
  mutable std::atomic<uint64_t> checked_run{0};
  mutable std::atomic<bool> verdict{false};
};

// Interned guard sets: identical nodes (same pods, same quotas) share one.
class GuardIntern {
 public:
  std::shared_ptr<EQGuards> intern(std::shared_ptr<EQGuards> g) {
    Shard& sh = shards_[g->hash % kShards];
    std::lock_guard<std::mutex> lk(sh.mu);
    auto& bucket = sh.m[g->hash];
    for (const auto& c : bucket)
      if (c->v.size() == g->v.size() &&
          std::equal(c->v.begin(), c->v.end(), g->v.begin(), same_guard))
        return c;
    if (sh.m.size() > 4096) {  // bounded: memo entries keep their own reference
      sh.m.clear();
      sh.m[g->hash].push_back(g);
      return g;
    }
    bucket.push_back(g);
    return g;
  }

 private:
  static constexpr size_t kShards = 64;
  struct Shard {
    std::mutex mu;
    std::unordered_map<uint64_t, std::vector<std::shared_ptr<EQGuards>>> m;
  };
  std::array<Shard, kShards> shards_;
};
thread_local std::shared_ptr<EQGuards> t_guards;  // recording on this worker (null: off)

const Res& guard_arg(const CSPreFilterState& pfs, GuardArg a) {
  static const Res kNone;
  switch (a) {
    case kArgPodReq: return pfs.pod_req;
    case kArgInEq: return pfs.nominated_in_eq_with_req;
    case kArgGlobal: return pfs.nominated_with_req;
    default: return kNone;
  }
}

// The predicate on the snapshot's base quotas with `delta` applied. A
// namespace without a quota makes every quota predicate false (callers only
// ask after has(), which is itself a guard).
bool guard_eval(const EQSnapshot& snap, const CSPreFilterState& pfs, GuardKind k, GuardArg a, const std::string& ns,
                const Res& delta) {
  if (k == kGHas) return snap.has(ns);
  if (k == kGAggOverMinWith) {
    Res used = snap.base->sum_used;
    used += delta;
    used += guard_arg(pfs, a);
    return cmp(used, snap.base->sum_min);
  }
  const Quota* q = snap.find(ns);
  if (!q) return false;
  Res used = q->used;
  used += delta;
  switch (k) {
    case kGOverMin: return cmp(used, q->min);
    case kGOverMinWith: return cmp2(guard_arg(pfs, a), used, q->min);
    default: return cmp2(guard_arg(pfs, a), used, q->max);
  }
}

// Evaluates a predicate on the live dry-run state and logs it when recording.
bool guarded(const EQSnapshot& snap, const CSPreFilterState* pfs, GuardKind k, GuardArg a, const std::string& ns) {
  static const CSPreFilterState kNoSums;
  Res delta;
  if (k == kGAggOverMinWith) delta = snap.delta_sum;
  else if (k != kGHas)
    if (const Res* d = snap.delta_of(ns)) delta = *d;
  const bool out = guard_eval(snap, pfs ? *pfs : kNoSums, k, a, ns, delta);
  if (t_guards) t_guards->v.push_back(EQGuard{k, a, out, k == kGAggOverMinWith ? std::string() : ns, std::move(delta)});
  return out;
}

void EQSnapshot::add(const Pod& p, int sign) {
  if (!guarded(*this, nullptr, kGHas, kArgNone, p.ns()) ||
      !(p.phase.empty() || p.phase == "Running" || p.phase == "Pending"))
    return;
  Res& d = delta[p.ns()];
  if (sign > 0) {
    d += p.request();
    delta_sum += p.request();
  } else {
    d -= p.request();
    delta_sum -= p.request();
  }
}

constexpr const char* kSnapKey = "CapacityScheduling/ElasticQuotaSnapshot";
constexpr const char* kStateKey = "PreFilterCapacityScheduling";

class CapacityScheduling : public Plugin, public PreemptionPolicy {
 public:
  explicit CapacityScheduling(Handle& h)
      : Plugin("CapacityScheduling", kPreFilter | kPostFilter | kReserve), h_(h), ev_("CapacityScheduling", h, this) {}

  // ---- informer handlers (capacity_scheduling.go:646-751) ----
  std::vector<std::string> watched_kinds() const override { return {"elasticquotas", "pods"}; }

  void on_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr& old) override {
    EventType t = static_cast<EventType>(type);
    if (kind == "elasticquotas") {
      auto eq = ElasticQuota::from_json(*obj);
      std::lock_guard<std::mutex> g(mu_);
      ++version_;
      if (t == EventType::Deleted) {
        infos_.erase(eq->meta.ns);
        return;
      }
      auto it = infos_.find(eq->meta.ns);
      if (t == EventType::Added && it != infos_.end()) return;  // first listed wins
      EQInfo info{eq->meta.ns, {}, eq->min, eq->max, {}, nullptr};
      if (it != infos_.end()) {
        info.pods = it->second.pods;
        info.used = it->second.used;
      } else {
        // Pods and quotas arrive on separate watches: assigned pods seen before
        // their namespace's quota were not counted then, so count them now
        // (add_pod dedupes by key, so a later pod event cannot double count).
        for (const auto& p : h_.informers->all_pods())
          if (p->ns() == eq->meta.ns && !p->node_name.empty() && p->phase != "Succeeded" && p->phase != "Failed")
            info.add_pod(*p);
      }
      infos_[eq->meta.ns] = std::move(info);
      return;
    }
    // pods: FilteringResourceEventHandler over assigned pods. Only pods of a
    // namespace with a quota matter: decided before the pod is parsed.
    {
      const std::string& ns = (*obj)["metadata"]["namespace"].as_string();
      bool known;
      {
        std::lock_guard<std::mutex> g(mu_);
        known = infos_.count(ns) > 0;
      }
      if (!known && !h_.informers->elastic_quota_for_namespace(ns)) return;
    }
    auto np = Pod::from_json(*obj, *h_.gpu_names);
    bool now_assigned = !np->node_name.empty();
    PodPtr op = old ? Pod::from_json(*old, *h_.gpu_names) : nullptr;
    bool was_assigned = op && !op->node_name.empty();
    std::lock_guard<std::mutex> g(mu_);
    if (t == EventType::Deleted) {
      if (now_assigned) delete_pod_locked(*np);
      return;
    }
    if (now_assigned && !was_assigned) {
      add_pod_locked(*np);
    } else if (now_assigned && was_assigned) {
      if (op->phase == "Succeeded" || op->phase == "Failed") return;
      if (np->phase != "Running" && np->phase != "Pending") {
        auto it = infos_.find(np->ns());
        if (it != infos_.end() && it->second.delete_pod(*np)) ++version_;
      }
    } else if (!now_assigned && was_assigned) {
      delete_pod_locked(*op);
    }
  }

  void add_pod_locked(const Pod& p) {
    auto it = infos_.find(p.ns());
    if (it == infos_.end()) {
      auto eq = h_.informers->elastic_quota_for_namespace(p.ns());
      if (!eq) return;
      it = infos_.emplace(p.ns(), EQInfo{p.ns(), {}, eq->min, eq->max, {}, nullptr}).first;
      ++version_;
    }
    if (it->second.add_pod(p)) ++version_;
  }
  void delete_pod_locked(const Pod& p) {
    auto it = infos_.find(p.ns());
    if (it != infos_.end() && it->second.delete_pod(p)) ++version_;
  }

  // The view of the current live state (under mu_): republished only when
  // the live state changed since the last one, and then only the changed
  // namespaces get a new Quota.
  std::shared_ptr<const QuotaView> view_locked() {
    if (view_ && view_version_ == version_) return view_;
    auto v = std::make_shared<QuotaView>();
    v->q.reserve(infos_.size());
    for (auto& [ns, e] : infos_) {
      if (!e.published) e.published = std::make_shared<const Quota>(Quota{e.min, e.max, e.used});
      v->q.emplace(ns, e.published);
      v->sum_used += e.used;
      v->sum_min += e.min;
    }
    view_ = std::move(v);
    view_version_ = version_;
    return view_;
  }

  // ---- PreFilter (capacity_scheduling.go:201-275) ----
  Status pre_filter(CycleState& s, const Pod& pod) override {
    auto snap = std::make_shared<EQSnapshot>();
    {
      std::lock_guard<std::mutex> g(mu_);
      snap->base = view_locked();
    }
    s.write(kSnapKey, snap);
    auto pfs = std::make_shared<CSPreFilterState>();
    pfs->pod_req = pod.request();
    const Quota* own = snap->find(pod.ns());
    if (!own) {
      s.write(kStateKey, pfs);
      return {};
    }
    Res in_eq, global;
    // Pods nominated onto nodes of the snapshot (the reference walks every
    // node and asks for its nominations): the cycle's nominated map when it
    // has one (one snapshot lookup per node, not per pod), else the Nominator.
    // Quotas are looked up once per run of pods of one namespace.
    const std::string* last_ns = nullptr;
    const Quota* last_q = nullptr;
    auto count = [&](const PodPtr& np) {
      if (np->uid() == pod.uid()) return;
      if (!last_ns || *last_ns != np->ns()) {
        last_ns = &np->ns();
        last_q = snap->find(np->ns());
      }
      const Quota* q = last_q;
      if (!q) return;
      if (np->ns() == pod.ns() && np->priority >= pod.priority) {
        in_eq += np->request();
        global += np->request();
      } else if (np->ns() != pod.ns() && !q->used_over_min()) {
        global += np->request();
      }
    };
    if (h_.snapshot && s.nominated) {
      for (const auto& [node, pods] : *s.nominated)
        if (!pods.empty() && h_.snapshot->has(node))
          for (const auto& np : pods) count(np);
    } else if (h_.snapshot && h_.nominator && !h_.nominator->empty()) {
      h_.nominator->for_each([&](const std::string& node, const PodPtr& np) {
        if (h_.snapshot->has(node)) count(np);
      });
    }
    in_eq += pod.request();
    global += pod.request();
    pfs->nominated_in_eq_with_req = in_eq;
    pfs->nominated_with_req = global;
    s.write(kStateKey, pfs);
    if (own->used_over_max_with(in_eq))
      return Status::unschedulable("Pod " + pod.key() + " is rejected in PreFilter because ElasticQuota " + pod.ns() +
                                   " is more than Max");
    if (snap->aggregated_used_over_min_with(global))
      return Status::unschedulable("Pod " + pod.key() +
                                   " is rejected in PreFilter because total ElasticQuota used is more than min");
    return {};
  }

  bool has_pre_filter_extensions() const override { return true; }
  // AddPod/RemovePod touch only the quota of the other pod's namespace.
  bool pre_filter_extension_affects(const CycleState& s, const Pod&, const Pod& other) const override {
    auto* snap = s.read_as<EQSnapshot>(kSnapKey);
    return snap && snap->has(other.ns());
  }
  Status add_pod(CycleState& s, const Pod&, const PodPtr& to_add, const NodeInfo&) override {
    if (auto* snap = s.read_as<EQSnapshot>(kSnapKey)) snap->add(*to_add, +1);
    return {};
  }
  Status remove_pod(CycleState& s, const Pod&, const PodPtr& to_remove, const NodeInfo&) override {
    if (auto* snap = s.read_as<EQSnapshot>(kSnapKey)) snap->add(*to_remove, -1);
    return {};
  }

  // ---- PostFilter: quota-aware preemption ----
  std::pair<PostFilterResult, Status> post_filter(CycleState& s, const Pod& p, const NodeStatusMap& m) override {
    cur_state_ = &s;
    auto r = ev_.preempt(s, p, m);
    cur_state_ = nullptr;
    return r;
  }
  std::pair<int, int> offset_and_num_candidates(int n) override { return {0, n}; }

  // Dry-run memo guards (EQGuard above). Recording starts only when the
  // cycle's own snapshot carries no changes yet (a PostFilter's does not):
  // the logged deltas are then this node's alone.
  bool guarded_victims() const override { return true; }
  const std::string* guarded_plugin() const override { return &name_; }
  void start_guards(const CycleState& s) override {
    auto* snap = s.read_as<EQSnapshot>(kSnapKey);
    t_guards = snap && snap->delta.empty() && snap->delta_sum.mask == 0 ? std::make_shared<EQGuards>() : nullptr;
  }
  std::shared_ptr<const VictimGuards> take_guards() override {
    std::shared_ptr<EQGuards> g = std::exchange(t_guards, nullptr);
    if (!g) return nullptr;
    // Duplicates (the same namespace asked again at the same delta) add
    // nothing to the check; then intern by content.
    std::vector<EQGuard> u;
    u.reserve(g->v.size());
    for (auto& x : g->v)
      if (std::none_of(u.begin(), u.end(), [&](const EQGuard& y) { return same_guard(x, y); })) u.push_back(std::move(x));
    g->v = std::move(u);
    uint64_t h = 1469598103934665603ULL;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ULL; };
    for (const auto& x : g->v) {
      mix(x.kind | (x.arg << 8) | (uint64_t{x.out} << 16));
      mix(std::hash<std::string>{}(x.ns));
      mix(x.delta.mask);
      for (uint64_t m = x.delta.mask; m; m &= m - 1) mix(static_cast<uint64_t>(x.delta.v[__builtin_ctzll(m)]));
    }
    g->hash = h;
    return intern_.intern(std::move(g));
  }
  bool guards_hold(const CycleState& s, const VictimGuards& vg, uint64_t run) const override {
    const auto& g = static_cast<const EQGuards&>(vg);
    if (g.checked_run.load(std::memory_order_acquire) == run) return g.verdict.load(std::memory_order_relaxed);
    auto* snap = s.read_as<EQSnapshot>(kSnapKey);
    auto* pfs = s.read_as<CSPreFilterState>(kStateKey);
    bool ok = snap && pfs && snap->delta.empty() && snap->delta_sum.mask == 0;
    for (size_t i = 0; ok && i < g.v.size(); ++i) {
      const EQGuard& x = g.v[i];
      ok = guard_eval(*snap, *pfs, x.kind, x.arg, x.ns, x.delta) == x.out;
    }
    g.verdict.store(ok, std::memory_order_relaxed);
    g.checked_run.store(run, std::memory_order_release);
    return ok;
  }

  bool eligible(const Pod& pod, const Status* nom) override {
    if (pod.preemption_policy == "Never") return false;
    CycleState* s = cur_state_;
    auto* pfs = s ? s->read_as<CSPreFilterState>(kStateKey) : nullptr;
    if (!pfs) return false;
    if (pod.nominated_node_name.empty()) return true;
    if (nom && nom->code() == Code::UnschedulableAndUnresolvable) return true;
    auto* snap = s->read_as<EQSnapshot>(kSnapKey);
    if (!snap) return true;
    auto ni = h_.snapshot ? h_.snapshot->get(pod.nominated_node_name) : nullptr;
    if (!ni) return true;
    if (snap->has(pod.ns())) {
      bool more_than_min = snap->quota(pod.ns()).used_over_min_with(pfs->nominated_in_eq_with_req);
      for (const auto& p : ni->pods) {
        if (!p->terminating()) continue;
        if (!snap->has(p->ns())) continue;
        if (p->ns() == pod.ns() && p->priority < pod.priority) return false;
        if (p->ns() != pod.ns() && !more_than_min && snap->quota(p->ns()).used_over_min()) return false;
      }
    } else {
      for (const auto& p : ni->pods) {
        if (snap->has(p->ns())) continue;
        if (p->terminating() && p->priority < pod.priority) return false;
      }
    }
    return true;
  }

  // SelectVictimsOnNode (capacity_scheduling.go:465-644).
  Status select_victims_on_node(CycleState& s, const Pod& pod, NodeInfo& ni, const std::vector<PDBPtr>& pdbs,
                                std::vector<PodPtr>& victims, int& num_violating) override {
    auto* snap = s.read_as<EQSnapshot>(kSnapKey);
    auto* pfs = s.read_as<CSPreFilterState>(kStateKey);
    if (!snap) return Status::unschedulable("Failed to read elasticQuotaSnapshot from cycleState");
    if (!pfs) return Status::unschedulable("Failed to read preFilterState from cycleState");
    Framework& fw = *h_.framework;
    const bool with_eq = guarded(*snap, pfs, kGHas, kArgNone, pod.ns());
    auto remove = [&](const PodPtr& p) {
      ni.remove_pod(p->uid());
      return fw.run_pre_filter_remove_pod(s, pod, p, ni);
    };
    auto add = [&](const PodPtr& p) {
      ni.add_pod(p);
      return fw.run_pre_filter_add_pod(s, pod, p, ni);
    };
    std::vector<PodPtr> pods = ni.pods;
    // Least important first (the reference sorts with !MoreImportantPod, which
    // is not a strict weak order; the reversed comparator is).
    std::stable_sort(pods.begin(), pods.end(),
                     [](const PodPtr& a, const PodPtr& b) { return more_important_pod(*b, *a); });
    std::vector<PodPtr> potential;
    if (with_eq) {
      bool more_than_min = guarded(*snap, pfs, kGOverMinWith, kArgInEq, pod.ns());
      for (const auto& p : pods) {
        if (!guarded(*snap, pfs, kGHas, kArgNone, p->ns())) continue;
        bool victim = more_than_min ? (p->ns() == pod.ns() && p->priority < pod.priority)
                                    : (p->ns() != pod.ns() && guarded(*snap, pfs, kGOverMin, kArgNone, p->ns()));
        if (victim) {
          potential.push_back(p);
          Status st = remove(p);
          if (!st.is_success()) return st;
        }
      }
    } else {
      for (const auto& p : pods) {
        if (guarded(*snap, pfs, kGHas, kArgNone, p->ns())) continue;
        if (p->priority < pod.priority) {
          potential.push_back(p);
          Status st = remove(p);
          if (!st.is_success()) return st;
        }
      }
    }
    if (potential.empty())
      return Status::unresolvable("No victims found on node " + ni.name() + " for preemptor pod " + pod.name());
    Status fst = fw.run_filter_with_nominated_pods(s, pod, ni);
    if (!fst.is_success()) return fst;
    if (with_eq && (guarded(*snap, pfs, kGOverMaxWith, kArgPodReq, pod.ns()) ||
                    guarded(*snap, pfs, kGAggOverMinWith, kArgPodReq, pod.ns())))
      return Status::unschedulable("global quota max exceeded");
    std::stable_sort(potential.begin(), potential.end(),
              [](const PodPtr& a, const PodPtr& b) { return more_important_pod(*a, *b); });
    std::vector<PodPtr> violating, non_violating;
    filter_pods_with_pdb_violation(potential, pdbs, violating, non_violating);
    auto reprieve = [&](const PodPtr& p) -> std::pair<bool, Status> {
      Status ast = add(p);
      if (!ast.is_success()) return {false, ast};
      bool fits = fw.run_filter_with_nominated_pods(s, pod, ni).is_success();
      if (!fits) {
        Status rst = remove(p);
        if (!rst.is_success()) return {false, rst};
        victims.push_back(p);
      }
      // The reference re-removes (and double-lists) a pod that already
      // failed the fit check; only a reprieved pod is re-checked here.
      if (fits && with_eq && (guarded(*snap, pfs, kGOverMaxWith, kArgInEq, pod.ns()) ||
                              guarded(*snap, pfs, kGAggOverMinWith, kArgGlobal, pod.ns()))) {
        Status rst = remove(p);
        if (!rst.is_success()) return {false, rst};
        victims.push_back(p);
      }
      return {fits, Status()};
    };
    for (const auto& p : violating) {
      auto [fits, err] = reprieve(p);
      if (!err.is_success()) return err;
      if (!fits) ++num_violating;
    }
    for (const auto& p : non_violating) {
      auto [fits, err] = reprieve(p);
      if (!err.is_success()) return err;
    }
    return {};
  }

  // ---- Reserve / Unreserve (capacity_scheduling.go:340-366) ----
  Status reserve(CycleState&, const PodPtr& p, const std::string&) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = infos_.find(p->ns());
    if (it != infos_.end() && it->second.add_pod(*p)) ++version_;
    return {};
  }
  void unreserve(CycleState&, const PodPtr& p, const std::string&) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = infos_.find(p->ns());
    if (it != infos_.end() && it->second.delete_pod(*p)) ++version_;
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"ElasticQuota", kAll, ""}};
  }

  // Unit-test hooks: capacity_scheduling_test.go:166 TestDryRunPreemption
  // (the evaluator's dry run over every snapshot node, after PreFilter) and
  // elasticquota_test.go:27/79 (reserveResource / unreserveResource: args.used
  // plus each of args.pods' effective request, computePodResourceRequest).
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    if (what == "reserveResource" || what == "unreserveResource") {
      Res used = Res::from_json(args["used"]);
      for (const auto& j : args["pods"].items()) {
        auto q = Pod::from_json(j, *h_.gpu_names);
        if (what == "reserveResource") used += q->request();
        else used -= q->request();
      }
      Json out = Json::object();
      out.set("used", used.to_json());
      return out;
    }
    if (what != "dryRunPreemption") return Plugin::debug_call(what, s, p, args);
    cur_state_ = &s;
    std::vector<NodeInfoPtr> nodes = h_.snapshot->nodes;
    auto cands = ev_.dry_run(s, *p, nodes, h_.informers->pdbs(), 0, static_cast<int>(nodes.size()));
    cur_state_ = nullptr;
    Json out = Json::object();
    Json arr = Json::array();
    for (const auto& c : cands) {
      Json e = Json::object();
      e.set("node", Json(c.node));
      Json v = Json::array();
      for (const auto& x : c.victims) v.push_back(Json(x->name()));
      e.set("victims", std::move(v));
      e.set("numPDBViolations", Json(static_cast<int64_t>(c.num_pdb_violations)));
      arr.push_back(std::move(e));
    }
    out.set("candidates", std::move(arr));
    return out;
  }

 private:
  Handle& h_;
  Evaluator ev_;
  std::mutex mu_;
  EQInfos infos_;
  uint64_t version_ = 0;  // bumped on every change of infos_ (under mu_)
  std::shared_ptr<const QuotaView> view_;
  uint64_t view_version_ = ~0ULL;
  CycleState* cur_state_ = nullptr;  // PostFilter runs on the scheduling thread only
  GuardIntern intern_;
};

PluginRegistrar reg("CapacityScheduling", [](const Json&, Handle& h) { return std::make_shared<CapacityScheduling>(h); });

}  // namespace

void link_capacity_plugin() {}

}  // namespace xsched
