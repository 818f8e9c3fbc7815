// CrossNodePreemption: a PostFilter that may evict lower-priority pods on
// *other* nodes than the one the preemptor lands on.
//
// Reference: pkg/crossnodepreemption/cross_node_preemption.go:19-224 (the
// whole file is commented out upstream, as are its tests). What it sketches:
// collect every lower-priority pod on the nodes where preemption might help
// (:145-157, :211-223), try all 2^n victim subsets depth-first (:171-180),
// and for each subset remove the victims from cloned NodeInfos + a cloned
// CycleState through the PreFilter RemovePod extensions, then run the
// filters on the touched nodes (:184-207). This matters for constraints that
// span nodes — required anti-affinity and topology spread — where the pod
// that blocks node B lives on node A.
//
// The rebuild keeps those semantics but bounds the search so it can run in a
// production scheduling cycle:
//   * subsets are enumerated by increasing size and the search stops at the
//     first size that yields a candidate, so the result is a minimum-victim
//     eviction (the upstream DFS returns every feasible subset, including all
//     supersets of the minimal ones);
//   * the victim pool is the `maxPoolPods` least important lower-priority pods
//     (util.MoreImportantPod order), subsets are at most `maxVictims` pods and
//     at most `maxCombinations` subsets are tried per cycle;
//   * each subset is checked against every potential node, not just the nodes
//     the victims sit on (removing a pod on A can open B, which the upstream
//     sketch never looks at), and victims may sit on nodes the preemptor can
//     never use when they constrain it through anti-affinity / spread;
//   * combinations run on the scheduler's Parallelizer; candidates are ranked
//     with the shared Evaluator's pickOneNodeForPreemption order and prepared
//     (waiting victims rejected, others deleted, lower nominations cleared)
//     exactly as DefaultPreemption does.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>

#include "framework/framework.h"
#include "framework/plugin.h"
#include "scheduler/informers.h"
#include "scheduler/metrics.h"
#include "scheduler/preemption.h"

namespace xsched {
namespace {

class CrossNodePreemption : public Plugin, public PreemptionPolicy {
 public:
  CrossNodePreemption(const Json& args, Handle& h)
      : Plugin("CrossNodePreemption", kPostFilter), h_(h), ev_(name_, h, this) {
    max_victims_ = static_cast<int>(args["maxVictims"].as_int(3));
    max_pool_ = static_cast<int>(args["maxPoolPods"].as_int(32));
    max_combos_ = args["maxCombinations"].as_int(20000);
  }

  // PreemptionPolicy: only eligibility is used; candidate search is ours.
  std::pair<int, int> offset_and_num_candidates(int n) override { return {0, n}; }
  bool eligible(const Pod& pod, const Status* nom) override { return default_eligible(h_, pod, nom); }
  Status select_victims_on_node(CycleState&, const Pod&, NodeInfo&, const std::vector<PDBPtr>&, std::vector<PodPtr>&,
                                int&) override {
    return Status::unresolvable("CrossNodePreemption selects victims across nodes");
  }

  std::pair<PostFilterResult, Status> post_filter(CycleState& s, const Pod& pod_in, const NodeStatusMap& m) override {
    if (h_.metrics) h_.metrics->inc("scheduler_preemption_attempts_total", "");
    PodPtr latest = h_.informers ? h_.informers->pod(pod_in.ns(), pod_in.name()) : nullptr;
    const Pod& pod = latest ? *latest : pod_in;
    const Status* nom = nullptr;
    if (!pod.nominated_node_name.empty()) nom = m.status_of(pod.nominated_node_name);
    if (!eligible(pod, nom)) return {PostFilterResult{}, Status::unschedulable("Pod is not eligible for preemption")};
    if (!h_.snapshot || h_.snapshot->nodes.empty()) return {PostFilterResult{}, Status::error("no nodes available")};

    std::vector<PDBPtr> pdbs = h_.informers ? h_.informers->pdbs() : std::vector<PDBPtr>{};
    auto cands = find_candidates(s, pod, m, pdbs);
    if (cands.empty())
      return {PostFilterResult{}, Status::unschedulable("0/" + std::to_string(h_.snapshot->nodes.size()) +
                                                        " nodes are available: no cross-node preemption victims found.")};
    std::string node = Evaluator::pick_one_node(cands);
    for (const auto& c : cands) {
      if (c.node != node) continue;
      Status st = ev_.prepare_candidate(c, pod);
      if (!st.is_success()) return {PostFilterResult{}, st};
      break;
    }
    return {PostFilterResult{node}, Status()};
  }

  // Exposed through the plugin for tests (bindings call post_filter).
  std::vector<Candidate> find_candidates(CycleState& s, const Pod& pod, const NodeStatusMap& m,
                                         const std::vector<PDBPtr>& pdbs) {
    std::vector<NodeInfoPtr> filtered;
    const std::vector<NodeInfoPtr>& potential = nodes_where_preemption_might_help(*h_.snapshot, m, filtered);
    if (potential.empty()) return {};
    // Victim pool: lower-priority, not already terminating pods that sit on a
    // potential node or can constrain the preemptor from elsewhere (they
    // match one of its required anti-affinity / hard spread selectors, or
    // their own required anti-affinity matches it); least important first.
    std::unordered_map<std::string, bool> is_potential;
    for (const auto& ni : potential) is_potential[ni->name()] = true;
    auto constrains = [&](const Pod& q) {
      for (const auto& t : pod.pod_anti_affinity_required)
        if (t.selector.matches(q.meta.labels)) return true;
      for (const auto& c : pod.spread_constraints)
        if (c.hard && c.selector.matches(q.meta.labels)) return true;
      for (const auto& t : q.pod_anti_affinity_required)
        if (t.selector.matches(pod.meta.labels)) return true;
      return false;
    };
    std::vector<std::pair<PodPtr, NodeInfoPtr>> pool;
    for (const auto& ni : h_.snapshot->nodes) {
      bool on_potential = is_potential.count(ni->name()) > 0;
      for (const auto& p : ni->pods)
        if (p->priority < pod.priority && !p->terminating() && (on_potential || constrains(*p)))
          pool.emplace_back(p, ni);
    }
    std::stable_sort(pool.begin(), pool.end(),
                     [](const auto& a, const auto& b) { return more_important_pod(*b.first, *a.first); });
    if (static_cast<int>(pool.size()) > max_pool_) pool.resize(max_pool_);
    const int n = static_cast<int>(pool.size());
    int64_t budget = max_combos_;
    for (int k = 1; k <= std::min(max_victims_, n) && budget > 0; ++k) {
      std::vector<std::vector<int>> combos;
      std::vector<int> idx(k);
      for (int i = 0; i < k; ++i) idx[i] = i;
      while (budget > 0) {
        combos.push_back(idx);
        --budget;
        int i = k - 1;
        while (i >= 0 && idx[i] == n - k + i) --i;
        if (i < 0) break;
        ++idx[i];
        for (int j = i + 1; j < k; ++j) idx[j] = idx[j - 1] + 1;
      }
      auto found = try_combinations(s, pod, potential, pool, combos, pdbs);
      if (!found.empty()) return found;
    }
    return {};
  }

 private:
  std::vector<Candidate> try_combinations(CycleState& s, const Pod& pod, const std::vector<NodeInfoPtr>& potential,
                                          const std::vector<std::pair<PodPtr, NodeInfoPtr>>& pool,
                                          const std::vector<std::vector<int>>& combos,
                                          const std::vector<PDBPtr>& pdbs) {
    Framework& fw = *h_.framework;
    std::vector<Candidate> out;
    std::mutex mu;
    h_.parallelizer->until(static_cast<int>(combos.size()), [&](int ci) {
      const auto& combo = combos[ci];
      auto st = s.clone();
      std::unordered_map<std::string, NodeInfoPtr> touched;
      std::vector<PodPtr> victims;
      for (int vi : combo) {
        const auto& [victim, src] = pool[vi];
        auto& ni = touched[src->name()];
        if (!ni) ni = src->clone();
        ni->remove_pod(victim->uid());
        if (!fw.run_pre_filter_remove_pod(*st, pod, victim, *ni).is_success()) return;
        victims.push_back(victim);
      }
      std::stable_sort(victims.begin(), victims.end(),
                       [](const PodPtr& a, const PodPtr& b) { return more_important_pod(*a, *b); });
      std::vector<PodPtr> violating, non_violating;
      filter_pods_with_pdb_violation(victims, pdbs, violating, non_violating);
      std::vector<Candidate> local;
      for (const auto& base : potential) {
        auto it = touched.find(base->name());
        const NodeInfo& ni = it != touched.end() ? *it->second : *base;
        if (!fw.run_filter_with_nominated_pods(*st, pod, ni).is_success()) continue;
        Candidate c;
        c.node = ni.name();
        c.victims = victims;
        c.num_pdb_violations = static_cast<int>(violating.size());
        local.push_back(std::move(c));
      }
      if (local.empty()) return;
      std::lock_guard<std::mutex> g(mu);
      for (auto& c : local) out.push_back(std::move(c));
    });
    // Deterministic order (combination index is not preserved by the pool).
    std::stable_sort(out.begin(), out.end(), [](const Candidate& a, const Candidate& b) { return a.node < b.node; });
    return out;
  }

  Handle& h_;
  Evaluator ev_;
  int max_victims_ = 3, max_pool_ = 32;
  int64_t max_combos_ = 20000;
};

PluginRegistrar reg("CrossNodePreemption",
                    [](const Json& a, Handle& h) { return std::make_shared<CrossNodePreemption>(a, h); });

}  // namespace

void link_crossnode_plugin() {}

}  // namespace xsched
