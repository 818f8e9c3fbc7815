// Upstream default plugins that reason about where *other* pods are:
// PodTopologySpread, InterPodAffinity and ImageLocality.
//
// The reference runs them implicitly in every profile through the vendored
// kube-scheduler's default plugin set (vendor/k8s.io/kubernetes/pkg/scheduler/
// apis/config/v1beta2/default_plugins.go:34-106; implementations under
// vendor/k8s.io/kubernetes/pkg/scheduler/framework/plugins/{podtopologyspread,
// interpodaffinity,imagelocality}). Semantics follow k8s 1.23:
//  * PodTopologySpread: hard constraints filter on skew = matching pods in the
//    node's domain + self - the minimum over eligible domains (critical paths);
//    soft constraints score cnt*log(#domains+2) + maxSkew-1, normalised so
//    fewer matching pods is better; system default constraints need a
//    Service/ReplicaSet selector, which this API has none of, so they never
//    apply (as upstream for bare pods).
//  * InterPodAffinity: required (anti-)affinity of the incoming pod and the
//    required anti-affinity of existing pods, counted per topology pair in
//    PreFilter and kept current through AddPod/RemovePod for preemption
//    dry-runs; preferred terms (and existing pods' hard affinity with
//    hardPodAffinityWeight) score per topology value, min-max normalised.
//  * ImageLocality: Σ image size × spread over containers, clamped to
//    [23 MiB, 1000 MiB × containers] and scaled to 0..100.
// Fast paths: a profile whose pods use none of these features pays one
// emptiness check per cycle (no per-node work).
#include <algorithm>
#include <array>
#include <atomic>
#include <climits>
#include <cmath>
#include <shared_mutex>
#include <unordered_map>
#include <unordered_set>

#include "framework/plugin.h"
#include "store/store.h"

namespace xsched {
namespace {

int64_t count_matching(const std::vector<PodPtr>& pods, const LabelSelector& sel, const std::string& ns) {
  int64_t n = 0;
  for (const auto& q : pods)
    if (!q->terminating() && q->ns() == ns && sel.matches(q->meta.labels)) ++n;
  return n;
}

// Filter failures, built once: a failing node costs a Status copy (two
// refcount increments), not a string, vector and control block per node.
const Status& kSpreadMissingLabel() {
  static const Status st = Status::immortal(
      Code::UnschedulableAndUnresolvable,
      "node(s) didn't match pod topology spread constraints (missing required label)");
  return st;
}
const Status& kSpreadSkew() {
  static const Status st = Status::immortal(Code::Unschedulable, "node(s) didn't match pod topology spread constraints");
  return st;
}
const Status& kAffinityUnmet() {
  static const Status st = Status::immortal(Code::UnschedulableAndUnresolvable, "node(s) didn't match pod affinity rules");
  return st;
}
const Status& kAntiAffinityUnmet() {
  static const Status st = Status::immortal(Code::Unschedulable, "node(s) didn't match pod anti-affinity rules");
  return st;
}
const Status& kExistingAntiAffinityUnmet() {
  static const Status st = Status::immortal(Code::Unschedulable, "node(s) didn't satisfy existing pods anti-affinity rules");
  return st;
}

// ===================================================== PodTopologySpread ====
struct CriticalPath {
  std::string value;
  int64_t num = INT32_MAX;
};

// The pre-filter/pre-score state of a pod that has nothing to track (no
// constraints, no affinity terms in play) is one shared empty object handed
// out as a non-owning shared_ptr (aliasing an empty owner): no allocation and
// no refcount traffic per cycle. Filter/Score only read it; preemption dry
// runs mutate clones (CycleState::clone), never the original.
template <typename T>
std::shared_ptr<StateData> empty_state() {
  static T obj;
  return std::shared_ptr<StateData>(std::shared_ptr<StateData>(), &obj);
}

// PreFilter states kept across cycles (PodTopologySpread, InterPodAffinity).
// Counting the pods that match a pod's terms walks every pod of the cluster;
// a later pod with the same spec (and, where it matters, labels) in the same
// namespace gets the earlier state brought up to date by replaying the pod
// events since (Snapshot::replay_since), while the topology epoch (node set,
// node labels) and `aux` (InterPodAffinity: namespace labels) are unchanged.
//
// Used only by PreFilter, which runs on the scheduling thread (cycle or
// explain(), both under the scheduler's cycle lock). The reused object is the
// one the previous cycle's CycleState points at: that cycle's Filter/Score
// are over, binding cycles hold its CycleState but none of their plugins read
// these states, and preemption / nominated-pod checks mutate clones.
template <typename State>
class StateMemo {
 public:
  struct Entry {
    uint64_t key = 0, aux = 0, epoch = 0, seq = 0;
    std::string ns;
    std::shared_ptr<State> st;
  };
  Entry* find(uint64_t key, const std::string& ns, uint64_t aux, uint64_t epoch) {
    for (auto& x : e_)
      if (x.st && x.key == key && x.aux == aux && x.epoch == epoch && x.ns == ns) return &x;
    return nullptr;
  }
  // Records `st` as computed from `snap` and asks the cache to log pod
  // events from now on (Snapshot::deltas_wanted).
  void put(uint64_t key, const std::string& ns, uint64_t aux, const Snapshot& snap, std::shared_ptr<State> st) {
    snap.deltas_wanted = true;
    Entry* slot = nullptr;
    for (auto& x : e_)
      if (x.st && x.key == key && x.ns == ns) slot = &x;
    if (!slot) slot = &e_[next_++ % e_.size()];
    *slot = Entry{key, aux, snap.topology_epoch, snap.delta_end, ns, std::move(st)};
  }

 private:
  std::array<Entry, 8> e_;
  size_t next_ = 0;
};

uint64_t labels_hash(const StrMap& m) {
  uint64_t h = 1469598103934665603ULL;
  std::hash<std::string> hs;
  for (const auto& [k, v] : m) h = (h ^ hs(k)) * 1099511628211ULL ^ (hs(v) * 0x9E3779B97F4A7C15ULL);
  return h;
}

// Topology key -> value -> count. Lookups take the node's own label strings,
// so Filter and Score build no key per node.
using TopoCounts = std::unordered_map<std::string, std::unordered_map<std::string, int64_t>>;

// Adds d to (key, value), dropping entries that reach 0 (an empty map means
// "no pair counted", which InterPodAffinity's Filter relies on).
void topo_add(TopoCounts& m, const std::string& key, const std::string& value, int64_t d) {
  auto& vals = m[key];
  int64_t& c = vals[value];
  c += d;
  if (c == 0) {
    vals.erase(value);
    if (vals.empty()) m.erase(key);
  }
}
int64_t topo_get(const TopoCounts& m, const std::string& key, const std::string& value) {
  auto kit = m.find(key);
  if (kit == m.end()) return 0;
  auto it = kit->second.find(value);
  return it == kit->second.end() ? 0 : it->second;
}

// Matching pods per (node, constraint) counted node-parallel on the
// framework's Parallelizer (upstream's PreFilter/PreScore also fan out over
// nodes): out[i * C + c] = count, or -1 where `eligible(node)` is false.
// Counting walks every pod of every node (O(pods in the cluster)), the part
// that dominates at thousands of nodes; the per-value sums stay serial.
template <typename Eligible>
void count_per_node(Parallelizer* par, const std::vector<NodeInfoPtr>& nodes,
                    const std::vector<TopologySpreadConstraint>& cs, const std::string& ns, Eligible eligible,
                    std::vector<int64_t>& out) {
  const size_t C = cs.size();
  out.assign(nodes.size() * C, -1);
  auto one = [&](int i) {
    const NodeInfo& ni = *nodes[i];
    if (!eligible(ni)) return;
    for (size_t c = 0; c < C; ++c) out[i * C + c] = count_matching(ni.pods, cs[c].selector, ns);
  };
  if (par && nodes.size() >= 256)
    par->until(static_cast<int>(nodes.size()), one);
  else
    for (size_t i = 0; i < nodes.size(); ++i) one(static_cast<int>(i));
}

struct SpreadFilterState : StateData {
  std::vector<TopologySpreadConstraint> constraints;
  TopoCounts pair_num;                                                    // key -> value -> matching pods
  std::unordered_map<std::string, std::array<CriticalPath, 2>> critical;  // topology key -> two smallest
  // Per constraint (index()): its value counts, the current minimum
  // (INT64_MIN: no critical paths) and whether the incoming pod matches its
  // own selector, so Filter does one hash lookup per constraint and node.
  std::vector<const std::unordered_map<std::string, int64_t>*> counts_c;
  std::vector<int64_t> min_c;
  std::vector<int64_t> self_c;
  std::shared_ptr<StateData> clone() const override {
    auto c = std::make_shared<SpreadFilterState>(*this);
    c->index();  // the copied pointers still point into this state's maps
    return c;
  }
  void index() {
    counts_c.clear();
    min_c.clear();
    for (const auto& c : constraints) {
      auto kit = pair_num.find(c.topology_key);
      counts_c.push_back(kit == pair_num.end() ? nullptr : &kit->second);
      auto cit = critical.find(c.topology_key);
      min_c.push_back(cit == critical.end() ? INT64_MIN : cit->second[0].num);
    }
  }
  void set_pod(const Pod& p) {
    self_c.clear();
    for (const auto& c : constraints) self_c.push_back(c.selector.matches(p.meta.labels) ? 1 : 0);
  }

  void recompute_critical() {
    for (auto& [key, p] : critical) p = {CriticalPath{}, CriticalPath{}};
    for (const auto& [key, values] : pair_num)
      for (const auto& [value, num] : values) update_critical(key, value, num);
  }
  void update_critical(const std::string& key, const std::string& value, int64_t num) {
    auto& p = critical[key];
    int i = value == p[0].value ? 0 : value == p[1].value ? 1 : -1;
    if (i >= 0) {
      p[i].num = num;
      if (p[0].num > p[1].num) std::swap(p[0], p[1]);
    } else if (num < p[0].num) {
      p[1] = p[0];
      p[0] = CriticalPath{value, num};
    } else if (num < p[1].num) {
      p[1] = CriticalPath{value, num};
    }
  }
};

struct SpreadScoreState : StateData {
  std::vector<TopologySpreadConstraint> constraints;
  std::unordered_set<std::string> ignored;
  TopoCounts pair_count;
  std::vector<double> weight;
  std::shared_ptr<StateData> clone() const override { return std::make_shared<SpreadScoreState>(*this); }
};

bool has_all_keys(const Node& n, const std::vector<TopologySpreadConstraint>& cs) {
  for (const auto& c : cs)
    if (!n.meta.label(c.topology_key)) return false;
  return true;
}

class PodTopologySpread : public Plugin {
 public:
  // Without constraints the pod's Filter/Score ignore other pods entirely.
  bool filter_node_local(const Pod& p, const Snapshot&) const override { return p.spread_constraints.empty(); }
  bool score_node_local(const Pod& p, const Snapshot&) const override { return p.spread_constraints.empty(); }
  bool score_all_zero(const Pod& p, const Snapshot&) const override {
    for (const auto& c : p.spread_constraints)
      if (!c.hard) return false;
    return true;
  }
  // NormalizeScore with no soft constraints: no ignored nodes and max 0, so
  // every node gets kMaxNodeScore.
  int64_t score_skip_value() const override { return kMaxNodeScore; }
  explicit PodTopologySpread(Handle& h)
      : Plugin("PodTopologySpread", kPreFilter | kFilter | kPreScore | kScore), h_(h) {}

  static constexpr const char* kFilterKey = "PreFilterPodTopologySpread";
  static constexpr const char* kScoreKey = "PreScorePodTopologySpread";

  Status pre_filter(CycleState& s, const Pod& p) override {
    bool any_hard = false;
    for (const auto& c : p.spread_constraints) any_hard = any_hard || c.hard;
    if (!any_hard) {
      s.write(kFilterKey, empty_state<SpreadFilterState>());
      return {};
    }
    if (h_.snapshot) {
      const Snapshot& snap = *h_.snapshot;
      if (auto* m = memo_.find(p.spec_hash, p.ns(), 0, snap.topology_epoch)) {
        SpreadFilterState& ms = *m->st;
        if (snap.replay_since(m->seq, [&](const PodDelta& d) { count_delta(ms, p, *d.pod, *d.node, d.d); })) {
          m->seq = snap.delta_end;
          ms.recompute_critical();
          ms.index();
          ms.set_pod(p);
          s.write(kFilterKey, m->st);
          return {};
        }
      }
    }
    auto st = std::make_shared<SpreadFilterState>();
    for (const auto& c : p.spread_constraints)
      if (c.hard) st->constraints.push_back(c);
    if (!st->constraints.empty() && h_.snapshot) {
      const auto& nodes = h_.snapshot->nodes;
      const size_t C = st->constraints.size();
      thread_local std::vector<int64_t> counts;
      count_per_node(h_.parallelizer, nodes, st->constraints, p.ns(), [&](const NodeInfo& ni) {
        return pod_matches_node_selector_and_affinity(p, *ni.node) && has_all_keys(*ni.node, st->constraints);
      }, counts);
      for (size_t c = 0; c < C; ++c) {
        auto& values = st->pair_num[st->constraints[c].topology_key];
        for (size_t i = 0; i < nodes.size(); ++i)
          if (counts[i * C + c] >= 0) values[*nodes[i]->node->meta.label(st->constraints[c].topology_key)] += counts[i * C + c];
      }
      for (const auto& c : st->constraints) st->critical[c.topology_key];
      for (const auto& [key, values] : st->pair_num)
        for (const auto& [value, num] : values) st->update_critical(key, value, num);
      memo_.put(p.spec_hash, p.ns(), 0, *h_.snapshot, st);
    }
    st->index();
    st->set_pod(p);
    s.write(kFilterKey, st);
    return {};
  }
  bool has_pre_filter_extensions() const override { return true; }

  // One pod event replayed into a memoized state: exactly what PreFilter's
  // count would have added for it (count_matching on eligible nodes).
  static void count_delta(SpreadFilterState& st, const Pod& p, const Pod& q, const Node& n, int d) {
    if (q.terminating() || q.ns() != p.ns()) return;
    if (!pod_matches_node_selector_and_affinity(p, n) || !has_all_keys(n, st.constraints)) return;
    for (const auto& c : st.constraints)
      if (c.selector.matches(q.meta.labels)) st.pair_num[c.topology_key][*n.meta.label(c.topology_key)] += d;
  }

  void update_with_pod(CycleState& s, const Pod& preemptor, const Pod& q, const NodeInfo& ni, int64_t delta) {
    auto* st = s.read_as<SpreadFilterState>(kFilterKey);
    if (!st || st->constraints.empty() || !ni.node) return;
    const Node& n = *ni.node;
    if (!pod_matches_node_selector_and_affinity(preemptor, n) || !has_all_keys(n, st->constraints)) return;
    if (q.ns() != preemptor.ns()) return;
    for (const auto& c : st->constraints) {
      if (!c.selector.matches(q.meta.labels)) continue;
      const std::string& v = *n.meta.label(c.topology_key);
      int64_t& num = st->pair_num[c.topology_key][v];
      num += delta;
      st->update_critical(c.topology_key, v, num);
    }
    st->index();
  }
  // update_with_pod changes nothing without hard constraints or across namespaces.
  bool pre_filter_extension_affects(const CycleState& s, const Pod& p, const Pod& q) const override {
    auto* st = s.read_as<SpreadFilterState>(kFilterKey);
    return st && !st->constraints.empty() && q.ns() == p.ns();
  }
  Status add_pod(CycleState& s, const Pod& p, const PodPtr& q, const NodeInfo& ni) override {
    update_with_pod(s, p, *q, ni, 1);
    return {};
  }
  Status remove_pod(CycleState& s, const Pod& p, const PodPtr& q, const NodeInfo& ni) override {
    update_with_pod(s, p, *q, ni, -1);
    return {};
  }

  Status filter(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    auto* st = s.read_as<SpreadFilterState>(kFilterKey);
    if (!st) return Status::error("PodTopologySpread: no PreFilter state");
    if (st->constraints.empty()) return {};
    const Node& n = *ni.node;
    for (size_t i = 0; i < st->constraints.size(); ++i) {
      const auto& c = st->constraints[i];
      const std::string* v = n.meta.label(c.topology_key);
      if (!v) return kSpreadMissingLabel();
      if (st->min_c[i] == INT64_MIN) return Status::error("PodTopologySpread: internal error: no critical paths");
      int64_t num = 0;
      if (const auto* counts = st->counts_c[i]) {
        auto it = counts->find(*v);
        if (it != counts->end()) num = it->second;
      }
      if (num + st->self_c[i] - st->min_c[i] > c.max_skew) return kSpreadSkew();
    }
    return {};
  }

  Status pre_score(CycleState& s, const Pod& p, const NodeList& nodes) override {
    bool any_soft = false;
    for (const auto& c : p.spread_constraints) any_soft = any_soft || !c.hard;
    if (!any_soft || nodes.empty()) {
      s.write(kScoreKey, empty_state<SpreadScoreState>());
      return {};
    }
    auto st = std::make_shared<SpreadScoreState>();
    for (const auto& c : p.spread_constraints)
      if (!c.hard) st->constraints.push_back(c);
    if (st->constraints.empty() || nodes.empty()) {
      s.write(kScoreKey, st);
      return {};
    }
    const size_t C = st->constraints.size();
    std::vector<int64_t> size(C, 0);
    for (const auto& ni : nodes) {
      const Node& n = *ni->node;
      if (!has_all_keys(n, st->constraints)) {
        st->ignored.insert(n.name());
        continue;
      }
      for (size_t i = 0; i < C; ++i) {
        const auto& c = st->constraints[i];
        if (c.topology_key == kHostnameLabel) {
          ++size[i];
          continue;
        }
        auto [it, fresh] = st->pair_count[c.topology_key].emplace(*n.meta.label(c.topology_key), 0);
        if (fresh) ++size[i];
      }
    }
    for (int64_t sz : size) st->weight.push_back(std::log(static_cast<double>(sz + 2)));
    // Hostname domains are counted per node in Score; the other domains take
    // their cluster-wide counts from the memoized per-value totals.
    if (h_.snapshot && !st->pair_count.empty()) {
      const TopoCounts& totals = soft_totals(p, st->constraints);
      for (auto& [key, values] : st->pair_count)
        for (auto& [value, cnt] : values) cnt = topo_get(totals, key, value);
    }
    s.write(kScoreKey, st);
    return {};
  }

  // Matching pods per (non-hostname topology key, value) over every node
  // eligible for p (node selector / affinity, all soft keys present): the
  // O(pods) part of PreScore, kept across cycles like the Filter state.
  struct SoftTotals {
    TopoCounts counts;  // zero entries dropped
  };
  static void count_soft(SoftTotals& t, const std::vector<TopologySpreadConstraint>& cs, const Pod& p, const Pod& q,
                         const Node& n, int64_t d) {
    if (q.terminating() || q.ns() != p.ns()) return;
    if (!pod_matches_node_selector_and_affinity(p, n) || !has_all_keys(n, cs)) return;
    for (const auto& c : cs)
      if (c.topology_key != kHostnameLabel && c.selector.matches(q.meta.labels))
        topo_add(t.counts, c.topology_key, *n.meta.label(c.topology_key), d);
  }
  const TopoCounts& soft_totals(const Pod& p, const std::vector<TopologySpreadConstraint>& cs) {
    const Snapshot& snap = *h_.snapshot;
    if (auto* m = soft_memo_.find(p.spec_hash, p.ns(), 0, snap.topology_epoch)) {
      SoftTotals& ms = *m->st;
      if (snap.replay_since(m->seq, [&](const PodDelta& d) { count_soft(ms, cs, p, *d.pod, *d.node, d.d); })) {
        m->seq = snap.delta_end;
        return ms.counts;
      }
    }
    auto t = std::make_shared<SoftTotals>();
    const auto& all = snap.nodes;
    const size_t C = cs.size();
    thread_local std::vector<int64_t> counts;
    count_per_node(h_.parallelizer, all, cs, p.ns(), [&](const NodeInfo& ni) {
      return pod_matches_node_selector_and_affinity(p, *ni.node) && has_all_keys(*ni.node, cs);
    }, counts);
    for (size_t c = 0; c < C; ++c) {
      const auto& key = cs[c].topology_key;
      if (key == kHostnameLabel) continue;
      for (size_t i = 0; i < all.size(); ++i)
        if (counts[i * C + c] > 0) topo_add(t->counts, key, *all[i]->node->meta.label(key), counts[i * C + c]);
    }
    soft_memo_.put(p.spec_hash, p.ns(), 0, snap, t);
    return t->counts;
  }

  std::pair<int64_t, Status> score(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    auto* st = s.read_as<SpreadScoreState>(kScoreKey);
    if (!st) return {0, Status::error("PodTopologySpread: no PreScore state")};
    if (st->constraints.empty() || st->ignored.count(ni.name())) return {0, {}};
    double score = 0;
    for (size_t i = 0; i < st->constraints.size(); ++i) {
      const auto& c = st->constraints[i];
      const std::string* v = ni.node->meta.label(c.topology_key);
      if (!v) continue;
      int64_t cnt;
      if (c.topology_key == kHostnameLabel) {
        cnt = count_matching(ni.pods, c.selector, p.ns());
      } else {
        cnt = 0;
        auto kit = st->pair_count.find(c.topology_key);
        if (kit != st->pair_count.end()) {
          auto it = kit->second.find(*v);
          if (it != kit->second.end()) cnt = it->second;
        }
      }
      score += static_cast<double>(cnt) * st->weight[i] + static_cast<double>(c.max_skew - 1);
    }
    return {static_cast<int64_t>(score), {}};
  }
  bool has_normalize_score() const override { return true; }
  bool normalize_uses_names() const override { return true; }  // ignored nodes are keyed by name
  Status normalize_score(CycleState& s, const Pod&, std::vector<NodeScore>& scores) override {
    auto* st = s.read_as<SpreadScoreState>(kScoreKey);
    if (!st) return Status::error("PodTopologySpread: no PreScore state");
    int64_t lo = INT64_MAX, hi = 0;
    std::vector<char> invalid(scores.size(), 0);
    for (size_t i = 0; i < scores.size(); ++i) {
      if (scores[i].name && st->ignored.count(*scores[i].name)) {
        invalid[i] = 1;
        continue;
      }
      lo = std::min(lo, scores[i].score);
      hi = std::max(hi, scores[i].score);
    }
    for (size_t i = 0; i < scores.size(); ++i) {
      if (invalid[i]) {
        scores[i].score = 0;
      } else if (hi == 0) {
        scores[i].score = kMaxNodeScore;
      } else {
        scores[i].score = kMaxNodeScore * (hi + lo - scores[i].score) / hi;
      }
    }
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kAll, ""}, {"Node", kAdd | kDelete | kUpdateNodeLabel, ""}};
  }

 private:
  Handle& h_;
  StateMemo<SpreadFilterState> memo_;
  StateMemo<SoftTotals> soft_memo_;
};

// ====================================================== InterPodAffinity ====
struct AffinityFilterState : StateData {
  TopoCounts existing_anti, affinity, anti;
  // The incoming pod's required (anti-)affinity term keys and, per term,
  // its value counts (nullptr: none), resolved once per cycle (index()) so
  // Filter does one hash lookup per term and node.
  std::vector<std::string> aff_keys, anti_keys;
  std::vector<const std::unordered_map<std::string, int64_t>*> aff_c, anti_c;
  std::shared_ptr<StateData> clone() const override {
    auto c = std::make_shared<AffinityFilterState>(*this);
    c->index();  // the copied pointers still point into this state's maps
    return c;
  }
  void set_pod(const Pod& p) {
    aff_keys.clear();
    anti_keys.clear();
    for (const auto& t : p.pod_affinity_required) aff_keys.push_back(t.topology_key);
    for (const auto& t : p.pod_anti_affinity_required) anti_keys.push_back(t.topology_key);
    index();
  }
  void index() {
    auto resolve = [](const TopoCounts& m, const std::vector<std::string>& keys,
                      std::vector<const std::unordered_map<std::string, int64_t>*>& out) {
      out.clear();
      for (const auto& k : keys) {
        auto it = m.find(k);
        out.push_back(it == m.end() ? nullptr : &it->second);
      }
    };
    resolve(affinity, aff_keys, aff_c);
    resolve(anti, anti_keys, anti_c);
  }
  void merge(const AffinityFilterState& o) {
    merge_into(existing_anti, o.existing_anti);
    merge_into(affinity, o.affinity);
    merge_into(anti, o.anti);
  }
  static void merge_into(TopoCounts& dst, const TopoCounts& src) {
    for (const auto& [k, vals] : src)
      for (const auto& [v, c] : vals) topo_add(dst, k, v, c);
  }
};
struct AffinityScoreState : StateData {
  TopoCounts topo_score;  // key -> value -> score (zero entries dropped)
  std::shared_ptr<StateData> clone() const override { return std::make_shared<AffinityScoreState>(*this); }
};

void bump(TopoCounts& m, const Node& n, const std::string& key, int64_t v) {
  if (const std::string* tv = n.meta.label(key)) topo_add(m, key, *tv, v);
}

class InterPodAffinity : public Plugin {
 public:
  // Node-local only when neither the pod nor any existing pod carries affinity terms.
  static bool no_terms(const Pod& p, const Snapshot& s) {
    return p.pod_affinity_required.empty() && p.pod_anti_affinity_required.empty() &&
           p.pod_affinity_preferred.empty() && p.pod_anti_affinity_preferred.empty() &&
           s.have_pods_with_affinity.empty() && s.have_pods_with_required_anti_affinity.empty();
  }
  bool filter_node_local(const Pod& p, const Snapshot& s) const override { return no_terms(p, s); }
  bool score_node_local(const Pod& p, const Snapshot& s) const override { return no_terms(p, s); }
  bool score_all_zero(const Pod& p, const Snapshot& s) const override { return no_terms(p, s); }
  InterPodAffinity(const Json& args, Handle& h)
      : Plugin("InterPodAffinity", kPreFilter | kFilter | kPreScore | kScore), h_(h) {
    hard_weight_ = static_cast<int32_t>(args["hardPodAffinityWeight"].as_int(1));
  }
  static constexpr const char* kFilterKey = "PreFilterInterPodAffinity";
  static constexpr const char* kScoreKey = "PreScoreInterPodAffinity";

  std::vector<std::string> watched_kinds() const override { return {"namespaces"}; }
  void on_object_event(const std::string&, int type, const JsonPtr& obj, const JsonPtr&) override {
    auto md = ObjectMeta::from_json(*obj);
    std::unique_lock<std::shared_mutex> g(ns_mu_);
    if (static_cast<EventType>(type) == EventType::Deleted)
      ns_labels_.erase(md.name);
    else
      ns_labels_[md.name] = md.labels;
    ns_version_.fetch_add(1, std::memory_order_release);
  }
  StrMap ns_labels(const std::string& ns) const {
    std::shared_lock<std::shared_mutex> g(ns_mu_);
    auto it = ns_labels_.find(ns);
    return it == ns_labels_.end() ? StrMap{} : it->second;
  }

  // AffinityTerm.Matches: namespace in the term's set (default: the owner's
  // namespace) or selected by namespaceSelector, and label selector match.
  bool term_matches(const PodAffinityTerm& t, const std::string& owner_ns, const Pod& q) const {
    bool ns_ok = false;
    if (t.namespaces.empty() && !t.namespace_selector.present) {
      ns_ok = q.ns() == owner_ns;
    } else {
      for (const auto& n : t.namespaces)
        if (n == q.ns()) {
          ns_ok = true;
          break;
        }
      if (!ns_ok && t.namespace_selector.present) ns_ok = t.namespace_selector.matches(ns_labels(q.ns()));
    }
    return ns_ok && t.selector.matches(q.meta.labels);
  }
  bool matches_all(const std::vector<PodAffinityTerm>& ts, const std::string& owner_ns, const Pod& q) const {
    if (ts.empty()) return false;
    for (const auto& t : ts)
      if (!term_matches(t, owner_ns, q)) return false;
    return true;
  }

  // Required anti-affinity terms whose topology domain is a single node
  // (hostname key, Snapshot::hostname_domains_are_nodes) are not counted in
  // the PreFilter state: Filter checks them against the node's own pods, so
  // PreFilter does no per-pod map work for the common "one per node" rule.
  bool counted(const PodAffinityTerm& t) const {
    return !(h_.snapshot && h_.snapshot->hostname_domains_are_nodes && t.topology_key == kHostnameLabel);
  }

  // updateWithPod: `q` (existing) entering/leaving node `n` for incoming `p`.
  // Callers add/remove q on the NodeInfo too, which node-local terms read.
  void update(AffinityFilterState& st, const Pod& p, const Pod& q, const Node& n, int64_t d) const {
    for (const auto& t : q.pod_anti_affinity_required)
      if (counted(t) && term_matches(t, q.ns(), p)) bump(st.existing_anti, n, t.topology_key, d);
    if (matches_all(p.pod_affinity_required, p.ns(), q))
      for (const auto& t : p.pod_affinity_required) bump(st.affinity, n, t.topology_key, d);
    for (const auto& t : p.pod_anti_affinity_required)
      if (counted(t) && term_matches(t, p.ns(), q)) bump(st.anti, n, t.topology_key, d);
  }

  Status pre_filter(CycleState& s, const Pod& p) override {
    const bool own_terms = !p.pod_affinity_required.empty() || !p.pod_anti_affinity_required.empty();
    if (!h_.snapshot || (h_.snapshot->have_pods_with_required_anti_affinity.empty() && !own_terms)) {
      if (!own_terms) {
        s.write(kFilterKey, empty_state<AffinityFilterState>());
      } else {  // no snapshot: nothing counted, but Filter indexes p's terms
        auto st = std::make_shared<AffinityFilterState>();
        st->set_pod(p);
        s.write(kFilterKey, st);
      }
      return {};
    }
    const Snapshot& snap = *h_.snapshot;
    const uint64_t key = p.spec_hash ^ labels_hash(p.meta.labels);
    const uint64_t nsv = ns_version_.load(std::memory_order_acquire);
    if (auto* m = memo_.find(key, p.ns(), nsv, snap.topology_epoch)) {
      AffinityFilterState& ms = *m->st;
      if (snap.replay_since(m->seq, [&](const PodDelta& d) { update(ms, p, *d.pod, *d.node, d.d); })) {
        m->seq = snap.delta_end;
        ms.set_pod(p);
        s.write(kFilterKey, m->st);
        return {};
      }
    }
    auto st = std::make_shared<AffinityFilterState>();
    // Existing pods' required anti-affinity against p, and p's own required
    // terms against every existing pod: O(pods in the cluster) term matches,
    // split into node chunks on the Parallelizer (as upstream's PreFilter
    // fans out over nodes) and merged.
    const auto& anti_nodes = h_.snapshot->have_pods_with_required_anti_affinity;
    const auto& all = h_.snapshot->nodes;
    bool own = !p.pod_affinity_required.empty();
    for (const auto& t : p.pod_anti_affinity_required) own = own || counted(t);
    const size_t work = anti_nodes.size() + (own ? all.size() : 0);
    const int chunks = h_.parallelizer && work >= 512 ? 16 : 1;
    std::vector<AffinityFilterState> part(chunks);
    auto run = [&](int k) {
      AffinityFilterState& ps = part[k];
      for (size_t i = anti_nodes.size() * k / chunks; i < anti_nodes.size() * (k + 1) / chunks; ++i) {
        const NodeInfo& ni = *anti_nodes[i];
        for (const auto& q : ni.pods_with_required_anti_affinity)
          for (const auto& t : q->pod_anti_affinity_required)
            if (counted(t) && term_matches(t, q->ns(), p)) bump(ps.existing_anti, *ni.node, t.topology_key, 1);
      }
      if (!own) return;
      for (size_t i = all.size() * k / chunks; i < all.size() * (k + 1) / chunks; ++i) {
        const NodeInfo& ni = *all[i];
        for (const auto& q : ni.pods) {
          if (matches_all(p.pod_affinity_required, p.ns(), *q))
            for (const auto& t : p.pod_affinity_required) bump(ps.affinity, *ni.node, t.topology_key, 1);
          for (const auto& t : p.pod_anti_affinity_required)
            if (counted(t) && term_matches(t, p.ns(), *q)) bump(ps.anti, *ni.node, t.topology_key, 1);
        }
      }
    };
    if (chunks > 1)
      h_.parallelizer->until(chunks, run);
    else
      run(0);
    for (const auto& ps : part) st->merge(ps);
    st->set_pod(p);
    memo_.put(key, p.ns(), nsv, snap, st);
    s.write(kFilterKey, st);
    return {};
  }
  bool has_pre_filter_extensions() const override { return true; }
  // update() bumps counts only through q's required anti-affinity terms or
  // p's own required (anti-)affinity terms.
  bool pre_filter_extension_affects(const CycleState&, const Pod& p, const Pod& q) const override {
    return !q.pod_anti_affinity_required.empty() || !p.pod_affinity_required.empty() ||
           !p.pod_anti_affinity_required.empty();
  }
  Status add_pod(CycleState& s, const Pod& p, const PodPtr& q, const NodeInfo& ni) override {
    if (auto* st = s.read_as<AffinityFilterState>(kFilterKey)) {
      update(*st, p, *q, *ni.node, 1);
      st->set_pod(p);  // a count map may have appeared or gone
    }
    return {};
  }
  Status remove_pod(CycleState& s, const Pod& p, const PodPtr& q, const NodeInfo& ni) override {
    if (auto* st = s.read_as<AffinityFilterState>(kFilterKey)) {
      update(*st, p, *q, *ni.node, -1);
      st->set_pod(p);
    }
    return {};
  }

  Status filter(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    auto* st = s.read_as<AffinityFilterState>(kFilterKey);
    if (!st) return Status::error("InterPodAffinity: no PreFilter state");
    const Node& n = *ni.node;
    // satisfyPodAffinity
    if (!p.pod_affinity_required.empty()) {
      bool exist = true;
      for (size_t i = 0; i < p.pod_affinity_required.size(); ++i) {
        const std::string* v = n.meta.label(p.pod_affinity_required[i].topology_key);
        if (!v) return kAffinityUnmet();
        const auto* counts = st->aff_c[i];
        auto it = counts ? counts->find(*v) : decltype(counts->end()){};
        if (!counts || it == counts->end() || it->second <= 0) exist = false;
      }
      // The first pod of a self-affine series may go anywhere.
      if (!exist && !(st->affinity.empty() && matches_all(p.pod_affinity_required, p.ns(), p)))
        return kAffinityUnmet();
    }
    // satisfyPodAntiAffinity
    for (size_t i = 0; i < p.pod_anti_affinity_required.size(); ++i) {
      const auto& t = p.pod_anti_affinity_required[i];
      if (counted(t)) {
        const auto* counts = st->anti_c[i];
        if (!counts) continue;
        const std::string* v = n.meta.label(t.topology_key);
        if (!v) continue;
        auto it = counts->find(*v);
        if (it != counts->end() && it->second > 0) return kAntiAffinityUnmet();
      } else if (n.meta.label(kHostnameLabel)) {
        for (const auto& q : ni.pods)
          if (term_matches(t, p.ns(), *q))
            return kAntiAffinityUnmet();
      }
    }
    // satisfyExistingPodsAntiAffinity: node-local terms of the node's own pods,
    // then per counted topology key the node's value (no key strings built).
    if (!ni.pods_with_required_anti_affinity.empty() && h_.snapshot && h_.snapshot->hostname_domains_are_nodes &&
        n.meta.label(kHostnameLabel))
      for (const auto& q : ni.pods_with_required_anti_affinity)
        for (const auto& t : q->pod_anti_affinity_required)
          if (!counted(t) && term_matches(t, q->ns(), p))
            return kExistingAntiAffinityUnmet();
    for (const auto& [key, values] : st->existing_anti) {
      const std::string* v = n.meta.label(key);
      if (!v) continue;
      auto it = values.find(*v);
      if (it != values.end() && it->second > 0)
        return kExistingAntiAffinityUnmet();
    }
    return {};
  }

  void add_term(AffinityScoreState& st, const PodAffinityTerm& t, int64_t w, const std::string& owner_ns,
                const Pod& q, const Node& n) const {
    if (w == 0 || !term_matches(t, owner_ns, q)) return;
    if (const std::string* v = n.meta.label(t.topology_key)) topo_add(st.topo_score, t.topology_key, *v, w);
  }
  // Everything existing pod `q` on node `n` adds to p's topology scores,
  // times d (+1 entering, -1 leaving): PreScore's per-pod body, and the
  // replay step of a memoized score state.
  void score_pod(AffinityScoreState& st, const Pod& p, const Pod& q, const Node& n, int64_t d) const {
    for (const auto& wt : p.pod_affinity_preferred) add_term(st, wt.term, d * wt.weight, p.ns(), q, n);
    for (const auto& wt : p.pod_anti_affinity_preferred) add_term(st, wt.term, -d * wt.weight, p.ns(), q, n);
    if (hard_weight_ > 0)
      for (const auto& t : q.pod_affinity_required) add_term(st, t, d * hard_weight_, q.ns(), p, n);
    for (const auto& wt : q.pod_affinity_preferred) add_term(st, wt.term, d * wt.weight, q.ns(), p, n);
    for (const auto& wt : q.pod_anti_affinity_preferred) add_term(st, wt.term, -d * wt.weight, q.ns(), p, n);
  }

  Status pre_score(CycleState& s, const Pod& p, const NodeList& nodes) override {
    bool has_pref = !p.pod_affinity_preferred.empty() || !p.pod_anti_affinity_preferred.empty();
    if (!h_.snapshot || nodes.empty() || (!has_pref && h_.snapshot->have_pods_with_affinity.empty())) {
      s.write(kScoreKey, empty_state<AffinityScoreState>());
      return {};
    }
    // The scores do not depend on the feasible `nodes`, only on the pods of
    // the cluster: memoized like the Filter state (same key and validity).
    const Snapshot& snap = *h_.snapshot;
    const uint64_t key = p.spec_hash ^ labels_hash(p.meta.labels);
    const uint64_t nsv = ns_version_.load(std::memory_order_acquire);
    if (auto* m = score_memo_.find(key, p.ns(), nsv, snap.topology_epoch)) {
      AffinityScoreState& ms = *m->st;
      if (snap.replay_since(m->seq, [&](const PodDelta& d) { score_pod(ms, p, *d.pod, *d.node, d.d); })) {
        m->seq = snap.delta_end;
        s.write(kScoreKey, m->st);
        return {};
      }
    }
    auto st = std::make_shared<AffinityScoreState>();
    const auto& scan = has_pref ? snap.nodes : snap.have_pods_with_affinity;
    for (const auto& ni : scan) {
      const auto& pods = has_pref ? ni->pods : ni->pods_with_affinity;
      for (const auto& q : pods) score_pod(*st, p, *q, *ni->node, 1);
    }
    score_memo_.put(key, p.ns(), nsv, snap, st);
    s.write(kScoreKey, st);
    return {};
  }
  std::pair<int64_t, Status> score(CycleState& s, const Pod&, const NodeInfo& ni) override {
    auto* st = s.read_as<AffinityScoreState>(kScoreKey);
    if (!st) return {0, Status::error("InterPodAffinity: no PreScore state")};
    int64_t score = 0;
    for (const auto& [key, vals] : st->topo_score) {
      const std::string* v = ni.node->meta.label(key);
      if (!v) continue;
      auto it = vals.find(*v);
      if (it != vals.end()) score += it->second;
    }
    return {score, {}};
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState& s, const Pod&, std::vector<NodeScore>& scores) override {
    auto* st = s.read_as<AffinityScoreState>(kScoreKey);
    if (!st || st->topo_score.empty()) return {};
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (const auto& x : scores) {
      lo = std::min(lo, x.score);
      hi = std::max(hi, x.score);
    }
    int64_t diff = hi - lo;
    for (auto& x : scores)
      x.score = diff > 0 ? static_cast<int64_t>(static_cast<double>(kMaxNodeScore) *
                                                (static_cast<double>(x.score - lo) / static_cast<double>(diff)))
                         : 0;
    return {};
  }
  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kAll, ""}, {"Node", kAdd | kUpdateNodeLabel, ""}};
  }

 private:
  Handle& h_;
  int32_t hard_weight_ = 1;
  mutable std::shared_mutex ns_mu_;
  std::unordered_map<std::string, StrMap> ns_labels_;
  std::atomic<uint64_t> ns_version_{0};  // memoized states depend on namespace labels
  StateMemo<AffinityFilterState> memo_;
  StateMemo<AffinityScoreState> score_memo_;
};

// ========================================================= ImageLocality ====
class ImageLocality : public Plugin {
 public:
  // Node images + cluster-wide image spread: both change only with Node objects (node epoch).
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  explicit ImageLocality(Handle& h) : Plugin("ImageLocality", kScore), h_(h) {}
  static constexpr int64_t kMB = 1024 * 1024;
  static constexpr int64_t kMinThreshold = 23 * kMB;
  static constexpr int64_t kMaxContainerThreshold = 1000 * kMB;

  static std::string normalized(const std::string& image) {
    size_t colon = image.rfind(':'), slash = image.rfind('/');
    bool has_tag = colon != std::string::npos && (slash == std::string::npos || colon > slash);
    return has_tag ? image : image + ":latest";
  }

  // No container image present on any node: sum is 0 on every node, which
  // clamps to kMinThreshold and scores 0. Reads the Snapshot's image spread,
  // the same view score() uses, so the skip and the score cannot disagree.
  bool score_all_zero(const Pod& p, const Snapshot& s) const override {
    if (kMaxContainerThreshold * static_cast<int64_t>(p.containers.size()) <= kMinThreshold) return true;
    if (s.image_spread->empty()) return true;
    for (const auto& c : p.containers)
      if (s.image_spread->count(normalized(c.image))) return false;
    return true;
  }

  // Upstream ImageLocality (vendor/.../plugins/imagelocality/image_locality.go):
  // Σ size·(numNodes/totalNodes) over the pod's images present on the node,
  // clamped to [23 MB, 1000 MB·containers] and scaled to [0, 100]. Node image
  // sizes come from the immutable Node object and spreads from the Snapshot.
  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    const Snapshot* snap = h_.snapshot;
    int64_t total_nodes = snap ? static_cast<int64_t>(snap->nodes.size()) : 1;
    int64_t sum = 0;
    if (ni.node && snap && total_nodes > 0 && !ni.node->image_sizes.empty())
      for (const auto& c : p.containers) {
        auto it = ni.node->image_sizes.find(normalized(c.image));
        if (it == ni.node->image_sizes.end()) continue;
        auto cnt = snap->image_spread->find(it->first);
        int64_t spread = cnt == snap->image_spread->end() ? 0 : cnt->second;
        sum += static_cast<int64_t>(static_cast<double>(it->second) * static_cast<double>(spread) /
                                    static_cast<double>(total_nodes));
      }
    int64_t max_threshold = kMaxContainerThreshold * static_cast<int64_t>(p.containers.size());
    if (max_threshold <= kMinThreshold) return {0, {}};
    sum = std::clamp(sum, kMinThreshold, max_threshold);
    return {kMaxNodeScore * (sum - kMinThreshold) / (max_threshold - kMinThreshold), {}};
  }

 private:
  Handle& h_;
};

PluginRegistrar r1("PodTopologySpread", [](const Json&, Handle& h) { return std::make_shared<PodTopologySpread>(h); });
PluginRegistrar r2("InterPodAffinity",
                   [](const Json& a, Handle& h) { return std::make_shared<InterPodAffinity>(a, h); });
PluginRegistrar r3("ImageLocality", [](const Json&, Handle& h) { return std::make_shared<ImageLocality>(h); });

}  // namespace

void link_topology_plugins() {}

}  // namespace xsched
