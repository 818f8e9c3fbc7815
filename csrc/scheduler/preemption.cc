#include "scheduler/preemption.h"

#include "common/log.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <map>
#include <mutex>
#include <tuple>

#include "framework/framework.h"
#include "framework/waiting_pods.h"
#include "scheduler/extender.h"
#include "scheduler/informers.h"
#include "scheduler/metrics.h"
#include "scheduler/queue.h"

namespace xsched {

// GetPodStartTime falls back to "now" for pods without status.startTime; a
// clock read per comparison would make sort comparators inconsistent, so use
// the latest timestamp we know instead (scheduled, created), else "latest".
int64_t pod_start_time(const Pod& p) {
  if (p.start_time) return p.start_time;
  if (p.scheduled_at) return p.scheduled_at;
  if (p.meta.creation) return p.meta.creation;
  return INT64_MAX;
}

bool more_important_pod(const Pod& a, const Pod& b) {
  if (a.priority != b.priority) return a.priority > b.priority;
  return pod_start_time(a) < pod_start_time(b);
}

void filter_pods_with_pdb_violation(const std::vector<PodPtr>& pods, const std::vector<PDBPtr>& pdbs,
                                    std::vector<PodPtr>& violating, std::vector<PodPtr>& non_violating) {
  std::vector<int64_t> allowed(pdbs.size());
  for (size_t i = 0; i < pdbs.size(); ++i) allowed[i] = pdbs[i]->disruptions_allowed;
  for (const auto& p : pods) {
    bool violated = false;
    if (!p->meta.labels.empty()) {
      for (size_t i = 0; i < pdbs.size(); ++i) {
        const auto& pdb = *pdbs[i];
        if (pdb.meta.ns != p->ns()) continue;
        // A nil or empty selector matches nothing.
        if (!pdb.selector.present || (pdb.selector.match_labels.empty() && pdb.selector.exprs.empty())) continue;
        if (!pdb.selector.matches(p->meta.labels)) continue;
        if (strmap_get(pdb.disrupted_pods, p->name())) continue;  // already processed by the API server
        if (--allowed[i] < 0) violated = true;
      }
    }
    (violated ? violating : non_violating).push_back(p);
  }
}

Status select_victims_default(Handle& h, CycleState& s, const Pod& preemptor, NodeInfo& ni,
                              const std::vector<PDBPtr>& pdbs, const std::function<bool(const Pod&)>& may_evict,
                              std::vector<PodPtr>& victims, int& num_violating) {
  Framework& fw = *h.framework;
  std::vector<PodPtr> potential;
  thread_local std::vector<PodPtr> pods;  // ni.pods changes while we walk it
  pods.assign(ni.pods.begin(), ni.pods.end());
  for (const auto& p : pods) {
    if (!may_evict(*p)) continue;
    potential.push_back(p);
    ni.remove_pod(p->uid());
    Status st = fw.run_pre_filter_remove_pod(s, preemptor, p, ni);
    if (!st.is_success()) return st;
  }
  if (potential.empty())
    return Status::unresolvable("No victims found on node " + ni.name() + " for preemptor pod " + preemptor.name());
  Status st = fw.run_filter_with_nominated_pods_inplace(s, preemptor, ni);
  if (!st.is_success()) return st;
  std::stable_sort(potential.begin(), potential.end(),
            [](const PodPtr& a, const PodPtr& b) { return more_important_pod(*a, *b); });
  std::vector<PodPtr> violating, non_violating;
  filter_pods_with_pdb_violation(potential, pdbs, violating, non_violating);
  auto reprieve = [&](const PodPtr& p) -> std::pair<bool, Status> {
    ni.add_pod(p);
    Status ast = fw.run_pre_filter_add_pod(s, preemptor, p, ni);
    if (!ast.is_success()) return {false, ast};
    bool fits = fw.run_filter_with_nominated_pods_inplace(s, preemptor, ni).is_success();
    if (!fits) {
      ni.remove_pod(p->uid());
      Status rst = fw.run_pre_filter_remove_pod(s, preemptor, p, ni);
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

bool default_eligible(Handle& h, const Pod& pod, const Status* nominated_status) {
  if (pod.preemption_policy == "Never") return false;
  if (!pod.nominated_node_name.empty()) {
    if (nominated_status && nominated_status->code() == Code::UnschedulableAndUnresolvable) return true;
    if (h.snapshot) {
      if (auto ni = h.snapshot->get(pod.nominated_node_name)) {
        for (const auto& p : ni->pods)
          if (p->terminating() && p->priority < pod.priority) return false;  // victims still terminating
      }
    }
  }
  return true;
}

int calculate_num_candidates(int num_nodes, int pct, int min_abs) {
  int n = num_nodes * pct / 100;
  if (n < min_abs) n = min_abs;
  if (n > num_nodes) n = num_nodes;
  return n;
}

const std::vector<NodeInfoPtr>& nodes_where_preemption_might_help(const Snapshot& snap, const NodeStatusMap& m,
                                                                  std::vector<NodeInfoPtr>& out) {
  if (m.count_code(Code::UnschedulableAndUnresolvable) == 0) return snap.nodes;  // no copy of the node list
  // The map may carry names outside this snapshot (a PostFilter handed a map
  // built elsewhere), so a node is only skipped on its own unresolvable entry.
  out.clear();
  out.reserve(snap.nodes.size());
  for (const auto& ni : snap.nodes) {
    const Status* st = m.status_of(ni->name());
    if (!st || st->code() != Code::UnschedulableAndUnresolvable) out.push_back(ni);
  }
  return out;
}

struct Evaluator::DryRun {
  // A slot holds a candidate of the run numbered `run` (older contents are
  // dead: slots are never reset, each write sets every field).
  struct Slot {
    uint64_t run = 0;
    const MemoEntry* memo = nullptr;
    const std::string* name = nullptr;  // memo hits: the node's name
    Candidate c;
    PickKey key;
  };
  std::vector<Slot> slots;
  std::vector<CandidateRef> refs;  // into slots / memo entries, non-violating first
};

namespace {

// The victims' share of a PickKey (victims sorted most important first).
void victim_key_parts(const std::vector<PodPtr>& v, int64_t& top, int64_t& sum, int64_t& earliest) {
  top = v.empty() ? 0 : v[0]->priority;
  sum = 0;
  earliest = LLONG_MAX;
  for (const auto& p : v) {
    sum += static_cast<int64_t>(p->priority) + INT32_MAX + 1;
    earliest = std::min(earliest, pod_start_time(*p));
  }
}

PickKey make_key(int npv, int64_t top, int64_t sum, size_t size, int64_t earliest) {
  return PickKey{npv, top, sum, static_cast<int64_t>(size), earliest == LLONG_MIN ? LLONG_MAX : -earliest};
}

PickKey key_of(const std::vector<PodPtr>& v, int npv) {
  int64_t top, sum, earliest;
  victim_key_parts(v, top, sum, earliest);
  return make_key(npv, top, sum, v.size(), earliest);
}

}  // namespace

Evaluator::Evaluator(std::string plugin_name, Handle& h, PreemptionPolicy* policy)
    : plugin_(std::move(plugin_name)), h_(h), policy_(policy), memo_(std::make_unique<Memo>()) {}
Evaluator::~Evaluator() = default;

std::vector<Candidate> Evaluator::dry_run(CycleState& s, const Pod& pod, const std::vector<NodeInfoPtr>& potential,
                                          const std::vector<PDBPtr>& pdbs, int offset, int num_candidates) {
  if (!scratch_) scratch_ = std::make_unique<DryRun>();
  DryRun& dr = *scratch_;
  dry_run_refs(s, pod, potential, pdbs, offset, num_candidates, dr);
  std::vector<Candidate> out;
  out.reserve(dr.refs.size());
  for (const auto& r : dr.refs) out.push_back(Candidate{*r.node, *r.victims, r.num_pdb_violations});
  return out;
}

void Evaluator::dry_run_refs(CycleState& s, const Pod& pod, const std::vector<NodeInfoPtr>& potential,
                             const std::vector<PDBPtr>& pdbs, int offset, int num_candidates, DryRun& dr) {
  std::atomic<bool> stop{false};
  int n = static_cast<int>(potential.size());
  // Reuse is sound when the policy's victims depend on the node alone, no
  // PDB can change the violation count, and every Filter is node-local for
  // this pod (the equivalence cache's condition); nodes with nominated pods
  // and nodes where a PreFilter extension reacts to a victim are recomputed.
  const bool guarded = policy_->guarded_victims();
  const uint64_t run = ++runs_;
  const bool memo_ok = (policy_->victims_depend_only_on_node() || guarded) && pdbs.empty() && pod.template_hash != 0 &&
                       h_.snapshot && h_.framework && h_.framework->filters_node_local(pod, *h_.snapshot) &&
                       (s.nominated || !h_.nominator || h_.nominator->empty());
  if (memo_ok) {
    // Bounded: entries of nodes that left the cluster are dropped here,
    // single-threaded, never while workers hold pointers into a shard.
    const size_t limit = 2 * (static_cast<size_t>(n) / Memo::kShards + 64);
    for (auto& sh : memo_->shards)
      if (sh.m.size() > limit) sh.m.clear();
  }
  // Candidates land in preallocated slots claimed with one atomic add: the
  // 16 workers never share a lock, and a remembered result is only a
  // pointer here (its victims are copied on this thread afterwards, so the
  // workers allocate nothing for it). Workers overshoot the stop by at most
  // one node each.
  using Slot = DryRun::Slot;
  // When every node is wanted (CapacityScheduling's offset 0, all nodes)
  // nothing stops early: node i writes slot i, with no shared counter for 16
  // workers to bounce (and the candidates keep the nodes' order).
  const bool by_index = num_candidates >= n;
  const int cap = by_index ? n : num_candidates + 64;
  std::vector<Slot>& slots = dr.slots;
  if (slots.size() < static_cast<size_t>(cap)) slots.resize(static_cast<size_t>(cap));
  std::atomic<int> used{0}, non_violating{0};
  auto claim = [&](int i, int num_pdb_violations) -> Slot* {
    if (by_index) return &slots[static_cast<size_t>(i)];
    int k = used.fetch_add(1, std::memory_order_relaxed);
    if (k >= cap) {
      stop.store(true);
      return nullptr;
    }
    int nv = num_pdb_violations == 0 ? non_violating.fetch_add(1) + 1 : non_violating.load();
    if (nv > 0 && k + 1 >= num_candidates) stop.store(true);
    return &slots[static_cast<size_t>(k)];
  };
  // One node's dry run. Memo hits and misses are counted by the caller per
  // chunk of nodes: a shared counter bumped per node serialised the 16
  // workers on one cache line (as the forked Filter walk did, round 6).
  auto one = [&](int i, uint64_t& hits, uint64_t& misses) {
    const NodeInfoPtr& src = potential[(offset + i) % n];
    Memo::Shard* shard = nullptr;
    const std::vector<PodPtr>* noms = nullptr;
    uint64_t nom_fp = 0;
    if (memo_ok) {
      if (s.nominated) {
        auto it = s.nominated->find(src->name());
        if (it != s.nominated->end() && !it->second.empty()) noms = &it->second;
      }
      // Nominated pods join the node in the Filters the dry run calls: a
      // guarded policy keys its entry on them (their pods' uid and priority),
      // the others recompute such nodes.
      if (noms && guarded) {
        nom_fp = 0x9e3779b97f4a7c15ULL;
        for (const auto& np : *noms)
          nom_fp += std::hash<std::string>{}(np->uid()) * 0xff51afd7ed558ccdULL ^ static_cast<uint64_t>(np->priority);
      }
      if (!noms || guarded) {
        shard = &memo_->shards[std::hash<std::string>{}(src->name()) % Memo::kShards];
        // Entries are stable for the run: only this worker writes this node's
        // entries during it, so they are checked outside the lock.
        std::array<const MemoEntry*, Memo::kVariants> match{};
        size_t nmatch = 0;
        {
          std::lock_guard<std::mutex> g(shard->mu);
          auto it = shard->m.find(src->name());
          if (it != shard->m.end())
            for (const MemoEntry& e : it->second.v)
              if (e.gen == src->generation && e.tmpl == pod.template_hash && e.nominated_fp == nom_fp &&
                  nmatch < match.size())
                match[nmatch++] = &e;
        }
        const MemoEntry* hit = nullptr;
        for (size_t j = 0; j < nmatch && !hit; ++j)
          if (!match[j]->guards || policy_->guards_hold(s, *match[j]->guards, run)) hit = match[j];
        if (hit) {
          ++hits;
          if (!hit->candidate) return;
          if (Slot* sl = claim(i, hit->num_pdb_violations)) {
            sl->run = run;
            sl->memo = hit;
            sl->name = &src->name();
            sl->key = make_key(hit->num_pdb_violations, hit->top, hit->sum, hit->victims.size(), hit->earliest);
          }
          return;
        }
        ++misses;
      }
    }
    // The candidate is evaluated on this worker's scratch NodeInfo: copy
    // assignment reuses its vectors' storage, so a dry run allocates nothing
    // per node (a fresh clone per candidate made the 16 workers contend on
    // the allocator: PreemptionBasic at 5,000 nodes, round-3 sample profile).
    thread_local NodeInfo scratch;
    scratch = *src;
    NodeInfo* ni = &scratch;
    // Victims leave and re-enter the node through the PreFilter extensions.
    // When none of them reacts to any pod here, those calls are skipped and
    // the candidate reads the cycle's state as every Filter worker does,
    // instead of deep-cloning it per node.
    std::shared_ptr<CycleState> cloned;
    CycleState* st = &s;
    // A guarded policy's own extensions are covered by its guards; any other
    // plugin's extension reacting to a pod here makes the result unmemoizable.
    bool others_react = false;
    for (const auto& q : ni->pods) {
      if (!cloned && h_.framework->pre_filter_extensions_affected(s, pod, *q)) {
        cloned = s.clone();
        st = cloned.get();
        if (!guarded) break;
      }
      if (cloned && guarded && h_.framework->pre_filter_extensions_affected(s, pod, *q, policy_->guarded_plugin())) {
        others_react = true;
        break;
      }
    }
    if (shard && guarded && noms && !others_react)
      for (const auto& np : *noms)
        if (h_.framework->pre_filter_extensions_affected(s, pod, *np, policy_->guarded_plugin())) {
          others_react = true;
          break;
        }
    if (shard && guarded) policy_->start_guards(s);
    Candidate c;
    c.node = ni->name();
    Status vs = policy_->select_victims_on_node(*st, pod, *ni, pdbs, c.victims, c.num_pdb_violations);
    std::shared_ptr<const VictimGuards> guards = shard && guarded ? policy_->take_guards() : nullptr;
    // An Error is not a property of the node: never remembered.
    const bool candidate = vs.is_success() && !c.victims.empty();
    const bool storable = guarded ? guards != nullptr && !others_react : !cloned;
    if (shard && storable && (candidate || vs.is_unschedulable())) {
      std::lock_guard<std::mutex> g(shard->mu);
      Memo::NodeMemo& nm = shard->m[c.node];
      // Results of an older node version are dead; then reuse the slot of
      // the same key (guarded: the same interned guard set) or rotate.
      nm.v.erase(std::remove_if(nm.v.begin(), nm.v.end(), [&](const MemoEntry& x) { return x.gen != src->generation; }),
                 nm.v.end());
      MemoEntry* slot = nullptr;
      for (MemoEntry& x : nm.v)
        if (x.tmpl == pod.template_hash && x.nominated_fp == nom_fp && (!guarded || x.guards == guards)) slot = &x;
      if (!slot && nm.v.size() < Memo::kVariants) slot = &nm.v.emplace_back();
      if (!slot) slot = &nm.v[nm.next++ % nm.v.size()];
      MemoEntry& e = *slot;
      e.gen = src->generation;
      e.tmpl = pod.template_hash;
      e.candidate = candidate;
      e.victims = c.victims;
      e.num_pdb_violations = c.num_pdb_violations;
      e.guards = std::move(guards);
      e.nominated_fp = nom_fp;
      victim_key_parts(e.victims, e.top, e.sum, e.earliest);
    }
    if (!candidate) return;
    if (Slot* sl = claim(i, c.num_pdb_violations)) {
      sl->run = run;
      sl->memo = nullptr;
      sl->key = key_of(c.victims, c.num_pdb_violations);
      sl->c.node = std::move(c.node);
      sl->c.victims.swap(c.victims);
      sl->c.num_pdb_violations = c.num_pdb_violations;
    }
  };
  auto range = [&](int b, int e) {
    uint64_t hits = 0, misses = 0;
    for (int i = b; i < e && !stop.load(std::memory_order_relaxed); ++i) one(i, hits, misses);
    if (hits) memo_->hits.fetch_add(hits, std::memory_order_relaxed);
    if (misses) memo_->misses.fetch_add(misses, std::memory_order_relaxed);
  };
  if (h_.parallelizer->plan_inline(n, nullptr))
    range(0, n);
  else
    h_.parallelizer->until_forked_ranges(n, range, &stop, nullptr);
  // Non-violating candidates first, then the violating ones (upstream order).
  const int k = by_index ? n : std::min(used.load(), cap);
  dr.refs.clear();
  dr.refs.reserve(static_cast<size_t>(k));
  for (int pass = 0; pass < 2; ++pass) {
    for (int j = 0; j < k; ++j) {
      const Slot& sl = slots[static_cast<size_t>(j)];
      if (sl.run != run) continue;
      if (sl.memo) {
        if ((sl.memo->num_pdb_violations == 0) != (pass == 0)) continue;
        dr.refs.push_back(CandidateRef{sl.name, &sl.memo->victims, sl.memo->num_pdb_violations, &sl.key});
      } else {
        if ((sl.c.num_pdb_violations == 0) != (pass == 0)) continue;
        dr.refs.push_back(CandidateRef{&sl.c.node, &sl.c.victims, sl.c.num_pdb_violations, &sl.key});
      }
    }
  }
  XS_LOGV(5, "preemption dry run").kv("pod", pod.key()).kv("potentialNodes", n).kv("candidates", dr.refs.size())
      .kv("memo", memo_ok).kv("memoHits", memo_->hits.load()).kv("memoMisses", memo_->misses.load());
}

std::string Evaluator::pick_one_node(const std::vector<Candidate>& cands) {
  std::vector<CandidateRef> refs;
  refs.reserve(cands.size());
  for (const auto& c : cands) refs.push_back(CandidateRef{&c.node, &c.victims, c.num_pdb_violations});
  size_t i = pick_one(refs);
  return i < cands.size() ? cands[i].node : std::string();
}

size_t Evaluator::pick_one(const std::vector<CandidateRef>& cands) {
  // pickOneNodeForPreemption's criteria in order, as one lexicographic key
  // per candidate and a single pass: fewest PDB violations, lowest
  // highest-priority victim, lowest priority sum, fewest victims, then the
  // latest "earliest victim start"; the first candidate wins a full tie.
  if (cands.empty()) return SIZE_MAX;
  using Key = PickKey;
  size_t best = SIZE_MAX;
  Key best_key{};
  for (size_t i = 0; i < cands.size(); ++i) {
    const auto& v = *cands[i].victims;
    if (v.empty()) return i;  // no preemption needed at all
    if (cands[i].key) {  // computed by the dry run's worker
      if (best == SIZE_MAX || *cands[i].key < best_key) {
        best = i;
        best_key = *cands[i].key;
      }
      continue;
    }
    // victims are sorted most-important first, so v[0] is the highest priority.
    Key k{cands[i].num_pdb_violations, v[0]->priority, 0, static_cast<int64_t>(v.size()), 0};
    if (best != SIZE_MAX && (k.npv > best_key.npv || (k.npv == best_key.npv && k.top > best_key.top))) continue;
    int64_t earliest = LLONG_MAX;
    for (const auto& p : v) {
      k.sum += static_cast<int64_t>(p->priority) + INT32_MAX + 1;
      earliest = std::min(earliest, pod_start_time(*p));
    }
    k.neg_earliest = earliest == LLONG_MIN ? LLONG_MAX : -earliest;
    if (best == SIZE_MAX || k < best_key) {
      best = i;
      best_key = k;
    }
  }
  return best;
}

Status Evaluator::prepare_candidate(const Candidate& c, const Pod& pod) {
  for (const auto& v : c.victims) {
    if (auto wp = h_.waiting_pods->get(v->uid())) {
      wp->reject(plugin_, "preempted");
    } else {
      try {
        h_.client->delete_pod(*v);
      } catch (const std::exception& e) {
        std::string msg = e.what();
        if (msg.find("not found") == std::string::npos) return Status::error(msg);
      }
    }
    h_.client->record_event("Pod", v->ns(), v->name(), "Normal", "Preempted",
                            "Preempted by " + pod.key() + " on node " + c.node);
  }
  if (h_.metrics) h_.metrics->histogram("scheduler_preemption_victims", "").observe(static_cast<double>(c.victims.size()));
  // Lower-priority pods nominated to this node may no longer fit.
  if (h_.nominator) {
    for (const auto& np : h_.nominator->nominated_pods_for_node(c.node)) {
      if (np->priority >= pod.priority || np->uid() == pod.uid()) continue;
      h_.nominator->remove(*np);
      Json patch = Json::object();
      Json st = Json::object();
      st.set("nominatedNodeName", Json());
      patch.set("status", std::move(st));
      try {
        h_.client->patch("pods", np->ns(), np->name(), patch);
      } catch (const std::exception&) {
      }
    }
  }
  return {};
}

Status Evaluator::call_extenders(const Pod& pod, std::vector<Candidate>& cands) {
  // preemption.go callExtenders: each interested extender with a preempt verb
  // gets the current node -> victims map and returns the subset it accepts;
  // the next extender sees that subset.
  std::map<std::string, Extender::NodeVictims> victims;
  for (const auto& c : cands) victims[c.node] = Extender::NodeVictims{c.victims, c.num_pdb_violations};
  if (victims.empty()) return {};
  Json pod_obj;
  bool have_pod = false;
  for (const auto& e : *h_.extenders) {
    if (!e->supports_preemption() || !e->interested(pod)) continue;
    if (!have_pod) {
      JsonPtr obj = h_.lookup ? h_.lookup("pods", pod.ns(), pod.name()) : nullptr;
      if (obj) {
        pod_obj = *obj;
      } else {
        Json md = Json::object();
        md.set("name", Json(pod.name()));
        md.set("namespace", Json(pod.ns()));
        md.set("uid", Json(pod.uid()));
        pod_obj = Json::object();
        pod_obj.set("metadata", std::move(md));
      }
      have_pod = true;
    }
    std::map<std::string, Extender::NodeVictims> got;
    try {
      got = e->process_preemption(pod_obj, victims, h_.lookup);
    } catch (const std::exception& ex) {
      if (e->ignorable()) continue;
      return Status::error(ex.what());
    }
    for (auto it = got.begin(); it != got.end();) {
      if (it->second.pods.empty()) {
        if (!e->ignorable()) return Status::error("expected at least one victim pod on node " + it->first);
        it = got.erase(it);
      } else {
        ++it;
      }
    }
    victims = std::move(got);
    if (victims.empty()) break;
  }
  std::vector<Candidate> out;
  out.reserve(victims.size());
  for (auto& [node, v] : victims) {
    Candidate c;
    c.node = node;
    c.victims = std::move(v.pods);
    c.num_pdb_violations = static_cast<int>(v.num_pdb_violations);
    out.push_back(std::move(c));
  }
  cands = std::move(out);
  return {};
}

std::pair<PostFilterResult, Status> Evaluator::preempt(CycleState& s, const Pod& pod_in, const NodeStatusMap& m) {
  if (h_.metrics) h_.metrics->inc("scheduler_preemption_attempts_total", "");
  // 0) latest version of the pod
  PodPtr latest = h_.informers ? h_.informers->pod(pod_in.ns(), pod_in.name()) : nullptr;
  const Pod& pod = latest ? *latest : pod_in;
  // 1) eligibility
  const Status* nom = nullptr;
  if (!pod.nominated_node_name.empty()) nom = m.status_of(pod.nominated_node_name);
  if (!policy_->eligible(pod, nom))
    return {PostFilterResult{}, Status::unschedulable("Pod is not eligible for preemption")};
  // 2) candidates: nodes where preemption might help
  if (!h_.snapshot || h_.snapshot->nodes.empty()) return {PostFilterResult{}, Status::error("no nodes available")};
  std::vector<NodeInfoPtr> filtered;
  const std::vector<NodeInfoPtr>& potential = nodes_where_preemption_might_help(*h_.snapshot, m, filtered);
  if (potential.empty())
    return {PostFilterResult{}, Status::unschedulable("0/" + std::to_string(h_.snapshot->nodes.size()) +
                                                      " nodes are available: preemption is not helpful for scheduling.")};
  if (policy_->victims_have_lower_priority() && h_.snapshot->min_pod_priority >= pod.priority)
    return {PostFilterResult{}, Status::unschedulable("0/" + std::to_string(h_.snapshot->nodes.size()) +
                                                      " nodes are available: no preemption victims found.")};
  std::vector<PDBPtr> pdbs = h_.informers ? h_.informers->pdbs() : std::vector<PDBPtr>{};
  auto [offset, num] = policy_->offset_and_num_candidates(static_cast<int>(potential.size()));
  if (!scratch_) scratch_ = std::make_unique<DryRun>();
  DryRun& dr = *scratch_;
  dry_run_refs(s, pod, potential, pdbs, offset, num, dr);
  if (dr.refs.empty())
    return {PostFilterResult{}, Status::unschedulable("0/" + std::to_string(h_.snapshot->nodes.size()) +
                                                      " nodes are available: no preemption victims found.")};
  Candidate best;
  if (h_.extenders && !h_.extenders->empty()) {
    // 3) extenders with a preempt verb narrow the candidates (they need the
    // whole node -> victims map, so the candidates are materialized)
    std::vector<Candidate> cands;
    cands.reserve(dr.refs.size());
    for (const auto& r : dr.refs) cands.push_back(Candidate{*r.node, *r.victims, r.num_pdb_violations});
    Status est = call_extenders(pod, cands);
    if (!est.is_success()) return {PostFilterResult{}, est};
    if (cands.empty()) return {PostFilterResult{}, Status::unschedulable("no candidate node for preemption")};
    std::string node = pick_one_node(cands);
    for (auto& c : cands)
      if (c.node == node) best = std::move(c);
  } else {
    // 4) best candidate, chosen over references; only it is copied
    const CandidateRef& r = dr.refs[pick_one(dr.refs)];
    best = Candidate{*r.node, *r.victims, r.num_pdb_violations};
  }
  // 5) prepare
  Status st = prepare_candidate(best, pod);
  if (!st.is_success()) return {PostFilterResult{}, st};
  return {PostFilterResult{best.node}, Status()};
}

}  // namespace xsched
