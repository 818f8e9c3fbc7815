// Preemption evaluator shared by DefaultPreemption, CapacityScheduling and
// PreemptionToleration.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/framework/preemption/
// preemption.go (Evaluator.Preempt: PodEligibleToPreemptOthers ->
// findCandidates (nodes where preemption might help, random offset,
// numCandidates = max(minAbsolute, n*pct/100)) -> DryRunPreemption (parallel
// SelectVictimsOnNode on cloned NodeInfo + CycleState) -> SelectCandidate
// (pickOneNodeForPreemption ordering) -> prepareCandidate (reject waiting
// victims, delete the others, clear lower-priority nominations)), and
// DefaultPreemption's SelectVictimsOnNode with the PDB-violation reprieve
// order (util.MoreImportantPod).
#pragma once

#include <array>
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "framework/plugin.h"

namespace xsched {

// What a guarded policy's victim selection read of cluster-wide state on one
// node, recorded so a later cycle can re-check it (PreemptionPolicy::
// guarded_victims). Policy-defined.
struct VictimGuards {
  virtual ~VictimGuards() = default;
};

// The per-plugin policy (preemption.Interface).
class PreemptionPolicy {
 public:
  virtual ~PreemptionPolicy() = default;
  virtual std::pair<int, int> offset_and_num_candidates(int num_nodes) = 0;
  virtual bool eligible(const Pod& pod, const Status* nominated_node_status) = 0;
  // Selects victims on a cloned NodeInfo (mutated), cloned state.
  virtual Status select_victims_on_node(CycleState& s, const Pod& preemptor, NodeInfo& ni,
                                        const std::vector<PDBPtr>& pdbs, std::vector<PodPtr>& victims,
                                        int& num_violating) = 0;
  // True when select_victims_on_node's outcome is a function of the node's
  // version, the preemptor's template and the node's nominated pods only
  // (no clock, no quota or other cluster-wide state): the evaluator may then
  // reuse a node's dry-run result across preemptors (Evaluator::dry_run).
  virtual bool victims_depend_only_on_node() const { return false; }
  // True when select_victims_on_node's outcome is a function of the node's
  // version, the preemptor's template and the outcomes of cluster-wide
  // predicates (quota comparisons) that the policy records on the worker's
  // thread while it runs (start_guards .. take_guards) and can re-evaluate
  // against a later cycle's state (guards_hold). The evaluator then reuses a
  // node's result while every recorded predicate still comes out the same:
  // identical predicate outcomes drive select_victims_on_node down the same
  // path to the same victims. `run` numbers the dry run (one at a time per
  // evaluator), so a policy may cache a verdict per guard set within a run.
  // Victims leaving and re-entering the node
  // through the PreFilter extensions of `guarded_plugin()` are covered by the
  // guards; any other plugin's extension reacting disqualifies the node.
  virtual bool guarded_victims() const { return false; }
  virtual void start_guards(const CycleState&) {}
  virtual std::shared_ptr<const VictimGuards> take_guards() { return nullptr; }
  virtual bool guards_hold(const CycleState&, const VictimGuards&, uint64_t /*run*/) const { return false; }
  virtual const std::string* guarded_plugin() const { return nullptr; }
  // True when every victim must have a lower priority than the preemptor:
  // with no such pod on any node the dry run is skipped (it could only find
  // no candidate), which keeps a scheduler overloaded with equal-priority
  // pods from dry-running every node for each failure.
  virtual bool victims_have_lower_priority() const { return false; }
};

struct Candidate {
  std::string node;
  std::vector<PodPtr> victims;
  int num_pdb_violations = 0;
};
// pickOneNodeForPreemption's criteria as one lexicographic key: fewest PDB
// violations, lowest highest-priority victim, lowest priority sum, fewest
// victims, then the latest "earliest victim start".
struct PickKey {
  int64_t npv = 0, top = 0, sum = 0, size = 0, neg_earliest = 0;
  bool operator<(const PickKey& o) const {
    return std::tie(npv, top, sum, size, neg_earliest) < std::tie(o.npv, o.top, o.sum, o.size, o.neg_earliest);
  }
};
// A candidate by reference (into a dry run's results or a Candidate); `key`
// when the dry run already computed it (on its worker, not serially in
// pick_one).
struct CandidateRef {
  const std::string* node = nullptr;
  const std::vector<PodPtr>* victims = nullptr;
  int num_pdb_violations = 0;
  const PickKey* key = nullptr;
};

class Evaluator {
 public:
  Evaluator(std::string plugin_name, Handle& h, PreemptionPolicy* policy);
  ~Evaluator();
  std::pair<PostFilterResult, Status> preempt(CycleState& s, const Pod& pod, const NodeStatusMap& m);

  // Exposed for tests / other plugins.
  std::vector<Candidate> dry_run(CycleState& s, const Pod& pod, const std::vector<NodeInfoPtr>& potential,
                                 const std::vector<PDBPtr>& pdbs, int offset, int num_candidates);
  static std::string pick_one_node(const std::vector<Candidate>& cands);
  // pickOneNodeForPreemption over references: the index of the chosen one.
  static size_t pick_one(const std::vector<CandidateRef>& cands);
  // prepareCandidate: reject waiting victims, delete the others, clear
  // lower-priority nominations on the node (also used by CrossNodePreemption).
  Status prepare_candidate(const Candidate& c, const Pod& pod);
  // callExtenders: the configured preempt-verb extenders filter `cands`.
  Status call_extenders(const Pod& pod, std::vector<Candidate>& cands);

  uint64_t memo_hits() const { return memo_->hits.load(std::memory_order_relaxed); }
  uint64_t memo_misses() const { return memo_->misses.load(std::memory_order_relaxed); }

 private:
  struct DryRun;
  // The dry run proper: candidates in `out` (non-violating first), each a
  // reference into `out`'s storage or the memo, nothing copied.
  void dry_run_refs(CycleState& s, const Pod& pod, const std::vector<NodeInfoPtr>& potential,
                    const std::vector<PDBPtr>& pdbs, int offset, int num_candidates, DryRun& out);
  // Dry-run results per node, valid while (node generation, preemptor
  // template) match and the node has no nominated pods (guarded policies:
  // the same nominated pods, and guards that still hold). PreemptionBasic-like
  // waves evaluate the same unchanged nodes for every preemptor of one
  // template: the reference recomputes each (cloning the NodeInfo and
  // re-running every Filter per reprieved victim), here the result is reused.
  struct MemoEntry {
    int64_t gen = -1;
    uint64_t tmpl = 0;
    bool candidate = false;
    std::vector<PodPtr> victims;
    int num_pdb_violations = 0;
    std::shared_ptr<const VictimGuards> guards;  // guarded policies: re-checked on every hit
    uint64_t nominated_fp = 0;                   // guarded policies: the node's nominated pods (0: none)
    // The victims' part of the PickKey (highest priority, priority sum,
    // earliest start), computed once when the entry is stored.
    int64_t top = 0, sum = 0, earliest = 0;
  };
  struct Memo {
    static constexpr size_t kShards = 256;  // 16 dry-run workers rarely meet on one
    // A node keeps a few results (for different templates, nominations or
    // guard outcomes: quota sums near a threshold flip a guard back and forth
    // as nominations come and go, and each side stays remembered).
    static constexpr size_t kVariants = 4;
    struct NodeMemo {
      std::vector<MemoEntry> v;
      size_t next = 0;  // round-robin victim once kVariants are held
    };
    struct Shard {
      std::mutex mu;
      std::unordered_map<std::string, NodeMemo> m;
    };
    std::array<Shard, kShards> shards;
    std::atomic<uint64_t> hits{0}, misses{0};
  };
  std::string plugin_;
  Handle& h_;
  PreemptionPolicy* policy_;
  std::unique_ptr<Memo> memo_;
  std::unique_ptr<DryRun> scratch_;  // reused across dry runs (slots keep their storage)
  uint64_t runs_ = 0;  // dry runs so far (PostFilter runs on the scheduling thread only)
};

// ---- helpers shared by policies ----
int64_t pod_start_time(const Pod& p);  // status.startTime, else "now"
bool more_important_pod(const Pod& a, const Pod& b);
void filter_pods_with_pdb_violation(const std::vector<PodPtr>& pods, const std::vector<PDBPtr>& pdbs,
                                    std::vector<PodPtr>& violating, std::vector<PodPtr>& non_violating);
// DefaultPreemption.SelectVictimsOnNode with a pluggable "may this pod be a
// victim" predicate (lower priority for the default; + quota / toleration
// rules for the other policies).
Status select_victims_default(Handle& h, CycleState& s, const Pod& preemptor, NodeInfo& ni,
                              const std::vector<PDBPtr>& pdbs, const std::function<bool(const Pod&)>& may_evict,
                              std::vector<PodPtr>& victims, int& num_violating);
bool default_eligible(Handle& h, const Pod& pod, const Status* nominated_status);
int calculate_num_candidates(int num_nodes, int pct, int min_abs);
// Snapshot nodes preemption might help on: all but those whose Filter status
// is UnschedulableAndUnresolvable (nodesWherePreemptionMightHelp). One pass
// over the diagnosis instead of a name lookup per node; usually no node is
// unresolvable and the snapshot's list is returned whole.
// Returns the snapshot's own list when no node is unresolvable, else `out`.
const std::vector<NodeInfoPtr>& nodes_where_preemption_might_help(const Snapshot& snap, const NodeStatusMap& m,
                                                                  std::vector<NodeInfoPtr>& out);

}  // namespace xsched
