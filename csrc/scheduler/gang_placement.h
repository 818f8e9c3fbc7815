// xGMI gang co-location: which nodes may take the next rank of a PodGroup.
//
// The reference aligns a pod's resources to one NUMA zone in Filter: a pod
// that cannot be aligned does not fit (pkg/noderesourcetopology/filter.go:
// 84-150, 190-216). SURVEY.md §2.1 C15 and §2.7 generalise the zone to the
// 8-GPU xGMI mesh of one MI355X node: every RCCL hop of a gang stays on xGMI
// only when all of its ranks share a node. The unit is the gang, not the pod,
// so the check reads cluster state (where the siblings sit, which free GPUs
// are already promised to other gangs in flight) and runs once per cycle in
// PreFilter; its answer is a node set (upstream's later PreFilterResult,
// NodeRestriction in framework/types.h):
//   * a gang with members placed: the node(s) hosting it that can still take
//     every remaining rank (else those with room for one more, else a new
//     node that takes the rest);
//   * a gang not started: the nodes that can take all of its ranks, counting
//     as taken the ranks still owed to gangs anchored on a node (started on
//     exactly one node and not complete), so two gangs in flight never count
//     on the same free GPUs;
//   * no such node: Preferred lets the scheduler use every node (the gang may
//     split), Required fails the cycle and Coscheduling parks the gang until
//     GPUs are released.
// Units are whole GPUs for GPU ranks and XCDs for XCD-partition ranks (a rank
// of `amount` XCDs occupies whole partitions: xcd_footprint).
#pragma once

#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common/clock.h"
#include "framework/types.h"

namespace xsched {

class SchedulerCache;

class GangPlacement {
 public:
  enum class Mode : uint8_t { Off, Preferred, Required };
  static Mode parse_mode(const std::string& s);  // Preferred | Required | None (throws otherwise)
  static const char* mode_name(Mode m);

  GangPlacement(SchedulerCache* cache, std::shared_ptr<Clock> clock) : cache_(cache), clock_(std::move(clock)) {}
  void set_mode(Mode m) { mode_ = m; }
  Mode mode() const { return mode_; }

  // A GPU or XCD rank (the kinds gangs are placed by).
  static bool gang_demand(const GpuDemand& d) {
    return (d.kind == GpuDemand::Gpu || d.kind == GpuDemand::Xcd) && d.amount > 0;
  }
  // XCDs one rank of `amount` XCDs occupies on a node whose free partitions
  // have the sizes in `mask` (bit b: 2^b-XCD partitions); 0 when none fits.
  static int64_t xcd_footprint(int64_t amount, uint8_t mask);

  struct Plan {
    bool gang = false;      // a GPU rank of a PodGroup with minMember > 1
    bool started = false;   // members of the gang are assumed or bound already
    int64_t remaining = 0;  // ranks still to place, this one included
    bool hostable = false;  // some node can take every remaining rank now
    std::shared_ptr<NodeRestriction> restriction;  // null: no restriction
  };
  // PreFilter (scheduling thread, `s` refreshed for the cycle). Registers
  // p's gang as in flight.
  Plan plan(const Snapshot& s, const Pod& p, int min_member);
  // Can one node take `remaining` ranks of p's kind now, counting the ranks
  // owed to anchored gangs (Coscheduling's gate in Required mode)?
  bool hostable(const Snapshot& s, const Pod& p, int64_t remaining);
  // The most ranks of p's kind one node of the cluster could hold if idle
  // (memoized per node epoch): a larger gang can never be co-located.
  int64_t node_capacity(const Snapshot& s, const Pod& p);
  // Gangs registered as in flight (tests, debug).
  size_t open_gangs() const;

 private:
  struct Open {
    GpuDemand::Kind kind = GpuDemand::None;
    int64_t amount = 0;
    int min_member = 0;
  };
  // Ranks owed to other gangs anchored on one node, as (position, units of
  // `kind`); prunes gangs that completed or went idle. Caller holds mu_.
  void reservations_locked(const Snapshot& s, uint64_t self, GpuDemand::Kind kind,
                           std::vector<std::pair<int, int64_t>>& out);
  // Nodes that can take `members` ranks of demand `d` after reservations:
  // count, plus a mask (when out_mask) and up to kList positions.
  int scan(const Snapshot& s, const GpuDemand& d, int64_t members, const std::vector<std::pair<int, int64_t>>& res,
           std::vector<char>* out_mask, std::vector<int>* out_list) const;

  // A restriction object from pool_ that no cycle holds any more (caller
  // holds mu_).
  std::shared_ptr<NodeRestriction> take_restriction(size_t nodes);

  static constexpr size_t kList = 16;  // restrictions up to this size are position lists
  static constexpr size_t kPool = 64;
  std::vector<std::shared_ptr<NodeRestriction>> pool_;
  size_t pool_next_ = 0;

  SchedulerCache* cache_;
  std::shared_ptr<Clock> clock_;
  Mode mode_ = Mode::Off;
  mutable std::mutex mu_;
  std::unordered_map<uint64_t, Open> open_;
  // node_capacity memo
  uint64_t cap_epoch_ = 0;
  size_t cap_nodes_ = 0;
  std::unordered_map<uint64_t, int64_t> cap_memo_;
};

}  // namespace xsched
