// Open-loop gang arrival driver (the benchmark's admission-latency mode).
//
// The headline bench creates a whole wave at once, so its gang-admit
// latency is mostly queueing behind the burst. Here gangs arrive one at a
// time at given offsets (a Poisson process drawn by the caller at a chosen
// fraction of the measured capacity), each gang is deleted a fixed hold time
// after its last member bound (so the cluster reaches a steady occupancy),
// and every gang's timeline is recorded:
//
//   create_us          the PodGroup and its pods written to the store
//   first_enqueue_us   first member entered the scheduling queue
//   admit_us           last member allowed at Permit (Coscheduling)
//   bound_us           last member bound
//
// so both intervals SURVEY.md Appendix D names can be reported:
// first-enqueue -> last-Allow (scheduler-internal) and PG-create -> last-Bind
// (end to end). Native, on its own thread, because a Python loop cannot pace
// ~10^4 gangs/s.
#pragma once

#include <array>

#include <cstdint>
#include <memory>
#include <vector>

#include "common/json.h"

namespace xsched {

class ObjectStore;
class Scheduler;

struct OpenLoopGang {
  Json pod_group;          // PodGroup object
  std::vector<Json> pods;  // its members
};

struct OpenLoopResult {
  struct Gang {
    int size = 0;
    int64_t create_us = 0, first_enqueue_us = 0, admit_us = 0, bound_us = 0;
    int nodes = 0, hostable = -1;  // placement (GangRecord)
  };
  std::vector<Gang> gangs;  // in arrival order; bound_us == 0: not admitted in time
  int64_t wall_us = 0;      // first arrival -> last gang done
  int64_t late_us = 0;      // total lag of arrivals behind their schedule (driver overload)
  int64_t delete_late_us = 0;  // total lag of deletions behind bound + hold
  // Peaks over the run, in pods: created but not yet bound (the scheduler's
  // backlog), and bound but not yet deleted (the held occupancy).
  int64_t max_in_flight_pods = 0, max_held_pods = 0;
  // Every 5 ms of the run: pods in flight and held at the end of the slice.
  // Per 5 ms slice: pods in flight, pods held, and the scheduler's attempts,
  // unschedulable attempts and parked groups during the slice, then the pods
  // the scheduler's cache accounts on nodes (assumed + bound, deletions not
  // yet seen included), of them the assumed ones, the pods waiting at Permit
  // and the binding cycles queued for the binders, at the end of the slice.
  std::vector<std::array<int32_t, 9>> timeline;
};

// Runs to completion on the calling thread. `offsets_us[i]` is gang i's
// arrival time after the start; gangs are deleted `hold_us` after binding;
// gangs not bound `timeout_us` after the last arrival are reported unbound.
OpenLoopResult run_open_loop(ObjectStore& store, Scheduler& sched, std::vector<OpenLoopGang> gangs,
                             const std::vector<int64_t>& offsets_us, int64_t hold_us, int64_t timeout_us);

}  // namespace xsched
