// Fork-join parallelizer for node-parallel Filter/Score/preemption dry runs.
//
// Equivalent role to the reference's framework/parallelize.Parallelizer
// (vendor/.../framework/parallelize/parallelism.go:27, 16 workers,
// workqueue.ParallelizeUntil with chunking). Workers are persistent; the
// calling thread participates; work is claimed in chunks from an atomic
// cursor so small node counts stay on the caller (no wakeups at all below
// `inline_below` items).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace xsched {

// Cost model of one call site (Filter, Score): an exponential moving average
// of the per-item time measured on the calling thread. Above `inline_below`
// items the site still runs inline while the estimated serial time is under
// Parallelizer::min_parallel_work_ns(): a fork/join round (waking helpers and
// joining them) costs ~15-25 us on the MI355X hosts, more than filtering a
// thousand nodes whose verdicts come from the equivalence cache
// (profiles/r1h_inline_ab.txt).
struct ParallelSite {
  std::atomic<int64_t> ns_per_item_x16{0};  // fixed point, 1/16 ns
  // Fraction of the n items a call actually runs before `stop` (Filter stops
  // at numFeasibleNodesToFind), fixed point 1/1024.
  std::atomic<int64_t> done_frac_x1024{1024};
  // Every kProbeEvery-th call runs inline to re-measure the serial cost, so
  // an estimate inflated by contention in parallel runs cannot lock it in.
  std::atomic<uint32_t> calls{0};
  static constexpr uint32_t kProbeEvery = 32;
};

class Parallelizer {
 public:
  explicit Parallelizer(int workers = 16, int inline_below = 128, const char* thread_name = "xs-filter");
  ~Parallelizer();
  Parallelizer(const Parallelizer&) = delete;
  Parallelizer& operator=(const Parallelizer&) = delete;

  // Runs fn(i) for i in [0, n). `stop` (optional) is polled between items to
  // allow early exit (e.g. enough feasible nodes found).
  void until(int n, const std::function<void(int)>& fn, const std::atomic<bool>* stop = nullptr,
             ParallelSite* site = nullptr);
  // The inline-vs-fork decision `until` makes for (n, site), exposed so a hot
  // call site can run its own serial loop (plain counters instead of the
  // atomics a parallel run needs) and report it with `record_inline`.
  // Counts as a call of the site (advances its probe cadence).
  bool plan_inline(int n, ParallelSite* site);
  // The fork/join half of `until`, for a caller that already got
  // plan_inline() == false (records the site's done fraction, no re-planning).
  void until_forked(int n, const std::function<void(int)>& fn, const std::atomic<bool>* stop, ParallelSite* site);
  // until_forked over claimed chunks: fn(begin, end) runs [begin, end) on one
  // thread, so the caller keeps per-chunk counters in locals and publishes
  // them once per chunk instead of touching a shared atomic per item. fn
  // polls `stop` itself between items.
  void until_forked_ranges(int n, const std::function<void(int, int)>& fn, const std::atomic<bool>* stop,
                           ParallelSite* site);
  static void record_inline(ParallelSite* site, int64_t elapsed_ns, int done, int n);
  static int64_t now_ns();
  int workers() const { return workers_; }
  // Serial-time estimate above which a site forks (XSCHED_MIN_PARALLEL_NS
  // overrides the default, for A/B runs).
  static constexpr int64_t kMinParallelWorkNs = 60'000;
  int64_t min_parallel_work_ns() const { return min_parallel_work_ns_; }

 private:
  struct Job {
    const std::function<void(int)>* fn = nullptr;
    const std::function<void(int, int)>* rfn = nullptr;  // chunk form (fn == nullptr)
    const std::atomic<bool>* stop = nullptr;
    int n = 0;
    int chunk = 1;
    int seats = 0;  // helpers allowed to join (guarded by mu_)
    std::atomic<int> next{0};
    std::atomic<int> active{0};
  };
  void worker_loop();
  void fork_join(Job& job, ParallelSite* site);
  int run_job(Job& job);  // items processed by this thread

  int workers_;
  int inline_below_;
  int64_t min_parallel_work_ns_ = kMinParallelWorkNs;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Job* job_ = nullptr;
  uint64_t job_gen_ = 0;
  bool stop_ = false;
  std::mutex call_mu_;  // one job at a time
  // The fork/join phases of one scheduling cycle (PreFilter, Filter, Score)
  // come back to back, so a few workers spin briefly for the next job and the
  // caller spins briefly for the join: both skip a futex round trip. Sleepers
  // are woken in a chain (each helper that takes a seat wakes the next), so
  // the caller pays at most two wake-ups per fork.
  static constexpr int64_t kSpinNs = 30'000;
  static constexpr int kMaxSpinners = 4;
  std::atomic<uint64_t> pub_gen_{0};  // job_gen_, readable without mu_
  std::atomic<int> spinners_{0};
  int sleepers_ = 0;             // guarded by mu_
  bool caller_waiting_ = false;  // guarded by mu_
};

}  // namespace xsched
