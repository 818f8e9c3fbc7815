#include "common/parallel.h"

#include "common/clock.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>

namespace xsched {

Parallelizer::Parallelizer(int workers, int inline_below, const char* thread_name)
    : workers_(std::max(1, workers)), inline_below_(inline_below) {
  if (const char* e = std::getenv("XSCHED_MIN_PARALLEL_NS")) min_parallel_work_ns_ = std::max<int64_t>(0, std::atoll(e));
  for (int i = 0; i < workers_ - 1; ++i) threads_.emplace_back([this, thread_name] {
    name_this_thread(thread_name);
    worker_loop();
  });
}

Parallelizer::~Parallelizer() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    pub_gen_.fetch_add(1, std::memory_order_release);  // ends spins
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

int64_t Parallelizer::now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

namespace {
inline void cpu_relax() { __builtin_ia32_pause(); }
void ema(std::atomic<int64_t>& v, int64_t sample, bool seed) {
  int64_t cur = v.load(std::memory_order_relaxed);
  v.store(seed ? sample : cur + (sample - cur) / 8, std::memory_order_relaxed);  // alpha 1/8
}
void observe(ParallelSite* site, int64_t ns, int items) {
  if (!site || items <= 0) return;
  ema(site->ns_per_item_x16, ns * 16 / items, site->ns_per_item_x16.load(std::memory_order_relaxed) == 0);
}
void observe_done(ParallelSite* site, int done, int n) {
  if (!site || n <= 0) return;
  ema(site->done_frac_x1024, static_cast<int64_t>(done) * 1024 / n, false);
}
}  // namespace

int Parallelizer::run_job(Job& job) {
  int done = 0;
  for (;;) {
    if (job.stop && job.stop->load(std::memory_order_relaxed)) return done;
    int start = job.next.fetch_add(job.chunk, std::memory_order_relaxed);
    if (start >= job.n) return done;
    int end = std::min(job.n, start + job.chunk);
    if (job.rfn) {
      (*job.rfn)(start, end);
      done += end - start;
      continue;
    }
    for (int i = start; i < end; ++i) {
      if (job.stop && job.stop->load(std::memory_order_relaxed)) return done;
      (*job.fn)(i);
      ++done;
    }
  }
}

void Parallelizer::worker_loop() {
  uint64_t seen = 0;
  for (;;) {
    if (spinners_.fetch_add(1, std::memory_order_relaxed) < kMaxSpinners) {
      int64_t end = now_ns() + kSpinNs;
      while (pub_gen_.load(std::memory_order_acquire) == seen && now_ns() < end) cpu_relax();
    }
    spinners_.fetch_sub(1, std::memory_order_relaxed);
    Job* job = nullptr;
    bool wake_next = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      ++sleepers_;
      cv_.wait(lk, [&] { return stop_ || (job_ != nullptr && job_gen_ != seen && job_->seats > 0); });
      --sleepers_;
      if (stop_) return;
      seen = job_gen_;
      job = job_;
      --job->seats;
      job->active.fetch_add(1);
      wake_next = job->seats > 0 && sleepers_ > 0;
    }
    if (wake_next) cv_.notify_one();
    run_job(*job);
    if (job->active.fetch_sub(1) == 1) {
      std::lock_guard<std::mutex> g(mu_);
      if (caller_waiting_) done_cv_.notify_one();
    }
  }
}

bool Parallelizer::plan_inline(int n, ParallelSite* site) {
  // Helpers only pay off when each gets >= inline_below_/2 items: a fork/join
  // round costs a few microseconds of wake-ups, more than filtering dozens of
  // nodes with the allocation-free plugins.
  int helpers = std::min<int>(static_cast<int>(threads_.size()), n / std::max(1, inline_below_ / 2) - 1);
  bool cheap = false;
  if (site) {
    int64_t est = site->ns_per_item_x16.load(std::memory_order_relaxed) * n / 16 *
                  site->done_frac_x1024.load(std::memory_order_relaxed) / 1024;
    bool probe = site->calls.fetch_add(1, std::memory_order_relaxed) % ParallelSite::kProbeEvery == 0;
    cheap = probe || est < min_parallel_work_ns_;
  }
  return n < inline_below_ || helpers <= 0 || cheap;
}

void Parallelizer::record_inline(ParallelSite* site, int64_t elapsed_ns, int done, int n) {
  observe(site, elapsed_ns, done);
  observe_done(site, done, n);
}

void Parallelizer::until(int n, const std::function<void(int)>& fn, const std::atomic<bool>* stop,
                         ParallelSite* site) {
  if (n <= 0) return;
  if (plan_inline(n, site)) {
    int64_t t0 = site ? now_ns() : 0;
    int done = 0;
    for (int i = 0; i < n; ++i) {
      if (stop && stop->load(std::memory_order_relaxed)) break;
      fn(i);
      ++done;
    }
    if (site) record_inline(site, now_ns() - t0, done, n);
    return;
  }
  until_forked(n, fn, stop, site);
}

void Parallelizer::until_forked(int n, const std::function<void(int)>& fn, const std::atomic<bool>* stop,
                                ParallelSite* site) {
  Job job;
  job.fn = &fn;
  job.stop = stop;
  job.n = n;
  fork_join(job, site);
}

void Parallelizer::until_forked_ranges(int n, const std::function<void(int, int)>& fn, const std::atomic<bool>* stop,
                                       ParallelSite* site) {
  Job job;
  job.rfn = &fn;
  job.stop = stop;
  job.n = n;
  fork_join(job, site);
}

void Parallelizer::fork_join(Job& job, ParallelSite* site) {
  const int n = job.n;
  if (n <= 0) return;
  int helpers = std::max(1, std::min<int>(static_cast<int>(threads_.size()), n / std::max(1, inline_below_ / 2) - 1));
  std::lock_guard<std::mutex> call(call_mu_);
  job.seats = helpers;
  // chunkSizeFor: sqrt(n), capped so every participant gets work.
  job.chunk = std::max(1, std::min(static_cast<int>(std::sqrt(static_cast<double>(n))), n / (helpers + 1)));
  job.active.store(1);  // the caller
  int wake = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &job;
    ++job_gen_;
    pub_gen_.store(job_gen_, std::memory_order_release);
    int spinning = static_cast<int>(threads_.size()) - sleepers_;
    if (helpers > spinning) wake = std::min({2, helpers - spinning, sleepers_});
  }
  for (int i = 0; i < wake; ++i) cv_.notify_one();
  // Per-item cost is learned from inline runs only (the periodic probes):
  // the caller's items in a parallel run are inflated by contention.
  run_job(job);
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = nullptr;  // no new worker can join after this point
  }
  if (job.active.fetch_sub(1, std::memory_order_acq_rel) != 1) {
    int64_t end = now_ns() + kSpinNs;
    while (job.active.load(std::memory_order_acquire) != 0 && now_ns() < end) cpu_relax();
    if (job.active.load(std::memory_order_acquire) != 0) {
      std::unique_lock<std::mutex> lk(mu_);
      caller_waiting_ = true;
      done_cv_.wait(lk, [&] { return job.active.load() == 0; });
      caller_waiting_ = false;
    }
  }
  if (site) observe_done(site, std::min(job.n, job.next.load(std::memory_order_relaxed)), job.n);
}

}  // namespace xsched
