// Clock and timer service.
//
// The reference leans on Go's time.AfterFunc for Permit timeouts
// (vendor/k8s.io/kubernetes/pkg/scheduler/framework/runtime/waiting_pods_map.go:100),
// go-cache janitors for TTL maps (pkg/coscheduling/core/core.go:103-104) and
// wait.Until tickers for queue flushes. Here one timer thread serves all of
// them from a deadline heap; the clock is injectable so tests can advance time
// deterministically instead of sleeping.
#pragma once

#include "common/adaptive_mutex.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <pthread.h>

namespace xsched {

// Names the calling thread (<= 15 chars) so per-thread CPU shows up by role
// in top -H, /proc/<pid>/task/*/comm and the stress driver's sampler.
inline void name_this_thread(const char* name) { pthread_setname_np(pthread_self(), name); }

class Clock {
 public:
  virtual ~Clock() = default;
  // Monotonic microseconds.
  virtual int64_t now_us() const = 0;
  virtual bool is_fake() const { return false; }
};

class RealClock : public Clock {
 public:
  int64_t now_us() const override {
    return std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
};

class FakeClock : public Clock {
 public:
  explicit FakeClock(int64_t start_us = 1'000'000'000) : t_(start_us) {}
  int64_t now_us() const override { return t_.load(); }
  bool is_fake() const override { return true; }
  void advance_us(int64_t d) { t_.fetch_add(d); }
  void set_us(int64_t t) { t_.store(t); }

 private:
  std::atomic<int64_t> t_;
};

// Single-threaded deadline scheduler. Callbacks run on the timer thread and
// must be short (they typically enqueue work elsewhere).
class TimerService {
 public:
  using Fn = std::function<void()>;
  explicit TimerService(std::shared_ptr<Clock> clock);
  ~TimerService();
  TimerService(const TimerService&) = delete;
  TimerService& operator=(const TimerService&) = delete;

  uint64_t schedule_at(int64_t deadline_us, Fn fn);
  uint64_t schedule_after(int64_t delay_us, Fn fn) { return schedule_at(clock_->now_us() + delay_us, std::move(fn)); }
  // Periodic timer; the period is measured from each firing.
  uint64_t every(int64_t period_us, Fn fn);
  bool cancel(uint64_t id);
  // Wake the thread (e.g. after a FakeClock advance) and wait until every
  // timer due at the current clock has run.
  void poke_and_drain();
  void stop();
  const Clock& clock() const { return *clock_; }

 private:
  struct Timer {
    Fn fn;
    int64_t period_us = 0;
    std::multimap<int64_t, uint64_t>::iterator pos;
  };
  void loop();

  std::shared_ptr<Clock> clock_;
  AdaptiveMutex mu_;  // schedule/cancel per waiting pod, from the scheduling and binder threads
  std::condition_variable_any cv_, drained_cv_;
  std::multimap<int64_t, uint64_t> heap_;
  std::unordered_map<uint64_t, Timer> timers_;
  uint64_t next_id_ = 1;
  bool stop_ = false;
  bool running_cb_ = false;
  uint64_t poke_gen_ = 0, drained_gen_ = 0, change_gen_ = 0;
  std::thread th_;
};

}  // namespace xsched
