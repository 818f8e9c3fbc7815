#include "common/clock.h"

namespace xsched {

TimerService::TimerService(std::shared_ptr<Clock> clock) : clock_(std::move(clock)) {
  th_ = std::thread([this] {
    name_this_thread("xs-timer");
    loop();
  });
}

TimerService::~TimerService() { stop(); }

void TimerService::stop() {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  drained_cv_.notify_all();
  if (th_.joinable() && std::this_thread::get_id() != th_.get_id()) th_.join();
}

uint64_t TimerService::schedule_at(int64_t deadline_us, Fn fn) {
  uint64_t id;
  bool earliest;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    id = next_id_++;
    Timer t;
    t.fn = std::move(fn);
    t.pos = heap_.emplace(deadline_us, id);
    // The loop sleeps until the earliest deadline; a later one needs no
    // wake-up (Permit timeouts arrive in deadline order, so this skips a
    // futex wake per waiting gang member).
    earliest = t.pos == heap_.begin();
    timers_.emplace(id, std::move(t));
    if (earliest) ++change_gen_;
  }
  if (earliest) cv_.notify_one();
  return id;
}

uint64_t TimerService::every(int64_t period_us, Fn fn) {
  uint64_t id;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    id = next_id_++;
    Timer t;
    t.fn = std::move(fn);
    t.period_us = period_us;
    t.pos = heap_.emplace(clock_->now_us() + period_us, id);
    timers_.emplace(id, std::move(t));
    ++change_gen_;
  }
  cv_.notify_one();
  return id;
}

bool TimerService::cancel(uint64_t id) {
  std::lock_guard<AdaptiveMutex> g(mu_);
  auto it = timers_.find(id);
  if (it == timers_.end()) return false;
  if (it->second.pos != heap_.end()) heap_.erase(it->second.pos);
  timers_.erase(it);
  return true;
}

void TimerService::poke_and_drain() {
  std::unique_lock<AdaptiveMutex> lk(mu_);
  uint64_t gen = ++poke_gen_;
  ++change_gen_;
  cv_.notify_all();
  drained_cv_.wait(lk, [&] { return drained_gen_ >= gen || stop_; });
}

void TimerService::loop() {
  std::unique_lock<AdaptiveMutex> lk(mu_);
  while (!stop_) {
    int64_t now = clock_->now_us();
    if (!heap_.empty() && heap_.begin()->first <= now) {
      auto hit = heap_.begin();
      uint64_t id = hit->second;
      heap_.erase(hit);
      auto tit = timers_.find(id);
      if (tit == timers_.end()) continue;
      Fn fn = tit->second.fn;
      if (tit->second.period_us > 0) {
        tit->second.pos = heap_.emplace(now + tit->second.period_us, id);
      } else {
        timers_.erase(tit);
      }
      running_cb_ = true;
      lk.unlock();
      fn();
      lk.lock();
      running_cb_ = false;
      continue;
    }
    // Nothing due: report drained for pokes issued so far, then sleep.
    if (drained_gen_ < poke_gen_) {
      drained_gen_ = poke_gen_;
      drained_cv_.notify_all();
    }
    uint64_t seen_change = change_gen_;
    int64_t wait_us = 50'000;
    if (!heap_.empty()) wait_us = std::min<int64_t>(wait_us, heap_.begin()->first - now);
    if (clock_->is_fake()) wait_us = std::min<int64_t>(wait_us, 5'000);
    if (wait_us < 0) wait_us = 0;
    cv_.wait_for(lk, std::chrono::microseconds(wait_us), [&] { return stop_ || change_gen_ != seen_change; });
  }
  drained_gen_ = poke_gen_;
  drained_cv_.notify_all();
}

}  // namespace xsched
