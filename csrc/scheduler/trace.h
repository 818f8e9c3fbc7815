// Per-cycle trace ring buffer (Chrome trace-event JSON export).
//
// The reference has no product tracing beyond verbosity-gated klog and
// upstream's sampled plugin metrics. Each scheduling/binding
// phase of a pod is recorded as a complete ("X") event with monotonic
// microsecond timestamps so a whole benchmark run can be opened in
// chrome://tracing / Perfetto.
#pragma once

#include <atomic>
#include <cstdint>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

namespace xsched {

struct TraceEvent {
  std::string name;   // phase: queue_wait, schedule, reserve, permit_wait, bind ...
  std::string pod;    // ns/name
  std::string detail; // node / status
  int64_t start_us = 0;
  int64_t dur_us = 0;
  int tid = 0;        // 0 = scheduling thread, 1 = binding workers, 2 = informer
};

class Tracer {
 public:
  explicit Tracer(size_t capacity = 1 << 16) : cap_(capacity) {}
  void enable(bool on) { enabled_.store(on); }
  bool enabled() const { return enabled_.load(std::memory_order_relaxed); }
  void record(TraceEvent ev);
  std::vector<TraceEvent> events() const;
  std::string chrome_json() const;
  void clear();
  // Linear recording of up to `cap` events (0: back to the default ring):
  // the slots are allocated up front and claimed with one atomic increment,
  // no lock, so a diagnosis run at full load is not serialized on the
  // tracer; events past the end are dropped (dropped()).
  void set_capacity(size_t cap);
  size_t dropped() const;

 private:
  size_t cap_;
  std::atomic<bool> enabled_{false};
  mutable std::mutex mu_;
  std::vector<TraceEvent> ring_;
  size_t head_ = 0;
  bool wrapped_ = false;
  // Linear mode (set_capacity): fixed slots, claimed by next_.
  std::unique_ptr<TraceEvent[]> slots_;
  size_t nslots_ = 0;
  std::atomic<size_t> next_{0};
};

}  // namespace xsched
