// Prometheus-compatible scheduler metrics with the upstream metric names.
//
// Names/labels follow vendor/k8s.io/kubernetes/pkg/scheduler/metrics/
// metrics.go:45-175 (scheduler_schedule_attempts_total,
// scheduler_e2e_scheduling_duration_seconds, scheduler_permit_wait_duration_seconds,
// scheduler_preemption_victims, ...). Added: xsched_gang_admit_seconds{size}
// — first-member-enqueue to last-member-bound for each PodGroup — the
// north-star latency metric (BASELINE.json).
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace xsched {

class Histogram {
 public:
  explicit Histogram(std::vector<double> bounds);
  void observe(double v);
  uint64_t count() const { return count_.load(); }
  double sum() const;
  std::vector<uint64_t> cumulative() const;
  const std::vector<double>& bounds() const { return bounds_; }

 private:
  std::vector<double> bounds_;
  std::unique_ptr<std::atomic<uint64_t>[]> buckets_;
  std::atomic<uint64_t> count_{0};
  std::atomic<uint64_t> sum_bits_{0};
};

std::vector<double> exponential_buckets(double start, double factor, int count);

// A counter/gauge cell; lock-free updates through a cached reference.
class Counter {
 public:
  void inc(double by = 1.0) { v_.fetch_add(by, std::memory_order_relaxed); }
  void set(double v) { v_.store(v, std::memory_order_relaxed); }
  double value() const { return v_.load(std::memory_order_relaxed); }

 private:
  std::atomic<double> v_{0.0};
};

class Metrics {
 public:
  Metrics();
  // Labelled families; labels is a canonical `k="v",k2="v2"` string.
  // References stay valid for the Metrics' lifetime: reset() retires cells
  // instead of freeing them and bumps epoch(), so hot paths cache references
  // per epoch and skip the name/label lookups under the lock.
  Histogram& histogram(const std::string& name, const std::string& labels);
  Counter& counter_ref(const std::string& name, const std::string& labels);
  uint64_t epoch() const { return epoch_.load(std::memory_order_acquire); }
  void inc(const std::string& name, const std::string& labels, double by = 1.0);
  void set_gauge(const std::string& name, const std::string& labels, double v);
  double counter(const std::string& name, const std::string& labels) const;
  std::string expose() const;  // Prometheus text format 0.0.4
  void reset();

 private:
  struct Family {
    std::string help, type;
    std::vector<double> bounds;
    std::map<std::string, std::unique_ptr<Histogram>> hists;
    std::map<std::string, std::unique_ptr<Counter>> values;
  };
  Family& family(const std::string& name);
  Counter& cell_locked(const std::string& name, const std::string& labels, const char* type);
  mutable std::mutex mu_;
  std::map<std::string, Family> fams_;
  std::atomic<uint64_t> epoch_{0};
  std::vector<std::unique_ptr<Histogram>> retired_hists_;
  std::vector<std::unique_ptr<Counter>> retired_cells_;
};

}  // namespace xsched
