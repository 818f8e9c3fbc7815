#include "scheduler/metrics.h"

#include <cstdio>
#include <cstring>

namespace xsched {

std::vector<double> exponential_buckets(double start, double factor, int count) {
  std::vector<double> b;
  double v = start;
  for (int i = 0; i < count; ++i) {
    b.push_back(v);
    v *= factor;
  }
  return b;
}

Histogram::Histogram(std::vector<double> bounds) : bounds_(std::move(bounds)) {
  buckets_.reset(new std::atomic<uint64_t>[bounds_.size() + 1]);
  for (size_t i = 0; i <= bounds_.size(); ++i) buckets_[i].store(0);
}

void Histogram::observe(double v) {
  size_t i = 0;
  while (i < bounds_.size() && v > bounds_[i]) ++i;
  buckets_[i].fetch_add(1, std::memory_order_relaxed);
  count_.fetch_add(1, std::memory_order_relaxed);
  uint64_t old_bits = sum_bits_.load(std::memory_order_relaxed);
  for (;;) {
    double old;
    std::memcpy(&old, &old_bits, sizeof old);
    double nv = old + v;
    uint64_t nb;
    std::memcpy(&nb, &nv, sizeof nb);
    if (sum_bits_.compare_exchange_weak(old_bits, nb, std::memory_order_relaxed)) break;
  }
}

double Histogram::sum() const {
  uint64_t b = sum_bits_.load();
  double d;
  std::memcpy(&d, &b, sizeof d);
  return d;
}

std::vector<uint64_t> Histogram::cumulative() const {
  std::vector<uint64_t> out(bounds_.size() + 1);
  uint64_t acc = 0;
  for (size_t i = 0; i <= bounds_.size(); ++i) {
    acc += buckets_[i].load();
    out[i] = acc;
  }
  return out;
}

namespace {
struct Def {
  const char* name;
  const char* type;
  const char* help;
  double start, factor;
  int count;
};
const Def kDefs[] = {
    {"scheduler_schedule_attempts_total", "counter", "Number of attempts to schedule pods, by the result.", 0, 0, 0},
    {"scheduler_e2e_scheduling_duration_seconds", "histogram",
     "E2e scheduling latency in seconds (scheduling algorithm + binding)", 0.001, 2, 15},
    {"scheduler_scheduling_attempt_duration_seconds", "histogram", "Scheduling attempt latency in seconds", 0.001, 2, 15},
    {"scheduler_scheduling_algorithm_duration_seconds", "histogram", "Scheduling algorithm latency in seconds", 0.001, 2, 15},
    {"scheduler_pod_scheduling_duration_seconds", "histogram",
     "E2e latency for a pod being scheduled which may include multiple scheduling attempts.", 0.01, 2, 20},
    {"scheduler_pod_scheduling_attempts", "histogram", "Number of attempts to successfully schedule a pod.", 1, 2, 5},
    {"scheduler_framework_extension_point_duration_seconds", "histogram",
     "Latency for running all plugins of a specific extension point.", 0.0001, 2, 12},
    {"scheduler_plugin_execution_duration_seconds", "histogram",
     "Duration for running a plugin at a specific extension point.", 0.00001, 1.5, 20},
    {"scheduler_permit_wait_duration_seconds", "histogram", "Duration of waiting on permit.", 0.001, 2, 15},
    {"scheduler_preemption_victims", "histogram", "Number of selected preemption victims", 1, 2, 7},
    {"scheduler_preemption_attempts_total", "counter", "Total preemption attempts in the cluster till now", 0, 0, 0},
    {"scheduler_pending_pods", "gauge", "Number of pending pods, by the queue type.", 0, 0, 0},
    {"scheduler_scheduler_goroutines", "gauge",
     "Number of running goroutines split by the work they do such as binding.", 0, 0, 0},
    {"scheduler_scheduler_cache_size", "gauge", "Number of nodes, pods, and assumed (bound) pods in the scheduler cache.",
     0, 0, 0},
    {"scheduler_queue_incoming_pods_total", "counter",
     "Number of pods added to scheduling queues by event and queue type.", 0, 0, 0},
    {"xsched_gang_admit_seconds", "histogram",
     "PodGroup gang-admit latency: first member enqueued to last member bound.", 0.0001, 2, 22},
    {"xsched_binding_duration_seconds", "histogram", "Binding cycle latency (PreBind+Bind+PostBind).", 0.00001, 2, 20},
};
}  // namespace

Metrics::Metrics() {
  for (const auto& d : kDefs) {
    Family& f = fams_[d.name];
    f.type = d.type;
    f.help = d.help;
    if (d.count > 0) f.bounds = exponential_buckets(d.start, d.factor, d.count);
  }
}

Metrics::Family& Metrics::family(const std::string& name) {
  auto it = fams_.find(name);
  if (it != fams_.end()) return it->second;
  Family& f = fams_[name];
  f.type = "histogram";
  f.bounds = exponential_buckets(0.0001, 2, 20);
  return f;
}

Histogram& Metrics::histogram(const std::string& name, const std::string& labels) {
  std::lock_guard<std::mutex> g(mu_);
  Family& f = family(name);
  auto& h = f.hists[labels];
  if (!h) h.reset(new Histogram(f.bounds));
  return *h;
}

Counter& Metrics::cell_locked(const std::string& name, const std::string& labels, const char* type) {
  auto it = fams_.find(name);
  Family& f = it != fams_.end() ? it->second : fams_[name];
  if (f.type.empty()) f.type = type;
  auto& c = f.values[labels];
  if (!c) c.reset(new Counter());
  return *c;
}

Counter& Metrics::counter_ref(const std::string& name, const std::string& labels) {
  std::lock_guard<std::mutex> g(mu_);
  return cell_locked(name, labels, "counter");
}

void Metrics::inc(const std::string& name, const std::string& labels, double by) {
  std::lock_guard<std::mutex> g(mu_);
  cell_locked(name, labels, "counter").inc(by);
}

void Metrics::set_gauge(const std::string& name, const std::string& labels, double v) {
  std::lock_guard<std::mutex> g(mu_);
  cell_locked(name, labels, "gauge").set(v);
}

double Metrics::counter(const std::string& name, const std::string& labels) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = fams_.find(name);
  if (it == fams_.end()) return 0;
  auto vit = it->second.values.find(labels);
  return vit == it->second.values.end() ? 0 : vit->second->value();
}

void Metrics::reset() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : fams_) {
    for (auto& h : kv.second.hists) retired_hists_.push_back(std::move(h.second));
    for (auto& v : kv.second.values) retired_cells_.push_back(std::move(v.second));
    kv.second.hists.clear();
    kv.second.values.clear();
  }
  epoch_.fetch_add(1, std::memory_order_release);
}

std::string Metrics::expose() const {
  std::lock_guard<std::mutex> g(mu_);
  std::string out;
  char buf[128];
  for (const auto& [name, f] : fams_) {
    if (f.hists.empty() && f.values.empty()) continue;
    out += "# HELP " + name + " " + f.help + "\n# TYPE " + name + " " + f.type + "\n";
    for (const auto& [labels, v] : f.values) {
      std::snprintf(buf, sizeof buf, "%.17g", v->value());
      out += name + (labels.empty() ? "" : "{" + labels + "}") + " " + buf + "\n";
    }
    for (const auto& [labels, h] : f.hists) {
      auto cum = h->cumulative();
      std::string sep = labels.empty() ? "" : labels + ",";
      for (size_t i = 0; i < h->bounds().size(); ++i) {
        std::snprintf(buf, sizeof buf, "%g", h->bounds()[i]);
        out += name + "_bucket{" + sep + "le=\"" + buf + "\"} " + std::to_string(cum[i]) + "\n";
      }
      out += name + "_bucket{" + sep + "le=\"+Inf\"} " + std::to_string(cum.back()) + "\n";
      std::snprintf(buf, sizeof buf, "%.17g", h->sum());
      out += name + "_sum" + (labels.empty() ? "" : "{" + labels + "}") + " " + buf + "\n";
      out += name + "_count" + (labels.empty() ? "" : "{" + labels + "}") + " " + std::to_string(h->count()) + "\n";
    }
  }
  return out;
}

}  // namespace xsched
