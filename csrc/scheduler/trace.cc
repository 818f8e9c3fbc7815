#include "scheduler/trace.h"

#include <algorithm>

#include "common/json.h"

namespace xsched {

void Tracer::set_capacity(size_t cap) {
  std::lock_guard<std::mutex> g(mu_);
  ring_.clear();
  head_ = 0;
  wrapped_ = false;
  slots_.reset(cap ? new TraceEvent[cap] : nullptr);
  nslots_ = cap;
  next_.store(0);
}

size_t Tracer::dropped() const {
  const size_t n = next_.load();
  return nslots_ && n > nslots_ ? n - nslots_ : 0;
}

void Tracer::record(TraceEvent ev) {
  if (!enabled()) return;
  if (nslots_) {
    const size_t i = next_.fetch_add(1, std::memory_order_relaxed);
    if (i < nslots_) slots_[i] = std::move(ev);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (ring_.size() < cap_) {
    ring_.push_back(std::move(ev));
    return;
  }
  ring_[head_] = std::move(ev);
  head_ = (head_ + 1) % cap_;
  wrapped_ = true;
}

std::vector<TraceEvent> Tracer::events() const {
  std::lock_guard<std::mutex> g(mu_);
  if (nslots_) {  // read after recording stopped (enable(false))
    const size_t n = std::min(next_.load(), nslots_);
    return std::vector<TraceEvent>(slots_.get(), slots_.get() + n);
  }
  if (!wrapped_) return ring_;
  std::vector<TraceEvent> out;
  out.reserve(ring_.size());
  for (size_t i = 0; i < ring_.size(); ++i) out.push_back(ring_[(head_ + i) % ring_.size()]);
  return out;
}

std::string Tracer::chrome_json() const {
  Json arr = Json::array();
  for (const auto& e : events()) {
    Json o = Json::object();
    o.set("name", Json(e.name));
    o.set("cat", Json("xsched"));
    o.set("ph", Json("X"));
    o.set("ts", Json(e.start_us));
    o.set("dur", Json(e.dur_us));
    o.set("pid", Json(1));
    o.set("tid", Json(e.tid));
    Json args = Json::object();
    args.set("pod", Json(e.pod));
    if (!e.detail.empty()) args.set("detail", Json(e.detail));
    o.set("args", std::move(args));
    arr.push_back(std::move(o));
  }
  Json doc = Json::object();
  doc.set("traceEvents", std::move(arr));
  doc.set("displayTimeUnit", Json("ms"));
  return doc.dump();
}

void Tracer::clear() {
  std::lock_guard<std::mutex> g(mu_);
  next_.store(0);
  ring_.clear();
  head_ = 0;
  wrapped_ = false;
}

}  // namespace xsched
