#include "scheduler/trace.h"

#include "common/json.h"

namespace xsched {

void Tracer::record(TraceEvent ev) {
  if (!enabled()) return;
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
  ring_.clear();
  head_ = 0;
  wrapped_ = false;
}

}  // namespace xsched
