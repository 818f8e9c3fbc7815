#include "common/log.h"

#include <sys/time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <ctime>
#include <deque>
#include <mutex>

namespace xsched::log {

std::atomic<int> g_verbosity{0};

namespace {
std::atomic<bool> g_json{true};
std::mutex g_mu;  // one line at a time; guards the capture ring
size_t g_capture_max = 0;
std::deque<std::string> g_captured;

const char* basename_of(const char* path) {
  const char* s = std::strrchr(path, '/');
  return s ? s + 1 : path;
}
}  // namespace

void set_verbosity(int v) { g_verbosity.store(v, std::memory_order_relaxed); }
void set_json(bool json) { g_json.store(json, std::memory_order_relaxed); }

void set_capture(size_t max_lines) {
  std::lock_guard<std::mutex> g(g_mu);
  g_capture_max = max_lines;
  if (!max_lines) g_captured.clear();
}

std::vector<std::string> drain_captured() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<std::string> out(g_captured.begin(), g_captured.end());
  g_captured.clear();
  return out;
}

Entry::Entry(char severity, int v, const char* file, int line, std::string_view msg)
    : severity_(severity), v_(v), file_(file), line_(line), msg_(msg) {}

Entry& Entry::kv(std::string_view key, Json value) {
  kvs_.emplace_back(std::string(key), std::move(value));
  return *this;
}

Entry::~Entry() {
  timeval tv;
  gettimeofday(&tv, nullptr);
  tm t;
  gmtime_r(&tv.tv_sec, &t);
  char ts[40];
  std::string caller = std::string(basename_of(file_)) + ":" + std::to_string(line_);
  std::string out;
  if (g_json.load(std::memory_order_relaxed)) {
    std::snprintf(ts, sizeof ts, "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ", t.tm_year + 1900, t.tm_mon + 1, t.tm_mday,
                  t.tm_hour, t.tm_min, t.tm_sec, static_cast<long>(tv.tv_usec));
    Json o = Json::object();
    o.set("ts", Json(ts));
    o.set("level", Json(severity_ == 'E' ? "ERROR" : severity_ == 'W' ? "WARNING" : "INFO"));
    o.set("v", Json(v_));
    o.set("logger", Json("xsched.native"));
    o.set("caller", Json(caller));
    o.set("msg", Json(msg_));
    for (auto& [k, v] : kvs_) o.set(k, std::move(v));
    out = o.dump();
  } else {
    // klog text: Lmmdd hh:mm:ss.uuuuuu pid file:line] "msg" key="value" ...
    std::snprintf(ts, sizeof ts, "%c%02d%02d %02d:%02d:%02d.%06ld %7d ", severity_, t.tm_mon + 1, t.tm_mday,
                  t.tm_hour, t.tm_min, t.tm_sec, static_cast<long>(tv.tv_usec), static_cast<int>(getpid()));
    out = ts + caller + "] " + Json(msg_).dump();
    for (auto& [k, v] : kvs_) out += " " + k + "=" + v.dump();
  }
  std::lock_guard<std::mutex> g(g_mu);
  if (g_capture_max) {
    g_captured.push_back(std::move(out));
    while (g_captured.size() > g_capture_max) g_captured.pop_front();
    return;
  }
  out += '\n';
  std::fwrite(out.data(), 1, out.size(), stderr);
}

}  // namespace xsched::log
