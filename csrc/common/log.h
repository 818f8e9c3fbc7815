// Leveled structured logging for the native core (klog's V(n).InfoS).
//
// The reference logs its placement decisions with klog at V(6)
// (pkg/flexgpu/flex_gpu.go:42-50,103-107, pkg/noderesourcetopology/filter.go)
// and its dev chart runs --v=6. Here the verbosity is one relaxed atomic set
// from the CLI's --v (cli.py -> set_verbosity), so a disabled XS_LOGV costs
// one load and a branch and builds nothing:
//
//   XS_LOGV(6, "fit indexes").kv("pod", p.key()).kv("node", n).kv("indexes", s);
//   XS_WARN("informer dropped object").kv("kind", k).kv("err", e.what());
//
// Each entry is one line on stderr, JSON by default ({"ts","level","v",
// "logger","caller","msg", key/values...}; strings escaped by the Json
// writer) or klog's text form. Tests capture lines instead (set_capture).
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "common/json.h"

namespace xsched::log {

extern std::atomic<int> g_verbosity;
inline int verbosity() { return g_verbosity.load(std::memory_order_relaxed); }
void set_verbosity(int v);
void set_json(bool json);  // false: klog text format
// Keep up to `max_lines` lines in memory instead of writing stderr (0: off).
void set_capture(size_t max_lines);
std::vector<std::string> drain_captured();

class Entry {
 public:
  Entry(char severity, int v, const char* file, int line, std::string_view msg);
  ~Entry();
  Entry(const Entry&) = delete;
  Entry& operator=(const Entry&) = delete;
  Entry& kv(std::string_view key, Json value);

 private:
  char severity_;
  int v_;
  const char* file_;
  int line_;
  std::string msg_;
  std::vector<std::pair<std::string, Json>> kvs_;
};

}  // namespace xsched::log

#define XS_V(n) (::xsched::log::verbosity() >= (n))
#define XS_LOGV(n, msg) \
  if (!XS_V(n)) {       \
  } else                \
    ::xsched::log::Entry('I', (n), __FILE__, __LINE__, (msg))
#define XS_INFO(msg) ::xsched::log::Entry('I', 0, __FILE__, __LINE__, (msg))
#define XS_WARN(msg) ::xsched::log::Entry('W', 0, __FILE__, __LINE__, (msg))
#define XS_ERROR(msg) ::xsched::log::Entry('E', 0, __FILE__, __LINE__, (msg))
