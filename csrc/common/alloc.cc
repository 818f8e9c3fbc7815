#include "common/alloc.h"

#include <malloc.h>

#include <cstdlib>
#include <cstring>

namespace xsched {

const std::string& tune_allocator() {
  static const std::string applied = [] {
    const char* env = std::getenv("XSCHED_MALLOC_TUNE");
    if (env && std::strcmp(env, "0") == 0) return std::string("glibc defaults (XSCHED_MALLOC_TUNE=0)");
    constexpr int kMmapThreshold = 32 << 20;  // glibc caps M_MMAP_THRESHOLD at 32 MiB on 64-bit
    constexpr int kTrimThreshold = 1 << 30;
    constexpr int kTopPad = 64 << 20;
    bool ok = mallopt(M_MMAP_THRESHOLD, kMmapThreshold) == 1;
    ok = mallopt(M_TRIM_THRESHOLD, kTrimThreshold) == 1 && ok;
    ok = mallopt(M_TOP_PAD, kTopPad) == 1 && ok;
    return std::string(ok ? "glibc: mmap_threshold=32MiB trim_threshold=1GiB top_pad=64MiB"
                          : "glibc: mallopt refused a setting");
  }();
  return applied;
}

}  // namespace xsched
