// In-process sampling profiler for the native stress driver (no perf on the
// hosts). Every thread is sampled at a fixed wall-clock rate; the SIGPROF
// handler records the thread id and a glibc backtrace into a preallocated
// buffer. `dump` writes one sample per line (tid name pc...) plus
// the load address of the executable, for tools/sample_report.py to
// symbolize with `nm`.
//
// backtrace() is primed once before the timer starts so libgcc is already
// loaded when the handler first runs; the driver does no dlopen or throw in
// the measured region, which keeps the unwinder's locks uncontended.
#pragma once

#include <dirent.h>
#include <execinfo.h>
#include <link.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <map>
#include <string>
#include <thread>
#include <vector>

namespace xsched::sampler {

constexpr int kDepth = 32;
struct Sample {
  int32_t tid;
  int32_t depth;
  int64_t t_ns;  // CLOCK_MONOTONIC at the signal (stall windows: sample_report --timeline)
  void* pcs[kDepth];
};

inline std::vector<Sample>& buffer() {
  static std::vector<Sample> b;
  return b;
}
inline std::atomic<size_t>& next() {
  static std::atomic<size_t> n{0};
  return n;
}

inline void on_sigprof(int, siginfo_t*, void*) {
  int saved = errno;
  auto& b = buffer();
  size_t i = next().fetch_add(1, std::memory_order_relaxed);
  if (i < b.size()) {
    Sample& s = b[i];
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);  // async-signal-safe
    s.t_ns = static_cast<int64_t>(ts.tv_sec) * 1000000000 + ts.tv_nsec;
    s.tid = static_cast<int32_t>(syscall(SYS_gettid));
    s.depth = backtrace(s.pcs, kDepth);
  }
  errno = saved;
}

// Wall-clock sampling: a sampler thread signals every other thread of the
// process `hz` times a second with tgkill (kernel CPU timers are tick-bound,
// ~40-250 Hz, too coarse for microsecond cycles). Blocked threads are
// sampled too; sample_report.py classifies their waits as idle.
inline std::atomic<bool>& running() {
  static std::atomic<bool> r{false};
  return r;
}
// While paused (e.g. a driver's untimed setup phase) no samples are taken.
inline std::atomic<bool>& paused() {
  static std::atomic<bool> p{false};
  return p;
}
inline void pause(bool on) { paused().store(on, std::memory_order_relaxed); }
inline std::thread& sampler_thread() {
  static std::thread t;
  return t;
}

inline std::vector<int> list_tids(int self) {
  std::vector<int> tids;
  if (DIR* d = opendir("/proc/self/task")) {
    while (struct dirent* e = readdir(d)) {
      int t = std::atoi(e->d_name);
      if (t > 0 && t != self) tids.push_back(t);
    }
    closedir(d);
  }
  return tids;
}

inline void start(int hz, size_t max_samples = 1 << 21) {
  if (running().load()) return;
  buffer().resize(max_samples);
  next().store(0);
  void* warm[4];
  backtrace(warm, 4);  // load libgcc's unwinder outside the handler
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  running() = true;
  sampler_thread() = std::thread([hz] {
    const int self = static_cast<int>(syscall(SYS_gettid));
    const int pid = getpid();
    const auto period = std::chrono::nanoseconds(1000000000LL / std::max(1, hz));
    std::vector<int> tids = list_tids(self);
    auto next_list = std::chrono::steady_clock::now() + std::chrono::milliseconds(50);
    auto tick = std::chrono::steady_clock::now();
    while (running().load(std::memory_order_relaxed) && next().load(std::memory_order_relaxed) < buffer().size()) {
      if (!paused().load(std::memory_order_relaxed))
        for (int t : tids) syscall(SYS_tgkill, pid, t, SIGPROF);
      tick += period;
      std::this_thread::sleep_until(tick);
      if (std::chrono::steady_clock::now() > next_list) {
        tids = list_tids(self);
        next_list = std::chrono::steady_clock::now() + std::chrono::milliseconds(50);
      }
    }
  });
}

inline void stop() {
  if (!running().exchange(false)) return;
  if (sampler_thread().joinable()) sampler_thread().join();
}

inline uintptr_t exe_base() {
  uintptr_t base = 0;
  dl_iterate_phdr(
      [](struct dl_phdr_info* info, size_t, void* data) {
        if (info->dlpi_name == nullptr || info->dlpi_name[0] == '\0') {  // the executable itself
          *static_cast<uintptr_t*>(data) = info->dlpi_addr;
          return 1;
        }
        return 0;
      },
      &base);
  return base;
}

inline void dump(const std::string& path) {
  stop();
  size_t n = std::min(next().load(), buffer().size());
  std::map<int32_t, std::string> names;
  std::ofstream f(path);
  f << "exe_base " << std::hex << exe_base() << std::dec << "\n";
  {
    std::ifstream maps("/proc/self/maps");
    std::string line;
    while (std::getline(maps, line))
      if (line.find(" r-xp ") != std::string::npos) f << "map " << line << "\n";
  }
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = buffer()[i];
    auto it = names.find(s.tid);
    if (it == names.end()) {
      std::ifstream c("/proc/self/task/" + std::to_string(s.tid) + "/comm");
      std::string nm;
      std::getline(c, nm);
      if (nm.empty()) nm = "exited";
      for (auto& ch : nm)
        if (ch == ' ') ch = '_';
      it = names.emplace(s.tid, nm).first;
    }
    f << s.tid << ' ' << it->second << " @" << s.t_ns;
    for (int d = 0; d < s.depth; ++d) f << ' ' << std::hex << reinterpret_cast<uintptr_t>(s.pcs[d]) << std::dec;
    f << "\n";
  }
}

}  // namespace xsched::sampler
