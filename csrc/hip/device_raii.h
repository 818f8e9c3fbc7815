// Scoped owners for the probes' HIP resources. Every XS_CHECK/XS_MCHECK early
// return releases what was acquired so far: the node agent runs these probes
// repeatedly in one long-lived process, so an error path must not leak HBM.
#pragma once

#include <hip/hip_runtime.h>

namespace xsprobe {

struct DevMem {
  void* p = nullptr;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Stream {
  hipStream_t s = nullptr;
  Stream() = default;
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  ~Stream() {
    if (s) (void)hipStreamDestroy(s);
  }
};

struct Event {
  hipEvent_t e = nullptr;
  Event() = default;
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  ~Event() {
    if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace xsprobe
