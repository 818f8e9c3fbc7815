// MI355X (gfx950) device probes used by the node agent and the benchmarks.
//
// There is no GPU code in the reference: the scheduler only
// counts extended resources. An MI355X-native scheduler must validate what it
// promises, so the node agent runs these probes on the box:
//
//  * xs_hbm_bandwidth   streaming read / write / copy / triad over N bytes with
//                       16-byte lanes (global_load/store_dwordx4). Variants:
//                       unroll 1/4/8 (independent 16 B accesses in flight per
//                       lane), non-temporal vs default cache policy, 4/8/16
//                       persistent workgroups of 256 threads per CU or a
//                       one-shot grid (one workgroup per 4 KiB, no loop);
//                       probe_bench sweeps them and the node agent keeps the
//                       fastest (profiles/r5*_stream_sweep.md). HBM3E peak
//                       is 8 TB/s. Each launch is timed by its own event pair
//                       and the median is reported (the back-to-back batch
//                       rate, launch gaps included, is kept as a second
//                       figure); working sets default to 1 GiB, 4x the 256 MB
//                       Infinity Cache, so the rate is HBM's and not the
//                       cache's (profiles/r4*_pmc_probe_summary.md checks the
//                       median against rocprofv3's dispatch times and bytes).
//  * xs_hbm_bandwidth_xcd  the same traffic executed only by workgroups that
//                       land on the XCDs in `xcd_mask` (work handed out by an
//                       atomic chunk counter, so every launched workgroup
//                       exits): the HBM bandwidth one CPX partition (one XCD,
//                       32 CUs) or a QPX/DPX partition can pull, measured on
//                       an SPX device.
//  * xs_xcd_census      every workgroup records s_getreg(HW_REG_XCC_ID):
//                       counts XCDs visible to this device — verifies the
//                       compute-partition mode the node advertises (SPX -> 8
//                       XCDs, CPX -> 1).
//  * xs_health_check    deterministic integer checksum over a pattern buffer
//                       (catches a dead/ECC-faulting device before the node is
//                       advertised schedulable).
//
// Exposed as a C ABI (loaded with ctypes from flex_gpu_scheduler_amd/ops).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <vector>

#include "hip/device_raii.h"

#define XS_CHECK(x)                                                            \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::snprintf(g_err, sizeof g_err, "%s: %s", #x, hipGetErrorString(e_)); \
      return -static_cast<int>(e_) - 1;                                        \
    }                                                                          \
  } while (0)

namespace {

char g_err[512];

using xsprobe::DevMem;
using xsprobe::Event;
using xsprobe::Stream;

constexpr int kBlock = 256;  // 4 waves of 64 lanes

typedef uint32_t vec4 __attribute__((ext_vector_type(4)));  // 16 B/lane
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T v, T* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Grid-stride walk in rows of U*grid lanes: one wave-instruction touches
// 1 KiB contiguous, U independent 16-B accesses per lane in flight.
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_read(const vec4* __restrict__ src, size_t n, uint32_t* __restrict__ sink) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    vec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n; i += stride) {
    vec4 v = ld<NT>(&src[i]);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // defeats DCE without a store per lane
}

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_write(vec4* __restrict__ dst, size_t n, uint32_t seed) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  vec4 v = {seed, seed ^ 0x55555555u, seed + 1, ~seed};
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(v, &dst[i + u * stride]);
  }
  for (; i < n; i += stride) st<NT>(v, &dst[i]);
}

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_copy(const vec4* __restrict__ src, vec4* __restrict__ dst, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    vec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(v[u], &dst[i + u * stride]);
  }
  for (; i < n; i += stride) st<NT>(ld<NT>(&src[i]), &dst[i]);
}

// STREAM triad a = b + s*c on float4 lanes.
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_triad(f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                  const f32x4* __restrict__ c, float s, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = ld<NT>(&b[i + u * stride]);
      y[u] = ld<NT>(&c[i + u * stride]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(x[u] + s * y[u], &a[i + u * stride]);
  }
  for (; i < n; i += stride) st<NT>(ld<NT>(&b[i]) + s * ld<NT>(&c[i]), &a[i]);
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

__device__ __forceinline__ uint32_t hw_cu_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}

// XCD-pinned streaming: workgroups off the selected XCDs exit at once. The
// selected XCDs split the buffer into equal contiguous slices (by their rank
// in xcd_mask) and the workgroups of each XCD pull 256 KiB chunks of their
// slice from that XCD's own counter, so the launch always drains and no
// atomic is shared across XCDs (one counter per 128-B line: a single
// device-wide counter serialized the 8-XCD case at ~2 TB/s, round-3 pmc
// run). mode 0 read, 1 write, 2 copy.
constexpr int kCounterStride = 32;  // unsigned per XCD counter (128 B)
constexpr int kMaxXcds = 8;

__global__ __launch_bounds__(kBlock) void k_pinned(const vec4* __restrict__ src, vec4* __restrict__ dst, size_t n,
                                                   uint32_t xcd_mask, unsigned* __restrict__ counters, int mode,
                                                   uint32_t* __restrict__ sink) {
  const uint32_t x = xcc_id();
  if (x >= kMaxXcds || !((xcd_mask >> x) & 1u)) return;
  constexpr size_t kChunk = 16384;  // vec4s = 256 KiB
  const uint32_t sel = xcd_mask & 0xffu;
  const size_t nsel = static_cast<size_t>(__popc(sel));
  const size_t rank = static_cast<size_t>(__popc(sel & ((1u << x) - 1u)));
  const size_t nchunks = (n + kChunk - 1) / kChunk;
  const size_t c0 = nchunks * rank / nsel, c1 = nchunks * (rank + 1) / nsel;
  unsigned* ctr = counters + x * kCounterStride;
  __shared__ unsigned chunk;
  uint32_t acc = 0;
  const vec4 fill = {1u, 2u, 3u, 4u};
  for (;;) {
    if (threadIdx.x == 0) chunk = atomicAdd(ctr, 1u);
    __syncthreads();
    const size_t c = c0 + chunk;
    __syncthreads();
    if (c >= c1) break;
    size_t base = c * kChunk;
    size_t end = base + kChunk < n ? base + kChunk : n;
    size_t i = base + threadIdx.x;
    for (; i + 3 * kBlock < end; i += 4 * kBlock) {
      if (mode == 1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(fill, &dst[i + u * kBlock]);
      } else {
        vec4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * kBlock]);
        if (mode == 2) {
#pragma unroll
          for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], &dst[i + u * kBlock]);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
      }
    }
    for (; i < end; i += kBlock) {
      if (mode == 1) {
        __builtin_nontemporal_store(fill, &dst[i]);
      } else {
        vec4 v = __builtin_nontemporal_load(&src[i]);
        if (mode == 2) __builtin_nontemporal_store(v, &dst[i]);
        else acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ __launch_bounds__(64) void k_census(uint32_t* __restrict__ xcd_of_block, uint32_t* __restrict__ hwid_of_block) {
  if (threadIdx.x == 0) {
    xcd_of_block[blockIdx.x] = xcc_id();
    hwid_of_block[blockIdx.x] = hw_cu_id();
  }
}

__global__ __launch_bounds__(kBlock) void k_pattern(uint32_t* __restrict__ buf, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
    buf[i] = static_cast<uint32_t>(i * 2654435761u) ^ 0xa5a5a5a5u;
}

// Block-level sum of the pattern (wave64 shuffles, then LDS across 4 waves).
__global__ __launch_bounds__(kBlock) void k_checksum(const uint32_t* __restrict__ buf, size_t n,
                                                     unsigned long long* __restrict__ out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  unsigned long long acc = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) acc += buf[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  __shared__ unsigned long long part[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += part[w];
    atomicAdd(out, s);
  }
}

// Counter calibration (xs_segment_access): every wave touches segments of
// `seg_lanes` x 16 B, each at the start of its own `stride_vec`-vec4 slot, so
// a dispatch moves a known number of bytes in a known number of 128-B lines
// (touches x ceil(seg/128)); rocprofv3's L2 memory-side request counters are
// read against that count (scripts/pmc_calibrate.sh). Lanes >= seg_lanes
// idle; mode 0 reads, 1 writes.
template <int MODE, bool NT>
__global__ __launch_bounds__(kBlock) void k_segments(vec4* __restrict__ buf, size_t touches, size_t stride_vec,
                                                     int seg_lanes, uint32_t* __restrict__ sink) {
  const size_t wave = (static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const size_t nwaves = (static_cast<size_t>(gridDim.x) * kBlock) >> 6;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  const vec4 fill = {5u, 6u, 7u, 8u};
  if (lane < seg_lanes) {
    for (size_t t = wave; t < touches; t += nwaves) {
      vec4* p = buf + t * stride_vec + lane;
      if constexpr (MODE == 0) {
        vec4 v = ld<NT>(p);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else {
        st<NT>(fill, p);
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// Per-launch timing: `launch(i)` enqueues launch i; every launch sits
// between its own event pair on `s`. out: [median ms, min ms, batch ms per
// launch (first start to last end / iters)]. Events are created once.
template <typename F>
int time_launches(hipStream_t s, int iters, F&& launch, double out[3]) {
  std::vector<Event> ev(2 * static_cast<size_t>(iters));
  for (auto& e : ev) XS_CHECK(hipEventCreate(&e.e));
  for (int i = 0; i < iters; ++i) {
    XS_CHECK(hipEventRecord(ev[2 * i].e, s));
    launch(i);
    XS_CHECK(hipEventRecord(ev[2 * i + 1].e, s));
  }
  XS_CHECK(hipEventSynchronize(ev.back().e));
  XS_CHECK(hipGetLastError());
  std::vector<double> per(iters);
  for (int i = 0; i < iters; ++i) {
    float ms = 0;
    XS_CHECK(hipEventElapsedTime(&ms, ev[2 * i].e, ev[2 * i + 1].e));
    per[i] = ms;
  }
  float total = 0;
  XS_CHECK(hipEventElapsedTime(&total, ev.front().e, ev.back().e));
  std::vector<double> sorted = per;
  std::sort(sorted.begin(), sorted.end());
  out[0] = sorted[sorted.size() / 2];
  out[1] = sorted.front();
  out[2] = static_cast<double>(total) / iters;
  return 0;
}

int cu_count(int dev) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 256;
  return p.multiProcessorCount;
}

// variant = unroll(1|4|8) | (nt ? 0x100 : 0) | (one_shot ? 0x200 : 0) |
// (blocks_per_cu << 16); 0 = default.
struct Variant {
  int unroll = 4;
  bool nt = true;
  int bpc = 8;
  bool one_shot = false;  // grid = one workgroup per 256 x 16 B x unroll (bpc unused)
};
Variant decode(int v) {
  Variant o;
  if (v == 0) return o;
  int u = v & 0xff;
  o.unroll = (u == 1 || u == 4 || u == 8) ? u : 4;
  o.nt = (v & 0x100) != 0;
  o.one_shot = (v & 0x200) != 0;
  int b = (v >> 16) & 0xff;
  o.bpc = (b == 4 || b == 8 || b == 16) ? b : 8;
  return o;
}

// Workgroups of a launch over n vec4s: the persistent grid (CUs x bpc), or
// for a one-shot variant enough workgroups that each lane does `unroll`
// accesses and exits (capped at 2^22 workgroups, where the kernels' grid
// stride takes over: past 16 GiB per array).
int grid_for(const Variant& v, size_t n, int cus) {
  if (!v.one_shot) return cus * v.bpc;
  const size_t per = static_cast<size_t>(kBlock) * v.unroll;
  return static_cast<int>(std::min<size_t>((n + per - 1) / per, size_t{1} << 22));
}

constexpr uint32_t kWriteSeed = 7;
constexpr float kTriadScale = 3.0f;

// mode 0 read(a), 1 write(a <- pattern(seed)), 2 copy(b <- a), 3 triad(a <- b + scale*c).
template <int U, bool NT>
void launch_t(int mode, int grid, hipStream_t s, void* a, void* b, void* c, size_t n, uint32_t* sink, uint32_t seed,
              float scale) {
  switch (mode) {
    case 0: k_read<U, NT><<<grid, kBlock, 0, s>>>(static_cast<const vec4*>(a), n, sink); break;
    case 1: k_write<U, NT><<<grid, kBlock, 0, s>>>(static_cast<vec4*>(a), n, seed); break;
    case 2: k_copy<U, NT><<<grid, kBlock, 0, s>>>(static_cast<const vec4*>(a), static_cast<vec4*>(b), n); break;
    default:
      k_triad<U, NT><<<grid, kBlock, 0, s>>>(static_cast<f32x4*>(a), static_cast<const f32x4*>(b),
                                            static_cast<const f32x4*>(c), scale, n);
  }
}

void launch(const Variant& v, int mode, int grid, hipStream_t s, void* a, void* b, void* c, size_t n, uint32_t* sink,
            uint32_t seed = kWriteSeed, float scale = kTriadScale) {
  if (v.nt) {
    if (v.unroll == 1) launch_t<1, true>(mode, grid, s, a, b, c, n, sink, seed, scale);
    else if (v.unroll == 8) launch_t<8, true>(mode, grid, s, a, b, c, n, sink, seed, scale);
    else launch_t<4, true>(mode, grid, s, a, b, c, n, sink, seed, scale);
  } else {
    if (v.unroll == 1) launch_t<1, false>(mode, grid, s, a, b, c, n, sink, seed, scale);
    else if (v.unroll == 8) launch_t<8, false>(mode, grid, s, a, b, c, n, sink, seed, scale);
    else launch_t<4, false>(mode, grid, s, a, b, c, n, sink, seed, scale);
  }
}

Variant default_variant(int mode) {
  // Measured optimum per mode on MI355X at the 2 GiB working set
  // (profiles/r5_stream_sweep.md, 648 layouts x unroll x policy x grid):
  // read: a persistent grid of 8 workgroups per CU, one non-temporal 16-B
  // load per lane per iteration (~7.0 TB/s, 88%). Write and copy: a one-shot
  // grid, one workgroup per 4 KiB and no loop (write 6.83 TB/s plain, copy
  // 6.48 TB/s non-temporal, vs 5.7 / 5.95 for the best persistent grid):
  // freshly dispatched workgroups keep more stores in flight than a
  // persistent loop whose waves stall on their own store queue.
  Variant v;
  v.unroll = 1;
  v.nt = mode != 1;
  v.bpc = 8;
  v.one_shot = mode != 0;
  return v;
}

}  // namespace

extern "C" {

const char* xs_last_error() { return g_err; }

int xs_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// JSON description of device `dev` into out (len bytes). Returns bytes written or <0.
int xs_device_props(int dev, char* out, int len) {
  hipDeviceProp_t p;
  XS_CHECK(hipGetDeviceProperties(&p, dev));
  size_t free_b = 0, total_b = 0;
  XS_CHECK(hipSetDevice(dev));
  XS_CHECK(hipMemGetInfo(&free_b, &total_b));
  int n = std::snprintf(out, len,
                        "{\"name\":\"%s\",\"gcnArchName\":\"%s\",\"computeUnits\":%d,\"totalGlobalMem\":%zu,"
                        "\"freeMem\":%zu,\"clockRateKHz\":%d,\"memoryClockRateKHz\":%d,\"memoryBusWidth\":%d,"
                        "\"l2CacheSize\":%d,\"pciBusID\":%d,\"pciDeviceID\":%d,\"pciDomainID\":%d,"
                        "\"maxSharedMemoryPerMultiProcessor\":%zu,\"warpSize\":%d}",
                        p.name, p.gcnArchName, p.multiProcessorCount, p.totalGlobalMem, free_b, p.clockRate,
                        p.memoryClockRate, p.memoryBusWidth, p.l2CacheSize, p.pciBusID, p.pciDeviceID, p.pciDomainID,
                        p.maxSharedMemoryPerMultiProcessor, p.warpSize);
  return n;
}

// mode: 0 read, 1 write, 2 copy, 3 triad. bytes = working set per array.
// cu_limit > 0 caps the grid at cu_limit * blocks_per_cu workgroups.
// detail (optional, 3 doubles): min-launch GB/s, batch GB/s, batch ms/launch.
int xs_hbm_bandwidth_d(int dev, size_t bytes, int iters, int cu_limit, int mode, int variant, double* gbps,
                       double* ms_per_iter, double* detail) {
  XS_CHECK(hipSetDevice(dev));
  if (iters <= 0) iters = 10;
  size_t n = bytes / sizeof(vec4);
  if (n == 0 || mode < 0 || mode > 3) return -1000;
  bytes = n * sizeof(vec4);
  Variant v = variant == 0 ? default_variant(mode) : decode(variant);
  DevMem a, b, c, sink;
  XS_CHECK(hipMalloc(&a.p, bytes));
  XS_CHECK(hipMalloc(&b.p, bytes));
  if (mode == 3) XS_CHECK(hipMalloc(&c.p, bytes));
  XS_CHECK(hipMalloc(&sink.p, sizeof(uint32_t)));
  int cus = cu_count(dev);
  if (cu_limit > 0 && cu_limit < cus) {
    cus = cu_limit;
    v.one_shot = false;  // a CU budget needs the persistent grid
  }
  int grid = grid_for(v, n, cus);
  Stream s;
  XS_CHECK(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
  // Page everything in and warm the launch path.
  launch(Variant{}, 1, grid, s.s, a.p, nullptr, nullptr, n, sink.as<uint32_t>());
  launch(Variant{}, 1, grid, s.s, b.p, nullptr, nullptr, n, sink.as<uint32_t>());
  if (c.p) launch(Variant{}, 1, grid, s.s, c.p, nullptr, nullptr, n, sink.as<uint32_t>());
  XS_CHECK(hipGetLastError());
  launch(v, mode, grid, s.s, a.p, b.p, c.p, n, sink.as<uint32_t>());
  XS_CHECK(hipStreamSynchronize(s.s));
  double t[3];
  int rc = time_launches(s.s, iters, [&](int) { launch(v, mode, grid, s.s, a.p, b.p, c.p, n, sink.as<uint32_t>()); }, t);
  if (rc) return rc;
  const double moved = static_cast<double>(bytes) * (mode == 2 ? 2.0 : mode == 3 ? 3.0 : 1.0);
  if (gbps) *gbps = moved / (t[0] * 1e-3) / 1e9;
  if (ms_per_iter) *ms_per_iter = t[0];
  if (detail) {
    detail[0] = moved / (t[1] * 1e-3) / 1e9;
    detail[1] = moved / (t[2] * 1e-3) / 1e9;
    detail[2] = t[2];
  }
  return 0;
}

int xs_hbm_bandwidth_v(int dev, size_t bytes, int iters, int cu_limit, int mode, int variant, double* gbps,
                       double* ms_per_iter) {
  return xs_hbm_bandwidth_d(dev, bytes, iters, cu_limit, mode, variant, gbps, ms_per_iter, nullptr);
}

// One streaming kernel over caller-owned device buffers (e.g. torch tensors),
// run to completion: the GPU tier checks the kernels' results against a plain
// PyTorch fp32 reference. mode 1: a <- pattern(seed); 2: b <- a; 3: a <- b +
// scale*c (float4 lanes). bytes must be a multiple of 16 and every pointer
// 16-byte aligned. variant as in xs_hbm_bandwidth_v (0 = the tuned default).
int xs_stream_op(int dev, int mode, void* a, void* b, void* c, size_t bytes, uint32_t seed, float scale,
                 int variant) {
  XS_CHECK(hipSetDevice(dev));
  if (mode < 1 || mode > 3 || bytes == 0 || bytes % sizeof(vec4) != 0) return -1000;
  const uintptr_t align = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                          reinterpret_cast<uintptr_t>(c);
  if (!a || (mode >= 2 && !b) || (mode == 3 && !c) || (align & (sizeof(vec4) - 1))) return -1001;
  Variant v = variant == 0 ? default_variant(mode) : decode(variant);
  int grid = grid_for(v, bytes / sizeof(vec4), cu_count(dev));
  launch(v, mode, grid, nullptr, a, b, c, bytes / sizeof(vec4), nullptr, seed, scale);
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipDeviceSynchronize());
  return 0;
}

// XCD-pinned streaming over caller-owned buffers (mode 1 write dst, 2 copy
// src -> dst): only workgroups on the XCDs in xcd_mask do the work.
int xs_pinned_op(int dev, int mode, const void* src, void* dst, size_t bytes, uint32_t xcd_mask) {
  XS_CHECK(hipSetDevice(dev));
  if (mode < 1 || mode > 2 || xcd_mask == 0 || bytes == 0 || bytes % sizeof(vec4) != 0) return -1000;
  const size_t n = bytes / sizeof(vec4);
  if (n / 16384 >= 0xffffff00ull) return -1000;
  if (!dst || (mode == 2 && !src) ||
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & (sizeof(vec4) - 1)))
    return -1001;
  DevMem counter, sink;
  const size_t ctr_bytes = sizeof(unsigned) * kMaxXcds * kCounterStride;
  XS_CHECK(hipMalloc(&counter.p, ctr_bytes));
  XS_CHECK(hipMalloc(&sink.p, sizeof(uint32_t)));
  XS_CHECK(hipMemset(counter.p, 0, ctr_bytes));
  k_pinned<<<cu_count(dev) * 8, kBlock>>>(static_cast<const vec4*>(src), static_cast<vec4*>(dst), n, xcd_mask,
                                         counter.as<unsigned>(), mode, sink.as<uint32_t>());
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipDeviceSynchronize());
  return 0;
}

int xs_hbm_bandwidth(int dev, size_t bytes, int iters, int cu_limit, int mode, double* gbps, double* ms_per_iter) {
  return xs_hbm_bandwidth_v(dev, bytes, iters, cu_limit, mode, 0, gbps, ms_per_iter);
}

// Bandwidth pulled by the workgroups resident on the XCDs in xcd_mask
// (mode 0 read, 1 write, 2 copy). detail as in xs_hbm_bandwidth_d.
int xs_hbm_bandwidth_xcd_d(int dev, size_t bytes, int iters, uint32_t xcd_mask, int mode, double* gbps,
                           double* ms_per_iter, double* detail) {
  XS_CHECK(hipSetDevice(dev));
  if (iters <= 0) iters = 10;
  if (mode < 0 || mode > 2 || xcd_mask == 0) return -1000;
  size_t n = bytes / sizeof(vec4);
  if (n == 0 || n / 16384 >= 0xffffff00ull) return -1000;
  bytes = n * sizeof(vec4);
  DevMem a, b, counters, sink;
  XS_CHECK(hipMalloc(&a.p, bytes));
  XS_CHECK(hipMalloc(&b.p, bytes));
  const size_t per_launch = static_cast<size_t>(kMaxXcds) * kCounterStride;  // fresh counters per launch
  XS_CHECK(hipMalloc(&counters.p, sizeof(unsigned) * per_launch * (iters + 1)));
  XS_CHECK(hipMalloc(&sink.p, sizeof(uint32_t)));
  XS_CHECK(hipMemset(counters.p, 0, sizeof(unsigned) * per_launch * (iters + 1)));
  unsigned* ctr = counters.as<unsigned>();
  int grid = cu_count(dev) * 8;  // every CU gets 8 workgroups; only masked XCDs work
  Stream s;
  XS_CHECK(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
  k_write<4, true><<<grid, kBlock, 0, s.s>>>(a.as<vec4>(), n, 1);
  k_pinned<<<grid, kBlock, 0, s.s>>>(a.as<const vec4>(), b.as<vec4>(), n, xcd_mask, &ctr[iters * per_launch], mode,
                                     sink.as<uint32_t>());
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipStreamSynchronize(s.s));
  double t[3];
  int rc = time_launches(s.s, iters, [&](int i) {
    k_pinned<<<grid, kBlock, 0, s.s>>>(a.as<const vec4>(), b.as<vec4>(), n, xcd_mask, &ctr[i * per_launch], mode,
                                       sink.as<uint32_t>());
  }, t);
  if (rc) return rc;
  const double moved = static_cast<double>(bytes) * (mode == 2 ? 2.0 : 1.0);
  if (gbps) *gbps = moved / (t[0] * 1e-3) / 1e9;
  if (ms_per_iter) *ms_per_iter = t[0];
  if (detail) {
    detail[0] = moved / (t[1] * 1e-3) / 1e9;
    detail[1] = moved / (t[2] * 1e-3) / 1e9;
    detail[2] = t[2];
  }
  return 0;
}

int xs_hbm_bandwidth_xcd(int dev, size_t bytes, int iters, uint32_t xcd_mask, int mode, double* gbps,
                         double* ms_per_iter) {
  return xs_hbm_bandwidth_xcd_d(dev, bytes, iters, xcd_mask, mode, gbps, ms_per_iter, nullptr);
}

// Counter calibration: `touches` segments of `seg_bytes` (16..1024, a
// multiple of 16), one per `stride_bytes` slot (a multiple of 128, >=
// seg_bytes), read (mode 0) or written (mode 1), default or non-temporal
// policy; `iters` timed launches after one warm-up. out: [median ms, bytes
// per dispatch, 128-B lines per dispatch].
int xs_segment_access(int dev, int mode, int nt, int seg_bytes, size_t stride_bytes, size_t touches, int iters,
                      double* out) {
  XS_CHECK(hipSetDevice(dev));
  if (mode < 0 || mode > 1 || seg_bytes < 16 || seg_bytes > 1024 || seg_bytes % 16 || stride_bytes % 128 ||
      stride_bytes < static_cast<size_t>(seg_bytes) || touches == 0)
    return -1000;
  if (iters <= 0) iters = 10;
  const size_t bytes = stride_bytes * touches;
  const size_t n = bytes / sizeof(vec4);
  DevMem buf, sink;
  XS_CHECK(hipMalloc(&buf.p, bytes));
  XS_CHECK(hipMalloc(&sink.p, sizeof(uint32_t)));
  const int grid = cu_count(dev) * 8;
  Stream s;
  XS_CHECK(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
  k_write<4, true><<<grid, kBlock, 0, s.s>>>(buf.as<vec4>(), n, 1);  // page in
  const size_t sv = stride_bytes / sizeof(vec4);
  const int lanes = seg_bytes / 16;
  auto go = [&] {
    if (mode == 0 && nt) k_segments<0, true><<<grid, kBlock, 0, s.s>>>(buf.as<vec4>(), touches, sv, lanes, sink.as<uint32_t>());
    else if (mode == 0) k_segments<0, false><<<grid, kBlock, 0, s.s>>>(buf.as<vec4>(), touches, sv, lanes, sink.as<uint32_t>());
    else if (nt) k_segments<1, true><<<grid, kBlock, 0, s.s>>>(buf.as<vec4>(), touches, sv, lanes, sink.as<uint32_t>());
    else k_segments<1, false><<<grid, kBlock, 0, s.s>>>(buf.as<vec4>(), touches, sv, lanes, sink.as<uint32_t>());
  };
  go();
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipStreamSynchronize(s.s));
  double t[3];
  int rc = time_launches(s.s, iters, [&](int) { go(); }, t);
  if (rc) return rc;
  out[0] = t[0];
  out[1] = static_cast<double>(touches) * seg_bytes;
  out[2] = static_cast<double>(touches) * ((seg_bytes + 127) / 128);
  return 0;
}

// Launches `blocks` single-wave workgroups; returns the number of distinct
// XCDs observed and writes a 8-entry histogram of blocks per XCD.
int xs_xcd_census(int dev, int blocks, int* xcd_hist8, int* distinct_cus) {
  XS_CHECK(hipSetDevice(dev));
  if (blocks <= 0) blocks = 2048;
  DevMem dx, dh;
  XS_CHECK(hipMalloc(&dx.p, blocks * sizeof(uint32_t)));
  XS_CHECK(hipMalloc(&dh.p, blocks * sizeof(uint32_t)));
  k_census<<<blocks, 64>>>(dx.as<uint32_t>(), dh.as<uint32_t>());
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> hx(blocks), hh(blocks);
  XS_CHECK(hipMemcpy(hx.data(), dx.p, blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  XS_CHECK(hipMemcpy(hh.data(), dh.p, blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  int hist[16] = {0};
  for (int i = 0; i < blocks; ++i) hist[hx[i] & 0xf]++;
  int distinct = 0;
  for (int i = 0; i < 16; ++i) distinct += hist[i] > 0;
  if (xcd_hist8)
    for (int i = 0; i < 8; ++i) xcd_hist8[i] = hist[i];
  if (distinct_cus) {
    // Unique (xcd, HW_ID CU/SE bits) pairs approximate distinct CUs touched.
    int uniq = 0;
    for (int i = 0; i < blocks; ++i) {
      uint32_t key = ((hx[i] & 0xf) << 16) | (hh[i] & 0xfff0);
      bool seen = false;
      for (int j = 0; j < i && !seen; ++j) seen = ((((hx[j] & 0xf) << 16) | (hh[j] & 0xfff0)) == key);
      uniq += !seen;
    }
    *distinct_cus = uniq;
  }
  return distinct;
}

// Writes a pattern over `bytes` and verifies its checksum on the host.
// Returns 0 when healthy, 1 on mismatch, <0 on HIP errors.
int xs_health_check(int dev, size_t bytes, unsigned long long* device_sum, unsigned long long* host_sum) {
  XS_CHECK(hipSetDevice(dev));
  size_t n = bytes / sizeof(uint32_t);
  if (n == 0) n = 1 << 20;
  DevMem buf, out;
  XS_CHECK(hipMalloc(&buf.p, n * sizeof(uint32_t)));
  XS_CHECK(hipMalloc(&out.p, sizeof(unsigned long long)));
  XS_CHECK(hipMemset(out.p, 0, sizeof(unsigned long long)));
  int grid = cu_count(dev) * 8;
  k_pattern<<<grid, kBlock>>>(buf.as<uint32_t>(), n);
  k_checksum<<<grid, kBlock>>>(buf.as<uint32_t>(), n, out.as<unsigned long long>());
  XS_CHECK(hipGetLastError());
  unsigned long long d = 0;
  XS_CHECK(hipMemcpy(&d, out.p, sizeof d, hipMemcpyDeviceToHost));
  unsigned long long h = 0;
  for (size_t i = 0; i < n; ++i) h += static_cast<uint32_t>(static_cast<uint32_t>(i * 2654435761u) ^ 0xa5a5a5a5u);
  if (device_sum) *device_sum = d;
  if (host_sum) *host_sum = h;
  return d == h ? 0 : 1;
}

}  // extern "C"
