// MI355X (gfx950) device probes used by the node agent and the benchmarks.
//
// There is no GPU code in the reference: the scheduler only
// counts extended resources. An MI355X-native scheduler must validate what it
// promises, so the node agent runs these probes on the box:
//
//  * xs_hbm_bandwidth   streaming read / write / copy / triad over N bytes
//                       with 16-byte lanes (global_load/store_dwordx4),
//                       grid = cu_limit x 8 blocks of 256 threads. cu_limit
//                       emulates a compute partition's CU budget (CPX: 32
//                       CUs/XCD); the result is HBM GB/s that a slice can
//                       expect (HBM3E peak 8 TB/s, ~6.3 TB/s achievable).
//  * xs_xcd_census      every workgroup records s_getreg(HW_REG_XCC_ID):
//                       counts XCDs/CUs visible to this device — verifies the
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
#include <cstring>

#define XS_CHECK(x)                                  \
  do {                                               \
    hipError_t e_ = (x);                             \
    if (e_ != hipSuccess) {                          \
      std::snprintf(g_err, sizeof g_err, "%s: %s", #x, hipGetErrorString(e_)); \
      return -static_cast<int>(e_) - 1;             \
    }                                                \
  } while (0)

namespace {

char g_err[512];

constexpr int kBlock = 256;       // 4 waves of 64 lanes
constexpr int kBlocksPerCU = 8;   // enough waves in flight to cover HBM latency
constexpr int kUnroll = 4;        // 4 x 16 B in flight per lane per iteration

typedef uint32_t vec4 __attribute__((ext_vector_type(4)));  // 16 B/lane -> global_load_dwordx4
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Every kernel walks the buffer in grid-stride "rows" of kUnroll*grid lanes so
// each wave-instruction touches 1 KiB contiguous (full 128 B lines).

__global__ __launch_bounds__(kBlock) void k_read(const vec4* __restrict__ src, size_t n, uint32_t* __restrict__ sink) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (kUnroll - 1) * stride < n; i += kUnroll * stride) {
    vec4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n; i += stride) {
    vec4 v = __builtin_nontemporal_load(&src[i]);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // practically never true: defeats DCE without a store per lane
}

__global__ __launch_bounds__(kBlock) void k_write(vec4* __restrict__ dst, size_t n, uint32_t seed) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  vec4 v = {seed, seed ^ 0x55555555u, seed + 1, ~seed};
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(v, &dst[i]);
}

__global__ __launch_bounds__(kBlock) void k_copy(const vec4* __restrict__ src, vec4* __restrict__ dst, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < n; i += kUnroll * stride) {
    vec4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) __builtin_nontemporal_store(v[u], &dst[i + u * stride]);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

// STREAM triad a = b + s*c on float4 lanes.
__global__ __launch_bounds__(kBlock) void k_triad(f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                  const f32x4* __restrict__ c, float s, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    f32x4 x = __builtin_nontemporal_load(&b[i]);
    f32x4 y = __builtin_nontemporal_load(&c[i]);
    __builtin_nontemporal_store(x + s * y, &a[i]);
  }
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

__device__ __forceinline__ uint32_t hw_cu_id() {
  // HW_ID register: CU_ID in bits [11:8], SE_ID in [14:13] on CDNA.
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
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

int grid_for(int dev, int cu_limit) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 256 * kBlocksPerCU;
  int cus = p.multiProcessorCount;
  if (cu_limit > 0 && cu_limit < cus) cus = cu_limit;
  return cus * kBlocksPerCU;
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

// mode: 0 read, 1 write, 2 copy, 3 triad. bytes = working-set per array.
// Returns 0 and writes GB/s (bytes moved / time) and ms per iteration.
int xs_hbm_bandwidth(int dev, size_t bytes, int iters, int cu_limit, int mode, double* gbps, double* ms_per_iter) {
  XS_CHECK(hipSetDevice(dev));
  if (iters <= 0) iters = 10;
  size_t n = bytes / sizeof(vec4);
  if (n == 0) return -1000;
  bytes = n * sizeof(vec4);
  void *a = nullptr, *b = nullptr, *c = nullptr;
  uint32_t* sink = nullptr;
  XS_CHECK(hipMalloc(&a, bytes));
  XS_CHECK(hipMalloc(&b, bytes));
  if (mode == 3) XS_CHECK(hipMalloc(&c, bytes));
  XS_CHECK(hipMalloc(&sink, sizeof(uint32_t)));
  int grid = grid_for(dev, cu_limit);
  hipStream_t s;
  XS_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // Touch everything once (page-in) and warm the launch path.
  k_write<<<grid, kBlock, 0, s>>>(static_cast<vec4*>(a), n, 1);
  k_write<<<grid, kBlock, 0, s>>>(static_cast<vec4*>(b), n, 2);
  if (c) k_write<<<grid, kBlock, 0, s>>>(static_cast<vec4*>(c), n, 3);
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipStreamSynchronize(s));
  auto launch = [&]() {
    switch (mode) {
      case 0: k_read<<<grid, kBlock, 0, s>>>(static_cast<const vec4*>(a), n, sink); break;
      case 1: k_write<<<grid, kBlock, 0, s>>>(static_cast<vec4*>(a), n, 7); break;
      case 2: k_copy<<<grid, kBlock, 0, s>>>(static_cast<const vec4*>(a), static_cast<vec4*>(b), n); break;
      default:
        k_triad<<<grid, kBlock, 0, s>>>(static_cast<f32x4*>(a), static_cast<const f32x4*>(b),
                                        static_cast<const f32x4*>(c), 3.0f, n);
    }
  };
  launch();
  XS_CHECK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  XS_CHECK(hipEventCreate(&e0));
  XS_CHECK(hipEventCreate(&e1));
  XS_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) launch();
  XS_CHECK(hipEventRecord(e1, s));
  XS_CHECK(hipEventSynchronize(e1));
  XS_CHECK(hipGetLastError());
  float ms = 0;
  XS_CHECK(hipEventElapsedTime(&ms, e0, e1));
  double per = ms / iters;
  double moved = static_cast<double>(bytes) * (mode == 2 ? 2.0 : mode == 3 ? 3.0 : 1.0);
  if (gbps) *gbps = moved / (per * 1e-3) / 1e9;
  if (ms_per_iter) *ms_per_iter = per;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  (void)hipFree(a);
  (void)hipFree(b);
  if (c) hipFree(c);
  (void)hipFree(sink);
  return 0;
}

// Launches `blocks` single-wave workgroups; returns the number of distinct
// XCDs observed and writes a 8-entry histogram of blocks per XCD.
int xs_xcd_census(int dev, int blocks, int* xcd_hist8, int* distinct_cus) {
  XS_CHECK(hipSetDevice(dev));
  if (blocks <= 0) blocks = 2048;
  uint32_t *dx = nullptr, *dh = nullptr;
  XS_CHECK(hipMalloc(&dx, blocks * sizeof(uint32_t)));
  XS_CHECK(hipMalloc(&dh, blocks * sizeof(uint32_t)));
  k_census<<<blocks, 64>>>(dx, dh);
  XS_CHECK(hipGetLastError());
  XS_CHECK(hipDeviceSynchronize());
  uint32_t* hx = new uint32_t[blocks];
  uint32_t* hh = new uint32_t[blocks];
  XS_CHECK(hipMemcpy(hx, dx, blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  XS_CHECK(hipMemcpy(hh, dh, blocks * sizeof(uint32_t), hipMemcpyDeviceToHost));
  int hist[16] = {0};
  for (int i = 0; i < blocks; ++i) hist[hx[i] & 0xf]++;
  int distinct = 0;
  for (int i = 0; i < 16; ++i) distinct += hist[i] > 0;
  if (xcd_hist8)
    for (int i = 0; i < 8; ++i) xcd_hist8[i] = hist[i];
  if (distinct_cus) {
    // Unique (xcd, hw_id & 0xfff) pairs approximate distinct CUs touched.
    int uniq = 0;
    for (int i = 0; i < blocks; ++i) {
      uint32_t key = ((hx[i] & 0xf) << 16) | (hh[i] & 0xfff0);
      bool seen = false;
      for (int j = 0; j < i && !seen; ++j) seen = ((((hx[j] & 0xf) << 16) | (hh[j] & 0xfff0)) == key);
      uniq += !seen;
    }
    *distinct_cus = uniq;
  }
  delete[] hx;
  delete[] hh;
  (void)hipFree(dx);
  (void)hipFree(dh);
  return distinct;
}

// Writes a pattern over `bytes` and verifies its checksum on the host.
// Returns 0 when healthy, 1 on mismatch, <0 on HIP errors.
int xs_health_check(int dev, size_t bytes, unsigned long long* device_sum, unsigned long long* host_sum) {
  XS_CHECK(hipSetDevice(dev));
  size_t n = bytes / sizeof(uint32_t);
  if (n == 0) n = 1 << 20;
  uint32_t* buf = nullptr;
  unsigned long long* out = nullptr;
  XS_CHECK(hipMalloc(&buf, n * sizeof(uint32_t)));
  XS_CHECK(hipMalloc(&out, sizeof(unsigned long long)));
  XS_CHECK(hipMemset(out, 0, sizeof(unsigned long long)));
  int grid = grid_for(dev, 0);
  k_pattern<<<grid, kBlock>>>(buf, n);
  k_checksum<<<grid, kBlock>>>(buf, n, out);
  XS_CHECK(hipGetLastError());
  unsigned long long d = 0;
  XS_CHECK(hipMemcpy(&d, out, sizeof d, hipMemcpyDeviceToHost));
  unsigned long long h = 0;
  for (size_t i = 0; i < n; ++i) h += static_cast<uint32_t>(static_cast<uint32_t>(i * 2654435761u) ^ 0xa5a5a5a5u);
  if (device_sum) *device_sum = d;
  if (host_sum) *host_sum = h;
  (void)hipFree(buf);
  (void)hipFree(out);
  return d == h ? 0 : 1;
}

}  // extern "C"
