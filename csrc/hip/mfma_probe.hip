// Matrix-core probes for gfx950 (MI355X): the node agent's compute check.
//
//  * xs_mfma_check   one wave computes C[32x32] = A[32xK]·B[Kx32] with
//                    v_mfma_f32_32x32x16_bf16 from exact small-integer bf16
//                    inputs (asymmetric B); the host compares bit-exactly
//                    against an integer reference. A GPU whose matrix cores
//                    mis-compute fails health even when HBM checksums pass.
//  * xs_mfma_peak    back-to-back bf16 MFMA issue, 2 waves per SIMD and 4
//                    independent 32x32 accumulators per wave (hides the
//                    MFMA dependency latency), optionally restricted to the
//                    XCDs of a mask (blocks read HW_REG_XCC_ID and the others
//                    exit), so a CPX/QPX/DPX partition's matrix throughput can
//                    be measured directly. Dense bf16 only (no sparsity).
//
// Operand maps (cdna_hip_programming.md §3, gfx950): lane l, r = l&31,
// h = l>>5 holds A[r][k0+8h+j] and B[k0+8h+j][r] (j = 0..7); accumulator
// register q holds C[(q&3) + 8(q>>2) + 4h][r].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hip/device_raii.h"

namespace {

char g_mfma_err[512];

#define XS_MCHECK(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::snprintf(g_mfma_err, sizeof g_mfma_err, "%s: %s", #x, hipGetErrorString(e_)); \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kPeakBlock = 256;  // 4 waves: one per SIMD
constexpr int kAcc = 4;          // independent accumulators per wave

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

__global__ __launch_bounds__(64) void k_mfma_tile(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                  float* __restrict__ C, int K) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 acc = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = A[r * K + k0 + 8 * h + j];
      b[j] = B[(k0 + 8 * h + j) * 32 + r];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}

__global__ __launch_bounds__(kPeakBlock) void k_mfma_peak(int iters, uint32_t xcd_mask, unsigned* __restrict__ active,
                                                           float* __restrict__ sink) {
  if (!((xcd_mask >> xcc_id()) & 1u)) return;
  if (threadIdx.x == 0) atomicAdd(active, 1u);
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(0.125f * static_cast<float>((threadIdx.x + j) & 7));
    b[j] = static_cast<__bf16>(0.0625f * static_cast<float>((threadIdx.x * 3 + j) & 15));
  }
  f32x16 acc[kAcc];
#pragma unroll
  for (int n = 0; n < kAcc; ++n) acc[n] = f32x16{};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int n = 0; n < kAcc; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[n], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int n = 0; n < kAcc; ++n)
#pragma unroll
    for (int q = 0; q < 16; ++q) s += acc[n][q];
  // Data-dependent store: the accumulators stay live, the store almost never runs.
  if (s == -1.0f) sink[blockIdx.x] = s;
}

inline __bf16 to_bf16(float f) { return static_cast<__bf16>(f); }

}  // namespace

extern "C" {

const char* xs_mfma_last_error() { return g_mfma_err; }

// Exact-integer MFMA tile check. Returns the number of mismatching elements
// of the 32x32 result (0 = pass), or <0 on a HIP error.
int xs_mfma_check(int dev, int K) {
  if (K <= 0 || K % 16) K = 64;
  XS_MCHECK(hipSetDevice(dev));
  std::vector<__bf16> a(32 * K), b(K * 32);
  std::vector<int> ai(32 * K), bi(K * 32);
  for (int i = 0; i < 32; ++i)
    for (int k = 0; k < K; ++k) {
      ai[i * K + k] = (i * 3 + k * 7) % 17 - 8;
      a[i * K + k] = to_bf16(static_cast<float>(ai[i * K + k]));
    }
  for (int k = 0; k < K; ++k)
    for (int j = 0; j < 32; ++j) {
      bi[k * 32 + j] = (k * 5 + j * 11 + (j > k ? 3 : 0)) % 13 - 6;  // asymmetric
      b[k * 32 + j] = to_bf16(static_cast<float>(bi[k * 32 + j]));
    }
  xsprobe::DevMem da, db, dc;
  XS_MCHECK(hipMalloc(&da.p, a.size() * sizeof(__bf16)));
  XS_MCHECK(hipMalloc(&db.p, b.size() * sizeof(__bf16)));
  XS_MCHECK(hipMalloc(&dc.p, 32 * 32 * sizeof(float)));
  XS_MCHECK(hipMemcpy(da.p, a.data(), a.size() * sizeof(__bf16), hipMemcpyHostToDevice));
  XS_MCHECK(hipMemcpy(db.p, b.data(), b.size() * sizeof(__bf16), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_mfma_tile, dim3(1), dim3(64), 0, 0, da.as<const __bf16>(), db.as<const __bf16>(),
                     dc.as<float>(), K);
  XS_MCHECK(hipGetLastError());
  std::vector<float> c(32 * 32);
  XS_MCHECK(hipMemcpy(c.data(), dc.p, c.size() * sizeof(float), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      long ref = 0;
      for (int k = 0; k < K; ++k) ref += static_cast<long>(ai[i * K + k]) * bi[k * 32 + j];
      if (c[i * 32 + j] != static_cast<float>(ref)) ++bad;
    }
  return bad;
}

// Dense bf16 MFMA throughput on the XCDs of `xcd_mask` (0xff = whole GPU).
// `blocks` = launch size (0: 8 per CU = 8 waves per SIMD). With the clock
// ramped by the warm-up, 2-8 waves per SIMD all issue at 98-99% of the
// 2.5 PF rate (profiles/r4z_mfma_sweep.jsonl); the earlier 79% reading was a
// clock still ramping under a short warm-up (r4x/r4y sweeps: rate rising with
// launch size and length only because each point ran hotter). Returns 0 and TFLOP/s, ms and the
// number of workgroups that ran on the selected XCDs.
int xs_mfma_peak(int dev, int iters, uint32_t xcd_mask, int blocks, double* tflops, double* ms_out,
                 int* active_blocks) {
  XS_MCHECK(hipSetDevice(dev));
  hipDeviceProp_t p;
  XS_MCHECK(hipGetDeviceProperties(&p, dev));
  if (blocks <= 0) blocks = 8 * p.multiProcessorCount;
  if (iters <= 0) iters = 4096;
  xsprobe::DevMem active_mem, sink_mem;
  XS_MCHECK(hipMalloc(&active_mem.p, sizeof(unsigned)));
  XS_MCHECK(hipMalloc(&sink_mem.p, blocks * sizeof(float)));
  unsigned* d_active = active_mem.as<unsigned>();
  float* d_sink = sink_mem.as<float>();
  xsprobe::Stream stream;
  XS_MCHECK(hipStreamCreate(&stream.s));
  hipStream_t s = stream.s;
  xsprobe::Event ev0, ev1;
  XS_MCHECK(hipEventCreate(&ev0.e));
  XS_MCHECK(hipEventCreate(&ev1.e));
  hipEvent_t e0 = ev0.e, e1 = ev1.e;
  // Warm-up: code resident, then about 20 ms of the same load so the clock has
  // ramped before the timed launch: 2.11 -> 2.40-2.41 PF/s in a fresh process
  // (profiles/r4za_probe_warm_ab.jsonl). The HBM probes are memory-bound and
  // read the same with or without it (same file), so they keep their short one.
  float warm_ms = 0.f;
  XS_MCHECK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(kPeakBlock), 0, s, iters, xcd_mask, d_active, d_sink);
  XS_MCHECK(hipGetLastError());
  XS_MCHECK(hipEventRecord(e1, s));
  XS_MCHECK(hipEventSynchronize(e1));
  XS_MCHECK(hipEventElapsedTime(&warm_ms, e0, e1));
  const char* env = std::getenv("XS_PROBE_WARM_MS");  // as the HBM probes; 0 = one launch
  const float target = env ? static_cast<float>(std::atof(env)) : 20.f;
  const int warm = target <= 0.f ? 0 : warm_ms > 0.f ? std::min(64, static_cast<int>(target / warm_ms) + 1) : 4;
  for (int w = 0; w < warm; ++w)
    hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(kPeakBlock), 0, s, iters, xcd_mask, d_active, d_sink);
  XS_MCHECK(hipGetLastError());
  XS_MCHECK(hipMemsetAsync(d_active, 0, sizeof(unsigned), s));
  XS_MCHECK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(kPeakBlock), 0, s, iters, xcd_mask, d_active, d_sink);
  XS_MCHECK(hipGetLastError());
  XS_MCHECK(hipEventRecord(e1, s));
  XS_MCHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  XS_MCHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned active = 0;
  XS_MCHECK(hipMemcpy(&active, d_active, sizeof(unsigned), hipMemcpyDeviceToHost));
  const double flop_per_mfma = 2.0 * 32 * 32 * 16;
  double flops = static_cast<double>(active) * (kPeakBlock / 64) * kAcc * static_cast<double>(iters) * flop_per_mfma;
  *tflops = ms > 0 ? flops / (ms * 1e-3) / 1e12 : 0.0;
  *ms_out = ms;
  *active_blocks = static_cast<int>(active);
  return 0;
}

}  // extern "C"
