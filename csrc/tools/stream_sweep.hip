// Streaming-kernel design sweep for the HBM probe (csrc/hip/hbm_probe.hip).
//
// A standalone executable (built by build_ext.build_stream_sweep into ops/stream_sweep, run on the
// GPU box as ops/stream_sweep [modes] [GiB]): read / write / copy over 2 GiB arrays
// for every combination of
//   layout  0 grid-stride (a persistent grid walks the array in rows of
//             grid x 4 KiB; the probe's current shape)
//           1 block-contiguous (persistent grid, workgroup b owns the b-th
//             contiguous 1/grid of the array)
//           2 one-shot (no loop: one workgroup per 4 KiB x U tile, ~0.5M
//             workgroups over 2 GiB)
//   unroll  U independent 16-B accesses per lane in flight (1, 2, 4, 8)
//   policy  0 plain global, 1 nontemporal builtin, 2..5 buffer ops with cache
//             policy bits (none, nt, sc1, sc1 nt)
//   bpc     persistent workgroups per CU (2, 4, 8, 16; layouts 0 and 1)
// Each row: median of 15 launches timed by their own event pairs, GB/s of
// bytes moved (copy counts read + write), one JSON line per row.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

constexpr int kBlock = 256;
typedef uint32_t vec4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// Buffer-op cache-policy operand per policy 2..5 (gfx950: bit 1 nt, bit 4 sc1).
constexpr int kAux[6] = {0, 0, 0, 2, 16, 18};

template <int POL>
struct Mem {
  __amdgpu_buffer_rsrc_t rs, rd;
  const vec4* s;
  vec4* d;
  __device__ Mem(const vec4* src, vec4* dst, size_t n) : s(src), d(dst) {
    if constexpr (POL >= 2) {
      // 2 GiB arrays: byte offsets fit the 32-bit voffset and num_records.
      const int32_t bytes = static_cast<int32_t>(n * sizeof(vec4) > 0x7fffffffULL ? 0x7fffffff : n * sizeof(vec4));
      rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<vec4*>(src), 0, bytes, 0x00020000);
      rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, bytes, 0x00020000);
    }
  }
  __device__ __forceinline__ vec4 load(size_t i) const {
    if constexpr (POL == 0) return s[i];
    else if constexpr (POL == 1) return __builtin_nontemporal_load(&s[i]);
    else {
      i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(i * sizeof(vec4)), 0, kAux[POL]);
      return __builtin_bit_cast(vec4, v);
    }
  }
  __device__ __forceinline__ void store(vec4 v, size_t i) const {
    if constexpr (POL == 0) d[i] = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, &d[i]);
    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rd, static_cast<int>(i * sizeof(vec4)), 0,
                                                kAux[POL]);
  }
};

// mode 0 read, 1 write, 2 copy; [lo, hi) walked in tiles of U x 256 vec4s,
// tile t at lo + t * step.
template <int MODE, int U, int POL>
__device__ __forceinline__ void walk(const Mem<POL>& m, size_t lo, size_t hi, size_t step, uint32_t& acc) {
  const vec4 fill = {1u, 2u, 3u, 4u};
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * kBlock < hi; i += step) {
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) m.store(fill, i + u * kBlock);
    } else {
      vec4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = m.load(i + u * kBlock);
      if constexpr (MODE == 2) {
#pragma unroll
        for (int u = 0; u < U; ++u) m.store(v[u], i + u * kBlock);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
      }
    }
  }
}

template <int MODE, int U, int POL, int LAYOUT>
__global__ __launch_bounds__(kBlock) void k_stream(const vec4* __restrict__ src, vec4* __restrict__ dst, size_t n,
                                                   uint32_t* __restrict__ sink) {
  Mem<POL> m(src, dst, n);
  uint32_t acc = 0;
  const size_t tile = static_cast<size_t>(U) * kBlock;
  if constexpr (LAYOUT == 0) {
    // Tiles round-robin over the grid.
    walk<MODE, U, POL>(m, blockIdx.x * tile, n, gridDim.x * tile, acc);
  } else if constexpr (LAYOUT == 1) {
    const size_t per = (n / gridDim.x) / tile * tile;
    walk<MODE, U, POL>(m, blockIdx.x * per, (blockIdx.x + 1) * per, tile, acc);
  } else {
    walk<MODE, U, POL>(m, blockIdx.x * tile, std::min(n, (blockIdx.x + 1) * tile), tile, acc);
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

struct Ctx {
  vec4 *a, *b;
  uint32_t* sink;
  size_t n;
  int cus;
  hipStream_t s;
};

template <int MODE, int U, int POL, int LAYOUT>
void run(const Ctx& c, int bpc, int iters) {
  const size_t tile = static_cast<size_t>(U) * kBlock;
  const int grid = LAYOUT == 2 ? static_cast<int>(c.n / tile) : c.cus * bpc;
  auto go = [&] { k_stream<MODE, U, POL, LAYOUT><<<grid, kBlock, 0, c.s>>>(c.a, c.b, c.n, c.sink); };
  go();
  CK(hipStreamSynchronize(c.s));
  std::vector<hipEvent_t> ev(2 * iters);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(ev[2 * i], c.s));
    go();
    CK(hipEventRecord(ev[2 * i + 1], c.s));
  }
  CK(hipEventSynchronize(ev.back()));
  CK(hipGetLastError());
  std::vector<float> ms(iters);
  for (int i = 0; i < iters; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
  for (auto& e : ev) CK(hipEventDestroy(e));
  std::sort(ms.begin(), ms.end());
  // Layout 1 leaves the n % (grid * tile) tail undone: count only what moved.
  size_t done = c.n;
  if (LAYOUT == 1) done = (c.n / grid) / tile * tile * grid;
  const double bytes = static_cast<double>(done) * sizeof(vec4) * (MODE == 2 ? 2.0 : 1.0);
  const char* modes[] = {"read", "write", "copy"};
  std::printf("{\"mode\":\"%s\",\"layout\":%d,\"unroll\":%d,\"policy\":%d,\"bpc\":%d,\"grid\":%d,"
              "\"median_ms\":%.4f,\"min_ms\":%.4f,\"gbps\":%.1f,\"pct_of_8tbs\":%.1f}\n",
              modes[MODE], LAYOUT, U, POL, LAYOUT == 2 ? 0 : bpc, grid, ms[iters / 2], ms[0],
              bytes / (ms[iters / 2] * 1e-3) / 1e9, 100.0 * bytes / (ms[iters / 2] * 1e-3) / 8e12);
  std::fflush(stdout);
}

template <int MODE, int U, int POL>
void sweep_layouts(const Ctx& c, int iters) {
  for (int bpc : {2, 4, 8, 16}) run<MODE, U, POL, 0>(c, bpc, iters);
  for (int bpc : {2, 4, 8, 16}) run<MODE, U, POL, 1>(c, bpc, iters);
  run<MODE, U, POL, 2>(c, 0, iters);
}

template <int MODE, int POL>
void sweep_unroll(const Ctx& c, int iters) {
  sweep_layouts<MODE, 1, POL>(c, iters);
  sweep_layouts<MODE, 2, POL>(c, iters);
  sweep_layouts<MODE, 4, POL>(c, iters);
  sweep_layouts<MODE, 8, POL>(c, iters);
}

template <int MODE>
void sweep_policy(const Ctx& c, int iters) {
  sweep_unroll<MODE, 0>(c, iters);
  sweep_unroll<MODE, 1>(c, iters);
  sweep_unroll<MODE, 2>(c, iters);
  sweep_unroll<MODE, 3>(c, iters);
  sweep_unroll<MODE, 4>(c, iters);
  sweep_unroll<MODE, 5>(c, iters);
}

__global__ void k_fill(vec4* p, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    p[i] = vec4{static_cast<uint32_t>(i), 1u, 2u, 3u};
}

}  // namespace

int main(int argc, char** argv) {
  // argv[1]: modes to sweep ("rwc" default); argv[2]: GiB per array (2).
  const char* modes = argc > 1 ? argv[1] : "rwc";
  const double gib = argc > 2 ? std::atof(argv[2]) : 2.0;
  Ctx c{};
  c.n = static_cast<size_t>(gib * (1ULL << 30)) / sizeof(vec4);
  if (c.n * sizeof(vec4) > 0x7fffffffULL) c.n = 0x7fffffffULL / sizeof(vec4) / 4096 * 4096;  // 32-bit buffer offsets
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  c.cus = p.multiProcessorCount;
  CK(hipMalloc(&c.a, c.n * sizeof(vec4)));
  CK(hipMalloc(&c.b, c.n * sizeof(vec4)));
  CK(hipMalloc(&c.sink, sizeof(uint32_t)));
  CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
  k_fill<<<c.cus * 8, kBlock, 0, c.s>>>(c.a, c.n);
  k_fill<<<c.cus * 8, kBlock, 0, c.s>>>(c.b, c.n);
  CK(hipStreamSynchronize(c.s));
  std::printf("{\"device\":\"%s\",\"cus\":%d,\"bytes_per_array\":%zu}\n", p.gcnArchName, c.cus, c.n * sizeof(vec4));
  const int iters = 15;
  if (std::strchr(modes, 'r')) sweep_policy<0>(c, iters);
  if (std::strchr(modes, 'w')) sweep_policy<1>(c, iters);
  if (std::strchr(modes, 'c')) sweep_policy<2>(c, iters);
  CK(hipFree(c.a));
  CK(hipFree(c.b));
  CK(hipFree(c.sink));
  CK(hipStreamDestroy(c.s));
  return 0;
}
