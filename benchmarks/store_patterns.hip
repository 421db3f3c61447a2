// Store / load access-shape microbenchmark for GEMM epilogues (round-4 item: are the hand-written
// GEMMs' output stores bound by their 16-rows x 64-B-per-instruction shape?).
//
// Every workgroup (512 threads = 8 waves, the GEMM's geometry) writes (or reads) T bf16 tiles of
// 256 x 256 of an M x N row-major matrix; each wave covers the GEMM's 128-row x 64-column sub-tile
// (16 KB = 16 wave-instructions of 16 B per lane) in one of these shapes per instruction:
//   0  16 rows x 64 B   (what gemm_pt / gemm.hip epilogues issue today)
//   1   8 rows x 128 B  (whole 128-B lines)
//   2  64 rows x 16 B   (row per lane)
//   3   2 rows x 512 B  (wave region re-cut to 32 rows x 256 columns)
//   4   1 KB contiguous (the tile treated as a flat 128 KB block: the ideal)
// Prints microseconds per tile per workgroup and the chip-wide GB/s for grids of 256 / 128 / 64 / 32.
//
// build: hipcc --offload-arch=gfx950 -O3 -o build/store_patterns benchmarks/store_patterns.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__device__ __forceinline__ size_t elem_off(int inst, int lane, int wave, int ld /*elements*/) {
  const int wm = wave >> 2, wn = wave & 3;
  if constexpr (SHAPE == 0) {
    const int r = wm * 128 + (inst >> 1) * 16 + (lane & 15);
    const int c = wn * 64 + (inst & 1) * 32 + (lane >> 4) * 8;
    return (size_t)r * ld + c;
  } else if constexpr (SHAPE == 1) {
    const int r = wm * 128 + inst * 8 + (lane >> 3);
    const int c = wn * 64 + (lane & 7) * 8;
    return (size_t)r * ld + c;
  } else if constexpr (SHAPE == 2) {
    const int r = wm * 128 + (inst >> 3) * 64 + lane;
    const int c = wn * 64 + (inst & 7) * 8;
    return (size_t)r * ld + c;
  } else if constexpr (SHAPE == 3) {
    const int r = wave * 32 + inst * 2 + (lane >> 5);
    const int c = (lane & 31) * 8;
    return (size_t)r * ld + c;
  } else {
    return 0;  // flat, handled by the caller
  }
}

template <int SHAPE, bool LOAD>
__global__ __launch_bounds__(512, 1) void pattern_kernel(unsigned short* buf, int M, int N, int T, unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tiles_n = N / 256;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int t = 0; t < T; ++t) {
    const int id = blockIdx.x + t * gridDim.x;
    const int tm = id / tiles_n, tn = id % tiles_n;
    unsigned short* tile = buf + (size_t)tm * 256 * N + (size_t)tn * 256;
    unsigned short* flat = buf + (size_t)id * 65536;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      unsigned short* p = SHAPE == 4 ? flat + ((size_t)(wave * 16 + i) * 512 + lane * 8) : tile + elem_off<SHAPE>(i, lane, wave, N);
      if constexpr (LOAD) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(p);
        acc += v;
      } else {
        const u32x4 v = {(unsigned)(lane + i), (unsigned)t, (unsigned)id, 7u};
        *reinterpret_cast<u32x4*>(p) = v;
      }
    }
  }
  if constexpr (LOAD) {
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc.x;
  }
}

template <int SHAPE, bool LOAD>
static float run(unsigned short* buf, int M, int N, int G, int T, unsigned* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((pattern_kernel<SHAPE, LOAD>), dim3(G), dim3(512), 0, 0, buf, M, N, T, sink);
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((pattern_kernel<SHAPE, LOAD>), dim3(G), dim3(512), 0, 0, buf, M, N, T, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ts[ts.size() / 2];
}

template <int SHAPE, bool LOAD>
static void report(const char* name, unsigned short* buf, int M, int N, unsigned* sink) {
  const int tiles = (M / 256) * (N / 256);
  for (int G : {256, 128, 64, 32}) {
    const int T = tiles / G;
    const float ms = run<SHAPE, LOAD>(buf, M, N, G, T, sink);
    const double bytes = (double)G * T * 131072.0;
    printf("{\"op\": \"%s\", \"shape\": \"%s\", \"grid\": %d, \"tiles_per_wg\": %d, \"us_per_tile\": %.2f, \"chip_GBps\": %.0f, "
           "\"per_cu_B_per_clk_at_2.4GHz\": %.1f}\n",
           LOAD ? "load" : "store", name, G, T, ms * 1e3 / T, bytes / (ms * 1e-3) / 1e9, 131072.0 / (ms * 1e-3 / T) / 2.4e9);
    fflush(stdout);
  }
}

int main() {
  const int M = 40960, N = 4096;  // 2560 tiles, 320 MB bf16
  unsigned short* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, (size_t)M * N * 2));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 1, (size_t)M * N * 2));
  report<0, false>("16rows_x_64B", buf, M, N, sink);
  report<1, false>("8rows_x_128B", buf, M, N, sink);
  report<2, false>("64rows_x_16B", buf, M, N, sink);
  report<3, false>("2rows_x_512B", buf, M, N, sink);
  report<4, false>("1KB_contiguous", buf, M, N, sink);
  report<0, true>("16rows_x_64B", buf, M, N, sink);
  report<1, true>("8rows_x_128B", buf, M, N, sink);
  report<2, true>("64rows_x_16B", buf, M, N, sink);
  report<3, true>("2rows_x_512B", buf, M, N, sink);
  report<4, true>("1KB_contiguous", buf, M, N, sink);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
