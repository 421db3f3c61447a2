// MFMA energy probe: the same bf16 FLOPs as the GEMM's 128x128-per-wave block issued as 16x16x32 (64 per
// 64-deep half K-step, the shape the assembly GEMMs use) or as 32x32x16 (32 per half K-step), operands in
// registers (random bf16, no memory traffic), 4 waves per CU on every CU. Run under a power sampler
// (scripts/gpu_mfma_power.sh): at the board limit the achieved TFLOP/s is the energy-per-FLOP of the shape.
//
//   hipcc --offload-arch=gfx950 -O3 -o benchmarks/mfma_power benchmarks/mfma_power.hip && benchmarks/mfma_power [seconds]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <chrono>

static double now() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ bf16x8 rnd8(unsigned& s, int zero) {
  bf16x8 v;
  for (int e = 0; e < 8; ++e) {
    s = s * 1664525u + 1013904223u;
    const float f = zero ? 0.f : ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 22));
    v[e] = (__bf16)f;
  }
  return v;
}

// 16x16x32: 8 A x 8 B fragments, 64 accumulators of 4 -> 256 registers
__global__ __launch_bounds__(256) void mfma16(float* out, int iters, int zero) {
  unsigned s = blockIdx.x * 256 + threadIdx.x + 1;
  bf16x8 a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = rnd8(s, zero); b[i] = rnd8(s, zero); }
  f32x4 acc[8][8];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    // new operands every half K-step, as the GEMM's fragment reads give (cheap register rotation)
#pragma unroll
    for (int i = 0; i < 7; ++i) { const bf16x8 t = a[i]; a[i] = b[i + 1]; b[i + 1] = t; }
  }
  float r = 0.f;
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) r += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

// 32x32x16: the same 128x128x64-per-wave block: 4 A x 4 B fragments per 16-deep k-slice, 2 slices per
// half K-step (32 MFMAs of twice the FLOPs), 16 accumulators of 16 -> 256 registers
__global__ __launch_bounds__(256) void mfma32(float* out, int iters, int zero) {
  unsigned s = blockIdx.x * 256 + threadIdx.x + 1;
  bf16x8 a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = rnd8(s, zero); b[i] = rnd8(s, zero); }
  f32x16 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[4 * kk + i], b[4 * kk + j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 7; ++i) { const bf16x8 t = a[i]; a[i] = b[i + 1]; b[i + 1] = t; }
  }
  float r = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) r += acc[i][j][0] + acc[i][j][15];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? atof(argv[1]) : 5.0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int grid = p.multiProcessorCount;  // one 4-wave workgroup per CU
  float* out;
  hipMalloc(&out, grid * 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;  // per launch: 64 x 16x16x32 per iteration per wave
  const double flop_per_launch = (double)grid * 4 * iters * 64 * (16.0 * 16 * 32 * 2);
  for (int zero = 0; zero < 2; ++zero) {
    for (int v = 0; v < 2; ++v) {
      // warm-up, then as many launches as fit in `seconds`
      if (v == 0) hipLaunchKernelGGL(mfma16, dim3(grid), dim3(256), 0, 0, out, iters, zero);
      else hipLaunchKernelGGL(mfma32, dim3(grid), dim3(256), 0, 0, out, iters, zero);
      hipDeviceSynchronize();
      const double t0 = now();
      hipEventRecord(e0);
      int n = 0;
      float ms = 0.f;
      while (ms < seconds * 1000.0) {
        for (int r = 0; r < 10; ++r) {
          if (v == 0) hipLaunchKernelGGL(mfma16, dim3(grid), dim3(256), 0, 0, out, iters, zero);
          else hipLaunchKernelGGL(mfma32, dim3(grid), dim3(256), 0, 0, out, iters, zero);
        }
        n += 10;
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      printf("{\"shape\": \"%s\", \"zero_operands\": %d, \"launches\": %d, \"ms\": %.1f, \"tflops\": %.1f, \"t0\": %.2f, \"t1\": %.2f}\n",
             v == 0 ? "16x16x32" : "32x32x16", zero, n, ms, flop_per_launch * n / (ms * 1e-3) / 1e12, t0, now());
      fflush(stdout);
    }
  }
  hipFree(out);
  return 0;
}
