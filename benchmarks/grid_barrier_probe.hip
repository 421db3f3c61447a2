// Prices the building block of a persistent (one workgroup per CU) decode-layer kernel: a grid-wide
// barrier between phases, against what the decode chain pays today -- one dependent kernel launch per
// phase (profiles/r3_decode_reference_b64_top_kernels.txt: 5-7 us per skinny / LN kernel).
//
//   build: hipcc --offload-arch=gfx950 -O3 -o benchmarks/grid_barrier_probe benchmarks/grid_barrier_probe.hip
//   run:   timeout -k 10 60 benchmarks/grid_barrier_probe
//
// Every launch is cooperative (hipLaunchCooperativeKernel refuses a grid that cannot be co-resident) and
// every spin is bounded (a wave that waits 2^22 polls gives up, flags it and opens every later barrier), so no configuration can hang.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

struct Bar {
  unsigned* count;
  unsigned* gen;
  unsigned* timeout;
};

// sense-by-generation barrier: thread 0 of each workgroup reads the generation, arrives (device-scope
// fetch-add); the last arrival resets the count and publishes generation + 1 (release), the others poll it
__device__ __forceinline__ void grid_barrier(const Bar& b, unsigned nblocks) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived = __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nblocks - 1) {
      __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;  // a timed-out barrier stays open for every later one (the grid drains)
      while (__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g &&
             __hip_atomic_load(b.timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (++spins > (1u << 22)) {
          __hip_atomic_fetch_add(b.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

// two-level form: workgroups arrive on one of 8 group counters (blockIdx % 8: the XCD a workgroup is
// dispatched to), the last of each group arrives on the top counter; fewer same-address atomics in a row
__device__ __forceinline__ void grid_barrier2(const Bar& b, unsigned nblocks, int sleepy) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned grp = blockIdx.x & 7, per = nblocks / 8;
    unsigned* gc = b.count + 32 * (1 + grp);  // separate 128-B lines
    bool release = false;
    if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == per - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      release = __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 7;
    }
    if (release) {
      __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g &&
             __hip_atomic_load(b.timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (sleepy) __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 22)) {
          __hip_atomic_fetch_add(b.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void barrier2_kernel(Bar b, int iters, int sleepy) {
  for (int it = 0; it < iters; ++it) grid_barrier2(b, gridDim.x, sleepy);
}

// `iters` phases; in each, every workgroup streams `bytes_per_wg` of a read-only buffer (the phase's
// weight slice in a real decode layer) and writes one float, then all meet at the barrier
__global__ __launch_bounds__(256) void phases_kernel(Bar b, int iters, const float4* __restrict__ src, size_t n4, int per_wg4,
                                                     float* __restrict__ out) {
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (per_wg4 > 0) {
      const size_t base = ((size_t)(it * gridDim.x + blockIdx.x) * per_wg4) % (n4 - per_wg4);
      for (int i = threadIdx.x; i < per_wg4; i += 256) {
        const float4 v = src[base + i];
        acc += v.x + v.y + v.z + v.w;
      }
    }
    grid_barrier(b, gridDim.x);
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

// the launch-per-phase baseline: the same phase work, one kernel per phase
__global__ __launch_bounds__(256) void one_phase_kernel(int it, const float4* __restrict__ src, size_t n4, int per_wg4,
                                                        float* __restrict__ out) {
  float acc = 0.f;
  if (per_wg4 > 0) {
    const size_t base = ((size_t)(it * gridDim.x + blockIdx.x) * per_wg4) % (n4 - per_wg4);
    for (int i = threadIdx.x; i < per_wg4; i += 256) {
      const float4 v = src[base + i];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

int main() {
  int dev = 0, ncu = 0, coop = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phases_kernel, 256, 0));
  printf("{\"cus\": %d, \"cooperative\": %d, \"max_wg_per_cu\": %d}\n", ncu, coop, per_cu);
  if (!coop) return 1;

  const size_t nbytes = 256ull << 20;  // larger than the 256 MB MALL: phase reads come from HBM
  const size_t n4 = nbytes / 16;
  float4* src;
  float* out;
  Bar b;
  CK(hipMalloc(&src, nbytes));
  CK(hipMemset(src, 0, nbytes));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMalloc(&b.count, 4096));
  CK(hipMalloc(&b.gen, 4));
  CK(hipMalloc(&b.timeout, 4));
  CK(hipMemset(b.count, 0, 4096));
  CK(hipMemset(b.gen, 0, 4));
  CK(hipMemset(b.timeout, 0, 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  const int iters = 2000;
  for (int grid : {ncu, 2 * ncu}) {
    for (int sleepy : {0, 1}) {
      int it = iters;
      void* args[] = {&b, &it, &sleepy};
      CK(hipLaunchCooperativeKernel((const void*)barrier2_kernel, dim3(grid), dim3(256), args, 0, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)barrier2_kernel, dim3(grid), dim3(256), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned to = 0;
      CK(hipMemcpy(&to, b.timeout, 4, hipMemcpyDeviceToHost));
      printf("{\"grid\": %d, \"two_level_barrier\": true, \"sleepy_poll\": %d, \"us_per_barrier\": %.2f, \"spin_timeouts\": %u}\n",
             grid, sleepy, ms * 1e3 / iters, to);
      fflush(stdout);
    }
  }
  for (int grid : {ncu, 2 * ncu}) {
    if (grid > ncu * per_cu) continue;
    for (int kb : {0, 8, 32, 128}) {  // bytes streamed per workgroup per phase
      int per_wg4 = kb * 1024 / 16;
      int it = iters;
      void* args[] = {&b, &it, &src, (void*)&n4, &per_wg4, &out};
      // warm-up
      CK(hipLaunchCooperativeKernel((const void*)phases_kernel, dim3(grid), dim3(256), args, 0, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)phases_kernel, dim3(grid), dim3(256), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms_bar = 0.f;
      CK(hipEventElapsedTime(&ms_bar, e0, e1));

      // launch-per-phase baseline, plain stream and hipGraph
      for (int i = 0; i < 50; ++i)
        hipLaunchKernelGGL(one_phase_kernel, dim3(grid), dim3(256), 0, st, i, (const float4*)src, n4, per_wg4, out);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(one_phase_kernel, dim3(grid), dim3(256), 0, st, i, (const float4*)src, n4, per_wg4, out);
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms_launch = 0.f;
      CK(hipEventElapsedTime(&ms_launch, e0, e1));

      hipGraph_t g;
      hipGraphExec_t ge;
      const int gi = 500;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < gi; ++i)
        hipLaunchKernelGGL(one_phase_kernel, dim3(grid), dim3(256), 0, st, i, (const float4*)src, n4, per_wg4, out);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < iters / gi; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms_graph = 0.f;
      CK(hipEventElapsedTime(&ms_graph, e0, e1));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));

      unsigned to = 0;
      CK(hipMemcpy(&to, b.timeout, 4, hipMemcpyDeviceToHost));
      printf("{\"grid\": %d, \"kb_per_wg_per_phase\": %d, \"phase_MB\": %.2f, \"us_per_phase_barrier\": %.2f, "
             "\"us_per_phase_launch\": %.2f, \"us_per_phase_graph\": %.2f, \"spin_timeouts\": %u}\n",
             grid, kb, grid * kb / 1024.0, ms_bar * 1e3 / iters, ms_launch * 1e3 / iters, ms_graph * 1e3 / iters, to);
      fflush(stdout);
    }
  }
  return 0;
}
