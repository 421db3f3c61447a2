// Memory-bound fused elementwise kernels (SURVEY K9 GEGLU, K8/K10 LayerScale+residual, K17 finite
// checks). All bf16 traffic is 16 bytes per lane (Guideline 13).
#include "common.h"

namespace dalle {

void column_sum(const float* part, int nrows, int width, float* out, hipStream_t st);
constexpr int SR_BWD_BLOCKS = 512;

// GEGLU: h (M, 2F) -> out (M, F) = h[:, :F] * gelu(h[:, F:])   (exact erf GELU)
__global__ void geglu_fwd_kernel(const __bf16* __restrict__ h, __bf16* __restrict__ out, long M, int F) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = F / 8;
  if (gid >= M * per_row) return;
  const long r = gid / per_row;
  const int c = (gid - r * per_row) * 8;
  float a[8], gg[8], o[8];
  unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + c), a);
  unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + F + c), gg);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = a[i] * gelu_erf(gg[i]);
  *reinterpret_cast<s16x8*>(out + r * F + c) = pack8(o);
}

__global__ void geglu_bwd_kernel(const __bf16* __restrict__ h, const __bf16* __restrict__ dout, __bf16* __restrict__ dh,
                                 long M, int F) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = F / 8;
  if (gid >= M * per_row) return;
  const long r = gid / per_row;
  const int c = (gid - r * per_row) * 8;
  float a[8], gg[8], d[8], da[8], dg[8];
  unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + c), a);
  unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + F + c), gg);
  unpack8(*reinterpret_cast<const s16x8*>(dout + r * F + c), d);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    da[i] = d[i] * gelu_erf(gg[i]);
    dg[i] = d[i] * a[i] * gelu_erf_grad(gg[i]);
  }
  *reinterpret_cast<s16x8*>(dh + r * 2 * F + c) = pack8(da);
  *reinterpret_cast<s16x8*>(dh + r * 2 * F + F + c) = pack8(dg);
}

// x (fp32, M x D) += scale[D] * y (bf16)   -- LayerScale fused into the residual add, in place
__global__ void scale_residual_kernel(float* __restrict__ x, const __bf16* __restrict__ y, const float* __restrict__ scale,
                                      long M, int D) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = D / 8;
  if (gid >= M * per_row) return;
  const long r = gid / per_row;
  const int c = (gid - r * per_row) * 8;
  float yv[8];
  unpack8(*reinterpret_cast<const s16x8*>(y + r * D + c), yv);
  f32x4* xp = reinterpret_cast<f32x4*>(x + r * D + c);
  const f32x4* sp = reinterpret_cast<const f32x4*>(scale + c);
  f32x4 x0 = xp[0], x1 = xp[1];
  const f32x4 s0 = sp[0], s1 = sp[1];
#pragma unroll
  for (int i = 0; i < 4; ++i) { x0[i] += s0[i] * yv[i]; x1[i] += s1[i] * yv[4 + i]; }
  xp[0] = x0;
  xp[1] = x1;
}

// dy = bf16(scale * g); dscale partials: per block column sums of g * y -> atomics into dscale
__global__ __launch_bounds__(256) void scale_residual_bwd_kernel(const float* __restrict__ g, const __bf16* __restrict__ y,
                                                                 const float* __restrict__ scale, __bf16* __restrict__ dy,
                                                                 float* __restrict__ dscale, long M, int D) {
  // each thread owns 8 consecutive columns and walks rows with a grid stride
  const int cols8 = D / 8;
  const int tcol = threadIdx.x % cols8;
  const int rows_per_iter = blockDim.x / cols8;
  const int trow = threadIdx.x / cols8;
  const bool on = trow < rows_per_iter;
  const int c = tcol * 8;
  float acc[8] = {};
  float sc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sc[i] = scale[c + i];
  for (long r = (long)blockIdx.x * rows_per_iter + trow; on && r < M; r += (long)gridDim.x * rows_per_iter) {
    const f32x4* gp = reinterpret_cast<const f32x4*>(g + r * D + c);
    const f32x4 g0 = gp[0], g1 = gp[1];
    float yv[8], o[8];
    unpack8(*reinterpret_cast<const s16x8*>(y + r * D + c), yv);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] += g0[i] * yv[i];
      acc[4 + i] += g1[i] * yv[4 + i];
      o[i] = g0[i] * sc[i];
      o[4 + i] = g1[i] * sc[4 + i];
    }
    *reinterpret_cast<s16x8*>(dy + r * D + c) = pack8(o);
  }
  // deterministic reduction: threads of one column -> LDS -> one partial row per block (no atomics)
  __shared__ float red[256 * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x * 8 + i] = on ? acc[i] : 0.f;
  __syncthreads();
  if (on && trow == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float sum = 0.f;
      for (int r = 0; r < rows_per_iter; ++r) sum += red[(r * cols8 + tcol) * 8 + i];
      dscale[(size_t)blockIdx.x * D + c + i] = sum;
    }
  }
}

// Non-finite detector over an fp32 buffer: flag[0] = 1 if any element is NaN/Inf
__global__ void nonfinite_kernel(const float* __restrict__ x, long n, int* __restrict__ flag) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long stride = (long)gridDim.x * blockDim.x * 4;
  bool bad = false;
  for (; i + 3 < n; i += stride) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
    bad |= !isfinite(v[0]) | !isfinite(v[1]) | !isfinite(v[2]) | !isfinite(v[3]);
  }
  for (; i < n; ++i) bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void geglu_fwd(const void* h, void* out, long M, int F, hipStream_t st) {
  const long t = M * (F / 8);
  hipLaunchKernelGGL(geglu_fwd_kernel, dim3((t + 255) / 256), dim3(256), 0, st, (const __bf16*)h, (__bf16*)out, M, F);
}
void geglu_bwd(const void* h, const void* dout, void* dh, long M, int F, hipStream_t st) {
  const long t = M * (F / 8);
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3((t + 255) / 256), dim3(256), 0, st, (const __bf16*)h, (const __bf16*)dout,
                     (__bf16*)dh, M, F);
}
void scale_residual(float* x, const void* y, const float* scale, long M, int D, hipStream_t st) {
  const long t = M * (D / 8);
  hipLaunchKernelGGL(scale_residual_kernel, dim3((t + 255) / 256), dim3(256), 0, st, x, (const __bf16*)y, scale, M, D);
}
void scale_residual_bwd(const float* g, const void* y, const float* scale, void* dy, float* dscale, long M, int D,
                        hipStream_t st) {
  // dscale points at [SR_BWD_BLOCKS x D partial rows | D outputs]
  const int blocks = SR_BWD_BLOCKS;
  hipLaunchKernelGGL(scale_residual_bwd_kernel, dim3(blocks), dim3(256), 0, st, g, (const __bf16*)y, scale, (__bf16*)dy, dscale,
                     M, D);
  column_sum(dscale, blocks, D, dscale + (size_t)blocks * D, st);
}
void nonfinite(const float* x, long n, int* flag, hipStream_t st) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(nonfinite_kernel, dim3(blocks), dim3(256), 0, st, x, n, flag);
}

}  // namespace dalle
