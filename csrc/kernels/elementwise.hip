// Memory-bound fused elementwise kernels (SURVEY K9 GEGLU, K8/K10 LayerScale+residual, K17 finite
// checks). All bf16 traffic is 16 bytes per lane (Guideline 13).
#include "common.h"
#include "geom.h"

namespace dalle {

void column_sum(const float* part, int nrows, int width, const GradSink& sink, hipStream_t st);
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
    float ge, gr;
    gelu_and_grad(gg[i], ge, gr);
    da[i] = d[i] * ge;
    dg[i] = d[i] * a[i] * gr;
  }
  *reinterpret_cast<s16x8*>(dh + r * 2 * F + c) = pack8(da);
  *reinterpret_cast<s16x8*>(dh + r * 2 * F + F + c) = pack8(dg);
}

// GEGLU backward fused with the FF-in bias gradient: grid (row blocks, F/2048 column blocks); each
// thread owns 8 columns j (and F+j), walks its rows, and leaves one partial [2F] row per row block
// (column-summed afterwards) -- no separate reduction over the (M, 2F) gradient.
__global__ __launch_bounds__(256) void geglu_bwd_bias_kernel(const __bf16* __restrict__ h, const __bf16* __restrict__ dout,
                                                             __bf16* __restrict__ dh, float* __restrict__ part, long M, int F) {
  const int j = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (j >= F) return;
  float sa[8] = {}, sg[8] = {};
  // U rows per iteration: all 3*U 16-byte loads are issued before any math (memory-level parallelism)
  constexpr int U = 4;
  const long step = gridDim.x;
  long r = blockIdx.x;
  for (; r + (U - 1) * step < M; r += U * step) {
    s16x8 va[U], vg[U], vd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long rr = r + u * step;
      va[u] = *reinterpret_cast<const s16x8*>(h + rr * 2 * F + j);
      vg[u] = *reinterpret_cast<const s16x8*>(h + rr * 2 * F + F + j);
      vd[u] = *reinterpret_cast<const s16x8*>(dout + rr * F + j);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long rr = r + u * step;
      float a[8], gg[8], d[8], da[8], dg[8];
      unpack8(va[u], a);
      unpack8(vg[u], gg);
      unpack8(vd[u], d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float ge, gr;
        gelu_and_grad(gg[i], ge, gr);
        da[i] = d[i] * ge;
        dg[i] = d[i] * a[i] * gr;
      }
      const s16x8 pa = pack8(da), pg = pack8(dg);
      *reinterpret_cast<s16x8*>(dh + rr * 2 * F + j) = pa;
      *reinterpret_cast<s16x8*>(dh + rr * 2 * F + F + j) = pg;
      float ra[8], rg[8];
      unpack8(pa, ra);  // bias grad of the values actually propagated (bf16), as a GEMM epilogue would
      unpack8(pg, rg);
#pragma unroll
      for (int i = 0; i < 8; ++i) { sa[i] += ra[i]; sg[i] += rg[i]; }
    }
  }
  for (; r < M; r += step) {
    float a[8], gg[8], d[8], da[8], dg[8];
    unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + j), a);
    unpack8(*reinterpret_cast<const s16x8*>(h + r * 2 * F + F + j), gg);
    unpack8(*reinterpret_cast<const s16x8*>(dout + r * F + j), d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float ge, gr;
      gelu_and_grad(gg[i], ge, gr);
      da[i] = d[i] * ge;
      dg[i] = d[i] * a[i] * gr;
    }
    const s16x8 pa = pack8(da), pg = pack8(dg);
    *reinterpret_cast<s16x8*>(dh + r * 2 * F + j) = pa;
    *reinterpret_cast<s16x8*>(dh + r * 2 * F + F + j) = pg;
    float ra[8], rg[8];
    unpack8(pa, ra);
    unpack8(pg, rg);
#pragma unroll
    for (int i = 0; i < 8; ++i) { sa[i] += ra[i]; sg[i] += rg[i]; }
  }
  float* prow = part + (size_t)blockIdx.x * 2 * F;
#pragma unroll
  for (int i = 0; i < 8; ++i) { prow[j + i] = sa[i]; prow[F + j + i] = sg[i]; }
}

// x (fp32, M x D) += scale[D] * y (bf16)   -- LayerScale fused into the residual add, in place
__global__ void scale_residual_kernel(const float* x, const __bf16* __restrict__ y, const float* __restrict__ scale,
                                      float* out, long M, int D) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = D / 8;
  if (gid >= M * per_row) return;
  const long r = gid / per_row;
  const int c = (gid - r * per_row) * 8;
  float yv[8];
  unpack8(*reinterpret_cast<const s16x8*>(y + r * D + c), yv);
  const f32x4* xp = reinterpret_cast<const f32x4*>(x + r * D + c);
  const f32x4* sp = reinterpret_cast<const f32x4*>(scale + c);
  f32x4 x0 = xp[0], x1 = xp[1];
  const f32x4 s0 = sp[0], s1 = sp[1];
#pragma unroll
  for (int i = 0; i < 4; ++i) { x0[i] += s0[i] * yv[i]; x1[i] += s1[i] * yv[4 + i]; }
  f32x4* op = reinterpret_cast<f32x4*>(out + r * D + c);
  op[0] = x0;
  op[1] = x1;
}

// dy = bf16(scale * g); per block partial column sums of g * y and of g (reduced by column_sum)
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
  float acc[8] = {}, gsum[8] = {};
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
      gsum[i] += g0[i];
      gsum[4 + i] += g1[i];
      o[i] = g0[i] * sc[i];
      o[4 + i] = g1[i] * sc[4 + i];
    }
    *reinterpret_cast<s16x8*>(dy + r * D + c) = pack8(o);
  }
  // deterministic reduction: threads of one column -> LDS -> one partial row [sum g*y | sum g] per block
  __shared__ float red[256 * 8];
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[threadIdx.x * 8 + i] = on ? (pass ? gsum[i] : acc[i]) : 0.f;
    __syncthreads();
    if (on && trow == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float sum = 0.f;
        for (int r = 0; r < rows_per_iter; ++r) sum += red[(r * cols8 + tcol) * 8 + i];
        dscale[(size_t)blockIdx.x * 2 * D + pass * D + c + i] = sum;
      }
    }
    __syncthreads();
  }
}

// Split-K GEMM reduction: acc (n floats) [+]= sum_s part[s] (part = s x n, fp32), fixed summation
// order (deterministic). The weight-grad GEMMs have a long reduction dimension (B x 1280 tokens) and a
// small output (d x d): hipBLASLt fills 256 CUs only when that reduction is split into a batch of
// GEMMs, whose fp32 partial outputs this kernel folds into the fp32 grad arena.
__global__ void splitk_accum_kernel(const float* __restrict__ part, float* __restrict__ acc, long n, int s, int accumulate) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  f32x4 v = accumulate ? *reinterpret_cast<const f32x4*>(acc + i) : f32x4{0.f, 0.f, 0.f, 0.f};
  // the partial loads of up to 8 slabs are issued together (one memory round trip per 8 slabs)
  int k = 0;
  for (; k + 8 <= s; k += 8) {
    f32x4 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = *reinterpret_cast<const f32x4*>(part + (size_t)(k + u) * n + i);
#pragma unroll
    for (int u = 0; u < 8; ++u) { v[0] += p[u][0]; v[1] += p[u][1]; v[2] += p[u][2]; v[3] += p[u][3]; }
  }
  for (; k < s; ++k) {
    const f32x4 p = *reinterpret_cast<const f32x4*>(part + (size_t)k * n + i);
    v[0] += p[0]; v[1] += p[1]; v[2] += p[2]; v[3] += p[3];
  }
  *reinterpret_cast<f32x4*>(acc + i) = v;
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

// x[:] = 0 if flag != 0 (the flag written by nonfinite_kernel earlier on the same stream): the
// trainer's "zero the accumulated grads only if they are not finite" without a host round trip
__global__ void zero_if_flag_kernel(float* __restrict__ x, long n, const int* __restrict__ flag) {
  if (flag[0] == 0) return;
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long stride = (long)gridDim.x * blockDim.x * 4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (; i + 3 < n; i += stride) *reinterpret_cast<f32x4*>(x + i) = z;
  for (; i < n; ++i) x[i] = 0.f;
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
constexpr int GEGLU_ROW_BLOCKS = 512;  // must match the partial buffer rows allocated in binding.cpp
void geglu_bwd_bias(const void* h, const void* dout, void* dh, float* part, const GradSink& dbias, long M, int F,
                    hipStream_t st) {
  dim3 grid(GEGLU_ROW_BLOCKS, (F / 8 + 255) / 256);
  hipLaunchKernelGGL(geglu_bwd_bias_kernel, grid, dim3(256), 0, st, (const __bf16*)h, (const __bf16*)dout, (__bf16*)dh, part, M, F);
  column_sum(part, GEGLU_ROW_BLOCKS, 2 * F, dbias, st);
}
void scale_residual(const float* x, const void* y, const float* scale, float* out, long M, int D, hipStream_t st) {
  const long t = M * (D / 8);
  hipLaunchKernelGGL(scale_residual_kernel, dim3((t + 255) / 256), dim3(256), 0, st, x, (const __bf16*)y, scale, out, M, D);
}
void scale_residual_bwd(const float* g, const void* y, const float* scale, void* dy, float* part, const GradSink& sink, long M,
                        int D, hipStream_t st) {
  // part: SR_BWD_BLOCKS x 2D partial rows [g*y | g]; the sink receives (sum_rows g*y, sum_rows g [* mul1])
  const int blocks = SR_BWD_BLOCKS;
  hipLaunchKernelGGL(scale_residual_bwd_kernel, dim3(blocks), dim3(256), 0, st, g, (const __bf16*)y, scale, (__bf16*)dy, part, M,
                     D);
  column_sum(part, blocks, 2 * D, sink, st);
}
void splitk_accum(const float* part, float* acc, long n, int s, int accumulate, hipStream_t st) {
  const long t = n / 4;
  hipLaunchKernelGGL(splitk_accum_kernel, dim3((t + 255) / 256), dim3(256), 0, st, part, acc, n, s, accumulate);
}
void nonfinite(const float* x, long n, int* flag, hipStream_t st) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(nonfinite_kernel, dim3(blocks), dim3(256), 0, st, x, n, flag);
}

void zero_if_flag(float* x, long n, const int* flag, hipStream_t st) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(zero_if_flag_kernel, dim3(blocks), dim3(256), 0, st, x, n, flag);
}

// fp32 W (R x C) -> bf16 W^T (C x R) in one pass: the transposed operand copy of the input-gradient GEMMs
// (hip_ops.bf16_weight_t). 32 x 32 tiles through LDS (row stride 33: conflict-free column reads); reads
// and writes are both row-contiguous across the 32 lanes of a tile row. Replaces a cast kernel plus
// a strided elementwise copy (~25 us per 8 MB weight, measured) with one ~2 us pass.
__global__ __launch_bounds__(256) void transpose_cast_bf16_kernel(const float* __restrict__ w, __bf16* __restrict__ wt,
                                                                  int R, int C) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    tile[ty + k][tx] = (r < R && c < C) ? w[(size_t)r * C + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (c < C && r < R) wt[(size_t)c * R + r] = (__bf16)tile[tx][ty + k];
  }
}

void transpose_cast_bf16(const float* w, void* wt, int R, int C, hipStream_t st) {
  hipLaunchKernelGGL(transpose_cast_bf16_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, st, w, (__bf16*)wt, R, C);
}

// bf16 X (R x C) -> X^T (C x R): the token-contiguous copy of a saved GEMM input (hip_ops WGRAD_XT). The
// weight-grad product g^T x runs 18-33 % faster on hipBLASLt when x arrives token-contiguous
// (profiles/r3s5_wgrad_nt_vs_tn_m81920.txt), so the LN output is kept transposed for the backward.
// 64 x 64 tiles through LDS (row stride 66 bf16: the column gathers spread over the banks); every global
// access is a 16-byte vector, 8 lanes per 128-byte tile row.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ xt, int R,
                                                             int C) {
  __shared__ uint16_t tile[64][66];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const int seg = threadIdx.x & 7, row = threadIdx.x >> 3;  // 8 x 16-byte segments per row, 32 rows per pass
#pragma unroll
  for (int k = 0; k < 64; k += 32) {
    const uint4 v = *reinterpret_cast<const uint4*>(x + (size_t)(r0 + row + k) * C + c0 + 8 * seg);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      tile[row + k][8 * seg + 2 * i] = (uint16_t)(w[i] & 0xffffu);
      tile[row + k][8 * seg + 2 * i + 1] = (uint16_t)(w[i] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 64; k += 32) {
    const int c = row + k;  // output row (input column)
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)tile[8 * seg + 2 * i][c] | ((uint32_t)tile[8 * seg + 2 * i + 1][c] << 16);
    *reinterpret_cast<uint4*>(xt + (size_t)(c0 + c) * R + r0 + 8 * seg) = uint4{w[0], w[1], w[2], w[3]};
  }
}

void transpose_bf16(const void* x, void* xt, int R, int C, hipStream_t st) {
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(C / 64, R / 64), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)xt, R, C);
}

}  // namespace dalle
