// Fused PreNorm LayerNorm + PreShiftToken (SURVEY K3 + K4).
//
// Forward: x (rows = B*n, D) fp32 residual stream -> y bf16, where y is LN(x) after the token
// shift: text positions take channels [0, D/2) from the previous position; image positions
// (raster, S x S grid) take [0, D/4) from the token above and [D/4, D/2) from the token to the
// left; missing sources are zeros. One wave per source row: it normalises its row once and scatters
// each channel quarter to its destination row, and writes the zeros its own row is owed, so every
// output element is written exactly once (no memset, no second pass).
// Backward: one wave per source row gathers the shifted output grads back, then LN backward, and
// adds the residual-stream grad (dx = g_resid + dLN/dx) so the caller needs no separate add;
// dweight / dbias are reduced deterministically (per-block partial rows -> column_sum) straight
// into the parameters' fp32 grad buffers (GradSink).
#include "common.h"
#include "geom.h"

namespace dalle {

constexpr int LN_BWD_BLOCKS = 512;

// destination position of channel group `grp` (0: [0,D/4), 1: [D/4,D/2), 2: [D/2,D)) of source p,
// or -1 if dropped
__device__ __forceinline__ int shift_dest(const ShiftGeom& g, int p, int grp) {
  if (!g.shift || grp == 2) return p;
  if (p < g.T) return (p + 1 < g.T) ? p + 1 : -1;
  const int k = p - g.T;
  if (grp == 0) return (p + g.S < g.n) ? p + g.S : -1;
  const int col = k % g.S;
  return (col < g.S - 1 && p + 1 < g.n) ? p + 1 : -1;
}

// source position for destination p (inverse map) or -1 (zero)
__device__ __forceinline__ int shift_src(const ShiftGeom& g, int p, int grp) {
  if (!g.shift || grp == 2) return p;
  if (p < g.T) return p >= 1 ? p - 1 : -1;
  const int k = p - g.T;
  if (grp == 0) return (k >= g.S) ? p - g.S : -1;
  return (k % g.S) ? p - 1 : -1;
}

// RES (sublayer boundary of the fused sequential stack): the row is first finished as
// x = res + scale * y_prev (the previous sublayer's LayerScale residual, written to xout), then
// normalised -- one pass over the residual stream instead of scale_residual + ln_shift_fwd.
template <int D, bool RES = false>
__global__ __launch_bounds__(256) void ln_shift_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ bias, __bf16* __restrict__ y,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                           ShiftGeom g, int rows, float eps, const __bf16* __restrict__ yprev,
                                                           const float* __restrict__ sprev, float* __restrict__ xout) {
  constexpr int PER = D / 256;  // float4 per lane
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= rows) return;
  const int row = wave;
  const int b = row / g.n, p = row - b * g.n;
  const float* xr = x + (size_t)row * D;
  f32x4 v[PER];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = *reinterpret_cast<const f32x4*>(xr + 4 * (lane + 64 * j));
    if (RES) {
      const int c = 4 * (lane + 64 * j);
      float yv[4];
      unpack4(*reinterpret_cast<const s16x4*>(yprev + (size_t)row * D + c), yv);
      const f32x4 sv = *reinterpret_cast<const f32x4*>(sprev + c);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[j][i] += sv[i] * yv[i];
      *reinterpret_cast<f32x4*>(xout + (size_t)row * D + c) = v[j];
    }
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) { const float d = v[j][i] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = 4 * (lane + 64 * j);
    const int grp = c < D / 4 ? 0 : (c < D / 2 ? 1 : 2);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + c);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (v[j][i] - mean) * rstd * wv[i] + bv[i];
    const int gsh = (g.shift && p < g.T && grp == 1) ? 0 : grp;  // text: whole first half moves by one
    const int dst = shift_dest(g, p, gsh);
    if (dst >= 0) *reinterpret_cast<s16x4*>(y + ((size_t)b * g.n + dst) * D + c) = pack4(o);
    if (gsh != 2 && g.shift && shift_src(g, p, gsh) < 0) {
      const s16x4 z = {};
      *reinterpret_cast<s16x4*>(y + (size_t)row * D + c) = z;
    }
  }
}

// SR (sublayer boundary of the fused sequential stack): dx is also the upstream grad of the PREVIOUS
// sublayer's LayerScale residual, so the same pass emits its dy_prev = bf16(scale_prev * dx) and the
// column partials [sum dx * y_prev | sum dx] (-> dscale_prev, dbias_prev) into part2 -- no separate
// scale_residual_bwd re-reading dx.
// D <= 1024: held to 256 VGPRs (2 waves per SIMD; the SR form compiled to 258 = 1 wave per SIMD without the
// bound, half the rows in flight of the bandwidth-bound pass)
template <int D, bool SR = false>
__global__ __launch_bounds__(256, D <= 1024 ? 2 : 1) void ln_shift_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const __bf16* __restrict__ dy, const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in, const float* __restrict__ resid,
                                                           float* __restrict__ dx, float* __restrict__ dw, ShiftGeom g,
                                                           int rows, const __bf16* __restrict__ yprev,
                                                           const float* __restrict__ sprev, __bf16* __restrict__ dyprev,
                                                           float* __restrict__ part2) {
  constexpr int PER = D / 256;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int wave0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  float dwa[PER][4] = {}, dba[PER][4] = {};
  float sya[SR ? PER : 1][4] = {}, sga[SR ? PER : 1][4] = {};
  // software pipeline: the next row's x / shifted dy / residual-grad loads are in flight while this
  // row's two wave reductions run (the kernel is latency-bound at 2 waves per SIMD otherwise)
  auto fetch = [&](int row, f32x4 (&xv)[PER], f32x4 (&rv)[PER], s16x4 (&dv)[PER], float& mean, float& rstd) {
    const int b = row / g.n, p = row - b * g.n;
    mean = mean_in[row];
    rstd = rstd_in[row];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = 4 * (lane + 64 * j);
      const int grp = c < D / 4 ? 0 : (c < D / 2 ? 1 : 2);
      const int gsh = (g.shift && p < g.T && grp == 1) ? 0 : grp;
      const int dst = shift_dest(g, p, gsh);
      xv[j] = *reinterpret_cast<const f32x4*>(x + (size_t)row * D + c);
      rv[j] = resid ? *reinterpret_cast<const f32x4*>(resid + (size_t)row * D + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j] = dst >= 0 ? *reinterpret_cast<const s16x4*>(dy + ((size_t)b * g.n + dst) * D + c) : s16x4{0, 0, 0, 0};
    }
  };
  f32x4 xa[PER], ra[PER];
  s16x4 da[PER];
  float ma = 0.f, sa = 0.f;
  if (wave0 < rows) fetch(wave0, xa, ra, da, ma, sa);
  for (int row = wave0; row < rows; row += nwaves) {
    f32x4 xb[PER], rb[PER];
    s16x4 db[PER];
    float mb = 0.f, sb = 0.f;
    if (row + nwaves < rows) fetch(row + nwaves, xb, rb, db, mb, sb);
    const float mean = ma, rstd = sa;
    float xh[PER][4], gy[PER][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = 4 * (lane + 64 * j);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
      float gv[4];
      unpack4(da[j], gv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[j][i] = (xa[j][i] - mean) * rstd;
        gy[j][i] = gv[i] * wv[i];
        dwa[j][i] += gv[i] * xh[j][i];
        dba[j][i] += gv[i];
        s1 += gy[j][i];
        s2 += gy[j][i] * xh[j][i];
      }
    }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = 4 * (lane + 64 * j);
      f32x4 o = ra[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] += rstd * (gy[j][i] - s1 - xh[j][i] * s2);
      *reinterpret_cast<f32x4*>(dx + (size_t)row * D + c) = o;
      if (SR) {
        float yp[4], dp[4];
        unpack4(*reinterpret_cast<const s16x4*>(yprev + (size_t)row * D + c), yp);
        const f32x4 sv = *reinterpret_cast<const f32x4*>(sprev + c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dp[i] = o[i] * sv[i];
          sya[SR ? j : 0][i] += o[i] * yp[i];
          sga[SR ? j : 0][i] += o[i];
        }
        *reinterpret_cast<s16x4*>(dyprev + (size_t)row * D + c) = pack4(dp);
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) { xa[j] = xb[j]; ra[j] = rb[j]; da[j] = db[j]; }
    ma = mb;
    sa = sb;
  }
  // deterministic two-stage reduction of dweight / dbias (no atomics: every workgroup adding into the
  // same D columns is the worst case for float atomics): waves -> LDS -> one partial row per block.
  __shared__ float red[4][2 * D];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = 4 * (lane + 64 * j);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      red[wv][c + i] = dwa[j][i];
      red[wv][D + c + i] = dba[j][i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += blockDim.x)
    dw[(size_t)blockIdx.x * 2 * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  if (SR) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = 4 * (lane + 64 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[wv][c + i] = sya[SR ? j : 0][i];
        red[wv][D + c + i] = sga[SR ? j : 0][i];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * D; c += blockDim.x)
      part2[(size_t)blockIdx.x * 2 * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// sum `nrows` partial rows of width `width` (column-parallel, fixed order)
// 256 threads = 16 columns x 16 row groups (width / 16 workgroups: 128 for the 2 x 1024 LN partials,
// enough to keep every row group's loads in flight at once); 8 independent loads per thread per round;
// the 16 row-group sums are added in a fixed order through LDS, so the result is deterministic.
// The result goes to a GradSink: columns [0, split) -> out0, [split, width) -> out1 (optionally
// multiplied per column by mul1), written or ACCUMULATED into the destination -- the destinations
// are the parameters' fp32 .grad views in the flat arena, so no autograd add kernel follows.
constexpr int CS_COLS = 16, CS_RG = 16;
// blockIdx.y selects one of up to two independent (part, sink) tasks of the same shape: the LN+shift
// backward's two reductions (this sublayer's [dw | db], the previous one's [dscale | dbias]) in one launch
__global__ __launch_bounds__(256) void column_sum_kernel(const float* __restrict__ part0, const float* __restrict__ part1,
                                                         int nrows, int width, GradSink sink0, GradSink sink1) {
  const float* __restrict__ part = blockIdx.y ? part1 : part0;
  const GradSink& sink = blockIdx.y ? sink1 : sink0;
  __shared__ float red[CS_RG][CS_COLS];
  const int cl = threadIdx.x % CS_COLS, rg = threadIdx.x / CS_COLS;
  const int c = blockIdx.x * CS_COLS + cl;
  float s = 0.f;
  if (c < width) {
    int r = rg;
    for (; r + 7 * CS_RG < nrows; r += 8 * CS_RG) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(size_t)(r + CS_RG * u) * width + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; r < nrows; r += CS_RG) s += part[(size_t)r * width + c];
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < width) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < CS_RG; ++k) v += red[k][cl];
    float* dst;
    if (c < sink.split) {
      dst = sink.out0 + c;
    } else {
      if (sink.out1 == nullptr) return;
      dst = sink.out1 + (c - sink.split);
      if (sink.mul1) v *= sink.mul1[c - sink.split];
    }
    *dst = sink.accumulate ? *dst + v : v;
  }
}

void column_sum(const float* part, int nrows, int width, const GradSink& sink, hipStream_t st) {
  hipLaunchKernelGGL(column_sum_kernel, dim3((width + CS_COLS - 1) / CS_COLS, 1), dim3(256), 0, st, part, part, nrows, width, sink,
                     sink);
}
static void column_sum2(const float* part0, const GradSink& sink0, const float* part1, const GradSink& sink1, int nrows, int width,
                        hipStream_t st) {
  hipLaunchKernelGGL(column_sum_kernel, dim3((width + CS_COLS - 1) / CS_COLS, 2), dim3(256), 0, st, part0, part1, nrows, width,
                     sink0, sink1);
}
void column_sum(const float* part, int nrows, int width, float* out, hipStream_t st) {
  column_sum(part, nrows, width, GradSink{out, nullptr, nullptr, width, 0}, st);
}

// plain LayerNorm variants for the final norm (no shift): same kernels with shift = 0

template <int D>
static void launch_fwd(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd, const ShiftGeom& g,
                       int rows, float eps, hipStream_t st, const void* yprev, const float* sprev, float* xout) {
  if (yprev)
    hipLaunchKernelGGL((ln_shift_fwd_kernel<D, true>), dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, (__bf16*)y, mean, rstd, g,
                       rows, eps, (const __bf16*)yprev, sprev, xout);
  else
    hipLaunchKernelGGL((ln_shift_fwd_kernel<D, false>), dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, (__bf16*)y, mean, rstd,
                       g, rows, eps, (const __bf16*)nullptr, (const float*)nullptr, (float*)nullptr);
}

template <int D>
static void launch_bwd(const float* x, const float* w, const void* dy, const float* mean, const float* rstd, const float* resid,
                       float* dx, float* part, const GradSink& sink, const ShiftGeom& g, int rows, hipStream_t st,
                       const void* yprev, const float* sprev, void* dyprev, float* part2, const GradSink* sink2) {
  // part (and part2) are (LN_BWD_BLOCKS x 2D) partial buffers; the sink receives [dw | db], sink2 [dscale | dbias]_prev
  int blocks = (rows + 3) / 4;
  if (blocks > LN_BWD_BLOCKS) blocks = LN_BWD_BLOCKS;
  if (yprev) {
    hipLaunchKernelGGL((ln_shift_bwd_kernel<D, true>), dim3(blocks), dim3(256), 0, st, x, w, (const __bf16*)dy, mean, rstd, resid,
                       dx, part, g, rows, (const __bf16*)yprev, sprev, (__bf16*)dyprev, part2);
    column_sum2(part, sink, part2, *sink2, blocks, 2 * D, st);  // both reductions, one launch
    return;
  } else {
    hipLaunchKernelGGL((ln_shift_bwd_kernel<D, false>), dim3(blocks), dim3(256), 0, st, x, w, (const __bf16*)dy, mean, rstd, resid,
                       dx, part, g, rows, (const __bf16*)nullptr, (const float*)nullptr, (__bf16*)nullptr, (float*)nullptr);
  }
  column_sum(part, blocks, 2 * D, sink, st);
}

// yprev / sprev / xout (all or none): the fused boundary x = res + sprev * yprev (see ln_shift_fwd_kernel RES)
bool ln_shift_fwd(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd, const ShiftGeom& g, int rows,
                  int D, float eps, hipStream_t st, const void* yprev, const float* sprev, float* xout) {
  switch (D) {
    case 256: launch_fwd<256>(x, w, b, y, mean, rstd, g, rows, eps, st, yprev, sprev, xout); return true;
    case 512: launch_fwd<512>(x, w, b, y, mean, rstd, g, rows, eps, st, yprev, sprev, xout); return true;
    case 1024: launch_fwd<1024>(x, w, b, y, mean, rstd, g, rows, eps, st, yprev, sprev, xout); return true;
    case 2048: launch_fwd<2048>(x, w, b, y, mean, rstd, g, rows, eps, st, yprev, sprev, xout); return true;
    default: return false;
  }
}

// yprev / sprev / dyprev / part2 / sink2 (all or none): the fused boundary (see ln_shift_bwd_kernel SR)
bool ln_shift_bwd(const float* x, const float* w, const void* dy, const float* mean, const float* rstd, const float* resid,
                  float* dx, float* part, const GradSink& sink, const ShiftGeom& g, int rows, int D, hipStream_t st,
                  const void* yprev, const float* sprev, void* dyprev, float* part2, const GradSink* sink2) {
  switch (D) {
    case 256: launch_bwd<256>(x, w, dy, mean, rstd, resid, dx, part, sink, g, rows, st, yprev, sprev, dyprev, part2, sink2); return true;
    case 512: launch_bwd<512>(x, w, dy, mean, rstd, resid, dx, part, sink, g, rows, st, yprev, sprev, dyprev, part2, sink2); return true;
    case 1024: launch_bwd<1024>(x, w, dy, mean, rstd, resid, dx, part, sink, g, rows, st, yprev, sprev, dyprev, part2, sink2); return true;
    case 2048: launch_bwd<2048>(x, w, dy, mean, rstd, resid, dx, part, sink, g, rows, st, yprev, sprev, dyprev, part2, sink2); return true;
    default: return false;
  }
}

}  // namespace dalle
