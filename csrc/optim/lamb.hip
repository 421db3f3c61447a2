// Fused multi-tensor LAMB with blockwise 8-bit (bitsandbytes dynamic-map) or fp32 moments over a
// flat parameter arena. No host synchronisation anywhere:
//
//  1. grad_sumsq    : per-4096-block partial sums of g^2                       (one launch)
//  2. clip_coef     : total norm -> min(1, max_norm / (norm + 1e-6)) on device (1 workgroup)
//  3. lamb_pass<0> : per block: g *= coef; dequant m,v (code[q] * absmax); Adam moments;
//                     delta = m/(sqrt(v)+eps) + wd*p; per-block partial sums of delta^2 and p^2
//  4. lamb_trust    : per tensor: sum its block partials -> trust = clamp(|p|,0,c)/|delta| (1 if 0)
//  5. lamb_pass<1>  : the same moments/delta recomputed; p -= lr_t * trust_t * delta; new block
//                     absmax; nearest-code requant (binary search in LDS) / fp32 store of m, v
//
// Each 4096-element block belongs to exactly one tensor (the arena aligns tensors to 4096), which is
// exactly bnb's per-tensor blockwise layout, so the uint8 states / absmax are bnb-compatible.
#include "../kernels/common.h"

namespace dalle {

constexpr int QBLOCK = 4096;

__global__ __launch_bounds__(256) void grad_sumsq_kernel(const float* __restrict__ g, float* __restrict__ partial, long n) {
  __shared__ float red[8];
  const long base = (long)blockIdx.x * QBLOCK;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long e = base + 4 * (threadIdx.x + 256 * j);
    if (e < n) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(g + e);
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    }
  }
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void clip_coef_kernel(const float* __restrict__ partial, int nblocks, float max_norm,
                                                        float* __restrict__ coef_out, float* __restrict__ norm_out) {
  __shared__ float red[8];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblocks; i += 256) s += partial[i];
  float fs = block_sum_256((float)s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(fs);
    norm_out[0] = norm;
    float c = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.0f;
    coef_out[0] = c < 1.0f ? c : 1.0f;
  }
}

struct LambParams {
  float beta1, beta2, eps;
  int use_clip;
};

__device__ __forceinline__ int nearest_code(const float* code, float x) {
  // lower_bound over 256 sorted entries
  int lo = 0, hi = 256;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int mid = (lo + hi) >> 1;
    if (code[mid] < x) lo = mid + 1; else hi = mid;
  }
  int idx = lo < 1 ? 1 : (lo > 255 ? 255 : lo);
  const float a = code[idx - 1], b = code[idx];
  return (fabsf(x - a) <= fabsf(b - x)) ? idx - 1 : idx;
}

// One 4096-element block: dequantise / load the moments of its tensor's mode, apply the clipped
// gradient. The updated moments stay in registers (16 per lane); `APPLY` selects the pass:
//   APPLY = false : per-block partial sums of delta^2 and p^2 (nothing is written but the partials)
//   APPLY = true  : the SAME arithmetic again (bit-identical moments and delta), then
//                   p -= lr_t * trust_t * delta and the new moments are stored (requantised for 8-bit)
// Recomputing instead of storing delta between the passes keeps the optimizer state at exactly the
// reference's footprint (uint8 m, v + fp32 absmax per block for 8-bit tensors; fp32 m, v only for the
// small fp32-state tensors) with the same HBM traffic as a stored delta (26 vs 28 B/param).
// State arrays are compact per mode: block `blk` of the arena owns slot `bslot[blk]` of its mode's
// array (8-bit: q1/q2/absmax, fp32: m32/v32).
template <bool APPLY>
__global__ __launch_bounds__(256) void lamb_pass_kernel(
    float* __restrict__ p, const float* __restrict__ g, uint8_t* __restrict__ q1, uint8_t* __restrict__ q2,
    float* __restrict__ absmax1, float* __restrict__ absmax2, float* __restrict__ m32, float* __restrict__ v32,
    const float* __restrict__ code1, const float* __restrict__ code2, const int* __restrict__ block_tensor,
    const int* __restrict__ bslot, const long* __restrict__ tstart, const long* __restrict__ tsize,
    const int* __restrict__ tmode, const float* __restrict__ twd, const float* __restrict__ coef_ptr,
    float* __restrict__ partial, const float* __restrict__ tlr, const float* __restrict__ trust, LambParams hp) {
  __shared__ float c1[256], c2[256];
  __shared__ float red[8];
  const int tid = threadIdx.x;
  c1[tid] = code1[tid];
  c2[tid] = code2[tid];
  const long blk = blockIdx.x;
  const int t = block_tensor[blk];
  const long tend = tstart[t] + tsize[t];
  const int mode8 = tmode[t];
  const long slot = bslot[blk];
  const float wd = twd[t];
  const float coef = hp.use_clip ? coef_ptr[0] : 1.0f;
  const long base = blk * QBLOCK;      // arena offset of the block (params, grads)
  const long sbase = slot * QBLOCK;    // offset of the block in its mode's state array
  __syncthreads();

  float mv[16], vv[16], pv[16];
  bool valid[16];
  float am1 = 0.f, am2 = 0.f;
  if (mode8) { am1 = absmax1[slot]; am2 = absmax2[slot]; }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long o = 4 * (tid + 256 * j);
    const long e = base + o;
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + e);
    const f32x4 pp = *reinterpret_cast<const f32x4*>(p + e);
    float m4[4], v4[4];
    if (mode8) {
      const uint32_t a = *reinterpret_cast<const uint32_t*>(q1 + sbase + o);
      const uint32_t b = *reinterpret_cast<const uint32_t*>(q2 + sbase + o);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        m4[i] = c1[(a >> (8 * i)) & 255] * am1;
        v4[i] = c2[(b >> (8 * i)) & 255] * am2;
      }
    } else {
      const f32x4 mm = *reinterpret_cast<const f32x4*>(m32 + sbase + o);
      const f32x4 vv4 = *reinterpret_cast<const f32x4*>(v32 + sbase + o);
#pragma unroll
      for (int i = 0; i < 4; ++i) { m4[i] = mm[i]; v4[i] = vv4[i]; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * j + i;
      valid[k] = (e + i) < tend;
      const float gi = valid[k] ? gg[i] * coef : 0.f;
      pv[k] = valid[k] ? pp[i] : 0.f;
      mv[k] = m4[i] * hp.beta1 + gi * (1.0f - hp.beta1);
      vv[k] = v4[i] * hp.beta2 + (gi * gi) * (1.0f - hp.beta2);
      if (!valid[k]) { mv[k] = 0.f; vv[k] = 0.f; }
    }
  }
  float dl[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float d = mv[k] / (sqrtf(vv[k]) + hp.eps);
    if (wd != 0.f) d += wd * pv[k];
    dl[k] = valid[k] ? d : 0.f;
  }
  if (!APPLY) {
    float sd = 0.f, sp = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) { sd += dl[k] * dl[k]; sp += pv[k] * pv[k]; }
    sd = block_sum_256(sd, red);
    __syncthreads();
    sp = block_sum_256(sp, red);
    if (tid == 0) { partial[2 * blk] = sd; partial[2 * blk + 1] = sp; }
    return;
  }
  const float step = -tlr[t] * trust[t];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long e = base + 4 * (tid + 256 * j);
    f32x4 pp;
#pragma unroll
    for (int i = 0; i < 4; ++i) pp[i] = pv[4 * j + i] + step * dl[4 * j + i];
    // padding lanes past the tensor end stay zero (they were loaded as p = 0 and delta = 0)
    *reinterpret_cast<f32x4*>(p + e) = pp;
  }
  if (mode8) {
    float mx1 = 0.f, mx2 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) { mx1 = fmaxf(mx1, fabsf(mv[k])); mx2 = fmaxf(mx2, fabsf(vv[k])); }
    mx1 = wave_max(mx1);
    mx2 = wave_max(mx2);
    const int w = tid >> 6, l = tid & 63;
    if (l == 0) { red[w] = mx1; red[4 + w] = mx2; }
    __syncthreads();
    const float n1 = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float n2 = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
    if (tid == 0) { absmax1[slot] = n1; absmax2[slot] = n2; }
    const float d1 = fmaxf(n1, 1e-30f), d2 = fmaxf(n2, 1e-30f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long o = 4 * (tid + 256 * j);
      uint32_t a = 0, b = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * j + i;
        a |= (uint32_t)nearest_code(c1, mv[k] / d1) << (8 * i);
        b |= (uint32_t)nearest_code(c2, vv[k] / d2) << (8 * i);
      }
      *reinterpret_cast<uint32_t*>(q1 + sbase + o) = a;
      *reinterpret_cast<uint32_t*>(q2 + sbase + o) = b;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long o = 4 * (tid + 256 * j);
      f32x4 mm, vq;
#pragma unroll
      for (int i = 0; i < 4; ++i) { mm[i] = mv[4 * j + i]; vq[i] = vv[4 * j + i]; }
      *reinterpret_cast<f32x4*>(m32 + sbase + o) = mm;
      *reinterpret_cast<f32x4*>(v32 + sbase + o) = vq;
    }
  }
}

__global__ __launch_bounds__(256) void lamb_trust_kernel(const float* __restrict__ partial, const long* __restrict__ tstart,
                                                         const long* __restrict__ tsize, float clamp_value,
                                                         float* __restrict__ trust, float* __restrict__ wnorm,
                                                         float* __restrict__ snorm) {
  __shared__ float red[8];
  const int t = blockIdx.x;
  const long b0 = tstart[t] / QBLOCK;
  const long b1 = b0 + (tsize[t] + QBLOCK - 1) / QBLOCK;
  double sd = 0.0, sp = 0.0;
  for (long b = b0 + threadIdx.x; b < b1; b += 256) { sd += partial[2 * b]; sp += partial[2 * b + 1]; }
  float fd = block_sum_256((float)sd, red);
  __syncthreads();
  float fp = block_sum_256((float)sp, red);
  if (threadIdx.x == 0) {
    const float s = sqrtf(fd);
    float w = sqrtf(fp);
    w = fminf(fmaxf(w, 0.f), clamp_value);
    trust[t] = (w != 0.f && s != 0.f) ? w / s : 1.0f;
    wnorm[t] = w;
    snorm[t] = s;
  }
}

void lamb_grad_norm(const float* g, long n, float* partial, float max_norm, float* coef, float* norm, hipStream_t st) {
  const int nblocks = (int)(n / QBLOCK);
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(nblocks), dim3(256), 0, st, g, partial, n);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, st, partial, nblocks, max_norm, coef, norm);
}

void lamb_step(float* p, const float* g, uint8_t* q1, uint8_t* q2, float* absmax1, float* absmax2, float* m32, float* v32,
               const float* code1, const float* code2, const int* block_tensor, const int* bslot, const long* tstart,
               const long* tsize, const int* tmode, const float* twd, const float* tlr, const float* coef, float* partial,
               float* trust, float* wnorm, float* snorm, int ntensors, long n, float beta1, float beta2, float eps,
               float clamp_value, int use_clip, hipStream_t st) {
  const int nblocks = (int)(n / QBLOCK);
  LambParams hp{beta1, beta2, eps, use_clip};
  hipLaunchKernelGGL(lamb_pass_kernel<false>, dim3(nblocks), dim3(256), 0, st, p, g, q1, q2, absmax1, absmax2, m32, v32, code1,
                     code2, block_tensor, bslot, tstart, tsize, tmode, twd, coef, partial, tlr, trust, hp);
  hipLaunchKernelGGL(lamb_trust_kernel, dim3(ntensors), dim3(256), 0, st, partial, tstart, tsize, clamp_value, trust, wnorm,
                     snorm);
  hipLaunchKernelGGL(lamb_pass_kernel<true>, dim3(nblocks), dim3(256), 0, st, p, g, q1, q2, absmax1, absmax2, m32, v32, code1,
                     code2, block_tensor, bslot, tstart, tsize, tmode, twd, coef, partial, tlr, trust, hp);
}

}  // namespace dalle
