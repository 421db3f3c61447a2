// 3-axis rotary embedding on q, k AND v + head split into the padded attention storage layout
// (SURVEY K6). Forward: qkv (B, n, 3*H*64) bf16 [GEMM output] -> q (pre-scaled by 1/sqrt(64)),
// k, v: (B*H, Np, 64) bf16. Rows with no sequence position (text padding, the padded last image
// token) are written as zeros, so no memset is needed. Backward applies the transposed rotation
// and scatters back to (B, n, 3*H*64). One thread = one 16-byte chunk (8 dims) of q, k and v.
#include "common.h"
#include "geom.h"

namespace dalle {

__device__ __forceinline__ int rope_st2seq(const RopeGeom& g, int s) {
  if (s < g.T) return s;
  if (s < g.Tp) return -1;
  const int kst = s - g.Tp;
  const int k = g.col_major ? ((kst & (g.S - 1)) << g.logS) + (kst >> g.logS) : kst;
  const int p = g.T + k;
  return p < g.n ? p : -1;
}

__device__ __forceinline__ int rope_seq2st(const RopeGeom& g, int p) {
  if (p < g.T) return p;
  const int k = p - g.T;
  const int kst = g.col_major ? ((k & (g.S - 1)) << g.logS) + (k >> g.logS) : k;
  return g.Tp + kst;
}

__device__ __forceinline__ void rotate8(float* x, const float* c, const float* s) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const float a = x[i], b = x[i + 1];
    x[i] = a * c[i] + b * s[i];
    x[i + 1] = b * c[i + 1] + a * s[i + 1];
  }
}

__device__ __forceinline__ void rotate8_t(float* x, const float* c, const float* s) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const float a = x[i], b = x[i + 1];
    x[i] = a * c[i] + b * s[i + 1];
    x[i + 1] = b * c[i + 1] + a * s[i];
  }
}

__global__ void rope_fwd_kernel(const __bf16* __restrict__ qkv, const float* __restrict__ cosT, const float* __restrict__ sinT,
                                __bf16* __restrict__ q, __bf16* __restrict__ k, __bf16* __restrict__ v, RopeGeom g,
                                int BH, float qscale) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = gid & 7;
  const long row = gid >> 3;
  if (row >= (long)BH * g.Np) return;
  const int bh = row / g.Np, s = row - (long)bh * g.Np;
  const int b = bh / g.H, h = bh - b * g.H;
  const int p = rope_st2seq(g, s);
  const size_t dst = (size_t)row * 64 + chunk * 8;
  if (p < 0) {
    const s16x8 z = {};
    *reinterpret_cast<s16x8*>(q + dst) = z;
    *reinterpret_cast<s16x8*>(k + dst) = z;
    *reinterpret_cast<s16x8*>(v + dst) = z;
    return;
  }
  const int HD = g.H * 64;
  const size_t src = ((size_t)b * g.n + p) * (3 * HD) + h * 64 + chunk * 8;
  float c[8], sn[8];
  *reinterpret_cast<f32x4*>(c) = *reinterpret_cast<const f32x4*>(cosT + (size_t)p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(c + 4) = *reinterpret_cast<const f32x4*>(cosT + (size_t)p * 64 + chunk * 8 + 4);
  *reinterpret_cast<f32x4*>(sn) = *reinterpret_cast<const f32x4*>(sinT + (size_t)p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(sn + 4) = *reinterpret_cast<const f32x4*>(sinT + (size_t)p * 64 + chunk * 8 + 4);
  __bf16* outs[3] = {q, k, v};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float x[8];
    unpack8(*reinterpret_cast<const s16x8*>(qkv + src + t * HD), x);
    rotate8(x, c, sn);
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] *= qscale;
    }
    *reinterpret_cast<s16x8*>(outs[t] + dst) = pack8(x);
  }
}

__global__ void rope_bwd_kernel(const __bf16* __restrict__ dq, const __bf16* __restrict__ dk, const __bf16* __restrict__ dv,
                                const float* __restrict__ cosT, const float* __restrict__ sinT, __bf16* __restrict__ dqkv,
                                RopeGeom g, int B, float qscale) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = gid & 7;
  const long r = gid >> 3;  // (b, p, h)
  if (r >= (long)B * g.n * g.H) return;
  const int h = r % g.H;
  const long bp = r / g.H;
  const int p = bp % g.n, b = bp / g.n;
  const int s = rope_seq2st(g, p);
  const size_t src = (((size_t)b * g.H + h) * g.Np + s) * 64 + chunk * 8;
  const int HD = g.H * 64;
  const size_t dst = ((size_t)b * g.n + p) * (3 * HD) + h * 64 + chunk * 8;
  float c[8], sn[8];
  *reinterpret_cast<f32x4*>(c) = *reinterpret_cast<const f32x4*>(cosT + (size_t)p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(c + 4) = *reinterpret_cast<const f32x4*>(cosT + (size_t)p * 64 + chunk * 8 + 4);
  *reinterpret_cast<f32x4*>(sn) = *reinterpret_cast<const f32x4*>(sinT + (size_t)p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(sn + 4) = *reinterpret_cast<const f32x4*>(sinT + (size_t)p * 64 + chunk * 8 + 4);
  const __bf16* ins[3] = {dq, dk, dv};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float x[8];
    unpack8(*reinterpret_cast<const s16x8*>(ins[t] + src), x);
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] *= qscale;
    }
    rotate8_t(x, c, sn);
    *reinterpret_cast<s16x8*>(dqkv + dst + t * HD) = pack8(x);
  }
}

void rope_fwd(const void* qkv, const float* cosT, const float* sinT, void* q, void* k, void* v, const RopeGeom& g, int BH,
              float qscale, hipStream_t st) {
  const long threads = (long)BH * g.Np * 8;
  hipLaunchKernelGGL(rope_fwd_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, (const __bf16*)qkv, cosT, sinT,
                     (__bf16*)q, (__bf16*)k, (__bf16*)v, g, BH, qscale);
}

void rope_bwd(const void* dq, const void* dk, const void* dv, const float* cosT, const float* sinT, void* dqkv,
              const RopeGeom& g, int B, float qscale, hipStream_t st) {
  const long threads = (long)B * g.n * g.H * 8;
  hipLaunchKernelGGL(rope_bwd_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, (const __bf16*)dq, (const __bf16*)dk,
                     (const __bf16*)dv, cosT, sinT, (__bf16*)dqkv, g, B, qscale);
}

}  // namespace dalle
