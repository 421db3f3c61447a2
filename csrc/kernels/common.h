// Shared device helpers for the dalle_amd CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dalle {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef uint16_t bf16_raw;

constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;

__device__ __forceinline__ float bf2f(bf16_raw v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_raw f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(bf16_raw, b);
}
__device__ __forceinline__ float bfv2f(__bf16 v) { return (float)v; }

// 8 bf16 <-> 8 floats
__device__ __forceinline__ void unpack8(const s16x8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f((bf16_raw)v[i]);
}
__device__ __forceinline__ s16x8 pack8(const float* f) {
  s16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (short)f2bf(f[i]);
  return v;
}
__device__ __forceinline__ void unpack4(const s16x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = bf2f((bf16_raw)v[i]);
}
__device__ __forceinline__ s16x4 pack4(const float* f) {
  s16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (short)f2bf(f[i]);
  return v;
}

// Desynchronise the first wave of a one-tile-per-workgroup GEMM: workgroup b < first_wave waits
// ((b >> 3) & 3) * ticks of the 100 MHz real-time counter before it starts, so the CUs' tile boundaries
// (and the HBM bursts of their epilogues) fall at four different phases instead of all at once; every
// later workgroup inherits its CU's offset. Bounded spin, no inter-workgroup dependence.
__device__ __forceinline__ void stagger_start(int ticks, int first_wave) {
  if (ticks <= 0 || (int)blockIdx.x >= first_wave) return;
  const unsigned long long until = __builtin_amdgcn_s_memrealtime() + (unsigned long long)(((blockIdx.x >> 3) & 3) * ticks);
  while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(4);
}

// ---- epilogue stores with an explicit cache policy ----
// GEMM epilogues write their whole output once and never read it back inside the kernel. Plain (and
// `nt`) stores keep every written line in the XCD's 4 MB L2, so each wave of 256 x 256 output tiles
// (4 MB per XCD) evicts the operand panels the next tiles stream from; `sc1` / `sc0 sc1` stores drop the
// line from L2 after the write (MI355X_MICROARCH.md, "stores of each flavour"). cpol is the raw buffer
// store's aux immediate: 1 = sc0, 2 = nt, 16 = sc1 (17 = sc0 sc1); 0 = a plain flat store.
typedef unsigned u32x4_vs __attribute__((vector_size(16)));

// whole-buffer descriptor over a wave-uniform base: the 32-bit per-lane byte offset addresses up to 4 GiB
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, -1, 0x00020000);
}

template <int AUX>
__device__ __forceinline__ void bstore16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4_vs v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

// 16-byte store of v at base + off (bytes) under cache policy cpol (wave-uniform)
__device__ __forceinline__ void cstore16(void* base, __amdgpu_buffer_rsrc_t r, uint32_t off, u32x4_vs v, int cpol) {
  switch (cpol) {
    case 0: *reinterpret_cast<u32x4_vs*>((char*)base + off) = v; break;
    case 1: bstore16<1>(r, off, v); break;
    case 2: bstore16<2>(r, off, v); break;
    case 16: bstore16<16>(r, off, v); break;
    case 17: bstore16<17>(r, off, v); break;
    case 18: bstore16<18>(r, off, v); break;
    case 19: bstore16<19>(r, off, v); break;
    default: bstore16<0>(r, off, v); break;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 256 (4 waves); `red` must hold >= 8 floats of LDS.
__device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = red[0] + red[1] + red[2] + red[3];
  return r;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// gelu(x) alone by the same erf approximation (|erf error| <= 1.5e-7): ~12 VALU + exp + rcp instead of
// ocml erff's ~50 (the fused FF-in GEMM epilogue is VALU-bound on it)
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-0.5f * x * x * LOG2E);
  const float erf_abs = fmaf(-poly, e, 1.0f);
  return x * (0.5f + 0.5f * copysignf(erf_abs, x));
}
// gelu(x) and gelu'(x) together for the GEGLU backward, which is VALU-bound with two ocml erff + one
// expf per element (~80 VALU). erf(x/sqrt2) by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far
// below bf16 resolution), whose exp(-x^2/2) is shared with the normal pdf: one exp + one rcp.
__device__ __forceinline__ void gelu_and_grad(float x, float& gelu, float& grad) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-0.5f * x * x * LOG2E);  // exp(-x^2 / 2) = exp(-z^2)
  const float erf_abs = fmaf(-poly, e, 1.0f);
  const float cdf = 0.5f + 0.5f * copysignf(erf_abs, x);
  gelu = x * cdf;
  grad = fmaf(x * 0.3989422804014327f, e, cdf);
}

}  // namespace dalle
