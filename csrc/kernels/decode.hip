// Autoregressive decode kernels (SURVEY K7f, K4 cached token shift, K6 rotary into the KV cache,
// K19 VQGAN codebook embed). Every positional argument is a DEVICE scalar (`pos`) so one decode
// step -- all layers plus sampling -- can be captured once into a hipGraph and replayed for each of
// the 1024 image tokens.
#include "common.h"
#include "geom.h"

namespace dalle {

// ---- LayerNorm of the new token, append to the per-branch LN history, emit the shifted row ----
// Pending residual update of the stream a LayerNorm reads: x += scale * (sum_ks part[ks] + bias), the
// split-K partial slabs of the projection that produced it (skinny EPI 4) -- summed here, so that
// GEMM needs no cross-workgroup hand-off and its workgroups each read only a slice of K.
struct PendingRes {
  const float* part;  // (KS, B, D) fp32, or null
  const __bf16* bias; // (D) bf16, may be null
  const float* scale; // (D) LayerScale
  int KS;
};

// One workgroup per batch row, one thread per 4 columns (D / 4 threads: 4 waves at D = 1024), so the
// pending slab loads of a row are spread over 4x the lanes of a one-wave row.
template <int D>
__global__ __launch_bounds__(D / 4) void decode_ln_shift_kernel(float* __restrict__ x, const float* __restrict__ w,
                                                                const float* __restrict__ bias, __bf16* __restrict__ hist,
                                                                __bf16* __restrict__ y, const int* __restrict__ pos_ptr,
                                                                DecodeGeom g, int shift, PendingRes pr) {
  constexpr int NW = D / 256;  // waves per row
  __shared__ float red[2][NW];
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int pos = *pos_ptr;
  if (pos < 0 || pos >= g.n) return;  // a replay past the cache end is a no-op, never an OOB write
  float* xr = x + (size_t)b * D;
  __bf16* hb = hist + (size_t)b * g.n * D;
  const int c = 4 * tid;
  // every load is independent of the row statistics -- the row, the LN parameters, the pending slabs
  // and the shifted history row (an earlier position, written by an earlier step) -- so all of them
  // are issued before the first reduction: one memory round trip per step
  const int B = gridDim.x;
  // all loads unconditional and in one basic block (slab index clamped to KS - 1, shift row clamped to row 0 and
  // masked after): the guarded forms compiled to a vmcnt(0) round trip after the first slab load and after the
  // shift-row load, two extra memory latencies per call
  const bool pend = pr.part != nullptr;  // uniform
  // the row, the LN parameters first; then the slabs through a pointer that is valid either way (the row itself
  // when nothing is pending, slab index 0) and the bias through one that is (the scale vector: >= D bf16)
  f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
  const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + c);
  const float* pp = pend ? pr.part : x;
  const int klast = pend ? pr.KS - 1 : 0;
  f32x4 t[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = *reinterpret_cast<const f32x4*>(pp + ((size_t)min(k, klast) * B + b) * D + c);
  const float* scp = pend ? pr.scale : w;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scp + c);
  const __bf16* bpp = (pend && pr.bias != nullptr) ? pr.bias : reinterpret_cast<const __bf16*>(w);
  const s16x4 pbr = *reinterpret_cast<const s16x4*>(bpp + c);
  const bool has_pb = pend && pr.bias != nullptr;
  const bool shifted = shift && c < D / 2;
  int src;
  if (pos < g.T) {
    src = pos - 1;
  } else {
    const int k = pos - g.T;
    src = (c < D / 4) ? ((k >= g.S) ? pos - g.S : -1) : ((k % g.S) ? pos - 1 : -1);
  }
  const s16x4 shl = *reinterpret_cast<const s16x4*>(hb + (size_t)max(src, 0) * D + c);
  const s16x4 sh = (shifted && src >= 0) ? shl : s16x4{};
  if (pend) {
    float pb[4];
    unpack4(pbr, pb);
    if (!has_pb) pb[0] = pb[1] = pb[2] = pb[3] = 0.f;
    f32x4 acc = t[0];  // fixed ks order: deterministic
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < pr.KS) acc += t[k];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += sc[i] * (acc[i] + pb[i]);
    *reinterpret_cast<f32x4*>(xr + c) = v;
  }
  // one reduction round for both moments (a decode step is latency-bound: one barrier fewer per row);
  // the shifted second moment about this thread's first element keeps E[x^2] - mean^2 cancellation-free
  const float piv = __shfl(v[0], 0, 64);
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) { const float d = v[i] - piv; s += d; q += d * d; }
  s = wave_sum(s);
  q = wave_sum(q);
  __shared__ float pivs[NW];
  if (lane == 0) { red[0][wave] = s; red[1][wave] = q; pivs[wave] = piv; }
  __syncthreads();
  // combine the waves' (pivot, shifted sum, shifted sum of squares) about wave 0's pivot
  const float p0 = pivs[0];
  float S = 0.f, Q = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const float dp = pivs[i] - p0, si = red[0][i], n = (float)(D / NW);
    S += si + n * dp;
    Q += red[1][i] + 2.f * dp * si + n * dp * dp;
  }
  const float dm = S * (1.0f / D);           // mean - p0
  const float mean = p0 + dm;
  const float var = fmaxf(Q * (1.0f / D) - dm * dm, 0.f);
  const float rstd = rsqrtf(var + 1e-5f);
  float o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (v[i] - mean) * rstd * wv[i] + bv[i];
  const s16x4 packed = pack4(o);
  *reinterpret_cast<s16x4*>(hb + (size_t)pos * D + c) = packed;
  *reinterpret_cast<s16x4*>(y + (size_t)b * D + c) = shifted ? sh : packed;
}

// ---- rotary on q/k/v of the new token; k, v appended to the cache at `pos` ----
__global__ void decode_rope_kernel(const __bf16* __restrict__ qkv, const float* __restrict__ cosT, const float* __restrict__ sinT,
                                   __bf16* __restrict__ q_out, __bf16* __restrict__ kc, __bf16* __restrict__ vc,
                                   const int* __restrict__ pos_ptr, DecodeGeom g, int B, float qscale) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;  // (b, h, chunk)
  if (gid >= B * g.H * 8) return;
  const int chunk = gid & 7, bh = gid >> 3;
  const int b = bh / g.H, h = bh - b * g.H;
  const int pos = *pos_ptr;
  if (pos < 0 || pos >= g.n) return;  // a replay past the cache end is a no-op, never an OOB write
  const int HD = g.H * 64;
  const size_t src = (size_t)b * 3 * HD + h * 64 + chunk * 8;
  float c[8], sn[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { c[i] = cosT[pos * 64 + chunk * 8 + i]; sn[i] = sinT[pos * 64 + chunk * 8 + i]; }
  __bf16* dst[3] = {q_out + (size_t)bh * 64 + chunk * 8, kc + ((size_t)bh * g.n + pos) * 64 + chunk * 8,
                    vc + ((size_t)bh * g.n + pos) * 64 + chunk * 8};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float x[8];
    unpack8(*reinterpret_cast<const s16x8*>(qkv + src + t * HD), x);
    float r[8];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      r[i] = x[i] * c[i] + x[i + 1] * sn[i];
      r[i + 1] = x[i + 1] * c[i + 1] + x[i] * sn[i + 1];
    }
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] *= qscale;
    }
    *reinterpret_cast<s16x8*>(dst[t]) = pack8(r);
  }
}

// ---- batched caption prefill: rotary on q/k/v of positions 0..P-1; q (pre-scaled) to (B*H, P, 64),
// k / v straight into the KV caches (one pass instead of the PyTorch rotate / convert / scatter chain) ----
__global__ __launch_bounds__(256) void prefill_rope_kernel(const __bf16* __restrict__ qkv, const float* __restrict__ cosT,
                                                           const float* __restrict__ sinT, __bf16* __restrict__ q_out,
                                                           __bf16* __restrict__ kc, __bf16* __restrict__ vc, int B, int P,
                                                           int H, int n, float qscale) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, p, h, chunk)
  if (gid >= (long)B * P * H * 8) return;
  const int chunk = gid & 7;
  const long bph = gid >> 3;
  const int h = bph % H;
  const long bp = bph / H;
  const int p = bp % P, b = bp / P;
  const int HD = H * 64;
  const __bf16* src = qkv + bp * 3 * HD + h * 64 + chunk * 8;
  float c[8], sn[8];
  *reinterpret_cast<f32x4*>(c) = *reinterpret_cast<const f32x4*>(cosT + p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(c + 4) = *reinterpret_cast<const f32x4*>(cosT + p * 64 + chunk * 8 + 4);
  *reinterpret_cast<f32x4*>(sn) = *reinterpret_cast<const f32x4*>(sinT + p * 64 + chunk * 8);
  *reinterpret_cast<f32x4*>(sn + 4) = *reinterpret_cast<const f32x4*>(sinT + p * 64 + chunk * 8 + 4);
  const size_t bh = (size_t)b * H + h;
  __bf16* dst[3] = {q_out + (bh * P + p) * 64 + chunk * 8, kc + (bh * n + p) * 64 + chunk * 8, vc + (bh * n + p) * 64 + chunk * 8};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float x[8], r[8];
    unpack8(*reinterpret_cast<const s16x8*>(src + t * HD), x);
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      r[i] = x[i] * c[i] + x[i + 1] * sn[i];
      r[i + 1] = x[i + 1] * c[i + 1] + x[i] * sn[i + 1];
    }
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] *= qscale;
    }
    *reinterpret_cast<s16x8*>(dst[t]) = pack8(r);
  }
}

void prefill_rope(const void* qkv, const float* cosT, const float* sinT, void* q, void* kc, void* vc, int B, int P, int H, int n,
                  float qscale, hipStream_t st) {
  const long threads = (long)B * P * H * 8;
  hipLaunchKernelGGL(prefill_rope_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, (const __bf16*)qkv, cosT, sinT,
                     (__bf16*)q, (__bf16*)kc, (__bf16*)vc, B, P, H, n, qscale);
}

// ---- batched caption prefill: LayerNorm + text token shift of every (b, p) row, one wave per row ----
// x (B, P, D) fp32 -> hist[b, p] (the unshifted LN output, bf16: the history the decode steps shift from,
// hist is (B, n, D)) and out (B, P, D) bf16 with the shift applied by push: channels [0, D/2) of row p land
// in row p + 1 and row 0 gets zeros there (shift = 0: out = the LN output). Replaces the PyTorch chain
// layer_norm -> bf16 cast -> history copy -> clone -> two slice copies (six passes over the rows).
template <int D>
__global__ __launch_bounds__(256) void prefill_ln_shift_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ bias, __bf16* __restrict__ hist,
                                                               __bf16* __restrict__ out, int B, int P, int n, float eps, int shift) {
  constexpr int PER = D / 256;  // float4 per lane
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (row >= B * P) return;
  const int b = row / P, p = row - b * P;
  const float* xr = x + (size_t)row * D;
  f32x4 v[PER];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = *reinterpret_cast<const f32x4*>(xr + 4 * (lane + 64 * j));
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) { const float d = v[j][i] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  __bf16* hr = hist + ((size_t)b * n + p) * D;
  __bf16* orow = out + (size_t)row * D;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = 4 * (lane + 64 * j);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + c);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (v[j][i] - mean) * rstd * wv[i] + bv[i];
    const s16x4 pk = pack4(o);
    *reinterpret_cast<s16x4*>(hr + c) = pk;
    if (shift && c < D / 2) {
      if (p + 1 < P) *reinterpret_cast<s16x4*>(orow + D + c) = pk;
      if (p == 0) *reinterpret_cast<s16x4*>(orow + c) = s16x4{};
    } else {
      *reinterpret_cast<s16x4*>(orow + c) = pk;
    }
  }
}

void prefill_ln_shift(const float* x, const float* w, const float* b, void* hist, void* out, int B, int P, int n, int D, float eps,
                      int shift, hipStream_t st) {
  const dim3 grid(((long)B * P + 3) / 4);
  switch (D) {
    case 256: hipLaunchKernelGGL(prefill_ln_shift_kernel<256>, grid, dim3(256), 0, st, x, w, b, (__bf16*)hist, (__bf16*)out, B, P, n, eps, shift); break;
    case 512: hipLaunchKernelGGL(prefill_ln_shift_kernel<512>, grid, dim3(256), 0, st, x, w, b, (__bf16*)hist, (__bf16*)out, B, P, n, eps, shift); break;
    case 1024: hipLaunchKernelGGL(prefill_ln_shift_kernel<1024>, grid, dim3(256), 0, st, x, w, b, (__bf16*)hist, (__bf16*)out, B, P, n, eps, shift); break;
    case 2048: hipLaunchKernelGGL(prefill_ln_shift_kernel<2048>, grid, dim3(256), 0, st, x, w, b, (__bf16*)hist, (__bf16*)out, B, P, n, eps, shift); break;
  }
}

// ---- batched caption prefill: masked softmax of the fp32 scores (R, P, P) -> bf16 probabilities, one wave per
// row (query i = row % P reads mask row i: the layer's static pattern over the caption, true = attend). One pass
// instead of masked_fill -> softmax -> bf16 cast over the fp32 scores. P <= 512 (8 columns per lane). ----
__global__ __launch_bounds__(256) void prefill_softmax_kernel(const float* __restrict__ sc, const bool* __restrict__ mask,
                                                              __bf16* __restrict__ out, long rows, int P) {
  const long row = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int i = row % P;
  const float* sr = sc + row * P;
  const bool* mr = mask + (size_t)i * P;
  float v[8];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    v[t] = (j < P && mr[j]) ? sr[j] : -INFINITY;
    m = fmaxf(m, v[t]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    v[t] = v[t] == -INFINITY ? 0.f : __expf(v[t] - m);
    s += v[t];
  }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.0f / s : 0.f;
  __bf16* orow = out + row * P;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int j = lane + 64 * t;
    if (j < P) orow[j] = (__bf16)(v[t] * inv);
  }
}

void prefill_softmax(const float* sc, const bool* mask, void* out, long rows, int P, hipStream_t st) {
  hipLaunchKernelGGL(prefill_softmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, sc, mask, (__bf16*)out, rows, P);
}

// ---- batched caption prefill: the residual update x += scale * y of a sublayer (y: the projection's bf16
// output, bias included; scale: LayerScale (D,)), one pass instead of the bf16->fp32 cast, the scale and the add ----
__global__ __launch_bounds__(256) void prefill_residual_kernel(float* __restrict__ x, const __bf16* __restrict__ y,
                                                               const float* __restrict__ scale, long n4, int D) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n4) return;
  const int c = i % D;
  float yv[4];
  unpack4(*reinterpret_cast<const s16x4*>(y + i), yv);
  f32x4 xv = *reinterpret_cast<const f32x4*>(x + i);
  const f32x4 sv = *reinterpret_cast<const f32x4*>(scale + c);
#pragma unroll
  for (int t = 0; t < 4; ++t) xv[t] += sv[t] * yv[t];
  *reinterpret_cast<f32x4*>(x + i) = xv;
}

void prefill_residual(float* x, const void* y, const float* scale, long n, int D, hipStream_t st) {
  hipLaunchKernelGGL(prefill_residual_kernel, dim3((n / 4 + 255) / 256), dim3(256), 0, st, x, (const __bf16*)y, scale, n, D);
}

// the last pending update of a step (before the final LayerNorm): x += scale * (sum_ks part + bias)
__global__ __launch_bounds__(256) void residual_from_partials_kernel(float* __restrict__ x, PendingRes pr, int B, int D) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= (long)B * D) return;
  const int c = i % D;
  f32x4 acc = *reinterpret_cast<const f32x4*>(pr.part + i);
  for (int k = 1; k < pr.KS; ++k) acc += *reinterpret_cast<const f32x4*>(pr.part + (size_t)k * B * D + i);
  f32x4 xv = *reinterpret_cast<const f32x4*>(x + i);
#pragma unroll
  for (int t = 0; t < 4; ++t) xv[t] += pr.scale[c + t] * (acc[t] + (pr.bias ? (float)pr.bias[c + t] : 0.f));
  *reinterpret_cast<f32x4*>(x + i) = xv;
}

// q / k / v of the new token from the QKV projection's split-K partial slabs (KS, B, 3*H*64): summed,
// rotated (3-axis rotary at *pos), q pre-scaled; k / v appended to the caches.
struct QkvPartials {
  const float* part;
  const float* cosT;
  const float* sinT;
  int KS, B;
  float qscale;
  // device flag (may be null): every batch row carries the same caption, so the text positions' K / V are
  // identical in every row's cache and all rows read them from row 0's (one L2-resident copy per head instead of
  // B copies streamed from HBM: the reference's generation workload repeats one query over the batch)
  const int* text_shared;
};

__device__ __forceinline__ int decode_num_keys(const DecodeGeom& g, int pos, int& nloc, int& r0, int& c0, int& nr, int& nc) {
  // text keys [0, min(T, pos+1)), then an image-local rectangle (rows r0.., cols c0..) clipped by causality
  if (pos < g.T) { nloc = 0; return pos + 1; }
  const int k = pos - g.T, r = k / g.S, c = k % g.S;
  if (g.pattern == 0) { nloc = k + 1; r0 = 0; c0 = 0; nr = 0; nc = 0; return g.T + nloc; }
  if (g.pattern == 1) { r0 = r; nr = 1; c0 = 0; nc = c + 1; }
  else if (g.pattern == 2) { r0 = 0; nr = r + 1; c0 = c; nc = 1; }
  else { r0 = max(0, r - g.K + 1); nr = r - r0 + 1; c0 = max(0, c - g.K + 1); nc = c - c0 + 1; }
  nloc = nr * nc;
  return g.T + nloc;
}

// Cache row of key i of the key list (text keys, then the local rectangle row by row). Branch-free
// (selects only), so a loop of loads indexed by it stays one basic block and the compiler can count
// its vmcnt statically. l / nc by a float reciprocal: l < 2^20, nc <= S, the +0.5 keeps the quotient
// off integer edges (exact; checked against integer division for every nc <= 64, l < 2^16).
__device__ __forceinline__ int decode_key_at(const DecodeGeom& g, int i, int pos, int r0, int c0, int nc) {
  const int l = i - g.T;
  const int qd = (int)(((float)l + 0.5f) * __builtin_amdgcn_rcpf((float)nc));
  const int local = g.pattern == 0 ? g.T + l : g.T + (r0 + qd) * g.S + c0 + l - qd * nc;
  return (pos < g.T || i < g.T) ? i : local;
}

// ---- one query per (b, h) against its allowed cached keys ----
// Bandwidth-bound: ~290 keys x (K + V) x 128 B per (b, h) at the reference config. Layout: 8 lanes
// cover one 128-B key row (16 B each), so a wave reads 8 whole rows per instruction; key i of a
// chunk sits at (round u, wave w, slot s) = i / 32, (i / 8) % 4, i % 8. In the common case (all keys
// in one chunk of 32 * DA_U) every K AND V load of the lane is issued before the first score is
// formed -- V does not depend on the softmax -- so the whole (b, h) is one memory round trip. Longer
// key sets (full attention late in the sequence) take a chunked two-pass path with scores in LDS.
// 10 rounds per chunk = 320 keys: the reference geometry's 257 text + <= 32 axial (<= 25 conv) keys in one chunk at
// 128 VGPRs, so four (b, h) workgroups fit a CU (12 rounds: 146 VGPRs, three)
constexpr int DA_U = 10;
constexpr int DA_CHUNK = 32 * DA_U;
constexpr int DA_MAXN = 2048;

__device__ __forceinline__ float dot8(const float* q, const s16x8& k) {
  float f[8];
  unpack8(k, f);
  float a = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) a += q[e] * f[e];
  return a;
}

// q . k over a lane's 8 dims as four packed-bf16 dot products (v_dot2c_f32_bf16: no unpacking; q is bf16-exact)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__device__ __forceinline__ float dot8_bf(const uint32_t (&q)[4], const s16x8& k) {
  const uint32_t* kw = reinterpret_cast<const uint32_t*>(&k);
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, q[j]), __builtin_bit_cast(bf16x2, kw[j]), a, false);
  return a;
}

__device__ __forceinline__ float slot_sum(float v) {  // over the 8 lanes of one key row
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

template <bool FROM_PART>
__global__ __launch_bounds__(256) void decode_attn_kernel(const __bf16* __restrict__ q, __bf16* __restrict__ kc,
                                                          __bf16* __restrict__ vc, __bf16* __restrict__ out,
                                                          const int* __restrict__ pos_ptr, DecodeGeom g, QkvPartials qp) {
  __shared__ float sc[DA_MAXN];
  __shared__ float red[2][4];
  __shared__ float part[4][64];
  __shared__ float qsh[64];
  __shared__ __attribute__((aligned(16))) __bf16 kvsh[2][64];
  const int bh = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sub = lane & 7, slot = lane >> 3;
  const int pos = *pos_ptr;
  if (pos < 0 || pos >= g.n) return;  // a replay past the cache end is a no-op, never an OOB write
  int nloc, r0 = 0, c0 = 0, nr = 0, nc = 1;
  const int nkeys = decode_num_keys(g, pos, nloc, r0, c0, nr, nc);
  const bool one_chunk = nkeys <= DA_CHUNK;
  const __bf16* kb = kc + (size_t)bh * g.n * 64 + sub * 8;
  const __bf16* vb = vc + (size_t)bh * g.n * 64 + sub * 8;
  // shared caption: text keys before this position come from row 0 of the same head (< 2^31 elements back:
  // B <= 64, H <= 32, n <= 2048); the new key itself (a text query's last key) stays this row's own
  const int tshift = (qp.text_shared != nullptr && *qp.text_shared) ? -(bh / g.H) * g.H * g.n * 64 : 0;
  const int tlim = min(g.T, pos);

  // FROM_PART: q / k / v of the new token are split-K slabs of the QKV projection (threads 0..95: q | k
  // | v x dim pair). Every load the query needs before its first score -- q, or its slabs and rotary
  // row -- is issued ahead of the cache stream, and all loads are unconditional (threads >= 96 load
  // thread 95's slabs; slots past the key list re-read the last key and get probability 0), so in the
  // single-chunk path the compiler's vmcnt counts stay static: the slab round trip and the first
  // scores overlap the stream. The new key's cache row, read stale, is patched from LDS.
  const int pt = min(tid, 95) >> 5, pd = (min(tid, 95) & 31) * 2;
  float2 pv[8], cs = make_float2(0.f, 0.f), sn = make_float2(0.f, 0.f);
  s16x8 qraw = s16x8{};
  // issued at the top of each path's basic block, so the compiler's vmcnt counting sees them with the
  // stream that follows (an early, separate block makes it wait for everything)
  auto issue_q = [&]() {
    if (FROM_PART) {
      const int b = bh / g.H, h = bh - b * g.H, HD = g.H * 64;
      const size_t col = (size_t)pt * HD + h * 64 + pd;
#pragma unroll
      for (int k = 0; k < 8; ++k)  // slabs past KS re-read the last one and are weighted 0
        pv[k] = *reinterpret_cast<const float2*>(qp.part + ((size_t)min(k, qp.KS - 1) * qp.B + b) * 3 * HD + col);
      cs = *reinterpret_cast<const float2*>(qp.cosT + pos * 64 + pd);
      sn = *reinterpret_cast<const float2*>(qp.sinT + pos * 64 + pd);
    } else {
      qraw = *reinterpret_cast<const s16x8*>(q + (size_t)bh * 64 + sub * 8);
    }
    asm volatile("" ::: "memory");  // keeps these loads ahead of the cache stream (hipcc sinks them otherwise)
  };
  float qd[8];      // q (x log2 e) as floats: the chunked path
  uint32_t qb2[4];  // q as bf16 pairs: the single-chunk path's packed dot products
  // q / k / v of the new token: q to every lane (qd, qb2), k / v to LDS and the caches
  auto prologue = [&]() {
    if (FROM_PART) {
      if (tid < 96) {
        float y0 = 0.f, y1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // fixed ks order
          const float wk = k < qp.KS ? 1.f : 0.f;
          y0 += wk * pv[k].x;
          y1 += wk * pv[k].y;
        }
        const float ra = y0 * cs.x + y1 * sn.x, rb = y1 * cs.y + y0 * sn.y;
        if (pt == 0) {  // rounded to bf16 as the cached-q path stores it
          qsh[pd] = bf2f(f2bf(ra * qp.qscale));
          qsh[pd + 1] = bf2f(f2bf(rb * qp.qscale));
        } else {
          const uint32_t pk = (uint32_t)f2bf(ra) | ((uint32_t)f2bf(rb) << 16);
          *reinterpret_cast<uint32_t*>(&kvsh[pt - 1][pd]) = pk;
          __bf16* dst = (pt == 1 ? kc : vc) + ((size_t)bh * g.n + pos) * 64 + pd;
          *reinterpret_cast<uint32_t*>(dst) = pk;
        }
      }
      __threadfence_block();  // the chunked path reads the new row back from the cache
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) qd[e] = qsh[sub * 8 + e];
#pragma unroll
      for (int j = 0; j < 4; ++j) qb2[j] = (uint32_t)f2bf(qd[2 * j]) | ((uint32_t)f2bf(qd[2 * j + 1]) << 16);  // exact: bf16 values
#pragma unroll
      for (int e = 0; e < 8; ++e) qd[e] *= LOG2E;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) qb2[j] = reinterpret_cast<const uint32_t*>(&qraw)[j];
      unpack8(qraw, qd);
#pragma unroll
      for (int e = 0; e < 8; ++e) qd[e] *= LOG2E;
    }
  };
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  float m, inv;

  if (one_chunk) {
    // ---- single chunk: K and V of every key in flight at once ----
    s16x8 kf[DA_U], vf[DA_U];
    int kidx[DA_U];
    issue_q();
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int i = min(u * 32 + wave * 8 + slot, nkeys - 1);
      kidx[u] = decode_key_at(g, i, pos, r0, c0, nc) * 64 + (i < tlim ? tshift : 0);
    }
#pragma unroll
    for (int u = 0; u < DA_U; ++u) kf[u] = *reinterpret_cast<const s16x8*>(kb + kidx[u]);
    asm volatile("" ::: "memory");  // every K row ahead of every V row: the scores start while V streams
#pragma unroll
    for (int u = 0; u < DA_U; ++u) vf[u] = *reinterpret_cast<const s16x8*>(vb + kidx[u]);
    prologue();
    if (FROM_PART) {  // the new key is the last of the key list
      const s16x8 kn = *reinterpret_cast<const s16x8*>(&kvsh[0][sub * 8]);
      const s16x8 vn = *reinterpret_cast<const s16x8*>(&kvsh[1][sub * 8]);
#pragma unroll
      for (int u = 0; u < DA_U; ++u) {
        if (u * 32 + wave * 8 + slot == nkeys - 1) {
          kf[u] = kn;
          vf[u] = vn;
        }
      }
    }
    float sv[DA_U];
    float mloc = NEG_BIG;
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int i = u * 32 + wave * 8 + slot;
      sv[u] = i < nkeys ? slot_sum(dot8_bf(qb2, kf[u])) * LOG2E : NEG_BIG;
      mloc = fmaxf(mloc, sv[u]);
    }
    mloc = wave_max(mloc);
    if (lane == 0) red[0][wave] = mloc;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float ssum = 0.f;
    // P.V two rounds at a time: this lane's keys of rounds u and u + 1 (same 8 dims) as one packed-bf16 dot per
    // dim -- P rounded to bf16 (as the training kernels feed it to the MFMAs), summed for the denominator as rounded
    static_assert(DA_U % 2 == 0, "DA_U");
#pragma unroll
    for (int u = 0; u < DA_U; u += 2) {
      const bf16_raw p0 = f2bf(exp2f(sv[u] - m)), p1 = f2bf(exp2f(sv[u + 1] - m));  // 0 for invalid slots
      ssum += bf2f(p0) + bf2f(p1);
      const bf16x2 pp = __builtin_bit_cast(bf16x2, (uint32_t)p0 | ((uint32_t)p1 << 16));
      const uint32_t* va = reinterpret_cast<const uint32_t*>(&vf[u]);
      const uint32_t* vb2 = reinterpret_cast<const uint32_t*>(&vf[u + 1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = __builtin_amdgcn_perm(va[j], vb2[j], 0x01000504u);  // (v_u[2j], v_u+1[2j])
        const uint32_t hi = __builtin_amdgcn_perm(va[j], vb2[j], 0x03020706u);  // (v_u[2j+1], v_u+1[2j+1])
        acc[2 * j] = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2, lo), acc[2 * j], false);
        acc[2 * j + 1] = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2, hi), acc[2 * j + 1], false);
      }
    }
    ssum = wave_sum(ssum) * 0.125f;  // each key counted once per lane of its row
    if (lane == 0) red[1][wave] = ssum;
  } else {
    // ---- chunked: scores of every key into LDS, then softmax, then P.V ----
    issue_q();
    prologue();
    float mloc = NEG_BIG;
    for (int c = 0; c < nkeys; c += DA_CHUNK) {
      s16x8 kf[DA_U];
#pragma unroll
      for (int u = 0; u < DA_U; ++u) {
        const int i = c + u * 32 + wave * 8 + slot;
        kf[u] = i < nkeys ? *reinterpret_cast<const s16x8*>(kb + ((long)decode_key_at(g, i, pos, r0, c0, nc) * 64 + (i < tlim ? tshift : 0)))
                          : s16x8{};
      }
#pragma unroll
      for (int u = 0; u < DA_U; ++u) {
        const int i = c + u * 32 + wave * 8 + slot;
        if (i < nkeys) {
          const float sv = slot_sum(dot8(qd, kf[u]));
          mloc = fmaxf(mloc, sv);
          if (sub == 0) sc[i] = sv;
        }
      }
    }
    mloc = wave_max(mloc);
    if (lane == 0) red[0][wave] = mloc;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float ssum = 0.f;
    for (int c = 0; c < nkeys; c += DA_CHUNK) {
      s16x8 vf[DA_U];
#pragma unroll
      for (int u = 0; u < DA_U; ++u) {
        const int i = c + u * 32 + wave * 8 + slot;
        vf[u] = i < nkeys ? *reinterpret_cast<const s16x8*>(vb + ((long)decode_key_at(g, i, pos, r0, c0, nc) * 64 + (i < tlim ? tshift : 0)))
                          : s16x8{};
      }
#pragma unroll
      for (int u = 0; u < DA_U; ++u) {
        const int i = c + u * 32 + wave * 8 + slot;
        const float p = i < nkeys ? exp2f(sc[i] - m) : 0.f;
        ssum += p;
        float f[8];
        unpack8(vf[u], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += p * f[e];
      }
    }
    ssum = wave_sum(ssum) * 0.125f;
    if (lane == 0) red[1][wave] = ssum;
  }
  // ---- reduce acc over the 8 row slots of the wave, then over the 4 waves ----
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v = acc[e];
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    acc[e] = v;
  }
  if (slot == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wave][sub * 8 + e] = acc[e];
  }
  __syncthreads();
  inv = 1.0f / (red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  if (tid < 64) {
    const int b = bh / g.H, h = bh - b * g.H;
    const float o = (part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]) * inv;
    reinterpret_cast<bf16_raw*>(out)[(size_t)b * g.H * 64 + h * 64 + tid] = f2bf(o);
  }
}

// ---- VQGAN codebook embed: z[b, c, y, x] = codebook[idx[b, y*W + x], c]  (one_hot @ codebook) ----
__global__ void vq_embed_kernel(const int64_t* __restrict__ idx, const float* __restrict__ codebook, float* __restrict__ z,
                                int HW, int C, int B) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over (b, c, pixel): pixel fastest
  if (gid >= (long)B * C * HW) return;
  const int p = gid % HW;
  const long bc = gid / HW;
  const int c = bc % C, b = bc / C;
  const int64_t code = idx[(long)b * HW + p];
  z[gid] = codebook[code * C + c];
}

void decode_ln_shift(float* x, const float* w, const float* b, void* hist, void* y, const int* pos, const DecodeGeom& g,
                     int B, int D, int shift, hipStream_t st, const float* part, const void* pbias, const float* pscale, int KS) {
  const PendingRes pr{part, (const __bf16*)pbias, pscale, KS};
  switch (D) {
    case 256: hipLaunchKernelGGL(decode_ln_shift_kernel<256>, dim3(B), dim3(64), 0, st, x, w, b, (__bf16*)hist, (__bf16*)y, pos, g, shift, pr); break;
    case 512: hipLaunchKernelGGL(decode_ln_shift_kernel<512>, dim3(B), dim3(128), 0, st, x, w, b, (__bf16*)hist, (__bf16*)y, pos, g, shift, pr); break;
    case 1024: hipLaunchKernelGGL(decode_ln_shift_kernel<1024>, dim3(B), dim3(256), 0, st, x, w, b, (__bf16*)hist, (__bf16*)y, pos, g, shift, pr); break;
    case 2048: hipLaunchKernelGGL(decode_ln_shift_kernel<2048>, dim3(B), dim3(512), 0, st, x, w, b, (__bf16*)hist, (__bf16*)y, pos, g, shift, pr); break;
  }
}

void residual_from_partials(float* x, const float* part, const void* pbias, const float* pscale, int KS, int B, int D,
                            hipStream_t st) {
  const PendingRes pr{part, (const __bf16*)pbias, pscale, KS};
  const long t = (long)B * D / 4;
  hipLaunchKernelGGL(residual_from_partials_kernel, dim3((t + 255) / 256), dim3(256), 0, st, x, pr, B, D);
}

void decode_rope(const void* qkv, const float* cosT, const float* sinT, void* q, void* kc, void* vc, const int* pos,
                 const DecodeGeom& g, int B, float qscale, hipStream_t st) {
  const int threads = B * g.H * 8;
  hipLaunchKernelGGL(decode_rope_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, (const __bf16*)qkv, cosT, sinT,
                     (__bf16*)q, (__bf16*)kc, (__bf16*)vc, pos, g, B, qscale);
}

void decode_attn(const void* q, void* kc, void* vc, void* out, const int* pos, const DecodeGeom& g, int B, hipStream_t st,
                 const int* text_shared) {
  QkvPartials qp{};
  qp.text_shared = text_shared;
  hipLaunchKernelGGL(decode_attn_kernel<false>, dim3(B * g.H), dim3(256), 0, st, (const __bf16*)q, (__bf16*)kc, (__bf16*)vc,
                     (__bf16*)out, pos, g, qp);
}

void decode_attn_part(const float* part, int KS, const float* cosT, const float* sinT, float qscale, void* kc, void* vc, void* out,
                      const int* pos, const DecodeGeom& g, int B, hipStream_t st, const int* text_shared) {
  hipLaunchKernelGGL(decode_attn_kernel<true>, dim3(B * g.H), dim3(256), 0, st, (const __bf16*)nullptr, (__bf16*)kc, (__bf16*)vc,
                     (__bf16*)out, pos, g, QkvPartials{part, cosT, sinT, KS, B, qscale, text_shared});
}

void vq_embed(const int64_t* idx, const float* codebook, float* z, int HW, int C, int B, hipStream_t st) {
  const long t = (long)B * C * HW;
  hipLaunchKernelGGL(vq_embed_kernel, dim3((t + 255) / 256), dim3(256), 0, st, idx, codebook, z, HW, C, B);
}

}  // namespace dalle
