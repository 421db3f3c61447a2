// Skinny GEMM for the decode step: Y (M <= 64, N) = X (M, K) . W (N, K)^T with M the
// decode batch. At M = 64 every weight byte is used for 64 MACs only, so the op is bound by streaming
// W out of HBM once (QKV 6 MB, FF1 16 MB, FF2 8 MB, out 2 MB at d=1024) -- the library GEMMs' 32x64
// tiles walk K serially and reach ~10% of that. The layout here is built for "all of W in flight at
// once":
//   * a workgroup owns 16 output columns (one v_mfma_f32_16x16x32_bf16 N-block; two for GEGLU, the
//     value and gate halves) and WK waves split its K range; cross-workgroup split-K (KS) when the
//     column count alone cannot fill the 256 CUs;
//   * each lane issues all of its loads up front: 4 x 16 B of W rows (64 contiguous bytes per lane,
//     256 per row across the 4 lane groups) and 4 x 16 B per 16-row M-block of X (L2-resident);
//     the K order inside a wave's 128-wide chunk is permuted identically for X and W, so fragments
//     come straight from global memory in MFMA operand layout -- no LDS staging;
//   * the WK partial tiles reduce through LDS in a fixed order; the KS partials go to a workspace and
//     the LAST arriving workgroup (device-scope counter, self-resetting) sums them in ks order, so the
//     result is deterministic and the op is one launch;
//   * epilogues fuse what follows the projection in the decode step: bias (+fp32 out), GEGLU, the
//     LayerScale residual update x += scale * (y + b) on the fp32 stream, and the 3-axis rotary with
//     q/k/v scattered into the query buffer and the KV cache at the device-side position.
#include "common.h"
#include "geom.h"

#include <vector>

namespace dalle {

constexpr int SK_U = 4;            // MFMA steps per wave (K = 128 per wave)
constexpr int SK_KW = 32 * SK_U;   // K elements per wave
constexpr int SK_KSU = 8;          // in-launch split-K: slabs the last arriver reads in one batch (more: a loop)

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// ---- EPI 5 tail: one row of the pending residual update, then the decode LayerNorm + cached token shift ----
// (the same arithmetic as decode_ln_shift_kernel in decode.hip, which does it as a launch of its own). The KS
// split-K slabs of the row were stored write-through (sc1) by the other workgroups of this launch, so every
// load of them here is an agent-scope (sc1) load; everything else was written by earlier launches.
// NT threads, CH chunks of 4 columns per thread (N <= 4 * NT * CH; columns past N idle), KS <= KSM slabs.
template <int NT, int CH, int KSM>
__device__ __forceinline__ void ln_tail_row(const SkinnyArgs& a, int row, int pos) {
  constexpr int NW = NT / 64;
  __shared__ float tred[2][NW], tpiv[NW];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int D = a.N, B = a.M;
  float* xr = a.resid + (size_t)row * D;
  __bf16* hb = static_cast<__bf16*>(a.hist) + (size_t)row * a.n * D;
  const float* part = static_cast<const float*>(a.out);
  f32x4 v[CH], wv[CH], bv[CH], sc[CH];
  s16x4 sh[CH], pbr[CH];
  unsigned long long t[CH][KSM][2];
  // every load first (one memory round trip): slabs, the row, the LN and pending parameters, the shifted row
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) {
    const int c = 4 * (tid + ch * NT);
    const bool in = c < D;
    const int cc = in ? c : 0;  // idle columns re-read column 0 and are masked out of everything below
#pragma unroll
    for (int k = 0; k < KSM; ++k) {
      const int kk = k < a.KS ? k : a.KS - 1;  // slabs past KS re-read the last one and are weighted 0
      gu64* p = (gu64*)(part + ((size_t)kk * B + row) * D + cc);
      t[ch][k][0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t[ch][k][1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    v[ch] = *reinterpret_cast<const f32x4*>(xr + cc);
    wv[ch] = *reinterpret_cast<const f32x4*>(a.ln_w + cc);
    bv[ch] = *reinterpret_cast<const f32x4*>(a.ln_b + cc);
    sc[ch] = *reinterpret_cast<const f32x4*>(a.scale + cc);
    pbr[ch] = a.bias ? *reinterpret_cast<const s16x4*>(static_cast<const __bf16*>(a.bias) + cc) : s16x4{};
    sh[ch] = s16x4{};
    if (a.shift && cc < D / 2) {
      int src = -1;
      if (pos < a.T) {
        src = pos - 1;
      } else {
        const int k = pos - a.T;
        if (cc < D / 4) src = (k >= a.S) ? pos - a.S : -1;
        else src = (k % a.S) ? pos - 1 : -1;
      }
      if (src >= 0) sh[ch] = *reinterpret_cast<const s16x4*>(hb + (size_t)src * D + cc);
    }
  }
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) {
    const int c = 4 * (tid + ch * NT);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KSM; ++k) {  // fixed ks order: deterministic
      const float wk = k < a.KS ? 1.f : 0.f;
      acc[0] += wk * __uint_as_float((unsigned)t[ch][k][0]);
      acc[1] += wk * __uint_as_float((unsigned)(t[ch][k][0] >> 32));
      acc[2] += wk * __uint_as_float((unsigned)t[ch][k][1]);
      acc[3] += wk * __uint_as_float((unsigned)(t[ch][k][1] >> 32));
    }
    float pb[4];
    unpack4(pbr[ch], pb);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[ch][i] += sc[ch][i] * (acc[i] + pb[i]);
    if (c < D) *reinterpret_cast<f32x4*>(xr + c) = v[ch];
  }
  // both moments in one reduction round, shifted about each wave's first element (as decode_ln_shift); a wave's
  // element count from the columns it holds (every wave holds at least column 4 * 64 * wave < D, or none)
  const float piv = __shfl(v[0][0], 0, 64);
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int ch = 0; ch < CH; ++ch)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = 4 * (tid + ch * NT) < D ? v[ch][i] - piv : 0.f;
      s += d;
      q += d * d;
    }
  s = wave_sum(s);
  q = wave_sum(q);
  if (lane == 0) { tred[0][wave] = s; tred[1][wave] = q; tpiv[wave] = piv; }
  __syncthreads();
  const float p0 = tpiv[0];
  float S = 0.f, Q = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    int cnt = 0;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) cnt += min(max(D - 4 * (ch * NT + 64 * i), 0), 256);
    if (cnt == 0) continue;
    const float dp = tpiv[i] - p0, si = tred[0][i], n = (float)cnt;
    S += si + n * dp;
    Q += tred[1][i] + 2.f * dp * si + n * dp * dp;
  }
  const float inv_d = 1.0f / (float)D;
  const float dm = S * inv_d;
  const float mean = p0 + dm;
  const float var = fmaxf(Q * inv_d - dm * dm, 0.f);
  const float rstd = rsqrtf(var + 1e-5f);
  __bf16* yr = static_cast<__bf16*>(a.y) + (size_t)row * D;
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) {
    const int c = 4 * (tid + ch * NT);
    if (c >= D) continue;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (v[ch][i] - mean) * rstd * wv[ch][i] + bv[ch][i];
    const s16x4 packed = pack4(o);
    *reinterpret_cast<s16x4*>(hb + (size_t)pos * D + c) = packed;
    *reinterpret_cast<s16x4*>(yr + c) = (a.shift && c < D / 2) ? sh[ch] : packed;
  }
}

// MB: 16-row M-blocks; NBV: 16-column output blocks per wave (they share the wave's X fragments, so
// X bytes per W byte fall as 4 / NBV at M = 64); EPI 1 (GEGLU) adds NBV gate blocks; WK: waves per
// workgroup, each on its own 128-wide K chunk.
template <int MB, int NBV, int EPI, int WK>
__global__ __launch_bounds__(64 * WK) void skinny_gemm_kernel(SkinnyArgs a) {
  constexpr int G = EPI == 1 ? 2 : 1;  // value (+ gate) groups
  constexpr int NB = NBV * G;
  __shared__ float red[WK * MB * NB * 256];
  __shared__ int s_last;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const int tile = blockIdx.x, ks = blockIdx.y, ntiles = gridDim.x;
  const int n0 = tile * 16 * NBV;
  const int steps = a.steps;  // consecutive 128-wide K chunks per wave
  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[i][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int st = 0; st < steps; ++st) {
    // lane's K elements for MFMA step j: kb + j * jstr (8 each). Standard MFMA order (fq * 8, j * 32):
    // one load instruction reads 64 contiguous bytes of each of 16 rows
    const bool perm = (a.dbg & 4) != 0;
    const int kb = ((ks * WK + wave) * steps + st) * SK_KW + fq * (perm ? 8 * SK_U : 8);
    const int jstr = perm ? 8 : 32;
    bf16x8 w[NB][SK_U], x[MB][SK_U];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int wrow = (nb < NBV ? n0 + nb * 16 : a.N + n0 + (nb - NBV) * 16) + fr;
      const __bf16* wp = static_cast<const __bf16*>(a.W) + (size_t)wrow * a.K + kb;
      if (a.dbg & 2) {
#pragma unroll
        for (int j = 0; j < SK_U; ++j) w[nb][j] = bf16x8{};
        continue;
      }
#pragma unroll
      for (int j = 0; j < SK_U; ++j) w[nb][j] = *reinterpret_cast<const bf16x8*>(wp + jstr * j);
    }
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int row = i * 16 + fr;
      if (row < a.M && !(a.dbg & 1)) {
        const __bf16* xp = static_cast<const __bf16*>(a.X) + (size_t)row * a.ldx + kb;
#pragma unroll
        for (int j = 0; j < SK_U; ++j) x[i][j] = *reinterpret_cast<const bf16x8*>(xp + jstr * j);
      } else {
#pragma unroll
        for (int j = 0; j < SK_U; ++j) x[i][j] = bf16x8{};
      }
    }
#pragma unroll
    for (int j = 0; j < SK_U; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[i][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[i][j], w[nb][j], acc[i][nb], 0, 0, 0);
  }

  // ---- fixed-order reduction of the WK wave partials (through LDS: also the layout change to pairs) ----
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wave * MB * NB + i * NB + nb) * 256 + r * 64 + lane] = acc[i][nb][r];
  __syncthreads();

  // output pairs: (row, adjacent column pair) -> one thread each
  constexpr int PR = 8 * NBV;  // pairs per row
  constexpr int P = MB * 16 * PR;
  constexpr int NT = 64 * WK;
  constexpr int PPT = (P + NT - 1) / NT;
  float v[PPT][G][2];  // this thread's output pairs: idx = tid + c * NT
#pragma unroll
  for (int c = 0; c < PPT; ++c) {
    const int idx = tid + c * NT;
    if (idx >= P) break;
    const int row = idx / PR, cpair = idx % PR;
    const int cb = cpair >> 3, cp = cpair & 7;
    const int i = row >> 4, rr = row & 15;
    const int base = (rr & 3) * 64 + (rr >> 2) * 16 + 2 * cp;
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float s = 0.f;
#pragma unroll
        for (int ww = 0; ww < WK; ++ww) s += red[(ww * MB * NB + i * NB + gi * NBV + cb) * 256 + base + e];
        v[c][gi][e] = s;
      }
  }

  // ---- cross-workgroup split-K: partials to the workspace, the last arriver sums them in ks order ----
  // Partials are written and read with agent-scope (device-coherent, L2-bypassing `sc1`) accesses and
  // ordered by vmcnt + barrier only: a __threadfence() here would write back and invalidate the L2
  // of the XCD on every workgroup (measured 5x slower).
  // bias values of this thread's outputs, loaded ahead of the hand-off they do not depend on (in the epilogue each
  // bias read compiled to its own load -> vmcnt(0) round trip after the slab sum)
  const __bf16* bias = static_cast<const __bf16*>(a.bias);
  const __bf16* bsrc = bias != nullptr ? bias : static_cast<const __bf16*>(a.W);  // branch-free: a valid address either way
  float bvv[PPT][G][2];
#pragma unroll
  for (int c = 0; c < PPT; ++c) {
    const int idx = min(tid + c * NT, P - 1);
    const int col = n0 + 2 * (idx % PR);
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const uint32_t w2 = *reinterpret_cast<const uint32_t*>(bsrc + gi * a.N + col);  // the column pair (col even)
      bvv[c][gi][0] = bias != nullptr ? __uint_as_float(w2 << 16) : 0.f;
      bvv[c][gi][1] = bias != nullptr ? __uint_as_float(w2 & 0xffff0000u) : 0.f;
    }
  }
  if (a.KS > 1 && EPI != 4 && EPI != 5) {
#pragma unroll
    for (int c = 0; c < PPT; ++c) {
      const int idx = tid + c * NT;
      if (idx >= P) break;
      float* wp = a.ws + (((size_t)ks * ntiles + tile) * P + idx) * (2 * G);
#pragma unroll
      for (int gi = 0; gi < G; ++gi)
#pragma unroll
        for (int e = 0; e < 2; ++e) __hip_atomic_store(wp + 2 * gi + e, v[c][gi][e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_s_waitcnt(0);  // stores acknowledged (vmcnt(0) lgkmcnt(0))
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = (prev == a.KS - 1);
    }
    __syncthreads();
    if (!s_last) return;
#pragma unroll
    for (int c = 0; c < PPT; ++c) {
      const int idx = tid + c * NT;
      if (idx >= P) break;
#pragma unroll
      for (int gi = 0; gi < G; ++gi) { v[c][gi][0] = 0.f; v[c][gi][1] = 0.f; }
      if (a.KS <= SK_KSU) {
        // every slab's value loaded at once (slab index clamped, the extra slots not summed): one round trip
        // instead of one per slab
        float lv[SK_KSU][G][2];
#pragma unroll
        for (int s = 0; s < SK_KSU; ++s) {
          float* wp = a.ws + (((size_t)min(s, a.KS - 1) * ntiles + tile) * P + idx) * (2 * G);
#pragma unroll
          for (int gi = 0; gi < G; ++gi)
#pragma unroll
            for (int e = 0; e < 2; ++e) lv[s][gi][e] = __hip_atomic_load(wp + 2 * gi + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int s = 0; s < SK_KSU; ++s)
          if (s < a.KS)
#pragma unroll
            for (int gi = 0; gi < G; ++gi)
#pragma unroll
              for (int e = 0; e < 2; ++e) v[c][gi][e] += lv[s][gi][e];  // fixed ks order
      } else {
        for (int s = 0; s < a.KS; ++s) {
          float* wp = a.ws + (((size_t)s * ntiles + tile) * P + idx) * (2 * G);
#pragma unroll
          for (int gi = 0; gi < G; ++gi)
#pragma unroll
            for (int e = 0; e < 2; ++e) v[c][gi][e] += __hip_atomic_load(wp + 2 * gi + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if (tid == 0) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- epilogue ----
  int pos = 0;
  if (EPI == 3) {
    pos = *a.pos;
    if (pos < 0 || pos >= a.n) return;  // a replay past the cache end is a no-op, never an OOB write
  }
#pragma unroll
  for (int c = 0; c < PPT; ++c) {
    const int idx = tid + c * NT;
    if (idx >= P) break;
    const int row = idx / PR, col = n0 + 2 * (idx % PR);
    if (row >= a.M) continue;
    float y0 = v[c][0][0], y1 = v[c][0][1];
    if (EPI == 4) {  // raw split-K partial slab ks: the consuming kernel sums the KS slabs (+ bias)
      *reinterpret_cast<float2*>(reinterpret_cast<float*>(a.out) + ((size_t)ks * a.M + row) * a.N + col) = make_float2(y0, y1);
      continue;
    }
    if (EPI == 5) {  // the same slab, stored write-through (sc1): read back in this launch by the tail workgroups
      gu64* sp = (gu64*)(reinterpret_cast<float*>(a.out) + ((size_t)ks * a.M + row) * a.N + col);
      __hip_atomic_store(sp, (unsigned long long)__float_as_uint(y0) | ((unsigned long long)__float_as_uint(y1) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (bias != nullptr) { y0 += bvv[c][0][0]; y1 += bvv[c][0][1]; }
    if (EPI == 0) {
      if (a.out_f32) {
        *reinterpret_cast<float2*>(reinterpret_cast<float*>(a.out) + (size_t)row * a.N + col) = make_float2(y0, y1);
      } else {
        uint32_t pk = (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<__bf16*>(a.out) + (size_t)row * a.N + col) = pk;
      }
    } else if (EPI == 1) {
      float g0 = v[c][G - 1][0], g1 = v[c][G - 1][1];
      if (bias != nullptr) { g0 += bvv[c][G - 1][0]; g1 += bvv[c][G - 1][1]; }
      uint32_t pk = (uint32_t)f2bf(y0 * gelu_erf(g0)) | ((uint32_t)f2bf(y1 * gelu_erf(g1)) << 16);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<__bf16*>(a.out) + (size_t)row * a.N + col) = pk;
    } else if (EPI == 2) {
      float2* rp = reinterpret_cast<float2*>(a.resid + (size_t)row * a.N + col);
      float2 r = *rp;
      r.x += a.scale[col] * y0;
      r.y += a.scale[col + 1] * y1;
      *rp = r;
    } else {
      const int HD = a.H * 64;
      const int t = col / HD, h = (col - t * HD) >> 6, dh = col & 63;
      const float c0 = a.cosT[pos * 64 + dh], c1 = a.cosT[pos * 64 + dh + 1];
      const float s0 = a.sinT[pos * 64 + dh], s1 = a.sinT[pos * 64 + dh + 1];
      float r0 = y0 * c0 + y1 * s0, r1 = y1 * c1 + y0 * s1;
      const size_t bh = (size_t)row * a.H + h;
      __bf16* dst;
      if (t == 0) {
        r0 *= a.qscale;
        r1 *= a.qscale;
        dst = static_cast<__bf16*>(a.q) + bh * 64 + dh;
      } else {
        dst = static_cast<__bf16*>(t == 1 ? a.kc : a.vc) + (bh * a.n + pos) * 64 + dh;
      }
      *reinterpret_cast<uint32_t*>(dst) = (uint32_t)f2bf(r0) | ((uint32_t)f2bf(r1) << 16);
    }
  }
  if constexpr (EPI == 5) {
    // hand-off (guide Guideline 16, R1 with a ticket counter): every storing wave drains its sc1 slab stores,
    // the workgroup meets, ONE lane takes a ticket. Tickets of one launch are [e * total, (e + 1) * total)
    // for the e-th launch on this counter word (every workgroup takes exactly one), so the epoch comes from
    // the ticket itself and no per-launch reset or argument is needed under graph replay.
    __shared__ unsigned s_tk;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_tk = __hip_atomic_fetch_add((gu32*)a.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned total = gridDim.x * gridDim.y, tk = s_tk, within = tk % total;
    if (within < total - (unsigned)a.M) return;  // not one of the last M arrivers
    const int trow = (int)(within - (total - (unsigned)a.M));
    if (tid == 0) {
      // the last M arrivers wait for the rest of the launch: every workgroup with a smaller ticket has
      // already added, so this waits at most for the other tail workgroups' adds (all resident: they run)
      const unsigned target = (tk / total + 1) * total;
      unsigned spins = 0;
      while (__hip_atomic_load((gu32*)a.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 22)) {  // bounded: never hang the device on a lost arrival
          __hip_atomic_store((gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    const int pos = *a.pos;
    if (pos < 0 || pos >= a.n) return;  // a replay past the cache end is a no-op, as decode_ln_shift
    constexpr int NT = 64 * WK;
    const int ch = (a.N + 4 * NT - 1) / (4 * NT);
    if (ch == 1) ln_tail_row<NT, 1, 8>(a, trow, pos);
    else if (ch == 2) ln_tail_row<NT, 2, 8>(a, trow, pos);
    else if (ch == 4) ln_tail_row<NT, 4, 4>(a, trow, pos);
  }
}

// ---- launch shape: (NBV, WK, KS) ----
static int g_force_nbv = 0, g_force_wk = 0, g_force_ks = 0, g_dbg = 0;  // benchmark override

void skinny_force_config(int nbv, int wk, int ks, int dbg) {
  g_force_nbv = nbv;
  g_force_wk = wk;
  g_force_ks = ks;
  g_dbg = dbg;
}

static bool skinny_valid(int M, int N, int K, int G, int nbv, int wk) {
  const int mb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int chunks = K / SK_KW;
  // registers: MB * NB accumulators (<= 16 f32x4); LDS reduction tile: WK * MB * NB KiB (<= 64)
  return N % (16 * nbv) == 0 && chunks % wk == 0 && mb * nbv * G <= 16 && wk * mb * nbv * G <= 64 &&
         (wk == 1 || wk == 2 || wk == 4 || wk == 8);
}

// Default (measured, benchmarks/bench_skinny.py --sweep, M = 64): 8 waves per workgroup, each on its
// own 128-wide K chunk. The kernel is bound by the X bytes every CU must read (64 x K bf16 per
// workgroup, ~45 GB/s per CU), not by the weight stream, so: no cross-workgroup split-K while
// K <= 1024 (its partial hand-off costs 3-5 us of serialised latency, more than the halved X saves);
// at K = 4096 split-K 4 beats 4 chunks in a row per wave (10.5 vs 20.4 us); two column blocks per
// wave (X fragment reuse) only pays where the column tiles alone oversubscribe the CUs (N >= 8192).
static void skinny_shape(int M, int N, int K, int G, int& NBV, int& WK, int& KS, int& steps) {
  const int chunks = K / SK_KW;
  if (g_force_nbv > 0 && g_force_ks > 0 && skinny_valid(M, N, K, G, g_force_nbv, g_force_wk) &&
      chunks % (g_force_wk * g_force_ks) == 0) {
    NBV = g_force_nbv;
    WK = g_force_wk;
    KS = g_force_ks;
  } else {
    NBV = (G == 1 && N >= 8192 && skinny_valid(M, N, K, G, 2, 8)) ? 2 : 1;
    WK = 1;
    for (int wk : {8, 4, 2, 1})
      if (skinny_valid(M, N, K, G, NBV, wk)) { WK = wk; break; }
    KS = chunks / WK;
  }
  steps = chunks / (WK * KS);
}

std::vector<int> skinny_shape_info(int M, int N, int K, int G) {
  int NBV, WK, KS, steps;
  skinny_shape(M, N, K, G, NBV, WK, KS, steps);
  return {NBV, WK, KS, steps};
}

int skinny_ks(int M, int N, int K, int G) {
  int NBV, WK, KS, steps;
  skinny_shape(M, N, K, G, NBV, WK, KS, steps);
  return KS;
}

template <int MB, int NBV, int EPI>
static void skinny_launch_wk(const SkinnyArgs& a, dim3 grid, int WK, hipStream_t st) {
  switch (WK) {
    case 1: hipLaunchKernelGGL((skinny_gemm_kernel<MB, NBV, EPI, 1>), grid, dim3(64), 0, st, a); break;
    case 2: hipLaunchKernelGGL((skinny_gemm_kernel<MB, NBV, EPI, 2>), grid, dim3(128), 0, st, a); break;
    case 4:
      if constexpr (MB * NBV * (EPI == 1 ? 2 : 1) <= 16) hipLaunchKernelGGL((skinny_gemm_kernel<MB, NBV, EPI, 4>), grid, dim3(256), 0, st, a);
      break;
    default:
      if constexpr (MB * NBV * (EPI == 1 ? 2 : 1) <= 8) hipLaunchKernelGGL((skinny_gemm_kernel<MB, NBV, EPI, 8>), grid, dim3(512), 0, st, a);
      break;
  }
}

template <int MB, int EPI>
static void skinny_launch_nb(const SkinnyArgs& a, dim3 grid, int NBV, int WK, hipStream_t st) {
  switch (NBV) {
    case 1: skinny_launch_wk<MB, 1, EPI>(a, grid, WK, st); break;
    case 2: skinny_launch_wk<MB, 2, EPI>(a, grid, WK, st); break;
    default:
      if constexpr (MB * 4 * (EPI == 1 ? 2 : 1) <= 16) skinny_launch_wk<MB, 4, EPI>(a, grid, WK, st);
      break;
  }
}

template <int EPI>
static void skinny_launch(const SkinnyArgs& a, dim3 grid, int NBV, int WK, hipStream_t st) {
  if (a.M <= 16) skinny_launch_nb<1, EPI>(a, grid, NBV, WK, st);
  else if (a.M <= 32) skinny_launch_nb<2, EPI>(a, grid, NBV, WK, st);
  else skinny_launch_nb<4, EPI>(a, grid, NBV, WK, st);
}

// Split-K partials for a consumer that sums them (EPI 4): every workgroup covers 16 columns x a
// 128 * WK slice of K and stores its fp32 slab; no hand-off between workgroups, so K is split as finely
// as the X bytes per CU want (the kernel is bound by the X rows each CU reads, see skinny_shape).
int skinny_partials_ks(int M, int N, int K) {
  const int chunks = K / SK_KW;
  const int big = K >= 4096;
  int wk = big ? 4 : 2;  // waves per workgroup (measured: benchmarks/bench_skinny.py)
  while (wk > 1 && (chunks % wk || !skinny_valid(M, N, K, 1, 1, wk))) wk >>= 1;
  return chunks / wk;
}
bool skinny_partials(SkinnyArgs a, hipStream_t st) {
  if (a.M < 1 || a.M > 64 || a.N % 16 || a.K % SK_KW) return false;
  const int chunks = a.K / SK_KW;
  const int KS = skinny_partials_ks(a.M, a.N, a.K);
  const int WK = chunks / KS;
  if (KS != a.KS || !skinny_valid(a.M, a.N, a.K, 1, 1, WK)) return false;
  a.steps = 1;
  a.dbg = g_dbg;
  skinny_launch<4>(a, dim3(a.N / 16, KS), 1, WK, st);
  return true;
}

// The same split-K slabs with the consumer's LayerNorm in the launch's tail (EPI 5): the last M workgroups to
// finish each take one row (see ln_tail_row). False where the tail's register tiling does not fit (then the
// caller keeps the separate decode_ln_shift launch).
bool skinny_partials_ln(SkinnyArgs a, hipStream_t st) {
  if (a.M < 1 || a.M > 64 || a.N % 16 || a.K % SK_KW) return false;
  const int chunks = a.K / SK_KW;
  const int KS = skinny_partials_ks(a.M, a.N, a.K);
  const int WK = chunks / KS;
  if (KS != a.KS || !skinny_valid(a.M, a.N, a.K, 1, 1, WK)) return false;
  const int NT = 64 * WK, ch = (a.N + 4 * NT - 1) / (4 * NT);
  if (!(((ch == 1 || ch == 2) && KS <= 8) || (ch == 4 && KS <= 4))) return false;
  if ((a.N / 16) * KS < a.M) return false;  // fewer workgroups than tail rows
  a.steps = 1;
  a.dbg = g_dbg;
  const dim3 grid(a.N / 16, KS);
  if (a.M <= 16) skinny_launch_wk<1, 1, 5>(a, grid, WK, st);
  else if (a.M <= 32) skinny_launch_wk<2, 1, 5>(a, grid, WK, st);
  else skinny_launch_wk<4, 1, 5>(a, grid, WK, st);
  return true;
}
bool skinny_partials_ln_ok(int M, int N, int K) {
  if (M < 1 || M > 64 || N % 16 || K % SK_KW) return false;
  const int KS = skinny_partials_ks(M, N, K), WK = (K / SK_KW) / KS, NT = 64 * WK;
  const int ch = (N + 4 * NT - 1) / (4 * NT);
  return (((ch == 1 || ch == 2) && KS <= 8) || (ch == 4 && KS <= 4)) && (N / 16) * KS >= M;
}

// Host entry (the binding validates tensors); false for unsupported shapes.
bool skinny_gemm(int epi, SkinnyArgs a, hipStream_t st) {
  const int G = epi == 1 ? 2 : 1;
  if (a.M < 1 || a.M > 64 || a.N % 16 || a.K % SK_KW) return false;
  int NBV, WK, KS, steps;
  skinny_shape(a.M, a.N, a.K, G, NBV, WK, KS, steps);
  a.steps = steps;
  if (KS != a.KS || !skinny_valid(a.M, a.N, a.K, G, NBV, WK)) return false;  // workspace sized for this KS
  dim3 grid(a.N / (16 * NBV), KS);
  a.dbg = g_dbg;
  switch (epi) {
    case 0: skinny_launch<0>(a, grid, NBV, WK, st); break;
    case 1: skinny_launch<1>(a, grid, NBV, WK, st); break;
    case 2: skinny_launch<2>(a, grid, NBV, WK, st); break;
    case 3: skinny_launch<3>(a, grid, NBV, WK, st); break;
    default: return false;
  }
  return true;
}

}  // namespace dalle
