// Sparse causal attention for DALL-E (text-causal + axial-row / axial-col / conv-like / full image
// patterns) on CDNA4 MFMA (v_mfma_f32_32x32x16_bf16). SURVEY K7a-K7e.
//
// Storage layout (written by the rotary kernel): q/k/v are (B*H, Np, 64) bf16 with text rows
// [0, T) padded to Tp = ceil32(T), followed by the S*S image rows (row-major, or column-major for
// axial_col so that a column becomes 32 contiguous keys). All query/key blocks are 32 rows.
//
// Forward  : one workgroup = 4 waves = 4 consecutive 32-query blocks of one (b, h). The union of
//            their key tiles (text prefix + local image rows) is staged once per tile in LDS and
//            shared by the 4 waves (double buffered, register-staged loads issued before compute).
//            Per wave: S^T = K Q^T (keys on rows, queries on lanes: the softmax is lane-local),
//            online softmax in the exp2 domain, O^T += V^T P^T with V^T read by ds_read_b64_tr_b16
//            and P^T taken straight from the accumulator registers (no LDS round trip).
// Backward : dQ is query-centric (same schedule as the forward, recomputing P and dP);
//            dK/dV is key-centric (each wave owns 32 keys, loops over the query tiles that see them)
//            so no float atomics are needed anywhere.
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include <stdlib.h>
#include "geom.h"

#include "attn_tile.h"

namespace dalle {

// Both dim-halves of a wave's 32-token gradient tile (acc0: dims 0-31, acc1: dims 32-63, MFMA accumulator
// layout) staged once through 8 KB of the wave's LDS ([32 tokens][64 dims] fp32, 16-byte chunk c of row r at
// c ^ (r & 15)) and stored as whole 128-B token rows (8 lanes x 16 B per token, 8 tokens per instruction)
// with the rotary inverse applied (round 4: the half form wrote 64-B half rows, two store calls per tile).
__device__ __forceinline__ void rope_bwd_store_full(const RopeOut& ro, const AttnGeom& g, int bh, int s0, int t,
                                                    const f32x16& acc0, const f32x16& acc1, float scale, float* stage,
                                                    int lane) {
  const int hl = lane >> 5, c32 = lane & 31;
  const int b = bh / g.H, h = bh - b * g.H, HD = g.H * 64;
  const int q8 = lane & 7, d0 = 8 * q8;
  // the (cos, sin) rows of the lane's tokens, two passes ahead (the first two before the staging, so their
  // latency runs under it; each later pair right after the pass that frees its registers)
  int pp[4];
  f32x4 c0[2], c1[2], n0[2], n1[2];
  auto load_tab = [&](int it) {
    const int tok = it * 8 + (lane >> 3);
    const int p = st2seq(g, s0 + tok);
    pp[it] = p;
    const int pc = p < 0 ? 0 : p;
    const float* cp = ro.cosT + (size_t)pc * 64 + d0;
    const float* sp = ro.sinT + (size_t)pc * 64 + d0;
    c0[it & 1] = *reinterpret_cast<const f32x4*>(cp);
    c1[it & 1] = *reinterpret_cast<const f32x4*>(cp + 4);
    n0[it & 1] = *reinterpret_cast<const f32x4*>(sp);
    n1[it & 1] = *reinterpret_cast<const f32x4*>(sp + 4);
  };
  load_tab(0);
  load_tab(1);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& acc = dt ? acc1 : acc0;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int ch = (8 * dt + 2 * gq + hl) ^ (c32 & 15);
      *reinterpret_cast<f32x4*>(stage + c32 * 64 + 4 * ch) = f32x4{acc[4 * gq], acc[4 * gq + 1], acc[4 * gq + 2], acc[4 * gq + 3]};
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); the table loads stay in flight
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int tok = it * 8 + (lane >> 3), sl = it & 1;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stage + tok * 64 + 4 * ((2 * q8) ^ (tok & 15)));
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stage + tok * 64 + 4 * ((2 * q8 + 1) ^ (tok & 15)));
    const float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    const float c[8] = {c0[sl][0], c0[sl][1], c0[sl][2], c0[sl][3], c1[sl][0], c1[sl][1], c1[sl][2], c1[sl][3]};
    const float sn[8] = {n0[sl][0], n0[sl][1], n0[sl][2], n0[sl][3], n1[sl][0], n1[sl][1], n1[sl][2], n1[sl][3]};
    const int p = pp[it];
    if (it + 2 < 4) load_tab(it + 2);
    float y[8];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {  // transposed rotation of the pair (i, i + 1)
      const float a0 = x[i] * scale, a1 = x[i + 1] * scale;
      y[i] = a0 * c[i] + a1 * sn[i + 1];
      y[i + 1] = a1 * c[i + 1] + a0 * sn[i];
    }
    if (p >= 0) *reinterpret_cast<s16x8*>(ro.dqkv + ((size_t)b * g.n + p) * (3 * HD) + t * HD + h * 64 + d0) = pack8(y);
  }
  __builtin_amdgcn_wave_barrier();  // every lane has read the slot before it is rewritten
}

// ------------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------------
// Lazy rescale threshold (log2 units, T13): the running max is only moved when a tile's max exceeds
// it by more than this, so P <= 2^8 (exact in bf16's relative precision; fp32 sums have headroom).
constexpr float RESCALE_THR = 8.0f;

// max of x over the lane and its partner in the other 32-lane half (v_permlane32_swap, no LDS)
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Online-softmax state of one wave (32 queries on the lanes, keys on the accumulator rows).
struct SoftmaxState {
  float m = NEG_BIG;  // running max of RAW scores (q carries 1/sqrt(d))
  float lsum = 0.f;   // this lane half's partial row sum
  f32x16 o0 = {}, o1 = {};
};

// S^T tile(s) of one wave -> masked -> online update -> P^T (bf16) -> O^T += V^T P^T.
// NT key tiles at once (independent MFMA chains and one rescale decision for all of them).
template <int NT>
__device__ __forceinline__ void fwd_tiles(SoftmaxState& st, const __bf16* const (&Ks)[NT], const __bf16* const (&Vs)[NT],
                                          const int (&kt)[NT], const bf16x8 (&qf)[4], const AttnGeom& g, int qb, int qs,
                                          int lane) {
  const int hl = lane >> 5, c32 = lane & 31;
  constexpr float THR_RAW = RESCALE_THR / LOG2E;
  f32x16 s[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    s[j] = f32x16{};
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) s[j] = MFMA32(row_operand(Ks[j], ss, c32, hl), qf[ss], s[j]);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    if (!tile_full(g, qb, kt[j])) {
      const uint32_t mh = key_mask(g, qs, kt[j]) >> (4 * hl);
#pragma unroll
      for (int r = 0; r < 16; ++r) s[j][r] = mask_bit(mh, r) ? s[j][r] : NEG_BIG;
    }
  }
  float mt = NEG_BIG;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; r += 2) mt = fmaxf(fmaxf(mt, s[j][r]), s[j][r + 1]);
  mt = half_max(mt);
  if (!__all(mt <= st.m + THR_RAW)) {
    const float mnew = fmaxf(st.m, mt);
    const float alpha = fast_exp2((st.m - mnew) * LOG2E);
    st.m = mnew;
    st.lsum *= alpha;
#pragma unroll
    for (int r = 0; r < 16; ++r) { st.o0[r] *= alpha; st.o1[r] *= alpha; }
  }
  const float mc = st.m * LOG2E;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fast_exp2(fmaf(s[j][r], LOG2E, -mc));
      s[j][r] = p;
      ps += p;
    }
    st.lsum += ps;
    const bf16x8 p0 = cvt8(s[j], 0), p1 = cvt8(s[j], 8);
    st.o0 = MFMA32(tr_operand(Vs[j], 0, 0, lane), p0, st.o0);
    st.o0 = MFMA32(tr_operand(Vs[j], 1, 0, lane), p1, st.o0);
    st.o1 = MFMA32(tr_operand(Vs[j], 0, 1, lane), p0, st.o1);
    st.o1 = MFMA32(tr_operand(Vs[j], 1, 1, lane), p1, st.o1);
  }
}

// Forward. Workgroup = 4 waves = 4 consecutive 32-query blocks of one (b, h).
// Phase A (shared): the text key tiles every block needs, staged cooperatively two tiles per step
//   (double-buffered 2 x {Ka, Kb, Va, Vb}, register-staged loads issued before compute, T14).
// Phase B (wave-private): each image query block streams ITS OWN local key tiles through a private
//   LDS slot (reusing phase A's buffers) -- no workgroup barrier, no wave idling on other blocks' tiles.
// TPS: text tiles staged per barrier step (2: 32 KB of LDS; 3: 48 KB, 3 steps instead of 5 for 9 text tiles)
template <int MINB, bool PREFETCH_LOCAL = true, int TPS = 2>
__global__ __launch_bounds__(256, MINB) void attn_fwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                          const __bf16* __restrict__ V, __bf16* __restrict__ out,
                                                          float* __restrict__ lse, AttnGeom g) {
  static_assert(TPS == 2 || TPS == 3, "TPS");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TPS * TILE];  // 32 / 48 KB
  int grp, bh;
  xcd_remap(grp, bh);
  const int b = bh / g.H, h = bh - b * g.H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nqb = g.Np >> 5, ntext = g.Tp >> 5;
  const int qb0 = grp * 4;
  const int qb = qb0 + wave;
  const int qb_last = min(qb0 + 3, nqb - 1);
  const bool active = qb < nqb;
  const size_t base = (size_t)bh * g.Np * 64;

  const int n_text = qb_last < ntext ? qb_last + 1 : ntext;  // text tiles of the workgroup union
  const int my_text_end = active ? min(qb + 1, ntext) : 0;
  const int qs = qb * 32 + c32;
  bf16x8 qf[4];
  // this wave's Q tile (32 contiguous rows) by LDS-DMA into buffer 1, which the loop first refills at
  // step 0: 4 coalesced 1 KiB pieces instead of per-lane row reads that touch 32 lines per instruction
  dma_tile_wave(Q + base + (size_t)(active ? qb : 0) * 32 * 64, smem + 2 * TPS * TILE + wave * TILE, lane);
  SoftmaxState st;
  // phase B's first local (image) key tile, loaded NOW into registers: its HBM latency then hides under
  // phase A instead of being exposed after the last text pair (each local tile is read by one query tile)
  const bool has_local = active && qb >= ntext;
  const int lo = has_local ? local_lo_tile(g, qb) : 0;
  s16x8 kr[4], vr[4];
  auto load_loc = [&](int t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      const size_t off = base + (size_t)(t * 32 + row) * 64 + col;
      kr[j] = *reinterpret_cast<const s16x8*>(Kt + off);
      vr[j] = *reinterpret_cast<const s16x8*>(V + off);
    }
  };
  if (has_local && PREFETCH_LOCAL) load_loc(lo);

  // ---- phase A: shared text tiles, TPS per step ----
  const int nsteps = (n_text + TPS - 1) / TPS;
  // K tiles then V tiles of a step by LDS-DMA straight into buffer `buf` (dma_tile)
  auto dma_step = [&](int si, int buf) {
    __bf16* S0 = smem + buf * (2 * TPS * TILE);
#pragma unroll
    for (int t = 0; t < TPS; ++t) {
      const int tt = min(TPS * si + t, n_text - 1);
      dma_tile(Kt + base + (size_t)tt * 32 * 64, S0 + t * TILE, wave, lane);
      dma_tile(V + base + (size_t)tt * 32 * 64, S0 + (TPS + t) * TILE, wave, lane);
    }
  };
  dma_step(0, 0);
  __builtin_amdgcn_s_waitcnt(WAIT_VM0);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = row_operand(smem + 2 * TPS * TILE + wave * TILE, s, c32, hl);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): Q is in registers before step 0 refills buffer 1
  __syncthreads();
  for (int si = 0; si < nsteps; ++si) {
    const bool more = si + 1 < nsteps;
    if (more) dma_step(si + 1, (si + 1) & 1);  // that buffer was released by the previous step's barrier
    const __bf16* S0 = smem + (si & 1) * (2 * TPS * TILE);
    const int ta = TPS * si, tb = ta + 1;
    if (tb < my_text_end) {
      const __bf16* const Ks[2] = {S0, S0 + TILE};
      const __bf16* const Vs[2] = {S0 + TPS * TILE, S0 + (TPS + 1) * TILE};
      const int kt[2] = {ta, tb};
      fwd_tiles<2>(st, Ks, Vs, kt, qf, g, qb, qs, lane);
    } else if (ta < my_text_end) {
      const __bf16* const Ks[1] = {S0};
      const __bf16* const Vs[1] = {S0 + TPS * TILE};
      const int kt[1] = {ta};
      fwd_tiles<1>(st, Ks, Vs, kt, qf, g, qb, qs, lane);
    }
    if (TPS == 3 && ta + 2 < my_text_end) {
      const __bf16* const Ks[1] = {S0 + 2 * TILE};
      const __bf16* const Vs[1] = {S0 + (TPS + 2) * TILE};
      const int kt[1] = {ta + 2};
      fwd_tiles<1>(st, Ks, Vs, kt, qf, g, qb, qs, lane);
    }
    __builtin_amdgcn_s_waitcnt(WAIT_VM0);  // the next step's tiles landed (this wave's pieces) before the barrier
    __syncthreads();
  }

  // ---- phase B: this wave's local (image) key tiles, private LDS slot {K, V} ----
  if (has_local) {
    __bf16* P = smem + wave * (2 * TILE);
    if (!PREFETCH_LOCAL) load_loc(lo);
    for (int t = lo; t <= qb; ++t) {
      // the previous tile's LDS reads were consumed by its MFMAs (in program order before these stores)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
        *reinterpret_cast<s16x8*>(P + lds_idx(row, col)) = kr[j];
        *reinterpret_cast<s16x8*>(P + TILE + lds_idx(row, col)) = vr[j];
      }
      if (t < qb) load_loc(t + 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stores landed before any lane reads them
      __builtin_amdgcn_wave_barrier();
      const __bf16* const Ks[1] = {P};
      const __bf16* const Vs[1] = {P + TILE};
      const int kt[1] = {t};
      fwd_tiles<1>(st, Ks, Vs, kt, qf, g, qb, qs, lane);
      __builtin_amdgcn_wave_barrier();
    }
  }

  if (!active) return;
  const float ltot = half_sum(st.lsum);
  const float inv = 1.0f / ltot;
  lse[(size_t)bh * g.Np + qs] = st.m * LOG2E + log2f(ltot);
  // O through the wave's private slot (free: its last reads fed the MFMAs above), then stored as whole
  // 128-byte token rows (8 lanes x 16 B per row) instead of 8-byte pieces scattered over 32 rows
  __bf16* Os = smem + wave * (2 * TILE);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& o = dt ? st.o1 : st.o0;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      float f[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = o[4 * gq + i] * inv;
      *reinterpret_cast<s16x4*>(Os + lds_idx(c32, 32 * dt + 8 * gq + 4 * hl)) = pack4(f);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * i + (lane >> 3), col = (lane & 7) * 8;
    const s16x8 v = *reinterpret_cast<const s16x8*>(Os + lds_idx(row, col));
    const int p = st2seq(g, qb * 32 + row);
    if (p >= 0) *reinterpret_cast<s16x8*>(out + ((size_t)b * g.n + p) * (g.H * 64) + h * 64 + col) = v;
  }
}

// ------------------------------------------------------------------------------------------------
// delta = rowsum(dO * O) per storage row, for the concurrent backward (the dK/dV kernels start before
// the dQ kernel, which otherwise publishes it): one thread per (row, 16-byte chunk)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_delta_kernel(const __bf16* __restrict__ dout, const __bf16* __restrict__ out,
                                                         float* __restrict__ delta, AttnGeom g, int BH) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = gid & 7;
  const long row_g = gid >> 3;
  if (row_g >= (long)BH * g.Np) return;
  const int bh = row_g / g.Np, srow = row_g - (long)bh * g.Np;
  const int off = tok_row(g, srow);
  float acc = 0.f;
  if (off >= 0) {
    float fd[8], fo[8];
    unpack8(ld_tok(tok_base(dout, g, bh), off, chunk * 8), fd);
    unpack8(ld_tok(tok_base(out, g, bh), off, chunk * 8), fo);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc = fmaf(fd[i], fo[i], acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (chunk == 0) delta[row_g] = acc;
}

// ------------------------------------------------------------------------------------------------
// Backward dQ (query-centric)
// ------------------------------------------------------------------------------------------------
// dS for one key tile of the wave's 32 queries -> dQ^T += K^T dS^T (S^T layout as in the forward).
__device__ __forceinline__ void dq_tile(f32x16& dq0, f32x16& dq1, const __bf16* Ks, const __bf16* Vs, int tile,
                                        const bf16x8 (&qf)[4], const bf16x8 (&dof)[4], float lq, float dl,
                                        const AttnGeom& g, int qb, int qs, int lane) {
  const int hl = lane >> 5, c32 = lane & 31;
  f32x16 s = {}, dp = {};
#pragma unroll
  for (int ss = 0; ss < 4; ++ss) {
    s = MFMA32(row_operand(Ks, ss, c32, hl), qf[ss], s);
    dp = MFMA32(row_operand(Vs, ss, c32, hl), dof[ss], dp);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = fast_exp2(fmaf(s[r], LOG2E, -lq)) * (dp[r] - dl);
  if (!tile_full(g, qb, tile)) {
    const uint32_t mh = key_mask(g, qs, tile) >> (4 * hl);
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = mask_bit(mh, r) ? s[r] : 0.f;
  }
  const bf16x8 d0 = cvt8(s, 0), d1 = cvt8(s, 8);
  dq0 = MFMA32(tr_operand(Ks, 0, 0, lane), d0, dq0);
  dq0 = MFMA32(tr_operand(Ks, 1, 0, lane), d1, dq0);
  dq1 = MFMA32(tr_operand(Ks, 0, 1, lane), d0, dq1);
  dq1 = MFMA32(tr_operand(Ks, 1, 1, lane), d1, dq1);
}

// dQ (query-centric). Workgroup = 4 waves = 4 consecutive 32-query blocks of one (b, h), same two
// phases as the forward: (A) the text key tiles, staged cooperatively two per barrier step with the
// next pair's loads in flight; (B) each image query block streams ITS OWN local key tiles through a
// private LDS slot (no workgroup barrier, no wave idling on the other blocks' tiles).
// FUSE_LOCAL (axial row / col, rotary-fused output only): an image key tile is attended by exactly one
// query tile -- its own row's (column's) -- so that tile's dK / dV are produced right here, by the wave
// that owns the query tile, from the K / V it already staged and the Q / dO it already holds: the
// separate image-key dK/dV kernel (a launch that re-read Q, dO, K and V of every local tile) disappears.
// Text tiles are register-staged, two per barrier step (LDS-DMA staging two or three tiles per step, one or two
// steps ahead, measured no different: profiles/r6_attn_staging_depth.txt).
template <int MINB, bool FUSE_LOCAL, bool PREFETCH_LOCAL = false>
__global__ __launch_bounds__(256, MINB) void attn_bwd_dq_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                             const __bf16* __restrict__ V, const __bf16* __restrict__ dout,
                                                             const __bf16* __restrict__ out, const float* __restrict__ lse,
                                                             float* __restrict__ delta, __bf16* __restrict__ dQ, AttnGeom g,
                                                             RopeOut ro, int delta_ready) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * 2 * TILE];  // 32 KB
  __shared__ float fstats[FUSE_LOCAL ? 4 : 1][2][32];                 // fused dK/dV: per wave {lse, delta}
  __shared__ float dsh[4][32];                                          // prologue: per wave row deltas
  int grp, bh;
  xcd_remap(grp, bh);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5;
  const int nqb = g.Np >> 5, ntext = g.Tp >> 5;
  const int qb0 = grp * 4;
  const int qb = qb0 + wave;
  const int qb_last = min(qb0 + 3, nqb - 1);
  const bool active = qb < nqb;
  const size_t base = (size_t)bh * g.Np * 64;
  const __bf16* dob = tok_base(dout, g, bh);
  const __bf16* outb = tok_base(out, g, bh);

  const int n_text = qb_last < ntext ? qb_last + 1 : ntext;  // text tiles of the workgroup union
  const int my_text_end = active ? min(qb + 1, ntext) : 0;
  const int qs = qb * 32 + (lane & 31);
  const int qrow = active ? qs : 0;
  // Q from the storage layout; dO and O gathered from the token-major tensors (the former backward
  // prologue pass is folded in here): delta = rowsum(dO * O) of the wave's rows, published for the
  // dK/dV kernels that run next on the stream
  bf16x8 qf[4], dof[4];
  float dl = 0.f;
  {
  // Q (4 KB of contiguous storage rows) and dO (32 gathered 128-B token rows) of this wave through its 8 KB
  // LDS slot (phase A's buffers are not in use yet), 8 lanes per row: every load instruction covers 8 whole
  // 128-B lines, where the per-lane operand-layout loads touched 32 lines per instruction (round 4). delta
  // = rowsum(dO * O) from the same registers, reduced over each row's 8 lanes (fixed xor tree).
  // All twelve loads (Q, dO, O x 4) are issued before the first use: one HBM round trip per wave instead of
  // eight (the per-j load -> LDS store form compiled to a vmcnt(0) drain per load pair, ~330 us of the
  // kernel's memory skeleton at micro-batch 128). Padding rows load row 0 unconditionally and are zeroed
  // afterwards (no divergent load to hold the batch up).
  __bf16* Ps = smem + wave * (2 * TILE);
  float dpart[4];
  s16x8 qv[4], dv[4], ov[4];
  int toff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
    const int srow = (active ? qb * 32 : 0) + row;
    toff[j] = tok_row(g, srow);
    const int safe = toff[j] < 0 ? 0 : toff[j];
    qv[j] = *reinterpret_cast<const s16x8*>(Q + base + (size_t)srow * 64 + col);
    dv[j] = *reinterpret_cast<const s16x8*>(dob + safe + col);
    ov[j] = *reinterpret_cast<const s16x8*>(outb + safe + col);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
    if (toff[j] < 0) dv[j] = s16x8{};
    *reinterpret_cast<s16x8*>(Ps + lds_idx(row, col)) = qv[j];
    *reinterpret_cast<s16x8*>(Ps + TILE + lds_idx(row, col)) = dv[j];
    float fd[8], fo[8];
    unpack8(dv[j], fd);
    unpack8(ov[j], fo);
    dpart[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) dpart[j] = fmaf(fd[i], fo[i], dpart[j]);
  }
  if (!delta_ready) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dpart[j] += __shfl_xor(dpart[j], 1, 64);
      dpart[j] += __shfl_xor(dpart[j], 2, 64);
      dpart[j] += __shfl_xor(dpart[j], 4, 64);
      const int row = 8 * j + (lane >> 3);
      if ((lane & 7) == 0) {
        dsh[wave][row] = dpart[j];
        if (active) delta[(size_t)bh * g.Np + qb * 32 + row] = dpart[j];
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot and the row deltas are written
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    qf[s2] = row_operand(Ps, s2, lane & 31, hl);
    dof[s2] = row_operand(Ps + TILE, s2, lane & 31, hl);
  }
  dl = delta_ready ? delta[(size_t)bh * g.Np + qrow] : dsh[wave][lane & 31];
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();  // every wave has its operands in registers before phase A refills the buffers
  }
  const float lq = lse[(size_t)bh * g.Np + qrow];
  f32x16 dq0 = {}, dq1 = {};
  // PREFETCH_LOCAL: phase B's first local key tile loaded before phase A (see attn_fwd_kernel)
  const bool has_local = active && qb >= ntext;
  const int lo = has_local ? local_lo_tile(g, qb) : 0;
  s16x8 kr[4], vr[4];
  auto load_loc = [&](int t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      const size_t off = base + (size_t)(t * 32 + row) * 64 + col;
      kr[j] = *reinterpret_cast<const s16x8*>(Kt + off);
      vr[j] = *reinterpret_cast<const s16x8*>(V + off);
    }
  };
  if (has_local && PREFETCH_LOCAL) load_loc(lo);

  // ---- phase A: shared text tiles, two per step ----
  {
  const int st_row = tid >> 3, st_col = (tid & 7) * 8;
  const int st_off = lds_idx(st_row, st_col);
  const int npairs = (n_text + 1) >> 1;
  s16x8 sreg[4];  // Ka, Kb, Va, Vb chunks of this thread
  auto load_pair = [&](int pi) {
    const int ta = 2 * pi, tb = min(2 * pi + 1, n_text - 1);
    const size_t oa = base + (size_t)(ta * 32 + st_row) * 64 + st_col;
    const size_t ob = base + (size_t)(tb * 32 + st_row) * 64 + st_col;
    sreg[0] = *reinterpret_cast<const s16x8*>(Kt + oa);
    sreg[1] = *reinterpret_cast<const s16x8*>(Kt + ob);
    sreg[2] = *reinterpret_cast<const s16x8*>(V + oa);
    sreg[3] = *reinterpret_cast<const s16x8*>(V + ob);
  };
  auto store_pair = [&](int buf) {
    __bf16* S0 = smem + buf * (4 * TILE);
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<s16x8*>(S0 + i * TILE + st_off) = sreg[i];
  };
  load_pair(0);
  store_pair(0);
  __syncthreads();
  for (int pi = 0; pi < npairs; ++pi) {
    const bool more = pi + 1 < npairs;
    if (more) load_pair(pi + 1);
    const __bf16* S0 = smem + (pi & 1) * (4 * TILE);
    const int ta = 2 * pi, tb = 2 * pi + 1;
    if (ta < my_text_end) dq_tile(dq0, dq1, S0, S0 + 2 * TILE, ta, qf, dof, lq, dl, g, qb, qs, lane);
    if (tb < my_text_end) dq_tile(dq0, dq1, S0 + TILE, S0 + 3 * TILE, tb, qf, dof, lq, dl, g, qb, qs, lane);
    if (more) store_pair((pi + 1) & 1);
    __syncthreads();
  }
  }

  // ---- phase B: this wave's local (image) key tiles, private LDS slot {K, V} ----
  if (has_local) {
    __bf16* P = smem + wave * (2 * TILE);
    if (!PREFETCH_LOCAL) load_loc(lo);
    for (int t = lo; t <= qb; ++t) {
      // the previous tile's LDS reads were consumed by its MFMAs (in program order before these stores)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
        *reinterpret_cast<s16x8*>(P + lds_idx(row, col)) = kr[j];
        *reinterpret_cast<s16x8*>(P + TILE + lds_idx(row, col)) = vr[j];
      }
      if (t < qb) load_loc(t + 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stores landed before any lane reads them
      __builtin_amdgcn_wave_barrier();
      dq_tile(dq0, dq1, P, P + TILE, t, qf, dof, lq, dl, g, qb, qs, lane);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (FUSE_LOCAL && active && qb >= ntext && ro.dqkv) {
    // key-centric pass over the diagonal tile: K / V rows of the tile's keys (lane = key) from the slot,
    // then the slot is refilled with this wave's Q / dO tile (lane = query row) and the row stats
    __bf16* P = smem + wave * (2 * TILE);
    const int c32 = lane & 31;
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      kf[s2] = ld16(P + lds_idx(c32, 16 * s2 + 8 * hl));
      vf[s2] = ld16(P + TILE + lds_idx(c32, 16 * s2 + 8 * hl));
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot is read before it is rewritten
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      *reinterpret_cast<bf16x8*>(P + lds_idx(c32, 16 * s2 + 8 * hl)) = qf[s2];
      *reinterpret_cast<bf16x8*>(P + TILE + lds_idx(c32, 16 * s2 + 8 * hl)) = dof[s2];
    }
    if (hl == 0) {
      fstats[FUSE_LOCAL ? wave : 0][0][c32] = lq;
      fstats[FUSE_LOCAL ? wave : 0][1][c32] = dl;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const float(*st)[32] = fstats[FUSE_LOCAL ? wave : 0];
    const int ks = qb * 32 + c32;
    f32x16 sc = {}, dp = {};
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      sc = MFMA32(row_operand(P, s2, c32, hl), kf[s2], sc);
      dp = MFMA32(row_operand(P + TILE, s2, c32, hl), vf[s2], dp);
    }
    f32x16 ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = acc_row(r, hl);
      const float pr = fast_exp2(fmaf(sc[r], LOG2E, -st[0][ql]));
      sc[r] = pr;
      ds[r] = pr * (dp[r] - st[1][ql]);
    }
    const uint32_t mh = query_mask(g, ks, qb) >> (4 * hl);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool on = mask_bit(mh, r);
      sc[r] = on ? sc[r] : 0.f;
      ds[r] = on ? ds[r] : 0.f;
    }
    const bf16x8 p0 = cvt8(sc, 0), p1 = cvt8(sc, 8);
    const bf16x8 e0 = cvt8(ds, 0), e1 = cvt8(ds, 8);
    f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
    dv0 = MFMA32(tr_operand(P + TILE, 0, 0, lane), p0, dv0);
    dv0 = MFMA32(tr_operand(P + TILE, 1, 0, lane), p1, dv0);
    dv1 = MFMA32(tr_operand(P + TILE, 0, 1, lane), p0, dv1);
    dv1 = MFMA32(tr_operand(P + TILE, 1, 1, lane), p1, dv1);
    dk0 = MFMA32(tr_operand(P, 0, 0, lane), e0, dk0);
    dk0 = MFMA32(tr_operand(P, 1, 0, lane), e1, dk0);
    dk1 = MFMA32(tr_operand(P, 0, 1, lane), e0, dk1);
    dk1 = MFMA32(tr_operand(P, 1, 1, lane), e1, dk1);
    // the MFMAs consumed the slot's operands: it now stages this wave's dK / dV stores
    float* stage = reinterpret_cast<float*>(P);
    rope_bwd_store_full(ro, g, bh, qb * 32, 1, dk0, dk1, 1.0f, stage, lane);
    rope_bwd_store_full(ro, g, bh, qb * 32, 2, dv0, dv1, 1.0f, stage, lane);
  }
  // the epilogue's per-wave staging slot (4 KB at wave * 4 KB) overlaps other waves' phase-B slots
  __syncthreads();

  if (!active) return;
  if (ro.dqkv) {  // the loop's last barrier released smem: each wave stages through its own 8 KB
    float* stage = reinterpret_cast<float*>(smem) + wave * 2048;
    rope_bwd_store_full(ro, g, bh, qb * 32, 0, dq0, dq1, ro.qscale, stage, lane);
    return;
  }
  __bf16* qp = dQ + base + (size_t)qs * 64;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& o = dt ? dq1 : dq0;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      float f[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = o[4 * gq + i];
      *reinterpret_cast<s16x4*>(qp + 32 * dt + 8 * gq + 4 * hl) = pack4(f);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Backward dK / dV for the IMAGE key blocks (key-centric, no float atomics). Image keys are seen only
// by the few query tiles of their local pattern (axial: the key's own row tile; conv_like: the next
// K row tiles; full: every later tile), so each wave owns one 32-key block and streams ITS OWN query
// tiles {Q, dO, lse, delta} through a private LDS slot (register prefetch one tile ahead): no
// workgroup barrier and no wave idling on the other blocks' tiles.
// ------------------------------------------------------------------------------------------------
template <int MINB>
__global__ __launch_bounds__(256, MINB) void attn_bwd_dkdv_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                               const __bf16* __restrict__ V, const __bf16* __restrict__ dout,
                                                               const float* __restrict__ lse, const float* __restrict__ delta,
                                                               __bf16* __restrict__ dK, __bf16* __restrict__ dV, AttnGeom g,
                                                               RopeOut ro) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[4 * 2 * TILE];  // per wave {Q, dO}
  __shared__ float stats[4][2][32];                                   // per wave {lse, delta}
  int grp, bh;
  xcd_remap(grp, bh);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nkb = g.Np >> 5, ntext = g.Tp >> 5;
  const int kb = ntext + grp * 4 + wave;
  if (kb >= nkb) return;  // wave-uniform; no workgroup barrier below
  const size_t base = (size_t)bh * g.Np * 64;
  const __bf16* dob = tok_base(dout, g, bh);
  const int ks = kb * 32 + c32;
  const int q_hi = local_hi_qtile(g, kb);
  bf16x8 kf[4], vf[4];
  {
    const __bf16* kp = Kt + base + (size_t)ks * 64 + 8 * hl;
    const __bf16* vp = V + base + (size_t)ks * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) { kf[s] = ld16(kp + 16 * s); vf[s] = ld16(vp + 16 * s); }
  }
  __bf16* Qs = smem + wave * (2 * TILE);
  __bf16* Ds = Qs + TILE;
  s16x8 qr[4], dr[4];
  float sv = 0.f;
  auto load_tile = [&](int qt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      const size_t off = base + (size_t)(qt * 32 + row) * 64 + col;
      qr[j] = *reinterpret_cast<const s16x8*>(Q + off);
      dr[j] = ld_tok(dob, tok_row(g, qt * 32 + row), col);
    }
    sv = (hl ? delta : lse)[(size_t)bh * g.Np + qt * 32 + c32];
  };
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  load_tile(kb);
  for (int qt = kb; qt <= q_hi; ++qt) {
    // this tile's LDS image (the previous tile's reads were consumed by its MFMAs, earlier in order)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<s16x8*>(Qs + lds_idx(row, col)) = qr[j];
      *reinterpret_cast<s16x8*>(Ds + lds_idx(row, col)) = dr[j];
    }
    stats[wave][hl][c32] = sv;
    if (qt < q_hi) load_tile(qt + 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    f32x16 sc = {}, dp = {};
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      sc = MFMA32(row_operand(Qs, ss, c32, hl), kf[ss], sc);
      dp = MFMA32(row_operand(Ds, ss, c32, hl), vf[ss], dp);
    }
    f32x16 ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = acc_row(r, hl);
      const float pr = fast_exp2(fmaf(sc[r], LOG2E, -stats[wave][0][ql]));
      sc[r] = pr;
      ds[r] = pr * (dp[r] - stats[wave][1][ql]);
    }
    if (!tile_full(g, qt, kb)) {
      const uint32_t mh = query_mask(g, ks, qt) >> (4 * hl);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool on = mask_bit(mh, r);
        sc[r] = on ? sc[r] : 0.f;
        ds[r] = on ? ds[r] : 0.f;
      }
    }
    const bf16x8 p0 = cvt8(sc, 0), p1 = cvt8(sc, 8);
    const bf16x8 d0 = cvt8(ds, 0), d1 = cvt8(ds, 8);
    dv0 = MFMA32(tr_operand(Ds, 0, 0, lane), p0, dv0);
    dv0 = MFMA32(tr_operand(Ds, 1, 0, lane), p1, dv0);
    dv1 = MFMA32(tr_operand(Ds, 0, 1, lane), p0, dv1);
    dv1 = MFMA32(tr_operand(Ds, 1, 1, lane), p1, dv1);
    dk0 = MFMA32(tr_operand(Qs, 0, 0, lane), d0, dk0);
    dk0 = MFMA32(tr_operand(Qs, 1, 0, lane), d1, dk0);
    dk1 = MFMA32(tr_operand(Qs, 0, 1, lane), d0, dk1);
    dk1 = MFMA32(tr_operand(Qs, 1, 1, lane), d1, dk1);
    __builtin_amdgcn_wave_barrier();
  }
  if (ro.dqkv) {  // this wave's private {Q, dO} slot is free after its last tile
    float* stage = reinterpret_cast<float*>(Qs);
    rope_bwd_store_full(ro, g, bh, kb * 32, 1, dk0, dk1, 1.0f, stage, lane);
    rope_bwd_store_full(ro, g, bh, kb * 32, 2, dv0, dv1, 1.0f, stage, lane);
    return;
  }
  __bf16* kp = dK + base + (size_t)ks * 64;
  __bf16* vp = dV + base + (size_t)ks * 64;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& a = dt ? dk1 : dk0;
    const f32x16& c = dt ? dv1 : dv0;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      float fa[4], fc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { fa[i] = a[4 * gq + i]; fc[i] = c[4 * gq + i]; }
      *reinterpret_cast<s16x4*>(kp + 32 * dt + 8 * gq + 4 * hl) = pack4(fa);
      *reinterpret_cast<s16x4*>(vp + 32 * dt + 8 * gq + 4 * hl) = pack4(fc);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Backward dK / dV for the TEXT key blocks: every later query tile (all image queries see all text
// keys) attends to them. One workgroup owns TWO 32-key blocks; wave w handles key block kb0 + (w&1)
// over the query tiles of parity (w>>1). Each step stages two query tiles {Q, dO} (one per parity)
// cooperatively, so every staged tile serves two key blocks (half the Q/dO traffic of one block per
// workgroup) while the critical path stays at half the query tiles. The two parity partials of each
// key block are summed through LDS at the end (fixed order, deterministic).
// ------------------------------------------------------------------------------------------------
template <int MINB, int QT = 2>
__global__ __launch_bounds__(256, MINB) void attn_bwd_dkdv_text_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                                    const __bf16* __restrict__ V, const __bf16* __restrict__ dout,
                                                                    const float* __restrict__ lse, const float* __restrict__ delta,
                                                                    __bf16* __restrict__ dK, __bf16* __restrict__ dV, AttnGeom g,
                                                                    RopeOut ro) {
  // QT query tiles per step (2: one per parity; 4: two per parity, half the steps and barriers):
  // 2 stages x QT x {Q, dO} tile images + the per-query stats
  static_assert(QT == 2 || QT == 4, "QT");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * QT * 2 * TILE];
  __shared__ float stats[2][QT][2][32];  // [stage][tile][lse | delta][row]
  int grp, bh;
  xcd_remap(grp, bh);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nqb = g.Np >> 5, ntext = g.Tp >> 5;
  const int kb0 = grp * 2;
  // odd last key block (QT 4): all four waves work on it, wave w taking the query tile t = w of each
  // step, instead of two waves idling on the absent partner block
  const bool tail = QT == 4 && kb0 + 1 >= ntext;
  const int kb = tail ? kb0 : kb0 + (wave & 1), par = tail ? wave : wave >> 1;
  const bool active = kb < ntext;
  const size_t base = (size_t)bh * g.Np * 64;
  const __bf16* dob = tok_base(dout, g, bh);
  const int ks = kb * 32 + c32;
  bf16x8 kf[4], vf[4];
  {
    const int krow = active ? ks : 0;
    const __bf16* kp = Kt + base + (size_t)krow * 64 + 8 * hl;
    const __bf16* vp = V + base + (size_t)krow * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) { kf[s] = ld16(kp + 16 * s); vf[s] = ld16(vp + 16 * s); }
  }
  // query tiles kb0 .. nqb-1, QT per step: tile t of step i is kb0 + QT i + t, handled by the waves of
  // parity t & 1
  const int nsteps = (nqb - kb0 + QT - 1) / QT;
  // staging: thread tid moves chunk (row, col) of Q and dO of every tile of the step
  const int st_row = (tid & 255) >> 3, st_col = (tid & 7) * 8;
  const int st_off = lds_idx(st_row, st_col);
  s16x8 sreg[2 * QT];  // Q0, dO0, Q1, dO1, ...
  float sl = 0.f;
  auto load_step = [&](int i) {
#pragma unroll
    for (int pp = 0; pp < QT; ++pp) {
      const int qt = min(kb0 + QT * i + pp, nqb - 1);
      const size_t off = base + (size_t)(qt * 32 + st_row) * 64 + st_col;
      sreg[2 * pp] = *reinterpret_cast<const s16x8*>(Q + off);
      sreg[2 * pp + 1] = ld_tok(dob, tok_row(g, qt * 32 + st_row), st_col);
    }
    if (tid < QT * 64) {  // lse / delta rows of every tile: QT x 2 stats x 32
      const int pp = tid >> 6, which = (tid >> 5) & 1, r = tid & 31;
      const int qt = min(kb0 + QT * i + pp, nqb - 1);
      const float* src = which ? delta : lse;
      sl = src[(size_t)bh * g.Np + qt * 32 + r];
    }
  };
  auto store_step = [&](int buf) {
#pragma unroll
    for (int pp = 0; pp < QT; ++pp) {
      __bf16* T0 = smem + (buf * QT + pp) * (2 * TILE);
      *reinterpret_cast<s16x8*>(T0 + st_off) = sreg[2 * pp];
      *reinterpret_cast<s16x8*>(T0 + TILE + st_off) = sreg[2 * pp + 1];
    }
    if (tid < QT * 64) stats[buf][tid >> 6][(tid >> 5) & 1][tid & 31] = sl;
  };
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  if (nsteps > 0) {
    load_step(0);
    store_step(0);
  }
  // retire the K / V fragment loads here: with them possibly in flight at the loop entry (the
  // conditional prologue above), the compiler guards each MFMA of the loop with a vmcnt wait that
  // in fact drains the NEXT step's prefetch loads, exposing their latency every step
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  // one query tile: scores S^T / dP^T (key rows x query lanes), probabilities and dS, then the
  // dV += P^T dO / dK += dS^T Q products
  auto scores = [&](const __bf16* Qs, const __bf16* Ds, f32x16& sc, f32x16& dp) {
    sc = f32x16{};
    dp = f32x16{};
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      sc = MFMA32(row_operand(Qs, ss, c32, hl), kf[ss], sc);
      dp = MFMA32(row_operand(Ds, ss, c32, hl), vf[ss], dp);
    }
  };
  auto probs = [&](int buf, int tt, int qt, f32x16& sc, f32x16& dp) {  // sc <- P, dp <- dS
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = acc_row(r, hl);
      const float pr = fast_exp2(fmaf(sc[r], LOG2E, -stats[buf][tt][0][ql]));
      sc[r] = pr;
      dp[r] = pr * (dp[r] - stats[buf][tt][1][ql]);
    }
    if (!tile_full(g, qt, kb)) {
      const uint32_t mh = query_mask(g, ks, qt) >> (4 * hl);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool on = mask_bit(mh, r);
        sc[r] = on ? sc[r] : 0.f;
        dp[r] = on ? dp[r] : 0.f;
      }
    }
  };
  auto accum = [&](const __bf16* Qs, const __bf16* Ds, const f32x16& sc, const f32x16& ds) {
    const bf16x8 p0 = cvt8(sc, 0), p1 = cvt8(sc, 8);
    const bf16x8 d0 = cvt8(ds, 0), d1 = cvt8(ds, 8);
    dv0 = MFMA32(tr_operand(Ds, 0, 0, lane), p0, dv0);
    dv0 = MFMA32(tr_operand(Ds, 1, 0, lane), p1, dv0);
    dv1 = MFMA32(tr_operand(Ds, 0, 1, lane), p0, dv1);
    dv1 = MFMA32(tr_operand(Ds, 1, 1, lane), p1, dv1);
    dk0 = MFMA32(tr_operand(Qs, 0, 0, lane), d0, dk0);
    dk0 = MFMA32(tr_operand(Qs, 1, 0, lane), d1, dk0);
    dk1 = MFMA32(tr_operand(Qs, 0, 1, lane), d0, dk1);
    dk1 = MFMA32(tr_operand(Qs, 1, 1, lane), d1, dk1);
  };
  // (measured: issuing the second tile's score products ahead of the first tile's softmax -- a
  // two-tile software pipeline -- made this kernel slower at B128: 677-690 us against 642 us)
  for (int i = 0; i < nsteps; ++i) {
    const bool more = i + 1 < nsteps;
    if (more) load_step(i + 1);
    const int buf = i & 1;
#pragma unroll
    for (int u = 0; u < QT / 2; ++u) {
      const int tt = tail ? par : par + 2 * u;
      const int qt = kb0 + QT * i + tt;
      if (active && qt < nqb && qt >= kb && !(tail && u > 0)) {
        const __bf16* Qs = smem + (buf * QT + tt) * (2 * TILE);
        f32x16 sc, dp;
        scores(Qs, Qs + TILE, sc, dp);
        probs(buf, tt, qt, sc, dp);
        accum(Qs, Qs + TILE, sc, dp);
      }
    }
    if (more) store_step((i + 1) & 1);
    __syncthreads();
  }
  // the other parity's waves hand their partials to the parity 0 wave of the same key block through
  // LDS (value-major layout: consecutive lanes on consecutive banks), which sums (fixed order) and
  // stores; a tail workgroup sums three partials (waves 1..3) into wave 0
  float* red = reinterpret_cast<float*>(smem);  // up to 3 slots x 64 values x 64 lanes floats = 48 KB
  if (par != 0) {
    const int slot = tail ? wave - 1 : (wave & 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      red[(slot * 64 + r) * 64 + lane] = dk0[r];
      red[(slot * 64 + 16 + r) * 64 + lane] = dk1[r];
      red[(slot * 64 + 32 + r) * 64 + lane] = dv0[r];
      red[(slot * 64 + 48 + r) * 64 + lane] = dv1[r];
    }
  }
  __syncthreads();
  if (par == 0 && active) {
    const int s0 = tail ? 0 : (wave & 1), s1 = tail ? 3 : s0 + 1;
    for (int sl2 = s0; sl2 < s1; ++sl2) {
      const float* mine = red + sl2 * 64 * 64;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk0[r] += mine[r * 64 + lane];
        dk1[r] += mine[(16 + r) * 64 + lane];
        dv0[r] += mine[(32 + r) * 64 + lane];
        dv1[r] += mine[(48 + r) * 64 + lane];
      }
    }
    if (ro.dqkv) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // this key block's partials are consumed: stage through them
      __builtin_amdgcn_wave_barrier();
      float* stage = red + (wave & 1) * 64 * 64;
      rope_bwd_store_full(ro, g, bh, kb * 32, 1, dk0, dk1, 1.0f, stage, lane);
      rope_bwd_store_full(ro, g, bh, kb * 32, 2, dv0, dv1, 1.0f, stage, lane);
    } else {
      __bf16* kp = dK + base + (size_t)ks * 64;
      __bf16* vp = dV + base + (size_t)ks * 64;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const f32x16& a = dt ? dk1 : dk0;
        const f32x16& c = dt ? dv1 : dv0;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float fa[4], fc[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            fa[i] = a[4 * gq + i];
            fc[i] = c[4 * gq + i];
          }
          *reinterpret_cast<s16x4*>(kp + 32 * dt + 8 * gq + 4 * hl) = pack4(fa);
          *reinterpret_cast<s16x4*>(vp + 32 * dt + 8 * gq + 4 * hl) = pack4(fc);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// Occupancy per kernel (workgroups per CU the register budget is compiled for), measured at B48
// (profiles/r1_attn_occupancy.txt): the forward is latency-bound at 2 waves/SIMD (178 VGPRs) and runs
// 225 -> 183 us at 3 (168 VGPRs); dq fits 148 VGPRs at 3; the dK/dV kernels spill at 3 and slow down
// 1.9-2.8x, so they stay at 2. Staging per barrier step: forward 2 text tiles (3 measured slower), dQ
// register-staged text pairs (LDS-DMA no different, profiles/r6_attn_staging_depth.txt), text dK/dV 4 query tiles (-0.9 ms per bench24
// B128 step vs 2); local-tile prefetch off (more spills at occupancy 3). Round-4 numbers of every
// variant: profiles/r4ab_switches_b128.txt, profiles/INDEX.md.
void attn_fwd(const void* q, const void* k, const void* v, void* out, float* lse, const AttnGeom& g, int BH, hipStream_t st) {
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  hipLaunchKernelGGL((attn_fwd_kernel<3, false>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (__bf16*)out, lse, g);
}

// the fused one-workgroup-per-head backward (attention_fused.hip)
bool attn_bwd_fused_ok(const AttnGeom& g, bool rope_out, bool has_freqs);
void attn_bwd_fused_launch(const void* q, const void* k, const void* v, const void* dout, const void* out, const float* lse,
                           const AttnGeom& g, int BH, hipStream_t st, const RopeOut& ro, const RotSpec& rsp);

void attn_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout, const float* lse,
              float* delta, void* dq, void* dk, void* dv, const AttnGeom& g, int BH, hipStream_t st,
              const float* cosT, const float* sinT, void* dqkv, float qscale, const float* rotf, int rot_nl, int rot_np,
              float rot_img_text_pos, float rot_text_axial) {
  const RopeOut ro{cosT, sinT, static_cast<__bf16*>(dqkv), qscale};
  if (attn_bwd_fused_ok(g, dqkv != nullptr, rotf != nullptr)) {
    attn_bwd_fused_launch(q, k, v, dout, out, lse, g, BH, st, ro, RotSpec{rotf, rot_nl, rot_np, rot_img_text_pos, rot_text_axial});
    return;
  }
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  // axial row / col: every image key tile is attended by exactly its own query tile -> dK / dV of the
  // image keys inside the dQ kernel (rotary-fused output path)
  const bool fuse_local = dqkv != nullptr && (g.pattern == 1 || g.pattern == 2);
  const int ntext = g.Tp / 32, nimg = g.Np / 32 - ntext;
  if (fuse_local)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, true, false>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, (const __bf16*)dout, (const __bf16*)out, lse, delta, (__bf16*)dq, g, ro, 0);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, false, false>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, (const __bf16*)dout, (const __bf16*)out, lse, delta, (__bf16*)dq, g, ro, 0);
  // text key blocks (long, every image query attends them): one block per workgroup, queries split over waves
  hipLaunchKernelGGL((attn_bwd_dkdv_text_kernel<2, 4>), dim3((ntext + 1) / 2, BH), dim3(256), 0, st, (const __bf16*)q,
                     (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dk, (__bf16*)dv, g, ro);
  // image key blocks (short, local patterns): four blocks per workgroup -- unless the dQ kernel did them
  if (!fuse_local)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<2>), dim3((nimg + 3) / 4, BH), dim3(256), 0, st, (const __bf16*)q,
                       (const __bf16*)k, (const __bf16*)v, (const __bf16*)dout, lse, delta, (__bf16*)dk, (__bf16*)dv, g, ro);
}

}  // namespace dalle
