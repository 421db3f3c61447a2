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

namespace dalle {

// LDS tile image: rows of 64 bf16 (128 B, no padding); 16-byte chunk ch of row r lives at chunk
// ch ^ swz(r). With this XOR both MFMA operand reads are bank-conflict-free: the ds_read_b128 row
// reads (16-lane groups read 16 different rows, one chunk: the 8 same-parity rows of a group get 8
// distinct swz values) and the ds_read_b64_tr_b16 transposed reads (a 32-lane half reads rows
// R..R+3 x 4 chunks: rows R and R+2 share a bank row, and swz differs in bit 2 between them).
__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int lds_idx(int r, int col) { return r * 64 + ((((col >> 3) ^ swz(r)) << 3) | (col & 7)); }
constexpr int TILE = 32 * 64;  // elements of one 32-row tile image

// LDS-DMA staging of one 32-row tile image (no VGPRs, no ds_write): wave w moves rows 8w .. 8w+7 as one
// 1 KiB global_load_lds_dwordx4 piece. The DMA writes lane-linearly (lane l -> row 8w + l/8, physical
// chunk l%8), so the swizzle goes on the SOURCE: that lane fetches logical chunk (l%8) ^ swz(row).
__device__ __forceinline__ void dma_tile(const __bf16* src_rows, __bf16* tile, int wave, int lane) {
  const int row = 8 * wave + (lane >> 3);
  const __bf16* gp = src_rows + (size_t)row * 64 + (((lane & 7) ^ swz(row)) << 3);
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)gp,
                                   (void __attribute__((address_space(3)))*)(tile + 512 * wave), 16, 0, 0);
}
// a whole tile moved by ONE wave (4 pieces)
__device__ __forceinline__ void dma_tile_wave(const __bf16* src_rows, __bf16* tile, int lane) {
#pragma unroll
  for (int piece = 0; piece < 4; ++piece) dma_tile(src_rows, tile, piece, lane);
}
constexpr int WAIT_VM0 = 0x0F70;  // s_waitcnt vmcnt(0) (expcnt / lgkmcnt untouched)

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ int st2seq(const AttnGeom& g, int s) {
  if (s < g.T) return s;
  if (s < g.Tp) return -1;
  const int kst = s - g.Tp;
  const int k = (g.pattern == 2) ? ((kst & (g.S - 1)) << g.logS) + (kst >> g.logS) : kst;
  const int p = g.T + k;
  return p < g.n ? p : -1;
}

// Token-major [B, n, H*64] tensors (the attention output and its gradient) read by storage row.
// tok_base: the (b, h) slice's first element; tok_row: the element offset of storage row s within it
// (32-bit: B*n*H*64 < 2^31 for every supported shape), -1 for padding rows -- branch-free, since these
// sit in the dK/dV kernels' staging loops.
__device__ __forceinline__ const __bf16* tok_base(const __bf16* x, const AttnGeom& g, int bh) {
  const int b = bh / g.H, h = bh - b * g.H;
  return x + (size_t)b * g.n * (g.H * 64) + h * 64;
}
__device__ __forceinline__ int tok_row(const AttnGeom& g, int s) {
  const int k = s - g.Tp;
  const int kk = (g.pattern == 2) ? ((k & (g.S - 1)) << g.logS) + (k >> g.logS) : k;
  const int p = s < g.Tp ? (s < g.T ? s : -1) : (g.T + kk < g.n ? g.T + kk : -1);
  return p < 0 ? -1 : p * (g.H * 64);
}
__device__ __forceinline__ s16x8 ld_tok(const __bf16* __restrict__ xb, int row_off, int col) {
  return row_off < 0 ? s16x8{} : *reinterpret_cast<const s16x8*>(xb + row_off + col);
}

// bits [lo, hi] of a 32-bit word (empty when hi < lo; bounds clipped to [0, 31])
__device__ __forceinline__ uint32_t range_bits(int lo, int hi) {
  lo = max(lo, 0);
  hi = min(hi, 31);
  if (hi < lo) return 0u;
  const uint32_t upto = hi == 31 ? 0xffffffffu : ((1u << (hi + 1)) - 1u);
  return upto & ~((1u << lo) - 1u);
}

// Allowed keys of storage query qs within key tile kt, as a bit mask over the tile's 32 keys.
// Semantics: text query -> causal over the padded text rows; image query -> every
// real text key plus its local pattern (full: causal; axial row/col: same row of the (possibly
// column-major) storage, causal; conv_like: the upper-left K x K window).
__device__ __forceinline__ uint32_t key_mask(const AttnGeom& g, int qs, int kt) {
  const int k0 = kt * 32;
  if (qs < g.Tp) return range_bits(0, qs - k0);
  if (k0 < g.Tp) return range_bits(0, g.T - 1 - k0);
  const int qk = qs - g.Tp, kk0 = k0 - g.Tp;
  if (g.pattern == 0) return range_bits(0, qk - kk0);
  const int qr = qk >> g.logS;
  if (g.pattern != 3) return range_bits((qr << g.logS) - kk0, qk - kk0);
  const int qc = qk & (g.S - 1);
  const int c_lo = max(0, qc - g.K + 1);
  const int rows = g.S >= 32 ? 1 : (32 >> g.logS);
  uint32_t m = 0u;
  for (int i = 0; i < rows; ++i) {
    const int kr = (kk0 >> g.logS) + i;
    if (kr > qr - g.K && kr <= qr) m |= range_bits((kr << g.logS) + c_lo - kk0, (kr << g.logS) + qc - kk0);
  }
  return m;
}

// Allowed queries of storage key ks within query tile qt (the transpose of key_mask).
__device__ __forceinline__ uint32_t query_mask(const AttnGeom& g, int ks, int qt) {
  const int q0 = qt * 32;
  if (ks < g.Tp) {
    if (q0 < g.Tp) return range_bits(ks - q0, 31);
    return ks < g.T ? 0xffffffffu : 0u;
  }
  if (q0 < g.Tp) return 0u;
  const int kk = ks - g.Tp, qk0 = q0 - g.Tp;
  if (g.pattern == 0) return range_bits(kk - qk0, 31);
  const int kr = kk >> g.logS;
  if (g.pattern != 3) return range_bits(kk - qk0, ((kr + 1) << g.logS) - 1 - qk0);
  const int kc = kk & (g.S - 1);
  const int c_hi = min(g.S - 1, kc + g.K - 1);
  const int rows = g.S >= 32 ? 1 : (32 >> g.logS);
  uint32_t m = 0u;
  for (int i = 0; i < rows; ++i) {
    const int qr = (qk0 >> g.logS) + i;
    if (qr >= kr && qr < kr + g.K) m |= range_bits((qr << g.logS) + kc - qk0, (qr << g.logS) + c_hi - qk0);
  }
  return m;
}

// wave-uniform: every (query, key) pair of the 32x32 tile (query tile qt, key tile kt) is allowed, so
// the mask can be skipped (all text tiles but the padded boundary one for image queries, tiles
// strictly below the diagonal for text queries / the dense pattern)
__device__ __forceinline__ bool tile_full(const AttnGeom& g, int qt, int kt) {
  const int ntext = g.Tp >> 5;
  if (kt < ntext) {
    if (kt * 32 + 31 >= g.T) return false;
    return qt >= ntext || kt < qt;
  }
  return g.pattern == 0 && qt >= ntext && kt < qt;
}

// XCD-aware workgroup order (guide §1 "Workgroups, grid, and XCD partitioning"): the dispatcher
// deals linear workgroup ids round-robin over the 8 XCDs, each with its own L2. Remap so every
// workgroup of one (b, h) runs on the same XCD, consecutively: its K/V (or Q/dO) stay L2-resident.
__device__ __forceinline__ void xcd_remap(int& grp, int& bh) {
  const int ng = gridDim.x, BH = gridDim.y;
  if (BH & 7) { grp = blockIdx.x; bh = blockIdx.y; return; }
  const int L = blockIdx.x + blockIdx.y * ng;
  const int x = L & 7, j = L >> 3;
  bh = x + 8 * (j / ng);
  grp = j - (j / ng) * ng;
}

// first local (image) key tile needed by image query block qb
__device__ __forceinline__ int local_lo_tile(const AttnGeom& g, int qb) {
  const int kq0 = qb * 32 - g.Tp;
  int lo;
  if (g.pattern == 0) lo = 0;
  else if (g.pattern == 3) lo = max(0, (kq0 >> g.logS) - (g.K - 1)) << g.logS;
  else lo = (kq0 >> g.logS) << g.logS;
  return (g.Tp + lo) >> 5;
}

// last query tile that attends to image key block kb
__device__ __forceinline__ int local_hi_qtile(const AttnGeom& g, int kb) {
  const int kk1 = kb * 32 + 31 - g.Tp;
  int hi;
  if (g.pattern == 0) hi = g.I - 1;
  else if (g.pattern == 3) hi = min(g.I, ((kk1 >> g.logS) + g.K) << g.logS) - 1;
  else hi = (((kk1 >> g.logS) + 1) << g.logS) - 1;
  return (g.Tp + hi) >> 5;
}

__device__ __forceinline__ bf16x8 ld16(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// transposed 4x16 block read (T10): lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3
__device__ __forceinline__ s16x4 tr_read(const __bf16* lds) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds));
}

// A operand X^T (32 x 16) for k-step `ss` of a [row][64] swizzled LDS tile, where the MFMA K index is
// the tile row in the accumulator-permuted order (element j of lane half h = row 16ss + 8(j>>2) + 4h + (j&3)).
__device__ __forceinline__ bf16x8 tr_operand(const __bf16* tile, int ss, int dt, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 16 * ss + 4 * (g >> 1) + (i >> 2);
  const int col = 32 * dt + 16 * (g & 1) + 4 * (i & 3);
  const s16x4 lo = tr_read(tile + lds_idx(row, col));
  const s16x4 hi = tr_read(tile + lds_idx(row + 8, col));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// B operand rows: row c32 of the tile, chunk 2ss + hl (the K index of the S / dP products)
__device__ __forceinline__ bf16x8 row_operand(const __bf16* tile, int ss, int c32, int hl) {
  return ld16(tile + lds_idx(c32, 16 * ss + 8 * hl));
}

// bit of accumulator register r (rows acc_row(r, hl)) in a mask already shifted right by 4*hl
__device__ __forceinline__ bool mask_bit(uint32_t mh, int r) { return (mh >> ((r & 3) + 8 * (r >> 2))) & 1u; }

__device__ __forceinline__ bf16x8 cvt8(const f32x16& a, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)a[base + j];
  return r;
}

__device__ __forceinline__ int acc_row(int r, int hl) { return (r & 3) + 8 * (r >> 2) + 4 * hl; }

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)


// Fused rotary backward (replaces rope_bwd_kernel when `dqkv` is set): each backward kernel's dQ / dK
// / dV tile is rotated back with its tokens' (cos, sin) rows -- rotary pairs are adjacent dims -- and
// written straight into the token-major projection gradient dqkv (B, n, 3*H*64), slot t (0 q, 1 k,
// 2 v). No (B*H, Np, 64) dq / dk / dv intermediates and no separate rotary pass (a 750 MB round trip
// per layer at B48). The tile is re-laid out through LDS first (rope_bwd_store_half) so the table
// reads and the stores are contiguous per token.
struct RopeOut {
  const float* cosT;
  const float* sinT;
  __bf16* dqkv;  // nullptr: write dq / dk / dv in storage layout instead
  float qscale;
  // the rotary frequencies for angles computed in-kernel (fused backward; null: tables only): per rotary pair j
  // of the head, its frequency in revolutions per position unit split hi (12-bit mantissa, so that position x
  // hi is exact) + lo; pairs [0, n_lang) turn with the text position (image tokens: img_text_pos), pairs
  // [n_lang, n_lang + n_pix) with the image row coordinate, the next n_pix with the column coordinate (text
  // tokens: text_axial on both), the rest not at all (dalle_amd/models/rotary.py)
  const float* rotf;   // [64]: hi[32], lo[32]
  int n_lang, n_pix;
  float img_text_pos, text_axial;
};

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
// STAGE: 0 = text tiles register-staged two per barrier step (round 1-3 form); 2 / 3 = LDS-DMA'd (no
// staging VGPRs, no ds_write) two / three per step (the forward's scheme)
template <int MINB, bool FUSE_LOCAL, bool PREFETCH_LOCAL = false, int STAGE = 0>
__global__ __launch_bounds__(256, MINB) void attn_bwd_dq_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                             const __bf16* __restrict__ V, const __bf16* __restrict__ dout,
                                                             const __bf16* __restrict__ out, const float* __restrict__ lse,
                                                             float* __restrict__ delta, __bf16* __restrict__ dQ, AttnGeom g,
                                                             RopeOut ro, int delta_ready) {
  static_assert(STAGE == 0 || STAGE == 2 || STAGE == 3, "STAGE");
  constexpr int TPS = STAGE == 3 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TPS * TILE];  // 32 / 48 KB
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

  // ---- phase A: shared text tiles, two (three) per step ----
  if constexpr (STAGE != 0) {
    const int nsteps = (n_text + TPS - 1) / TPS;
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
    for (int si = 0; si < nsteps; ++si) {
      const bool more = si + 1 < nsteps;
      if (more) dma_step(si + 1, (si + 1) & 1);  // that buffer was released by the previous step's barrier
      const __bf16* S0 = smem + (si & 1) * (2 * TPS * TILE);
#pragma unroll
      for (int t = 0; t < TPS; ++t) {
        const int tile = TPS * si + t;
        if (tile < my_text_end)
          dq_tile(dq0, dq1, S0 + t * TILE, S0 + (TPS + t) * TILE, tile, qf, dof, lq, dl, g, qb, qs, lane);
      }
      __builtin_amdgcn_s_waitcnt(WAIT_VM0);  // the next step's tiles landed (this wave's pieces) before the barrier
      __syncthreads();
    }
  } else {
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
// Fused backward for the axial patterns at S = 32 (the bench / reference geometry): ONE workgroup per (b, h)
// does dQ, dK and dV of every tile, so S and dP are computed once per (query tile, key tile) pair (the
// two-kernel form computes them twice: once query-centric for dQ, once key-centric for dK / dV) and Q / dO
// stream from HBM once (the text dK/dV kernel re-read them per key pair).
//
//   * 8 waves (2 per SIMD). Wave w OWNS text key tile w: its dK^T / dV^T accumulate in registers over every
//     query tile (key on the MFMA lane, S = Q K^T and dP = dO V^T; their accumulators are directly the B
//     operands of dV^T += dO^T P and dK^T += Q^T dS). A 9th text tile (T = 257: one real key) is processed
//     by wave 0 / 4 in turn, its real keys' dK / dV accumulated in LDS (fp32, a fixed order).
//   * the image query tile i attends its own image key tile i only (axial, S = 32): that "local" pair is
//     processed by wave 1 / 5 in turn, and its dK / dV (complete after this one pair) are stored at once.
//   * every pair leaves dS (bf16) transposed in an LDS panel [key][query]; dQ^T of query tile i = K^T dS^T
//     over the panel's key tiles is computed in the NEXT iteration by waves 2 / 6 (dims 0-31) and 3 / 7
//     (dims 32-63), so every SIMD carries one extra unit of work per iteration (tile 8, local, dQ half).
//   * Q, dO (gathered from the token-major dO), and the local K / V tiles stream by LDS-DMA into a 4-slot
//     ring two query tiles ahead; each tile's row constants (-lse ln2, -delta with delta = rowsum(dO O))
//     are prepared one tile ahead and preload the S / dP accumulators, so P = exp2(S' log2e), dS = P dP'.
//   * padding query rows (text rows >= T, the last image slot) get -1e30 as their row constant: P = 0, so
//     they add nothing to dK / dV whatever their dO staging row holds.
// All outputs go through the rotary inverse into the token-major projection gradient dqkv. One
// __syncthreads-free barrier per query tile; the DMA of tile i + 2 stays in flight across it.
// ------------------------------------------------------------------------------------------------
namespace fbwd {
constexpr int NW = 8;
constexpr int KT_OFF = 0;                          // text K tiles (<= 9 x 4 KB)
constexpr int V8_OFF = KT_OFF + 9 * TILE;          // text V tile 8
constexpr int RING_OFF = V8_OFF + TILE;            // 4 slots x {Q, dO, K_loc, V_loc}
constexpr int PANEL_OFF = RING_OFF + 4 * 4 * TILE; // 2 x 10 dS^T tiles [key][query] (32 x 32 bf16)
constexpr int PANEL_TILE = 32 * 32;
constexpr int SMEM_BF16 = PANEL_OFF + 2 * 10 * PANEL_TILE;
constexpr int ACC8_KEYS = 4;                       // tile 8's real keys (host: T - 256 <= 4)
constexpr int ACC8_FLOATS = ACC8_KEYS * 128;       // dK (64) + dV (64) fp32 per real key
constexpr int STG_BYTES = 2048;                    // one rotary half-store staging slot ([32 tokens][32 dims] bf16)
constexpr int ROLE_STG = 6;                        // local dV / dK halves (4), dQ halves (2)
}  // namespace fbwd

// byte offset of the 8-byte piece (key, 4 queries from q) in a 64-B-row [key][query] tile (16-B chunks swizzled)
__device__ __forceinline__ int panel_off(int key, int q) {
  return key * 64 + ((((q >> 3) ^ ((key >> 2) & 3)) << 4) | (((q >> 2) & 1) << 3));
}


// The in-loop form of the rotary stores: CDNA's vmcnt counts loads and stores together, in issue order, so a
// load waited on mid-iteration also waits for every older store and for the ring's HBM prefetch. The loop
// therefore issues no mid-iteration loads: the rotary angles are computed in-kernel (rot_cs / rot_stage), the
// rotated bf16 tile is staged in LDS, and its stores go out together at the end of the iteration (stage_flush:
// 2 buffer stores per lane, always issued -- a padding token's offset is out of range and the store is
// dropped -- so the iteration's closing vmcnt counts them exactly).
// (cos, sin) of rotary pair j at sequence position p (p >= T: an image token), from the frequencies in LDS
__device__ __forceinline__ void rot_cs(const float* rf, const RopeOut& ro, const AttnGeom& g, int p, int j, float& c, float& s) {
  const bool txt = p < g.T;
  const int k = p - g.T;
  const float inv = 2.0f / (float)(g.S - 1);
  const float pos = j < ro.n_lang ? (txt ? (float)p : ro.img_text_pos)
                                  : (txt ? ro.text_axial : -1.0f + inv * (float)(j < ro.n_lang + ro.n_pix ? k >> g.logS : k & (g.S - 1)));
  float r = pos * rf[j];
  r -= __builtin_rintf(r);
  r = fmaf(pos, rf[32 + j], r);
  c = __builtin_amdgcn_cosf(r);
  s = __builtin_amdgcn_sinf(r);
}
// rotary inverse (dx[2i] = dy[2i] c + dy[2i+1] s, dx[2i+1] = dy[2i+1] c - dy[2i] s) of one dims half of a
// 32-token gradient tile held as an accumulator (rows = dims, lanes = tokens), angles computed in-kernel (no
// table loads: a load issued here would wait, in vmcnt order, for the ring's HBM prefetch), packed to bf16 and
// staged in LDS ([token][32 dims], 64-B rows) for stage_flush
__device__ __forceinline__ void rot_stage(const float* rf, const RopeOut& ro, const AttnGeom& g, int s0, int dt,
                                          const f32x16& acc, float scale, char* stage, int lane) {
  const int hl = lane >> 5, c32 = lane & 31;
  const int p0 = st2seq(g, s0 + c32);
  const int p = p0 < 0 ? 0 : p0;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    float y[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float c, s;
      rot_cs(rf, ro, g, p, 16 * dt + 4 * gq + 2 * hl + e, c, s);
      const float x0 = acc[4 * gq + 2 * e] * scale, x1 = acc[4 * gq + 2 * e + 1] * scale;
      y[2 * e] = x0 * c + x1 * s;
      y[2 * e + 1] = x1 * c - x0 * s;
    }
    *reinterpret_cast<s16x4*>(stage + c32 * 64 + (((gq ^ ((c32 >> 2) & 3)) << 4) | (hl << 3))) = pack4(y);
  }
}
// stores of a staged dims half of tokens s0 .. s0 + 31, part t (0 q, 1 k, 2 v) into sample b's dqkv rows (rsrc:
// that sample's n x 3HD bf16 block, exact size); the stage must have been written and lgkmcnt-waited
__device__ __forceinline__ void stage_flush(const char* stage, const AttnGeom& g, int h, int s0, int t, int dt,
                                            __amdgpu_buffer_rsrc_t rs, int lane) {
  const int HD = g.H * 64;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int tk = (lane >> 2) + 16 * it, ch = lane & 3;
    const u32x4_vs v = *reinterpret_cast<const u32x4_vs*>(stage + tk * 64 + ((ch ^ ((tk >> 2) & 3)) << 4));
    const int pt = st2seq(g, s0 + tk);
    const uint32_t off = pt < 0 ? 0x80000000u : (uint32_t)((pt * 3 * HD + t * HD + h * 64 + 32 * dt + 8 * ch) * 2);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
  }
}
// s_waitcnt vmcnt(n) lgkmcnt(0) for the iteration's closing wait (the immediate must be a constant)
__device__ __forceinline__ void wait_vm_lgkm0(int n) {
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(0x0070); break;
    case 1: __builtin_amdgcn_s_waitcnt(0x0071); break;
    case 2: __builtin_amdgcn_s_waitcnt(0x0072); break;
    case 3: __builtin_amdgcn_s_waitcnt(0x0073); break;
    case 4: __builtin_amdgcn_s_waitcnt(0x0074); break;
    case 8: __builtin_amdgcn_s_waitcnt(0x0078); break;
    case 9: __builtin_amdgcn_s_waitcnt(0x0079); break;
    case 10: __builtin_amdgcn_s_waitcnt(0x007A); break;
    default: __builtin_amdgcn_s_waitcnt(0x0070); break;   // (never: waits for everything -- safe)
  }
}

// one (query tile, key tile) pair, key on the lane. Qs / Ds: the query tile's Q and dO images; Ks / Vs: the key
// tile's K / V images (Vs null: vreg holds V's B operands); st: the tile's row constants [2][32]; mask: 0 none,
// 1 causal (key <= query within the tile) + key < kmax, 2 key < kmax. Leaves P and dS (bf16 B operands of the
// dV^T / dK^T products, fbwd_dv / fbwd_dk) and writes dS^T into the panel.
struct PairOut {
  bf16x8 p0, p1, e0, e1;
};
__device__ __forceinline__ PairOut fbwd_pair(const __bf16* Qs, const __bf16* Ds, const __bf16* Ks, const __bf16* Vs,
                                             const bf16x8 (&vreg)[4], const float* st, int mask, int kmax, char* panel,
                                             int lane) {
  const int hl = lane >> 5, c32 = lane & 31;
  f32x16 sc, dp;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(st + 8 * gq + 4 * hl);
    const f32x4 d = *reinterpret_cast<const f32x4*>(st + 32 + 8 * gq + 4 * hl);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[4 * gq + e] = a[e];
      dp[4 * gq + e] = d[e];
    }
  }
#pragma unroll
  for (int ss = 0; ss < 4; ++ss) {
    sc = MFMA32(row_operand(Qs, ss, c32, hl), row_operand(Ks, ss, c32, hl), sc);
    dp = MFMA32(row_operand(Ds, ss, c32, hl), Vs ? row_operand(Vs, ss, c32, hl) : vreg[ss], dp);
  }
  if (mask) {
    const bool kin = c32 < kmax;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool on = kin && (mask == 2 || c32 <= acc_row(r, hl));
      sc[r] = on ? sc[r] : NEG_BIG;
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float pr = fast_exp2(sc[r] * LOG2E);
    sc[r] = pr;
    dp[r] = pr * dp[r];
  }
  PairOut o;
  o.p0 = cvt8(sc, 0);
  o.p1 = cvt8(sc, 8);
  o.e0 = cvt8(dp, 0);
  o.e1 = cvt8(dp, 8);
  // dS^T into the panel: registers 4gq .. 4gq + 3 (queries 8gq + 4hl + 0..3) at [key c32][query 8gq + 4hl]
  const s16x8 s0 = __builtin_bit_cast(s16x8, o.e0), s1 = __builtin_bit_cast(s16x8, o.e1);
  *reinterpret_cast<s16x4*>(panel + panel_off(c32, 4 * hl)) = s16x4{s0[0], s0[1], s0[2], s0[3]};
  *reinterpret_cast<s16x4*>(panel + panel_off(c32, 8 + 4 * hl)) = s16x4{s0[4], s0[5], s0[6], s0[7]};
  *reinterpret_cast<s16x4*>(panel + panel_off(c32, 16 + 4 * hl)) = s16x4{s1[0], s1[1], s1[2], s1[3]};
  *reinterpret_cast<s16x4*>(panel + panel_off(c32, 24 + 4 * hl)) = s16x4{s1[4], s1[5], s1[6], s1[7]};
  return o;
}
// dV^T half dt += dO^T P (Ds: the query tile's dO image) / dK^T half dt += Q^T dS (Qs: its Q image)
__device__ __forceinline__ void fbwd_acc(f32x16& acc, const __bf16* Xs, const bf16x8& b0, const bf16x8& b1, int dt, int lane) {
  acc = MFMA32(tr_operand(Xs, 0, dt, lane), b0, acc);
  acc = MFMA32(tr_operand(Xs, 1, dt, lane), b1, acc);
}

// dst[8 gq + e] += acc[4 gq + e] (one dims half of an accumulator column, this lane's rows)
__device__ __forceinline__ void acc8_add(float* dst, const f32x16& acc) {
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    f32x4 v = *reinterpret_cast<f32x4*>(dst + 8 * gq);
    v[0] += acc[4 * gq];
    v[1] += acc[4 * gq + 1];
    v[2] += acc[4 * gq + 2];
    v[3] += acc[4 * gq + 3];
    *reinterpret_cast<f32x4*>(dst + 8 * gq) = v;
  }
}

// B operand of dQ^T = K^T dS^T: dS^T of a panel tile (lane = query, elements = keys in the accumulator-permuted
// order of tr_operand: 16ss + 8(j >> 2) + 4h + (j & 3))
__device__ __forceinline__ bf16x8 panel_operand(const char* panel, int ss, int lane) {
  const int g16 = lane >> 4, i = lane & 15;
  const int key = 16 * ss + 4 * (g16 >> 1) + (i >> 2);
  const int q = 16 * (g16 & 1) + 4 * (i & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(panel + panel_off(key, q)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(panel + panel_off(key + 8, q)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// 8 storage rows of a 32-row token-major tile gathered by LDS-DMA (padding rows read the slice's row 0)
__device__ __forceinline__ void dma_tok_piece(const __bf16* xb, const AttnGeom& g, int s0, __bf16* tile, int piece, int lane) {
  const int row = 8 * piece + (lane >> 3);
  const int off = tok_row(g, s0 + row);
  const __bf16* gp = xb + (off < 0 ? 0 : off) + (((lane & 7) ^ swz(row)) << 3);
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)gp,
                                   (void __attribute__((address_space(3)))*)(tile + 512 * piece), 16, 0, 0);
}

// query tile t's ring slot by LDS-DMA: Q, dO (+ the local K, V of an image tile), 1 KB pieces spread over the waves
__device__ __forceinline__ void fbwd_dma_qtile(const __bf16* Q, const __bf16* Kt, const __bf16* V, const __bf16* dob,
                                               const AttnGeom& g, size_t base, __bf16* smem, int t, int NT, int wave, int lane) {
  const int slot = t & 3, npieces = t >= NT ? 16 : 8;
  for (int pc = wave; pc < npieces; pc += fbwd::NW) {
    const int part = pc >> 2, sub = pc & 3;
    __bf16* dst = smem + fbwd::RING_OFF + (slot * 4 + part) * TILE;
    if (part == 1) dma_tok_piece(dob, g, t * 32, dst, sub, lane);
    else dma_tile((part == 0 ? Q : part == 2 ? Kt : V) + base + (size_t)t * 32 * 64, dst, sub, lane);
  }
}

// row constants of query tile t (rows 4 wave .. + 3): the dO / O pieces and lse, loaded one tile ahead ...
__device__ __forceinline__ void fbwd_stats_load(const __bf16* dob, const __bf16* outb, const float* lse, const AttnGeom& g,
                                                int bh, int t, int wave, int lane, s16x4& pd, s16x4& po, float& plse,
                                                int& poff) {
  const int row = 4 * wave + (lane >> 4);
  poff = tok_row(g, t * 32 + row);
  const int safe = poff < 0 ? 0 : poff;
  pd = *reinterpret_cast<const s16x4*>(dob + safe + 4 * (lane & 15));
  po = *reinterpret_cast<const s16x4*>(outb + safe + 4 * (lane & 15));
  plse = lse[(size_t)bh * g.Np + t * 32 + row];
}
// ... and stored as [-lse ln2 | -delta] (padding rows: -1e30, so P = 0)
__device__ __forceinline__ void fbwd_stats_store(float* st, const s16x4& pd, const s16x4& po, float plse, int poff, int wave,
                                                 int lane) {
  float fd[4], fo[4];
  unpack4(pd, fd);
  unpack4(po, fo);
  float d = fd[0] * fo[0] + fd[1] * fo[1] + fd[2] * fo[2] + fd[3] * fo[3];
  d += __shfl_xor(d, 1, 64);
  d += __shfl_xor(d, 2, 64);
  d += __shfl_xor(d, 4, 64);
  d += __shfl_xor(d, 8, 64);
  if ((lane & 15) == 0) {
    const int row = 4 * wave + (lane >> 4);
    st[row] = poff < 0 ? NEG_BIG : -plse * 0.6931471805599453f;
    st[32 + row] = -d;
  }
}

__global__ __launch_bounds__(512, 1) void attn_bwd_fused_axial_kernel(
    const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt, const __bf16* __restrict__ V, const __bf16* __restrict__ dout,
    const __bf16* __restrict__ out, const float* __restrict__ lse, AttnGeom g, RopeOut ro) {
  using namespace fbwd;
  __shared__ __attribute__((aligned(16))) __bf16 smem[SMEM_BF16];
  __shared__ __attribute__((aligned(16))) float acc8[ACC8_FLOATS];
  __shared__ __attribute__((aligned(16))) char stg[ROLE_STG * STG_BYTES];
  __shared__ __attribute__((aligned(16))) float stats[4][64];  // per ring slot: -lse ln2 [32], -delta [32]
  __shared__ __attribute__((aligned(16))) float rotf[64];       // rotary frequencies (RopeOut::rotf)
  const int bh = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int NT = g.Tp >> 5, nq = g.Np >> 5;
  const int r8 = NT == 9 ? g.T - 256 : 0;   // real keys of text tile 8 (host: <= ACC8_KEYS)
  const size_t base = (size_t)bh * g.Np * 64;
  const __bf16* dob = tok_base(dout, g, bh);
  const __bf16* outb = tok_base(out, g, bh);
  const int bb = bh / g.H, hh = bh - bb * g.H;
  // sample bb's block of the projection gradient, exact size: out-of-range stores (padding tokens) are dropped
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
      ro.dqkv + (size_t)bb * g.n * 3 * g.H * 64, (short)0, g.n * 3 * g.H * 64 * 2, 0x00020000);
  __bf16* KT = smem + KT_OFF;
  __bf16* V8 = smem + V8_OFF;
#define FB_RING(slot, part) (smem + RING_OFF + ((slot) * 4 + (part)) * TILE)
#define FB_PANEL(buf, ks) (reinterpret_cast<char*>(smem + PANEL_OFF + ((buf) * 10 + (ks)) * PANEL_TILE))
  // row constants of query tile t: wave w takes rows 4w .. 4w + 3, 16 lanes per row (4 dims each)
  // two register sets by tile parity: tile t's pieces are loaded two iterations before they are reduced
  s16x4 pd = {}, po = {}, pd1 = {}, po1 = {};
  float plse = 0.f, plse1 = 0.f;
  int poff = -1, poff1 = -1;
  // ---- prologue: text K tiles (+ V tile 8), query tiles 0 and 1, tile 0's row constants, the owned V rows
  for (int pc = wave; pc < 4 * (NT + (r8 > 0 ? 1 : 0)); pc += NW) {
    const int tile = pc >> 2, sub = pc & 3;
    if (tile < NT) dma_tile(Kt + base + (size_t)tile * 32 * 64, KT + tile * TILE, sub, lane);
    else dma_tile(V + base + (size_t)8 * 32 * 64, V8, sub, lane);
  }
  fbwd_dma_qtile(Q, Kt, V, dob, g, base, smem, 0, NT, wave, lane);
  if (nq > 1) fbwd_dma_qtile(Q, Kt, V, dob, g, base, smem, 1, NT, wave, lane);
  for (int e = tid; e < ACC8_FLOATS; e += 512) acc8[e] = 0.f;
  if (tid < 64) rotf[tid] = ro.rotf[tid];
  const bool owner = wave < NT && wave < 8;
  bf16x8 vf[4];
  {
    const int kr = owner ? wave * 32 + c32 : 0;
    const __bf16* vp = V + base + (size_t)kr * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) vf[s] = ld16(vp + 16 * s);
  }
  fbwd_stats_load(dob, outb, lse, g, bh, 0, wave, lane, pd, po, plse, poff);
  if (nq > 1) fbwd_stats_load(dob, outb, lse, g, bh, 1, wave, lane, pd1, po1, plse1, poff1);
  __builtin_amdgcn_s_waitcnt(WAIT_VM0);
  fbwd_stats_store(stats[0], pd, po, plse, poff, wave, lane);
  __syncthreads();

  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  for (int i = 0; i <= nq; ++i) {
    const int slot = i & 3, par = i & 1;
    if (i + 2 < nq) {   // into the set tile i's constants came from (stored last iteration)
      if (par) fbwd_stats_load(dob, outb, lse, g, bh, i + 2, wave, lane, pd1, po1, plse1, poff1);
      else fbwd_stats_load(dob, outb, lse, g, bh, i + 2, wave, lane, pd, po, plse, poff);
    }
    if (i < nq) {
      const __bf16* Qs = FB_RING(slot, 0);
      const __bf16* Ds = FB_RING(slot, 1);
      const float* st = stats[slot];
      const bool img = i >= NT;
      if (owner && (img || wave <= i)) {
        // text diag: causal; an owned tile past T's last real key (NT <= 8, T % 32): keys < T
        const int kmax = min(32, g.T - wave * 32);
        const int mask = (wave == i) ? 1 : (kmax < 32 ? 2 : 0);
        const PairOut o = fbwd_pair(Qs, Ds, KT + wave * TILE, nullptr, vf, st, mask, kmax, FB_PANEL(par, wave), lane);
        fbwd_acc(dv0, Ds, o.p0, o.p1, 0, lane);
        fbwd_acc(dv1, Ds, o.p0, o.p1, 1, lane);
        fbwd_acc(dk0, Qs, o.e0, o.e1, 0, lane);
        fbwd_acc(dk1, Qs, o.e0, o.e1, 1, lane);
      }
      if (r8 > 0 && i >= 8 && wave == 4 * par) {
        const PairOut o = fbwd_pair(Qs, Ds, KT + 8 * TILE, V8, vf, st, i == 8 ? 1 : 2, r8, FB_PANEL(par, 8), lane);
        // this pair's contribution to the real keys' dK / dV, summed in LDS in query-tile order (one half at a time)
        float* ak = acc8 + c32 * 128 + 4 * hl;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          f32x16 a = {};
          if (q4 < 2) fbwd_acc(a, Ds, o.p0, o.p1, q4, lane);
          else fbwd_acc(a, Qs, o.e0, o.e1, q4 - 2, lane);
          if (c32 < r8) acc8_add(ak + (q4 < 2 ? 64 : 0) + 32 * (q4 & 1), a);
        }
      }
      if (img && wave == 1 + 4 * par) {
        const __bf16* Ks = FB_RING(slot, 2);
        const PairOut o = fbwd_pair(Qs, Ds, Ks, FB_RING(slot, 3), vf, st, 1, 32, FB_PANEL(par, 9), lane);
        // the local key tile's dK / dV are complete after this pair: rotated per dims half (the tables of both
        // halves loaded at once), staged for the end-of-iteration stores
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          f32x16 av = {};
          if (q4 < 2) fbwd_acc(av, Ds, o.p0, o.p1, q4, lane);
          else fbwd_acc(av, Qs, o.e0, o.e1, q4 - 2, lane);
          rot_stage(rotf, ro, g, i * 32, q4 & 1, av, 1.0f, stg + q4 * STG_BYTES, lane);
        }
      }
    }
    if (i >= 1 && (wave & 3) >= 2 && (wave >> 2) == par) {
      // dQ^T of query tile j = i - 1, dims half dt: K^T dS^T over the panel's key tiles
      const int j = i - 1, dt = wave & 1, pb = j & 1;
      f32x16 dq = {};
      const int ntext = j >= NT ? NT : j + 1;
      for (int ks = 0; ks < ntext; ++ks) {
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) dq = MFMA32(tr_operand(KT + ks * TILE, ss, dt, lane), panel_operand(FB_PANEL(pb, ks), ss, lane), dq);
      }
      if (j >= NT) {
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) dq = MFMA32(tr_operand(FB_RING(j & 3, 2), ss, dt, lane), panel_operand(FB_PANEL(pb, 9), ss, lane), dq);
      }
      rot_stage(rotf, ro, g, j * 32, dt, dq, ro.qscale, stg + (4 + dt) * STG_BYTES, lane);
    }

    // ---- end of iteration: the next tile's row constants, the DMA of tile i + 2, then the barrier that
    //      publishes tile i + 1 (its pieces are older than tile i + 2's, which may stay in flight)
    //      Order: DMA of tile i + 2 (d pieces), then this iteration's staged stores (s), then vmcnt(d + s):
    //      everything older -- tile i + 1's pieces among them -- has landed; the d + s newest stay in flight.
    if (i + 1 < nq) {   // tile i + 1's constants (loaded in iteration i - 1, or the prologue)
      if (par) fbwd_stats_store(stats[(i + 1) & 3], pd, po, plse, poff, wave, lane);
      else fbwd_stats_store(stats[(i + 1) & 3], pd1, po1, plse1, poff1, wave, lane);
    }
    int nvm = 0;
    if (i + 2 < nq) {
      fbwd_dma_qtile(Q, Kt, V, dob, g, base, smem, i + 2, NT, wave, lane);
      nvm = i + 2 >= NT ? 2 : 1;
    }
    const bool st_local = i < nq && i >= NT && wave == 1 + 4 * par;
    const bool st_dq = i >= 1 && (wave & 3) >= 2 && (wave >> 2) == par;
    if (st_local || st_dq) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the staged tiles are written (each wave reads its own)
      __builtin_amdgcn_wave_barrier();
    }
    if (st_local) {
      stage_flush(stg + 0 * STG_BYTES, g, hh, i * 32, 2, 0, rs_out, lane);
      stage_flush(stg + 1 * STG_BYTES, g, hh, i * 32, 2, 1, rs_out, lane);
      stage_flush(stg + 2 * STG_BYTES, g, hh, i * 32, 1, 0, rs_out, lane);
      stage_flush(stg + 3 * STG_BYTES, g, hh, i * 32, 1, 1, rs_out, lane);
      nvm += 8;
    }
    if (st_dq) {
      stage_flush(stg + (4 + (wave & 1)) * STG_BYTES, g, hh, (i - 1) * 32, 0, wave & 1, rs_out, lane);
      nvm += 2;
    }
    wait_vm_lgkm0(nvm);
    __builtin_amdgcn_s_barrier();
  }

  // ---- owned text tiles' dK / dV (the ring is free now: 4 x 2 KB of staging per wave), then tile 8's real keys
  char* mystg = reinterpret_cast<char*>(smem + RING_OFF) + wave * 4 * STG_BYTES;
  if (owner) {
    rot_stage(rotf, ro, g, wave * 32, 0, dk0, 1.0f, mystg, lane);
    rot_stage(rotf, ro, g, wave * 32, 1, dk1, 1.0f, mystg + STG_BYTES, lane);
    rot_stage(rotf, ro, g, wave * 32, 0, dv0, 1.0f, mystg + 2 * STG_BYTES, lane);
    rot_stage(rotf, ro, g, wave * 32, 1, dv1, 1.0f, mystg + 3 * STG_BYTES, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    stage_flush(mystg, g, hh, wave * 32, 1, 0, rs_out, lane);
    stage_flush(mystg + STG_BYTES, g, hh, wave * 32, 1, 1, rs_out, lane);
    stage_flush(mystg + 2 * STG_BYTES, g, hh, wave * 32, 2, 0, rs_out, lane);
    stage_flush(mystg + 3 * STG_BYTES, g, hh, wave * 32, 2, 1, rs_out, lane);
  }
  if (r8 > 0 && wave == NW - 1) {
    const int HD = g.H * 64;
    for (int it = lane; it < r8 * 16; it += 64) {
      const int k = it >> 4, t = 1 + ((it >> 3) & 1), ch = it & 7;
      const int p = 256 + k;
      const float* src = acc8 + k * 128 + (t - 1) * 64 + 8 * ch;
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        float c, s;
        rot_cs(rotf, ro, g, p, 4 * ch + e / 2, c, s);
        y[e] = src[e] * c + src[e + 1] * s;
        y[e + 1] = src[e + 1] * c - src[e] * s;
      }
      *reinterpret_cast<s16x8*>(ro.dqkv + ((size_t)bb * g.n + p) * (3 * HD) + t * HD + hh * 64 + 8 * ch) = pack8(y);
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
// register-staged text pairs (LDS-DMA measured slower), text dK/dV 4 query tiles (-0.9 ms per bench24
// B128 step vs 2); local-tile prefetch off (more spills at occupancy 3). Round-4 numbers of every
// variant: profiles/r4ab_switches_b128.txt, profiles/INDEX.md.
void attn_fwd(const void* q, const void* k, const void* v, void* out, float* lse, const AttnGeom& g, int BH, hipStream_t st) {
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  hipLaunchKernelGGL((attn_fwd_kernel<3, false>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (__bf16*)out, lse, g);
}

// the fused one-workgroup-per-head backward: axial row / col at S = 32 (one image row or column = one 32-key
// tile), rotary-fused output with the angles computed in-kernel (rotary frequencies given), at most 9 text tiles
// with at most ACC8_KEYS real keys in a 9th (T <= 260; the reference's T = 257). DALLE_AMD_ATTN_FUSED_BWD=0
// keeps the two-kernel form (A/B).
bool attn_bwd_fused_ok(const AttnGeom& g, bool rope_out, bool has_freqs) {
  // opt-in (default off): at B128 the isolated backward is at parity with the two-kernel form (1536 vs 1545 us
  // axial row) and the whole bench24 step is 5 % slower with it (306 vs 322 samples/s, same box, alternating;
  // profiles/r6_attn_fused_bwd.txt): at one workgroup per CU its waves wait ~66 % of their cycles (SQ_WAIT_ANY)
  // -- the ring's one-iteration HBM lead and the per-tile barrier behind the role waves' VALU -- where the
  // two-kernel form keeps 3 (dQ) / 2 (dK/dV) waves per SIMD in flight. Read per call: a test / A/B may flip it.
  const char* s = getenv("DALLE_AMD_ATTN_FUSED_BWD");
  const int env = s ? atoi(s) : 0;
  const int NT = g.Tp / 32;
  return env != 0 && rope_out && has_freqs && (g.pattern == 1 || g.pattern == 2) && g.S == 32 && g.I == 1024 && NT >= 1 && NT <= 9 &&
         (NT < 9 || g.T - 256 <= fbwd::ACC8_KEYS) && g.n == g.T + g.I - 1;
}

void attn_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout, const float* lse,
              float* delta, void* dq, void* dk, void* dv, const AttnGeom& g, int BH, hipStream_t st,
              const float* cosT, const float* sinT, void* dqkv, float qscale, const float* rotf, int rot_nl, int rot_np,
              float rot_img_text_pos, float rot_text_axial) {
  const RopeOut ro{cosT, sinT, static_cast<__bf16*>(dqkv), qscale, rotf, rot_nl, rot_np, rot_img_text_pos, rot_text_axial};
  if (attn_bwd_fused_ok(g, dqkv != nullptr, rotf != nullptr)) {
    hipLaunchKernelGGL(attn_bwd_fused_axial_kernel, dim3(BH), dim3(512), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, (const __bf16*)dout, (const __bf16*)out, lse, g, ro);
    return;
  }
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  // axial row / col: every image key tile is attended by exactly its own query tile -> dK / dV of the
  // image keys inside the dQ kernel (rotary-fused output path)
  const bool fuse_local = dqkv != nullptr && (g.pattern == 1 || g.pattern == 2);
  const int ntext = g.Tp / 32, nimg = g.Np / 32 - ntext;
  if (fuse_local)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, true, false, 0>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, (const __bf16*)dout, (const __bf16*)out, lse, delta, (__bf16*)dq, g, ro, 0);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, false, false, 0>), grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
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
