// Tile-level helpers shared by the sparse attention kernels (attention.hip: forward, two-kernel backward) and
// the fused one-workgroup-per-head backward (attention_fused.hip). SURVEY K7a-K7e.
#pragma once
#include "common.h"
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
};
// The rotary frequencies for angles computed in-kernel (the fused backward; a separate argument, so the
// two-kernel form's RopeOut and code stay as they were): per rotary pair j of the head, its frequency in
// revolutions per position unit split hi (12-bit mantissa, so that position x hi is exact) + lo; pairs
// [0, n_lang) turn with the text position (image tokens: img_text_pos), pairs [n_lang, n_lang + n_pix) with
// the image row coordinate, the next n_pix with the column coordinate (text tokens: text_axial on both), the
// rest not at all (dalle_amd/models/rotary.py)
struct RotSpec {
  const float* rotf;   // [64]: hi[32], lo[32]
  int n_lang, n_pix;
  float img_text_pos, text_axial;
};


}  // namespace dalle
