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

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ int st2seq(const AttnGeom& g, int s) {
  if (s < g.T) return s;
  if (s < g.Tp) return -1;
  const int kst = s - g.Tp;
  const int k = (g.pattern == 2) ? ((kst & (g.S - 1)) << g.logS) + (kst >> g.logS) : kst;
  const int p = g.T + k;
  return p < g.n ? p : -1;
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

// ------------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------------
// Lazy rescale threshold (log2 units, T13): the running max is only moved when a tile's max exceeds
// it by more than this, so P <= 2^8 (exact in bf16's relative precision; fp32 sums have headroom).
constexpr float RESCALE_THR = 8.0f;

__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                          const __bf16* __restrict__ V, __bf16* __restrict__ out,
                                                          float* __restrict__ lse, AttnGeom g) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TILE];
  const int bh = blockIdx.y;
  const int b = bh / g.H, h = bh - b * g.H;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nqb = g.Np >> 5, ntext = g.Tp >> 5;
  const int qb0 = blockIdx.x * 4;
  const int qb = qb0 + wave;
  const int qb_last = min(qb0 + 3, nqb - 1);
  const bool active = qb < nqb;
  const size_t base = (size_t)bh * g.Np * 64;

  // union of key tiles of the workgroup
  const int u_text_end = qb_last < ntext ? qb_last + 1 : ntext;
  const int first_img_qb = max(qb0, ntext);
  const int u_loc_lo = (qb_last >= ntext) ? local_lo_tile(g, first_img_qb) : 0;
  const int n_loc = (qb_last >= ntext) ? (qb_last - u_loc_lo + 1) : 0;
  const int ntiles = u_text_end + n_loc;
  // this wave's ranges
  int my_text_end = 0, my_lo = 1, my_hi = 0;
  if (active) {
    if (qb < ntext) my_text_end = qb + 1;
    else { my_text_end = ntext; my_lo = local_lo_tile(g, qb); my_hi = qb; }
  }

  const int qs = qb * 32 + c32;
  bf16x8 qf[4];
  {
    const __bf16* qp = Q + base + (size_t)(active ? qs : 0) * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = ld16(qp + 16 * s);
  }

  // staging: each thread moves one 16-B chunk of K and of V per tile (swizzled image)
  const int st_row = tid >> 3, st_col = (tid & 7) * 8;
  const int st_off = lds_idx(st_row, st_col);
  auto tile_id = [&](int t) { return t < u_text_end ? t : u_loc_lo + (t - u_text_end); };
  s16x8 kreg, vreg;
  {
    const int t0 = tile_id(0);
    const size_t off = base + (size_t)(t0 * 32 + st_row) * 64 + st_col;
    kreg = *reinterpret_cast<const s16x8*>(Kt + off);
    vreg = *reinterpret_cast<const s16x8*>(V + off);
    *reinterpret_cast<s16x8*>(smem + st_off) = kreg;
    *reinterpret_cast<s16x8*>(smem + TILE + st_off) = vreg;
  }
  __syncthreads();

  // m: running max of the RAW scores (q carries 1/sqrt(d)); p = 2^(s*log2e - m*log2e) via one fma
  float m = NEG_BIG, lsum = 0.f;
  f32x16 o0 = {}, o1 = {};
  constexpr float THR_RAW = RESCALE_THR / LOG2E;

  for (int t = 0; t < ntiles; ++t) {
    const int tile = tile_id(t);
    const bool more = t + 1 < ntiles;
    if (more) {
      const size_t off = base + (size_t)(tile_id(t + 1) * 32 + st_row) * 64 + st_col;
      kreg = *reinterpret_cast<const s16x8*>(Kt + off);
      vreg = *reinterpret_cast<const s16x8*>(V + off);
    }
    const __bf16* Ks = smem + (t & 1) * (2 * TILE);
    const __bf16* Vs = Ks + TILE;
    const bool need = (tile < my_text_end) || (tile >= my_lo && tile <= my_hi);
    if (need) {
      f32x16 s = {};
#pragma unroll
      for (int ss = 0; ss < 4; ++ss) s = MFMA32(row_operand(Ks, ss, c32, hl), qf[ss], s);
      if (!tile_full(g, qb, tile)) {
        const uint32_t mh = key_mask(g, qs, tile) >> (4 * hl);
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = mask_bit(mh, r) ? s[r] : NEG_BIG;
      }
      float mt = fmaxf(fmaxf(s[0], s[1]), s[2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) mt = fmaxf(fmaxf(mt, s[r]), s[r + 1]);
      mt = fmaxf(mt, s[15]);
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      if (!__all(mt <= m + THR_RAW)) {
        const float mnew = fmaxf(m, mt);
        const float alpha = fast_exp2((m - mnew) * LOG2E);
        m = mnew;
        lsum *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      }
      const float mc = m * LOG2E;
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(fmaf(s[r], LOG2E, -mc));
        s[r] = p;
        ps += p;
      }
      lsum += ps;
      const bf16x8 p0 = cvt8(s, 0), p1 = cvt8(s, 8);
      o0 = MFMA32(tr_operand(Vs, 0, 0, lane), p0, o0);
      o0 = MFMA32(tr_operand(Vs, 1, 0, lane), p1, o0);
      o1 = MFMA32(tr_operand(Vs, 0, 1, lane), p0, o1);
      o1 = MFMA32(tr_operand(Vs, 1, 1, lane), p1, o1);
    }
    if (more) {
      __bf16* Kn = smem + ((t + 1) & 1) * (2 * TILE);
      *reinterpret_cast<s16x8*>(Kn + st_off) = kreg;
      *reinterpret_cast<s16x8*>(Kn + TILE + st_off) = vreg;
    }
    __syncthreads();
  }

  if (!active) return;
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = 1.0f / ltot;
  lse[(size_t)bh * g.Np + qs] = m * LOG2E + log2f(ltot);
  const int p = st2seq(g, qs);
  if (p < 0) return;
  __bf16* op = out + ((size_t)b * g.n + p) * (g.H * 64) + h * 64;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& o = dt ? o1 : o0;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      float f[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) f[i] = o[4 * gq + i] * inv;
      *reinterpret_cast<s16x4*>(op + 32 * dt + 8 * gq + 4 * hl) = pack4(f);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Backward preprocessing: dO -> storage layout, delta = rowsum(dO * O) (fp32)
// ------------------------------------------------------------------------------------------------
__global__ void attn_bwd_prep_kernel(const __bf16* __restrict__ dout, const __bf16* __restrict__ out,
                                     __bf16* __restrict__ do_st, float* __restrict__ delta, AttnGeom g, int BH) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;  // one thread per (bh, row, 8-chunk)
  const int chunk = gid & 7;
  const int row_g = gid >> 3;
  if (row_g >= BH * g.Np) return;
  const int bh = row_g / g.Np, s = row_g - bh * g.Np;
  const int b = bh / g.H, h = bh - b * g.H;
  const int p = st2seq(g, s);
  s16x8 d = {};
  float acc = 0.f;
  if (p >= 0) {
    const size_t off = ((size_t)b * g.n + p) * (g.H * 64) + h * 64 + chunk * 8;
    d = *reinterpret_cast<const s16x8*>(dout + off);
    const s16x8 o = *reinterpret_cast<const s16x8*>(out + off);
    float fd[8], fo[8];
    unpack8(d, fd);
    unpack8(o, fo);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += fd[i] * fo[i];
  }
  *reinterpret_cast<s16x8*>(do_st + (size_t)row_g * 64 + chunk * 8) = d;
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (chunk == 0) delta[row_g] = acc;
}

// ------------------------------------------------------------------------------------------------
// Backward dQ (query-centric)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                             const __bf16* __restrict__ V, const __bf16* __restrict__ dO,
                                                             const float* __restrict__ lse, const float* __restrict__ delta,
                                                             __bf16* __restrict__ dQ, AttnGeom g) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TILE];
  const int bh = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nqb = g.Np >> 5, ntext = g.Tp >> 5;
  const int qb0 = blockIdx.x * 4;
  const int qb = qb0 + wave;
  const int qb_last = min(qb0 + 3, nqb - 1);
  const bool active = qb < nqb;
  const size_t base = (size_t)bh * g.Np * 64;

  const int u_text_end = qb_last < ntext ? qb_last + 1 : ntext;
  const int first_img_qb = max(qb0, ntext);
  const int u_loc_lo = (qb_last >= ntext) ? local_lo_tile(g, first_img_qb) : 0;
  const int n_loc = (qb_last >= ntext) ? (qb_last - u_loc_lo + 1) : 0;
  const int ntiles = u_text_end + n_loc;
  int my_text_end = 0, my_lo = 1, my_hi = 0;
  if (active) {
    if (qb < ntext) my_text_end = qb + 1;
    else { my_text_end = ntext; my_lo = local_lo_tile(g, qb); my_hi = qb; }
  }

  const int qs = qb * 32 + c32;
  const int qrow = active ? qs : 0;
  bf16x8 qf[4], dof[4];
  {
    const __bf16* qp = Q + base + (size_t)qrow * 64 + 8 * hl;
    const __bf16* dp = dO + base + (size_t)qrow * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) { qf[s] = ld16(qp + 16 * s); dof[s] = ld16(dp + 16 * s); }
  }
  const float lq = lse[(size_t)bh * g.Np + qrow];
  const float dl = delta[(size_t)bh * g.Np + qrow];

  const int st_row = tid >> 3, st_col = (tid & 7) * 8;
  const int st_off = lds_idx(st_row, st_col);
  auto tile_id = [&](int t) { return t < u_text_end ? t : u_loc_lo + (t - u_text_end); };
  s16x8 kreg, vreg;
  {
    const size_t off = base + (size_t)(tile_id(0) * 32 + st_row) * 64 + st_col;
    kreg = *reinterpret_cast<const s16x8*>(Kt + off);
    vreg = *reinterpret_cast<const s16x8*>(V + off);
    *reinterpret_cast<s16x8*>(smem + st_off) = kreg;
    *reinterpret_cast<s16x8*>(smem + TILE + st_off) = vreg;
  }
  __syncthreads();

  f32x16 dq0 = {}, dq1 = {};
  for (int t = 0; t < ntiles; ++t) {
    const int tile = tile_id(t);
    const bool more = t + 1 < ntiles;
    if (more) {
      const size_t off = base + (size_t)(tile_id(t + 1) * 32 + st_row) * 64 + st_col;
      kreg = *reinterpret_cast<const s16x8*>(Kt + off);
      vreg = *reinterpret_cast<const s16x8*>(V + off);
    }
    const __bf16* Ks = smem + (t & 1) * (2 * TILE);
    const __bf16* Vs = Ks + TILE;
    const bool need = (tile < my_text_end) || (tile >= my_lo && tile <= my_hi);
    if (need) {
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
    if (more) {
      __bf16* Kn = smem + ((t + 1) & 1) * (2 * TILE);
      *reinterpret_cast<s16x8*>(Kn + st_off) = kreg;
      *reinterpret_cast<s16x8*>(Kn + TILE + st_off) = vreg;
    }
    __syncthreads();
  }
  if (!active) return;
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
// Backward dK / dV (key-centric)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                               const __bf16* __restrict__ V, const __bf16* __restrict__ dO,
                                                               const float* __restrict__ lse, const float* __restrict__ delta,
                                                               __bf16* __restrict__ dK, __bf16* __restrict__ dV, AttnGeom g) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TILE];
  __shared__ float stats[2][2][32];
  const int bh = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nkb = g.Np >> 5, ntext = g.Tp >> 5;
  // image (local) key blocks only: text key blocks go to attn_bwd_dkdv_text_kernel
  const int kb0 = ntext + blockIdx.x * 4;
  const int kb = kb0 + wave;
  const int kb_last = min(kb0 + 3, nkb - 1);
  const bool active = kb < nkb;
  const size_t base = (size_t)bh * g.Np * 64;

  auto hi_of = [&](int k) { return k < ntext ? nkb - 1 : local_hi_qtile(g, k); };
  const int q_lo = kb0;
  const int q_hi = hi_of(kb_last) > hi_of(kb0) ? hi_of(kb_last) : hi_of(kb0);
  int u_hi = q_hi;
  for (int k = kb0; k <= kb_last; ++k) u_hi = max(u_hi, hi_of(k));
  const int ntiles = u_hi - q_lo + 1;
  const int my_hi = active ? hi_of(kb) : -1;

  const int ks = kb * 32 + c32;
  const int krow = active ? ks : 0;
  bf16x8 kf[4], vf[4];
  {
    const __bf16* kp = Kt + base + (size_t)krow * 64 + 8 * hl;
    const __bf16* vp = V + base + (size_t)krow * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) { kf[s] = ld16(kp + 16 * s); vf[s] = ld16(vp + 16 * s); }
  }

  const int st_row = tid >> 3, st_col = (tid & 7) * 8;
  const int st_off = lds_idx(st_row, st_col);
  s16x8 qreg, doreg;
  float lreg = 0.f, dreg = 0.f;
  {
    const size_t off = base + (size_t)(q_lo * 32 + st_row) * 64 + st_col;
    qreg = *reinterpret_cast<const s16x8*>(Q + off);
    doreg = *reinterpret_cast<const s16x8*>(dO + off);
    *reinterpret_cast<s16x8*>(smem + st_off) = qreg;
    *reinterpret_cast<s16x8*>(smem + TILE + st_off) = doreg;
    if (tid < 32) stats[0][0][tid] = lse[(size_t)bh * g.Np + q_lo * 32 + tid];
    else if (tid < 64) stats[0][1][tid - 32] = delta[(size_t)bh * g.Np + q_lo * 32 + tid - 32];
  }
  __syncthreads();

  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  for (int t = 0; t < ntiles; ++t) {
    const int qt = q_lo + t;
    const bool more = t + 1 < ntiles;
    if (more) {
      const size_t off = base + (size_t)((qt + 1) * 32 + st_row) * 64 + st_col;
      qreg = *reinterpret_cast<const s16x8*>(Q + off);
      doreg = *reinterpret_cast<const s16x8*>(dO + off);
      if (tid < 32) lreg = lse[(size_t)bh * g.Np + (qt + 1) * 32 + tid];
      else if (tid < 64) dreg = delta[(size_t)bh * g.Np + (qt + 1) * 32 + tid - 32];
    }
    const int buf = t & 1;
    const __bf16* Qs = smem + buf * (2 * TILE);
    const __bf16* Ds = Qs + TILE;
    const bool need = active && qt >= kb && qt <= my_hi;
    if (need) {
      f32x16 s = {}, dp = {};
#pragma unroll
      for (int ss = 0; ss < 4; ++ss) {
        s = MFMA32(row_operand(Qs, ss, c32, hl), kf[ss], s);
        dp = MFMA32(row_operand(Ds, ss, c32, hl), vf[ss], dp);
      }
      f32x16 ds;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = acc_row(r, hl);
        const float p = fast_exp2(fmaf(s[r], LOG2E, -stats[buf][0][ql]));
        s[r] = p;
        ds[r] = p * (dp[r] - stats[buf][1][ql]);
      }
      if (!tile_full(g, qt, kb)) {
        const uint32_t mh = query_mask(g, ks, qt) >> (4 * hl);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool on = mask_bit(mh, r);
          s[r] = on ? s[r] : 0.f;
          ds[r] = on ? ds[r] : 0.f;
        }
      }
      const bf16x8 p0 = cvt8(s, 0), p1 = cvt8(s, 8);
      const bf16x8 d0 = cvt8(ds, 0), d1 = cvt8(ds, 8);
      dv0 = MFMA32(tr_operand(Ds, 0, 0, lane), p0, dv0);
      dv0 = MFMA32(tr_operand(Ds, 1, 0, lane), p1, dv0);
      dv1 = MFMA32(tr_operand(Ds, 0, 1, lane), p0, dv1);
      dv1 = MFMA32(tr_operand(Ds, 1, 1, lane), p1, dv1);
      dk0 = MFMA32(tr_operand(Qs, 0, 0, lane), d0, dk0);
      dk0 = MFMA32(tr_operand(Qs, 1, 0, lane), d1, dk0);
      dk1 = MFMA32(tr_operand(Qs, 0, 1, lane), d0, dk1);
      dk1 = MFMA32(tr_operand(Qs, 1, 1, lane), d1, dk1);
    }
    if (more) {
      const int nb = (t + 1) & 1;
      __bf16* Qn = smem + nb * (2 * TILE);
      *reinterpret_cast<s16x8*>(Qn + st_off) = qreg;
      *reinterpret_cast<s16x8*>(Qn + TILE + st_off) = doreg;
      if (tid < 32) stats[nb][0][tid] = lreg;
      else if (tid < 64) stats[nb][1][tid - 32] = dreg;
    }
    __syncthreads();
  }
  if (!active) return;
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
// Backward dK / dV for the TEXT key blocks: every later query tile (all image queries see all
// text keys) attends to them, so one workgroup owns ONE 32-key block and its 4 waves split the
// query tiles round-robin (balanced; 4x shorter critical path than one wave per key block). Each
// wave stages its own Q/dO tile (wave-private double buffer, register prefetch one tile ahead);
// the four partial dK/dV accumulators are summed through LDS at the end.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_text_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ Kt,
                                                                    const __bf16* __restrict__ V, const __bf16* __restrict__ dO,
                                                                    const float* __restrict__ lse, const float* __restrict__ delta,
                                                                    __bf16* __restrict__ dK, __bf16* __restrict__ dV, AttnGeom g) {
  // per wave: 2 buffers x {Q, dO} tile images   +  2 buffers x {lse, delta} x 32
  __shared__ __attribute__((aligned(16))) __bf16 smem[4 * 2 * 2 * TILE];
  __shared__ float stats[4][2][2][32];
  const int bh = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hl = lane >> 5, c32 = lane & 31;
  const int nqb = g.Np >> 5;
  const int kb = blockIdx.x;
  const size_t base = (size_t)bh * g.Np * 64;
  const int ks = kb * 32 + c32;
  bf16x8 kf[4], vf[4];
  {
    const __bf16* kp = Kt + base + (size_t)ks * 64 + 8 * hl;
    const __bf16* vp = V + base + (size_t)ks * 64 + 8 * hl;
#pragma unroll
    for (int s = 0; s < 4; ++s) { kf[s] = ld16(kp + 16 * s); vf[s] = ld16(vp + 16 * s); }
  }
  __bf16* wsm = smem + wave * (2 * 2 * TILE);
  const int first = kb + wave;
  const int ntiles = first < nqb ? (nqb - first + 3) / 4 : 0;
  // lane-private staging: 4 chunks of Q and 4 of dO per tile (32 rows x 8 chunks of 16 B)
  s16x8 qreg[4], dreg[4];
  float lreg = 0.f, dlreg = 0.f;
  auto load_tile = [&](int qt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      const size_t off = base + (size_t)(qt * 32 + row) * 64 + col;
      qreg[j] = *reinterpret_cast<const s16x8*>(Q + off);
      dreg[j] = *reinterpret_cast<const s16x8*>(dO + off);
    }
    if (lane < 32) {
      lreg = lse[(size_t)bh * g.Np + qt * 32 + lane];
      dlreg = delta[(size_t)bh * g.Np + qt * 32 + lane];
    }
  };
  auto store_tile = [&](int buf) {
    __bf16* Qs = wsm + buf * (2 * TILE);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = lane + 64 * j, row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<s16x8*>(Qs + lds_idx(row, col)) = qreg[j];
      *reinterpret_cast<s16x8*>(Qs + TILE + lds_idx(row, col)) = dreg[j];
    }
    if (lane < 32) { stats[wave][buf][0][lane] = lreg; stats[wave][buf][1][lane] = dlreg; }
  };
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  if (ntiles > 0) {
    load_tile(first);
    store_tile(0);
  }
  for (int i = 0; i < ntiles; ++i) {
    const int qt = first + 4 * i;
    const bool more = i + 1 < ntiles;
    if (more) load_tile(qt + 4);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS stores of the current tile landed
    __builtin_amdgcn_wave_barrier();
    const int buf = i & 1;
    const __bf16* Qs = wsm + buf * (2 * TILE);
    const __bf16* Ds = Qs + TILE;
    f32x16 s = {}, dp = {};
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      s = MFMA32(row_operand(Qs, ss, c32, hl), kf[ss], s);
      dp = MFMA32(row_operand(Ds, ss, c32, hl), vf[ss], dp);
    }
    f32x16 ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = acc_row(r, hl);
      const float p = fast_exp2(fmaf(s[r], LOG2E, -stats[wave][buf][0][ql]));
      s[r] = p;
      ds[r] = p * (dp[r] - stats[wave][buf][1][ql]);
    }
    if (!tile_full(g, qt, kb)) {
      const uint32_t mh = query_mask(g, ks, qt) >> (4 * hl);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool on = mask_bit(mh, r);
        s[r] = on ? s[r] : 0.f;
        ds[r] = on ? ds[r] : 0.f;
      }
    }
    const bf16x8 p0 = cvt8(s, 0), p1 = cvt8(s, 8);
    const bf16x8 d0 = cvt8(ds, 0), d1 = cvt8(ds, 8);
    dv0 = MFMA32(tr_operand(Ds, 0, 0, lane), p0, dv0);
    dv0 = MFMA32(tr_operand(Ds, 1, 0, lane), p1, dv0);
    dv1 = MFMA32(tr_operand(Ds, 0, 1, lane), p0, dv1);
    dv1 = MFMA32(tr_operand(Ds, 1, 1, lane), p1, dv1);
    dk0 = MFMA32(tr_operand(Qs, 0, 0, lane), d0, dk0);
    dk0 = MFMA32(tr_operand(Qs, 1, 0, lane), d1, dk0);
    dk1 = MFMA32(tr_operand(Qs, 0, 1, lane), d0, dk1);
    dk1 = MFMA32(tr_operand(Qs, 1, 1, lane), d1, dk1);
    if (more) {
      __builtin_amdgcn_wave_barrier();  // every lane finished reading the other buffer (tile i-1)
      store_tile(buf ^ 1);
    }
  }
  // reduce the 4 waves' partial dK^T / dV^T through LDS (reuse the staging area: 4 waves x 64 values
  // x 64 lanes floats = 64 KB), laid out value-major so consecutive lanes hit consecutive banks
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    red[(wave * 64 + r) * 64 + lane] = dk0[r];
    red[(wave * 64 + 16 + r) * 64 + lane] = dk1[r];
    red[(wave * 64 + 32 + r) * 64 + lane] = dv0[r];
    red[(wave * 64 + 48 + r) * 64 + lane] = dv1[r];
  }
  __syncthreads();
  if (wave == 0) {
    __bf16* kp = dK + base + (size_t)ks * 64;
    __bf16* vp = dV + base + (size_t)ks * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        float fa[4], fc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * gq + i;
          fa[i] = fc[i] = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            fa[i] += red[(w * 64 + dt * 16 + r) * 64 + lane];
            fc[i] += red[(w * 64 + 32 + dt * 16 + r) * 64 + lane];
          }
        }
        *reinterpret_cast<s16x4*>(kp + 32 * dt + 8 * gq + 4 * hl) = pack4(fa);
        *reinterpret_cast<s16x4*>(vp + 32 * dt + 8 * gq + 4 * hl) = pack4(fc);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
void attn_fwd(const void* q, const void* k, const void* v, void* out, float* lse, const AttnGeom& g, int BH, hipStream_t st) {
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k, (const __bf16*)v,
                     (__bf16*)out, lse, g);
}

void attn_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout, const float* lse,
              void* do_st, float* delta, void* dq, void* dk, void* dv, const AttnGeom& g, int BH, hipStream_t st) {
  const int rows = BH * g.Np;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, st, (const __bf16*)dout,
                     (const __bf16*)out, (__bf16*)do_st, delta, g, BH);
  dim3 grid((g.Np / 32 + 3) / 4, BH);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k, (const __bf16*)v,
                     (const __bf16*)do_st, lse, delta, (__bf16*)dq, g);
  const int ntext = g.Tp / 32, nimg = g.Np / 32 - ntext;
  // text key blocks (long, every image query attends them): one block per workgroup, queries split over waves
  hipLaunchKernelGGL(attn_bwd_dkdv_text_kernel, dim3(ntext, BH), dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (const __bf16*)do_st, lse, delta, (__bf16*)dk, (__bf16*)dv, g);
  // image key blocks (short, local patterns): four blocks per workgroup
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((nimg + 3) / 4, BH), dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (const __bf16*)do_st, lse, delta, (__bf16*)dk, (__bf16*)dv, g);
}

}  // namespace dalle
