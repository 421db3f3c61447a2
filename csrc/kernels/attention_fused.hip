// The fused one-workgroup-per-head backward of the axial attention patterns (its own translation unit: in
// attention.hip the same source changed the code the compiler emits for the two-kernel dQ kernel).
#include <cstdlib>

#include "attn_tile.h"

namespace dalle {

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
__device__ __forceinline__ void rot_cs(const float* rf, const RotSpec& ro, const AttnGeom& g, int p, int j, float& c, float& s) {
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
__device__ __forceinline__ void rot_stage(const float* rf, const RotSpec& ro, const AttnGeom& g, int s0, int dt,
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
    const __bf16* __restrict__ out, const float* __restrict__ lse, AttnGeom g, RopeOut ro, RotSpec rsp) {
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
  if (tid < 64) rotf[tid] = rsp.rotf[tid];
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
          rot_stage(rotf, rsp, g, i * 32, q4 & 1, av, 1.0f, stg + q4 * STG_BYTES, lane);
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
      rot_stage(rotf, rsp, g, j * 32, dt, dq, ro.qscale, stg + (4 + dt) * STG_BYTES, lane);
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
    rot_stage(rotf, rsp, g, wave * 32, 0, dk0, 1.0f, mystg, lane);
    rot_stage(rotf, rsp, g, wave * 32, 1, dk1, 1.0f, mystg + STG_BYTES, lane);
    rot_stage(rotf, rsp, g, wave * 32, 0, dv0, 1.0f, mystg + 2 * STG_BYTES, lane);
    rot_stage(rotf, rsp, g, wave * 32, 1, dv1, 1.0f, mystg + 3 * STG_BYTES, lane);
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
        rot_cs(rotf, rsp, g, p, 4 * ch + e / 2, c, s);
        y[e] = src[e] * c + src[e + 1] * s;
        y[e + 1] = src[e + 1] * c - src[e] * s;
      }
      *reinterpret_cast<s16x8*>(ro.dqkv + ((size_t)bb * g.n + p) * (3 * HD) + t * HD + hh * 64 + 8 * ch) = pack8(y);
    }
  }
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

void attn_bwd_fused_launch(const void* q, const void* k, const void* v, const void* dout, const void* out, const float* lse,
                           const AttnGeom& g, int BH, hipStream_t st, const RopeOut& ro, const RotSpec& rsp) {
  hipLaunchKernelGGL(attn_bwd_fused_axial_kernel, dim3(BH), dim3(512), 0, st, (const __bf16*)q, (const __bf16*)k,
                     (const __bf16*)v, (const __bf16*)dout, (const __bf16*)out, lse, g, ro, rsp);
}

}  // namespace dalle
