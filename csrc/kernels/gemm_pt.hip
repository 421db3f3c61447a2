// Persistent bf16 GEMM with register-direct fused epilogues (SURVEY K5/K6, K8, K9, K10 GEMM +
// epilogue fusion targets).
//
//   C[M, N] = A[M, K] . B[N, K]^T     (both operands K-contiguous; fp32 accumulate)
//
// Main loop: the 256 x 256 x 64 8-phase schedule of gemm.hip (8 waves, 2 along M x 4 along N,
// half-tile LDS-DMA images, counted vmcnt, the two wave rows staggered by one barrier), with three
// changes that target the epilogue, which cost the one-tile-per-workgroup kernel 16-26 % of its time
// (profiles/r2_gemm_epilogue_cost.jsonl):
//
//   1. Persistent: one workgroup per CU walks its tiles (XCD-aware order), and the DMA stream is ONE
//      sequence of K-steps across tile boundaries -- the next tile's first K-tiles are already in flight
//      while a tile's last K-step computes, so there is no per-tile prologue bubble.
//   2. Transposed accumulators: the MFMA is issued as B-fragment x A-fragment, so every lane ends up
//      holding 4 CONSECUTIVE output columns of one row (C^T layout) instead of 4 rows of one column.
//      The epilogue converts straight from the accumulators: no LDS staging pass (no 2-byte
//      ds_write per element), and v_permlane16_swap pairs two 16-column sub-tiles so each lane
//      issues one 16-byte store per pair.
//   3. The epilogue of tile i runs at the start of tile i+1's first phase (LDS is not touched, the
//      accumulators are re-zeroed right after), so its global stores drain while the next tile's
//      MFMAs run.
//
// Epilogues (template EPI): 0 = bf16 store (+bias), 1 = QKV + 3-axis rotary scattered into the
// attention storage (q pre-scaled), 2 = GEGLU backward (FF-out dgrad: dh = GEGLU'(h, du) + per-64-row
// bias-grad partials), 3 = GEGLU forward (FF-in: W1 rows interleaved per 64-column group, writes the
// pre-activation a = [value | gate] and u = value * gelu(gate)), 5 = none (measurement only).
#include "common.h"

#include <cstdlib>

namespace dalle {

namespace pt {

typedef __attribute__((ext_vector_type(4))) float f4;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int THREADS = 512;
constexpr int HALF = 128 * BK;  // elements of one half-tile image (128 operand rows x 64 k)

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// Half-tile image of 128 operand rows (see gemm.hip stage_half): image row hr <-> tile row
// (hr / blk) * 2 blk + off + hr % blk; the 16-byte chunk index is XOR-swizzled by image row on the
// per-lane SOURCE address (the DMA writes LDS lane-linearly).
__device__ __forceinline__ void stage_half(const __bf16* __restrict__ src, int ld, int row0, int k0, __bf16* lds_half,
                                           int wave, int lane, int blk, int off) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;
    const int hr = piece * 8 + (lane >> 3);
    const int row = (hr / blk) * 2 * blk + off + (hr % blk);
    const int lchunk = (lane & 7) ^ swz(hr);
    const __bf16* g = src + (size_t)(row0 + row) * ld + k0 + lchunk * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)(lds_half + piece * 512), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const __bf16* tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(tile + row * 64 + ((chunk ^ swz(row)) << 3));
}

// persistent tile id -> (tm, tn): XCD slot first (blocks b and b + 8 share an XCD, and the grid is a
// multiple of 8, so a workgroup stays on one XCD's contiguous range), then column groups of `group`
// panels swept along M (group > 0) or row groups of -group panels swept along N (group < 0)
__device__ __forceinline__ void tile_of(int id, int tiles_m, int tiles_n, int group, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  if ((nwg & 7) == 0) id = (id & 7) * (nwg >> 3) + (id >> 3);
  if (group > 0) {
    const int g = id / (group * tiles_m);
    const int first_n = g * group;
    const int gn = min(tiles_n - first_n, group);
    const int in_group = id - g * group * tiles_m;
    tn = first_n + in_group % gn;
    tm = in_group / gn;
  } else {
    const int gm_size = -group;
    const int g = id / (gm_size * tiles_n);
    const int first_m = g * gm_size;
    const int gm = min(tiles_m - first_m, gm_size);
    const int in_group = id - g * gm_size * tiles_n;
    tm = first_m + in_group % gm;
    tn = in_group / gm;
  }
}

__device__ __forceinline__ unsigned pk2(float a, float b) {
  const __bf16 x = (__bf16)a, y = (__bf16)b;
  return (unsigned)__builtin_bit_cast(unsigned short, x) | ((unsigned)__builtin_bit_cast(unsigned short, y) << 16);
}
__device__ __forceinline__ float lo_f(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi_f(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// v_permlane16_swap: rows (16 lanes) 1 and 3 of x trade places with rows 0 and 2 of y. Applied to
// the packed columns of sub-tiles j (x) and j + 1 (y) it leaves lanes of row q = 0, 2 holding 8
// consecutive columns of j and lanes of row 1, 3 holding 8 consecutive columns of j + 1; the swap is
// an involution, so the same call turns 16-byte loads of that arrangement back into per-lane columns.
__device__ __forceinline__ void swap16(unsigned& x, unsigned& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

// DPP row_ror:8 -- lane l of every 16-lane row reads lane (l + 8) & 15 of the same row
__device__ __forceinline__ unsigned ror8(unsigned v) { return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false); }

// Whole-line re-layout of one 16-row sub-tile (round 4, profiles/r4_store_patterns.jsonl): on entry lane
// (fr, q) holds two 16-byte chunks of ITS row fr, c0 from column pair jp = 0 and c1 from jp = 1 (the
// layout after swap16); on exit c0 is the chunk of row (fr & 7) and c1 the chunk of row 8 + (fr & 7), both
// at element column lines_col(lane) of the wave's 64. The lanes of row halves fr < 8 / fr >= 8 trade their
// jp = 1 / jp = 0 chunks through one DPP row rotate per dword, so each store instruction covers 8 rows x
// 128 B (whole lines) instead of 16 rows x 64 B: 41-51 vs 14-15 B/clk of store issue per CU.
__device__ __forceinline__ void lines16(u32x4_vs& c0, u32x4_vs& c1, bool low) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned r = ror8(low ? c1[k] : c0[k]);
    const unsigned a = low ? c0[k] : r, b = low ? r : c1[k];
    c0[k] = a;
    c1[k] = b;
  }
}
__device__ __forceinline__ int lines_col(int lane) {
  const int fr = lane & 15, q = lane >> 4;
  return (fr >> 3) * 32 + (q & 1) * 16 + (q >> 1) * 8;
}

// epilogue output stream: a wave-uniform base, its buffer descriptor and the store cache policy
struct Out {
  __bf16* base;
  __amdgpu_buffer_rsrc_t rsrc;
  int cpol;
  __device__ __forceinline__ Out(__bf16* b, int cp) : base(b), rsrc(uniform_rsrc(b)), cpol(cp) {}
  __device__ __forceinline__ void st(__bf16* p, unsigned x0, unsigned x1, unsigned y0, unsigned y1) const {
    const u32x4_vs v = {x0, x1, y0, y1};
    cstore16(base, rsrc, (uint32_t)((char*)p - (char*)base), v, cpol);
  }
  __device__ __forceinline__ void st4(__bf16* p, const u32x4_vs& v) const {
    cstore16(base, rsrc, (uint32_t)((char*)p - (char*)base), v, cpol);
  }
};

}  // namespace pt

struct PtArgs {
  // EPI 0: C (M, ldc) bf16 (+ bias (N,) bf16, may be null)
  __bf16* C;
  const __bf16* bias;
  int ldc;
  // EPI 1 (QKV + rotary): storage (B*H, Np, 64); cs (n + 1, 32, 2) fp32 = (cos, sin) per rotary pair
  __bf16* q;
  __bf16* k;
  __bf16* v;
  const float* cs;
  int T, Tp, S, logS, n, Np, H, col_major;
  float qscale;
  // EPI 2 (GEGLU backward): h = FF-in pre-activation (M, 2F) [value | gate], dh its gradient,
  // part (M / 64, 2F) fp32 partial column sums of dh (the FF-in bias gradient)
  const __bf16* h;
  __bf16* dh;
  float* part;
  int F;
  // EPI 3 (GEGLU forward): a (M, 2F) pre-activation in the ORIGINAL [value | gate] column order, u (M, F)
  __bf16* a;
  __bf16* u;
  int group;
  int stagger, first_wave;  // per-tile mode: start-time stagger of the first wave (stagger_start)
  int cpol;                 // cache policy of the output stores (common.h cstore16)
  // measurement only (one tile per workgroup): per workgroup {start, epilogue start, stores issued,
  // stores complete, CU id} in 10 ns real-time ticks; skip_odd = odd workgroups issue no stores
  unsigned long long* stamps;
  int skip_odd;
  int drain;  // wait for the output stores before the workgroup ends (gemm_set_drain)
  int prefetch;  // EPI 2: pull the tile's pre-activation lines toward the caches during its main loop
  int overlap;   // persistent: a tile's epilogue stores drain beside the next tile's first K-steps (pt_overlap)
};

__device__ __forceinline__ int pt_seq2st(const PtArgs& e, int p) {
  if (p < e.T) return p;
  const int kk = p - e.T;
  const int kst = e.col_major ? ((kk & (e.S - 1)) << e.logS) + (kk >> e.logS) : kk;
  return e.Tp + kst;
}

// Epilogue of one finished tile (origin r0, c0) straight from the transposed accumulators: lane l of
// wave (wm, wn) holds, for sub-tile (i, j), row r0 + wm*128 + i*16 + (l & 15) and the 4 columns
// c0 + wn*64 + j*16 + (l >> 4)*4 + 0..3.
template <int EPI, bool LINES>
__device__ __forceinline__ void pt_epilogue(pt::f4 (&acc)[8][4], int r0, int c0, int wm, int wn, int lane, const PtArgs& e) {
  using namespace pt;
  const int fr = lane & 15, q = lane >> 4;
  const int cw = c0 + wn * 64;  // first column of the wave's 64
  if constexpr (EPI == 5) {  // measurement: keep the results live, store nothing
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (e.ldc < 0) e.C[lane] = (__bf16)t;
    return;
  }
  if constexpr (EPI == 0) {
    if (e.skip_odd && (blockIdx.x & 1)) return;
    const pt::Out oc(e.C, e.cpol);
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
    if (e.bias != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 b = *reinterpret_cast<const uint2*>(e.bias + cw + j * 16 + q * 4);
        bv[j][0] = lo_f(b.x); bv[j][1] = hi_f(b.x); bv[j][2] = lo_f(b.y); bv[j][3] = hi_f(b.y);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __bf16* rowp = e.C + (size_t)(r0 + wm * 128 + i * 16 + fr) * e.ldc + cw + (q & 2) * 4;
      u32x4_vs ch[2];
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int j0 = 2 * jp, j1 = j0 + 1;
        unsigned x0 = pk2(acc[i][j0][0] + bv[j0][0], acc[i][j0][1] + bv[j0][1]);
        unsigned x1 = pk2(acc[i][j0][2] + bv[j0][2], acc[i][j0][3] + bv[j0][3]);
        unsigned y0 = pk2(acc[i][j1][0] + bv[j1][0], acc[i][j1][1] + bv[j1][1]);
        unsigned y1 = pk2(acc[i][j1][2] + bv[j1][2], acc[i][j1][3] + bv[j1][3]);
        swap16(x0, y0);
        swap16(x1, y1);
        if constexpr (LINES) ch[jp] = u32x4_vs{x0, x1, y0, y1};
        else oc.st(rowp + ((q & 1) ? j1 : j0) * 16, x0, x1, y0, y1);
      }
      if constexpr (LINES) {
        lines16(ch[0], ch[1], fr < 8);
        __bf16* lp = e.C + (size_t)(r0 + wm * 128 + i * 16 + (fr & 7)) * e.ldc + cw + lines_col(lane);
        oc.st4(lp, ch[0]);
        oc.st4(lp + (size_t)8 * e.ldc, ch[1]);
      }
    }
  } else if constexpr (EPI == 1) {
    // the wave's 64 columns are one (part, head); rotary pairs (2t, 2t+1) sit in one lane
    const int HD = e.H * 64;
    const int part = cw / HD, hh = (cw - part * HD) >> 6;
    __bf16* dstT = part == 0 ? e.q : (part == 1 ? e.k : e.v);
    const float sc = part == 0 ? e.qscale : 1.0f;
    const pt::Out oc(dstT, e.cpol);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = r0 + wm * 128 + i * 16 + fr;
      const int b = r / e.n, p = r - b * e.n;
      __bf16* rowp = dstT + ((size_t)(b * e.H + hh) * e.Np + pt_seq2st(e, p)) * 64 + (q & 2) * 4;
      const float* csp = e.cs + (size_t)p * 64 + q * 4;  // (cos, sin) of pairs j*8 + 2q, j*8 + 2q + 1
      f4 t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = *reinterpret_cast<const f4*>(csp + j * 16);
      unsigned w[4][2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x0 = acc[i][j][0], x1 = acc[i][j][1], x2 = acc[i][j][2], x3 = acc[i][j][3];
        w[j][0] = pk2((x0 * t[j][0] - x1 * t[j][1]) * sc, (x1 * t[j][0] + x0 * t[j][1]) * sc);
        w[j][1] = pk2((x2 * t[j][2] - x3 * t[j][3]) * sc, (x3 * t[j][2] + x2 * t[j][3]) * sc);
      }
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int j0 = 2 * jp, j1 = j0 + 1;
        swap16(w[j0][0], w[j1][0]);
        swap16(w[j0][1], w[j1][1]);
        if constexpr (!LINES) oc.st(rowp + ((q & 1) ? j1 : j0) * 16, w[j0][0], w[j0][1], w[j1][0], w[j1][1]);
      }
      if constexpr (LINES) {
        // the 16 rows of a sub-tile are 16 consecutive positions of one sample (n % 16 == 0, host-checked)
        u32x4_vs c0v = {w[0][0], w[0][1], w[1][0], w[1][1]}, c1v = {w[2][0], w[2][1], w[3][0], w[3][1]};
        lines16(c0v, c1v, fr < 8);
        const int p0 = p - (fr & 8);
        __bf16* base = dstT + (size_t)(b * e.H + hh) * e.Np * 64 + lines_col(lane);
        oc.st4(base + (size_t)pt_seq2st(e, p0) * 64, c0v);
        oc.st4(base + (size_t)pt_seq2st(e, p0 + 8) * 64, c1v);
      }
      __builtin_amdgcn_sched_barrier(0);  // bound the live loads to one row sub-tile
    }
  } else if constexpr (EPI == 2) {
    // GEGLU backward: the tile is du for feature columns f = cw + j*16 + q*4 + r (bf16-rounded, as the
    // unfused path stores it). da = du * gelu(gate), dg = du * value * gelu'(gate) into dh, and the
    // column sums of the (bf16) results over each 64-row half of the wave's 128 rows -> part. One
    // sub-tile pair (j0, j0 + 1) of one 64-row half at a time keeps the live set small.
    const int F = e.F;
    const pt::Out od(e.dh, e.cpol);
    u32x4_vs hold[4][2];  // LINES: the jp = 0 [da | dg] chunks of the half's 4 sub-tiles, paired with jp = 1
#pragma unroll
    for (int half = 0; half < 2; ++half)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int j0 = 2 * jp, j1 = j0 + 1;
        const int jo = ((q & 1) ? j1 : j0) * 16;
        float sv[2][4], sg[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) sv[t][r] = sg[t][r] = 0.f;
        // every [value | gate] load of the half first: one wait for 8 loads, not one per 16 rows
        uint4 lvs[4], lgs[4];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const size_t row = (size_t)(r0 + wm * 128 + (half * 4 + ii) * 16 + fr);
          const size_t off = row * 2 * F + cw + (q & 2) * 4 + jo;
          lvs[ii] = *reinterpret_cast<const uint4*>(e.h + off);
          lgs[ii] = *reinterpret_cast<const uint4*>(e.h + off + F);
        }
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = half * 4 + ii;
          const size_t row = (size_t)(r0 + wm * 128 + i * 16 + fr);
          const size_t off = row * 2 * F + cw + (q & 2) * 4 + jo;
          const uint4 lv = lvs[ii], lg = lgs[ii];
          unsigned va[2][2] = {{lv.x, lv.y}, {lv.z, lv.w}}, ga[2][2] = {{lg.x, lg.y}, {lg.z, lg.w}};
          swap16(va[0][0], va[1][0]); swap16(va[0][1], va[1][1]);
          swap16(ga[0][0], ga[1][0]); swap16(ga[0][1], ga[1][1]);
          unsigned da[2][2], dg[2][2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int j = j0 + t;
            float d[4], av[4], gv[4], ra[4], rg[4];
            const unsigned d01 = pk2(acc[i][j][0], acc[i][j][1]), d23 = pk2(acc[i][j][2], acc[i][j][3]);
            d[0] = lo_f(d01); d[1] = hi_f(d01); d[2] = lo_f(d23); d[3] = hi_f(d23);
            av[0] = lo_f(va[t][0]); av[1] = hi_f(va[t][0]); av[2] = lo_f(va[t][1]); av[3] = hi_f(va[t][1]);
            gv[0] = lo_f(ga[t][0]); gv[1] = hi_f(ga[t][0]); gv[2] = lo_f(ga[t][1]); gv[3] = hi_f(ga[t][1]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float ge, gr;
              gelu_and_grad(gv[r], ge, gr);
              ra[r] = d[r] * ge;
              rg[r] = d[r] * av[r] * gr;
            }
            da[t][0] = pk2(ra[0], ra[1]); da[t][1] = pk2(ra[2], ra[3]);
            dg[t][0] = pk2(rg[0], rg[1]); dg[t][1] = pk2(rg[2], rg[3]);
            sv[t][0] += lo_f(da[t][0]); sv[t][1] += hi_f(da[t][0]); sv[t][2] += lo_f(da[t][1]); sv[t][3] += hi_f(da[t][1]);
            sg[t][0] += lo_f(dg[t][0]); sg[t][1] += hi_f(dg[t][0]); sg[t][2] += lo_f(dg[t][1]); sg[t][3] += hi_f(dg[t][1]);
          }
          swap16(da[0][0], da[1][0]); swap16(da[0][1], da[1][1]);
          swap16(dg[0][0], dg[1][0]); swap16(dg[0][1], dg[1][1]);
          if constexpr (LINES) {
            u32x4_vs ca = {da[0][0], da[0][1], da[1][0], da[1][1]}, cg = {dg[0][0], dg[0][1], dg[1][0], dg[1][1]};
            if (jp == 0) {
              hold[ii][0] = ca;
              hold[ii][1] = cg;
            } else {
              lines16(hold[ii][0], ca, fr < 8);
              lines16(hold[ii][1], cg, fr < 8);
              const size_t lrow = (size_t)(r0 + wm * 128 + i * 16 + (fr & 7));
              __bf16* lp = e.dh + lrow * 2 * F + cw + lines_col(lane);
              od.st4(lp, hold[ii][0]);
              od.st4(lp + (size_t)16 * F, ca);
              od.st4(lp + F, hold[ii][1]);
              od.st4(lp + (size_t)16 * F + F, cg);
            }
          } else {
            od.st(e.dh + off, da[0][0], da[0][1], da[1][0], da[1][1]);
            od.st(e.dh + off + F, dg[0][0], dg[0][1], dg[1][0], dg[1][1]);
          }
        }
        // reduce over the 16 rows held by lanes 16q .. 16q+15 (fixed xor tree: deterministic)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1)
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              sv[t][r] += __shfl_xor(sv[t][r], o, 64);
              sg[t][r] += __shfl_xor(sg[t][r], o, 64);
            }
        if (fr == 0) {
          float* pr = e.part + (size_t)((r0 + wm * 128 + half * 64) >> 6) * 2 * F + cw + q * 4;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            *reinterpret_cast<f4*>(pr + (j0 + t) * 16) = f4{sv[t][0], sv[t][1], sv[t][2], sv[t][3]};
            *reinterpret_cast<f4*>(pr + F + (j0 + t) * 16) = f4{sg[t][0], sg[t][1], sg[t][2], sg[t][3]};
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
  } else if constexpr (EPI == 3) {
    // GEGLU forward: the wave's 64 columns are [32 value | 32 gate] of features fb .. fb + 31
    // (W1 / b1 rows interleaved on the host); j = 0, 1 value, j = 2, 3 the matching gate
    const int F = e.F;
    const int fb = cw >> 1;
    const pt::Out oa(e.a, e.cpol), ou(e.u, e.cpol);
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
    if (e.bias != nullptr) {  // the interleaved bias (2F,)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 b = *reinterpret_cast<const uint2*>(e.bias + cw + j * 16 + q * 4);
        bv[j][0] = lo_f(b.x); bv[j][1] = hi_f(b.x); bv[j][2] = lo_f(b.y); bv[j][3] = hi_f(b.y);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const size_t row = (size_t)(r0 + wm * 128 + i * 16 + fr);
      __bf16* ap = e.a + row * 2 * F + fb + (q & 2) * 4;
      __bf16* up = e.u + row * F + fb + (q & 2) * 4;
      unsigned vv[2][2], gg[2][2], uu[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        vv[j][0] = pk2(acc[i][j][0] + bv[j][0], acc[i][j][1] + bv[j][1]);
        vv[j][1] = pk2(acc[i][j][2] + bv[j][2], acc[i][j][3] + bv[j][3]);
        gg[j][0] = pk2(acc[i][j + 2][0] + bv[j + 2][0], acc[i][j + 2][1] + bv[j + 2][1]);
        gg[j][1] = pk2(acc[i][j + 2][2] + bv[j + 2][2], acc[i][j + 2][3] + bv[j + 2][3]);
        float o[4];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          o[2 * h2] = lo_f(vv[j][h2]) * gelu_fast(lo_f(gg[j][h2]));
          o[2 * h2 + 1] = hi_f(vv[j][h2]) * gelu_fast(hi_f(gg[j][h2]));
        }
        uu[j][0] = pk2(o[0], o[1]);
        uu[j][1] = pk2(o[2], o[3]);
      }
      swap16(vv[0][0], vv[1][0]); swap16(vv[0][1], vv[1][1]);
      swap16(gg[0][0], gg[1][0]); swap16(gg[0][1], gg[1][1]);
      swap16(uu[0][0], uu[1][0]); swap16(uu[0][1], uu[1][1]);
      const int jo = (q & 1) * 16;
      oa.st(ap + jo, vv[0][0], vv[0][1], vv[1][0], vv[1][1]);
      oa.st(ap + F + jo, gg[0][0], gg[0][1], gg[1][0], gg[1][1]);
      ou.st(up + jo, uu[0][0], uu[0][1], uu[1][0], uu[1][1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// FF-in + GEGLU forward (EPI 3) with whole-line stores, one tile per workgroup: after the main loop the
// 128 KiB of operand LDS is free, so the tile goes out through it. Pass 1 writes value and gate (bf16, 8 B
// per lane: 4 consecutive features) into two [256 rows][128 features] images whose 16-byte chunks are
// XOR-swizzled by row (c ^ (row & 15): the 16 lanes of a write group hit 16 distinct chunks); pass 2 reads
// them back (each instruction covers 4 whole rows x 256 B) and stores whole 128-B lines of a (value | gate
// halves) and of u = value * gelu(gate), computed there from the same bf16 values (one barrier in all;
// round 3 held u in registers through pass 1 and needed a third LDS pass).
__device__ __forceinline__ int geglu_lds_idx(int row, int feat) {
  return row * 128 + ((((feat >> 3) ^ (row & 15)) << 3) | (feat & 7));
}

__device__ __forceinline__ void pt_epilogue_geglu_lds(pt::f4 (&acc)[8][4], __bf16* smem, int r0, int c0, int wm, int wn,
                                                      int lane, const PtArgs& e) {
  using namespace pt;
  const int fr = lane & 15, q = lane >> 4;
  const int tid = threadIdx.x;
  const int F = e.F;
  const int fw = c0 >> 1;  // the workgroup's first feature (128 features per tile)
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
  if (e.bias != nullptr) {  // the interleaved bias (2F,)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint2 b = *reinterpret_cast<const uint2*>(e.bias + c0 + wn * 64 + j * 16 + q * 4);
      bv[j][0] = lo_f(b.x); bv[j][1] = hi_f(b.x); bv[j][2] = lo_f(b.y); bv[j][3] = hi_f(b.y);
    }
  }
  __bf16* V = smem;              // [256][128] value image
  __bf16* G = smem + 256 * 128;  // [256][128] gate image
  asm volatile("s_barrier" ::: "memory");  // every wave is past its last operand read
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wm * 128 + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned v0 = pk2(acc[i][j][0] + bv[j][0], acc[i][j][1] + bv[j][1]);
      const unsigned v1 = pk2(acc[i][j][2] + bv[j][2], acc[i][j][3] + bv[j][3]);
      const unsigned g0 = pk2(acc[i][j + 2][0] + bv[j + 2][0], acc[i][j + 2][1] + bv[j + 2][1]);
      const unsigned g1 = pk2(acc[i][j + 2][2] + bv[j + 2][2], acc[i][j + 2][3] + bv[j + 2][3]);
      const int feat = wn * 32 + j * 16 + q * 4;
      *reinterpret_cast<uint2*>(V + geglu_lds_idx(row, feat)) = uint2{v0, v1};
      *reinterpret_cast<uint2*>(G + geglu_lds_idx(row, feat)) = uint2{g0, g1};
    }
  }
  __syncthreads();
  // one pass: each thread takes an 8-feature chunk of one row, stores its value and gate lines and the
  // product u = value * gelu(gate) of the same (bf16) values
  const pt::Out oa(e.a, e.cpol), ou(e.u, e.cpol);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 512 + tid, row = idx >> 4, ch = idx & 15;
    const int li = row * 128 + ((ch ^ (row & 15)) << 3);
    const u32x4_vs vv = *reinterpret_cast<const u32x4_vs*>(V + li);
    const u32x4_vs gg = *reinterpret_cast<const u32x4_vs*>(G + li);
    __bf16* ap = e.a + (size_t)(r0 + row) * 2 * F + fw + ch * 8;
    oa.st4(ap, vv);
    oa.st4(ap + F, gg);
    u32x4_vs uv;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      uv[k] = pk2(lo_f(vv[k]) * gelu_fast(lo_f(gg[k])), hi_f(vv[k]) * gelu_fast(hi_f(gg[k])));
    ou.st4(e.u + (size_t)(r0 + row) * F + fw + ch * 8, uv);
  }
}

// FF-out dgrad + GEGLU backward (EPI 2) through LDS, one tile per workgroup (the LDS-staged epilogue of the
// 8-phase kernel on this kernel's faster main loop): each wave parks its 128 x 64 du block (bf16, as the
// unfused path rounds it) in its own 16 KB of the free operand LDS -- 8-byte writes of 4 consecutive columns,
// 16-byte chunks XOR-swizzled by row -- then every lane owns one 8-column chunk of 16 rows: its 32
// pre-activation loads ([value | gate] halves) are issued together, da = du * gelu(gate) and
// dg = du * value * gelu'(gate) leave as whole 128-B lines (8 rows x 128 B per store instruction), and the
// column sums of the bf16 results over each 64-row half are reduced over the 8 lanes sharing a chunk
// (fixed xor tree) into part (M / 64, 2F).
__device__ __forceinline__ void pt_epilogue_geglu_bwd_lds(pt::f4 (&acc)[8][4], __bf16* smem, int r0, int c0, int wm, int wn,
                                                          int lane, const PtArgs& e) {
  using namespace pt;
  const int fr = lane & 15, q = lane >> 4;
  const int F = e.F;
  __bf16* ep = smem + (threadIdx.x >> 6) * (128 * 64);
  asm volatile("s_barrier" ::: "memory");  // every wave is past its last operand read
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = i * 16 + fr, c = j * 16 + q * 4;
      *reinterpret_cast<uint2*>(ep + row * 64 + ((((c >> 3) ^ (row & 7)) << 3) | (c & 7))) =
          uint2{pk2(acc[i][j][0], acc[i][j][1]), pk2(acc[i][j][2], acc[i][j][3])};
    }
  const int ch = lane & 7;
  const int gcol = c0 + wn * 64 + ch * 8;
  const size_t rw = (size_t)(r0 + wm * 128);
  s16x8 hv[16], hg[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const size_t r = rw + it * 8 + (lane >> 3);
    hv[it] = *reinterpret_cast<const s16x8*>(e.h + r * 2 * F + gcol);
    hg[it] = *reinterpret_cast<const s16x8*>(e.h + r * 2 * F + F + gcol);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's image is complete
  const pt::Out od(e.dh, e.cpol);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    float sv[8] = {}, sg[8] = {};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int it = half * 8 + k;
      const int row = it * 8 + (lane >> 3);
      const size_t r = rw + row;
      float d[8], a[8], gg[8], da[8], dg[8];
      unpack8(*reinterpret_cast<const s16x8*>(ep + row * 64 + ((ch ^ (row & 7)) << 3)), d);
      unpack8(hv[it], a);
      unpack8(hg[it], gg);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float ge, gr;
        gelu_and_grad(gg[i], ge, gr);
        da[i] = d[i] * ge;
        dg[i] = d[i] * a[i] * gr;
      }
      const s16x8 pa = pack8(da), pg = pack8(dg);
      od.st4(e.dh + r * 2 * F + gcol, __builtin_bit_cast(u32x4_vs, pa));
      od.st4(e.dh + r * 2 * F + F + gcol, __builtin_bit_cast(u32x4_vs, pg));
      unpack8(pa, da);
      unpack8(pg, dg);
#pragma unroll
      for (int i = 0; i < 8; ++i) { sv[i] += da[i]; sg[i] += dg[i]; }
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sv[i] += __shfl_xor(sv[i], o, 64);
        sg[i] += __shfl_xor(sg[i], o, 64);
      }
    if (lane < 8) {
      float* pr = e.part + ((rw + half * 64) >> 6) * 2 * F + gcol;
      *reinterpret_cast<f4*>(pr) = f4{sv[0], sv[1], sv[2], sv[3]};
      *reinterpret_cast<f4*>(pr + 4) = f4{sv[4], sv[5], sv[6], sv[7]};
      *reinterpret_cast<f4*>(pr + F) = f4{sg[0], sg[1], sg[2], sg[3]};
      *reinterpret_cast<f4*>(pr + F + 4) = f4{sg[4], sg[5], sg[6], sg[7]};
    }
  }
}

// PERSIST = false: one tile per workgroup (grid = tile count), the same main loop and register-direct
// epilogue -- a workgroup's stores then drain while the NEXT workgroup on that CU already streams its
// first K-tiles (the epilogue ends with the store issue; nothing waits for completion)
template <int EPI, bool PERSIST = true, bool LINES = false>
__global__ __launch_bounds__(pt::THREADS, 1) void gemm_pt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                                 int M, int N, int K, PtArgs e) {
  using namespace pt;
  // vector-memory instructions of one wave's overlapped epilogue (pt_epilogue, EPI 0 without bias: 8
  // row sub-tiles x 2 16-byte stores); 0 = this epilogue cannot overlap
  constexpr int EPI_VM = EPI == 0 ? 16 : 0;
  // [buf][A-lo | B-lo | B-hi | A-hi] half-tile images, 128 KiB in ONE array (a second __shared__
  // object can make hipcc drain vmcnt before every ds_read)
  // + 2 KiB: the landing area of the EPI 2 cache prefetch (8 waves x 256 B, never read)
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 4 * HALF + 1024];
  stagger_start(e.stagger, e.first_wave);
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_m = M / BM, tiles_n = N / BN, ntiles = tiles_m * tiles_n;
  const int nk = K / BK;  // >= 2 (host-checked)
  const int G = gridDim.x;
  const int my_tiles = PERSIST ? (ntiles - (int)blockIdx.x + G - 1) / G : 1;
  const int total = my_tiles * nk;

  auto origin = [&](int it, int& r0, int& c0) {
    int tm, tn;
    tile_of((int)blockIdx.x + it * G, tiles_m, tiles_n, e.group, tm, tn);
    r0 = tm * BM;
    c0 = tn * BN;
  };
  auto slot = [&](int buf, int which) { return smem + (buf * 4 + which) * HALF; };
  // which: 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi
  auto stage = [&](int r0, int c0, int kt, int buf, int which) {
    const int k0 = kt * BK;
    if (which == 0) stage_half(A, K, r0, k0, slot(buf, 0), wave, lane, 64, 0);
    else if (which == 1) stage_half(B, K, c0, k0, slot(buf, 1), wave, lane, 32, 0);
    else if (which == 2) stage_half(B, K, c0, k0, slot(buf, 2), wave, lane, 32, 32);
    else stage_half(A, K, r0, k0, slot(buf, 3), wave, lane, 64, 64);
  };
  auto fragA = [&](const __bf16* img, int i, int kk) { return frag(img, wm * 64 + i * 16 + (lane & 15), kk * 4 + (lane >> 4)); };
  auto fragB = [&](const __bf16* img, int j, int kk) { return frag(img, wn * 32 + j * 16 + (lane & 15), kk * 4 + (lane >> 4)); };

  int cr, cc, nr, nc;  // origins of the current and the next tile
  origin(0, cr, cc);
  if (my_tiles > 1) origin(1, nr, nc);
  else { nr = cr; nc = cc; }

  // prologue: K-step 0 complete, three halves of K-step 1 in flight
  stage(cr, cc, 0, 0, 1); stage(cr, cc, 0, 0, 0); stage(cr, cc, 0, 0, 2); stage(cr, cc, 0, 0, 3);
  stage(cr, cc, 1, 1, 1); stage(cr, cc, 1, 1, 0); stage(cr, cc, 1, 1, 2);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");
  if (wm == 1) asm volatile("s_barrier" ::: "memory");

  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a[4][2], b0[2][2], b1[2][2];
  int pr = 0, pc = 0;  // origin of the finished tile whose epilogue is pending
  int g = 0;
  for (int it = 0; it < my_tiles; ++it) {
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const int buf = g & 1;
      const __bf16* Alo = slot(buf, 0);
      const __bf16* Blo = slot(buf, 1);
      const __bf16* Bhi = slot(buf, 2);
      const __bf16* Ahi = slot(buf, 3);
      // sources of K-steps g + 1 and g + 2 (the next tile's first K-steps near the end of a tile)
      const bool x1 = PERSIST && kt + 1 >= nk, x2 = PERSIST && kt + 2 >= nk;
      const int r1 = x1 ? nr : cr, c1 = x1 ? nc : cc, k1 = x1 ? kt + 1 - nk : kt + 1;
      const int r2 = x2 ? nr : cr, c2 = x2 ? nc : cc, k2 = x2 ? kt + 2 - nk : kt + 2;
      const bool s1 = g + 1 < total, s2 = g + 2 < total;

      // ---- phase 1: B-lo then A-lo -> quadrant (lo, lo)
      // overlapped epilogue (persistent, e.overlap): the previous tile's stores go out HERE, after this
      // phase's DMA, so they are younger than every operand load the phase-4 wait must retire: that wait
      // then leaves them in flight (vmcnt(6 + EPI_VM)) and they drain beside this K-step's MFMAs
      const bool ovl = PERSIST && EPI_VM > 0 && e.overlap && kt == 0 && it > 0;
      if (ovl) {
        if (s1) stage(r1, c1, k1, buf ^ 1, 3);
        __builtin_amdgcn_sched_barrier(0);
        pt_epilogue<EPI, LINES>(acc, pr, pc, wm, wn, lane, e);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) b0[j][kk] = fragB(Blo, j, kk);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) a[i][kk] = fragA(Alo, i, kk);
      if (s1 && !ovl) stage(r1, c1, k1, buf ^ 1, 3);
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j][kk], a[i][kk], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_barrier" ::: "memory");

      // ---- phase 2: B-hi -> quadrant (lo, hi)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) b1[j][kk] = fragB(Bhi, j, kk);
      if (s2) stage(r2, c2, k2, buf, 1);
      asm volatile("s_barrier" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j][kk], a[i][kk], acc[i][2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_barrier" ::: "memory");

      // ---- phase 3: A-hi -> quadrant (hi, hi)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) a[i][kk] = fragA(Ahi, i, kk);
      if (s2) stage(r2, c2, k2, buf, 0);
      asm volatile("s_barrier" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j][kk], a[i][kk], acc[4 + i][2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_barrier" ::: "memory");

      // ---- phase 4: registers only -> quadrant (hi, lo); retire K-step g + 1
      if (s2) {
        stage(r2, c2, k2, buf, 2);
        if (ovl) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + EPI_VM) : "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if constexpr (EPI == 2) {
        // cache prefetch of the pre-activation lines the epilogue will read (2048 x 128 B per tile: the
        // value and gate halves of 256 rows), one 4-byte LDS-DMA piece per lane and line, at four K-steps
        // spread over the main loop: the HBM reads move from the epilogue (when every CU's epilogue
        // competes for them) into the MFMA-bound main loop. Issued after the counted wait, so the wait
        // structure is unchanged (a younger piece only ever makes a later vmcnt stricter).
        const int slot = nk >= 8 ? (kt * 4) / nk : -1;
        if (e.prefetch && slot >= 0 && kt == (slot * nk + 3) / 4) {
          const int L = slot * 512 + tid;  // line id in [0, 2048)
          const int row = L >> 3, ln = L & 7;
          const __bf16* src = e.h + (size_t)(cr + row) * 2 * e.F + (ln < 4 ? cc + ln * 64 : e.F + cc + (ln - 4) * 64);
          __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                           (void __attribute__((address_space(3)))*)(smem + 2 * 4 * HALF + wave * 128), 4, 0, 0);
        }
      }
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j][kk], a[i][kk], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_barrier" ::: "memory");
    }
    // ---- the finished tile's epilogue, straight from the accumulators (no LDS), while the next tile's
    // first K-steps are in flight; then re-zero
    if (it + 1 < my_tiles && !(EPI_VM > 0 && e.overlap)) {
      __builtin_amdgcn_sched_barrier(0);
      pt_epilogue<EPI, LINES>(acc, cr, cc, wm, wn, lane, e);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
    }
    pr = cr;
    pc = cc;
    cr = nr;
    cc = nc;
    if (it + 2 < my_tiles) origin(it + 2, nr, nc);
  }
  if (wm == 0) asm volatile("s_barrier" ::: "memory");
  const unsigned long long t_epi = __builtin_amdgcn_s_memrealtime();
  if constexpr (EPI == 3 && LINES && !PERSIST) pt_epilogue_geglu_lds(acc, smem, pr, pc, wm, wn, lane, e);
  else if constexpr (EPI == 2 && LINES && !PERSIST) pt_epilogue_geglu_bwd_lds(acc, smem, pr, pc, wm, wn, lane, e);
  else pt_epilogue<EPI, LINES>(acc, pr, pc, wm, wn, lane, e);
  if (e.drain && e.stamps == nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!PERSIST && e.stamps != nullptr) {
    const unsigned long long t_issued = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t_done = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      unsigned long long* o = e.stamps + (size_t)blockIdx.x * 5;
      o[0] = t_start; o[1] = t_epi; o[2] = t_issued; o[3] = t_done; o[4] = (unsigned long long)__smid();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int pt_grid(int ntiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  // one workgroup per CU (128 KiB of LDS); a multiple of 8 keeps each workgroup on one XCD's range.
  int g = cus < ntiles ? cus : ntiles;
  if (g > 8 && ntiles > g) g &= ~7;
  return g;
}

static int pt_persist_default() { return 0; }

static int pt_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

// former switch GEMM_STAGGER=<percent>: stagger the first wave by that fraction of one tile's main-loop time
// (10 ns ticks at ~1.3 PF/s chip-wide bf16), when the grid has more tiles than CUs. Off by default: it
// measured SLOWER on every training shape (e.g. M61440 N1024 K8192 874 vs 766 us, N3072 K1024 374 vs 359;
// profiles/r3_gemm_stagger.jsonl) -- the stores' cost is not the simultaneity of the epilogues.
int gemm_stagger_ticks(int ntiles, int K) {
  (void)ntiles;
  (void)K;
  return 0;
}

// former switch GEMM_CPOL: cache policy of every hand-written GEMM's output stores (common.h cstore16);
// gemm_set_cpol overrides it at run time (benchmarks)
static int g_gemm_cpol = 0;
void gemm_set_cpol(int c) { g_gemm_cpol = c; }
int gemm_cpol() { return g_gemm_cpol; }

// former switch GEMM_DRAIN=1: every hand-written GEMM workgroup waits for its output stores (s_waitcnt
// vmcnt(0)) before it ends. Measured: a one-tile-per-workgroup GEMM whose waves end with their
// epilogue stores still in flight runs 4-11 % slower than the same kernel draining them first
// (profiles/r3_gemm_epilogue_stamps.jsonl); gemm_set_drain overrides it at run time
static int g_gemm_drain = 1;
void gemm_set_drain(int d) { g_gemm_drain = d; }
int gemm_drain() { return g_gemm_drain; }

// former switch GEMM_LINES (default 1): epilogue stores of whole 128-B lines (8 rows x 128 B per store
// instruction, lines16) instead of 16 rows x 64 B
static const int g_gemm_lines = 1;
// former switch GEMM_PREFETCH (default 0 until measured): the FF-out dgrad + GEGLU-backward GEMM prefetches
// its epilogue's pre-activation lines during the main loop (off)
static const int g_gemm_prefetch = 0;
// former switch PT_OVERLAP (default 0; measured slower at every B128 shape): persistent plain GEMMs (no bias) issue a tile's stores beside the next
// tile's first K-step (see gemm_pt_kernel phase 1); former switch PT_STAGGER=<percent of one tile>: start the
// persistent workgroups at four phases so their epilogues do not all hit HBM at once
static int g_pt_overlap = 0;
static int g_pt_stagger = 0;
void gemm_set_pt_overlap(int v, int stagger_pct) {
  g_pt_overlap = v;
  g_pt_stagger = stagger_pct;
}

template <int EPI, bool LINES>
static void pt_launch_k(const void* A, const void* B, int M, int N, int K, PtArgs& e, hipStream_t st, int persist, int ntiles) {
  if (persist)
    hipLaunchKernelGGL((gemm_pt_kernel<EPI, true, LINES>), dim3(pt_grid(ntiles)), dim3(pt::THREADS), 0, st, (const __bf16*)A,
                       (const __bf16*)B, M, N, K, e);
  else
    hipLaunchKernelGGL((gemm_pt_kernel<EPI, false, LINES>), dim3(ntiles), dim3(pt::THREADS), 0, st, (const __bf16*)A,
                       (const __bf16*)B, M, N, K, e);
}

template <int EPI>
static void pt_launch(const void* A, const void* B, int M, int N, int K, PtArgs& e, hipStream_t st, int persist = -1,
                      bool lines_ok = true) {
  const int ntiles = (M / pt::BM) * (N / pt::BN);
  if (persist < 0) persist = pt_persist_default();
  if (!persist && e.stagger < 0) e.stagger = gemm_stagger_ticks(ntiles, K);
  if (e.stagger < 0) e.stagger = 0;
  e.first_wave = pt_cus();
  // buffer-store policies address the output with a 32-bit byte offset: plain stores past 2 GiB of output
  e.cpol = (size_t)M * N * 4 < (1ull << 32) ? g_gemm_cpol : 0;
  e.drain = g_gemm_drain;
  e.prefetch = g_gemm_prefetch;
  e.overlap = g_pt_overlap && (EPI != 0 || e.bias == nullptr);
  if (persist && g_pt_stagger > 0 && ntiles > 2 * pt_cus()) {
    // a quarter-phase offset per group of 8 workgroups: (b >> 3) & 3 quarters of stagger_pct % of one tile
    const double tile_s = 2.0 * 256.0 * 256.0 * K / (1.3e15 / pt_cus());
    e.stagger = (int)(tile_s * g_pt_stagger / 100.0 * 1e8);
  }
  if constexpr (EPI == 0 || EPI == 1 || EPI == 2 || EPI == 3) {
    // EPI 3: whole lines through LDS in the one-tile-per-workgroup form only (a persistent kernel's LDS
    // holds the next tile's operands)
    if (g_gemm_lines && lines_ok && (EPI != 3 || !persist)) {
      pt_launch_k<EPI, true>(A, B, M, N, K, e, st, persist, ntiles);
      return;
    }
  }
  pt_launch_k<EPI, false>(A, B, M, N, K, e, st, persist, ntiles);
}

static bool pt_shape_ok(int M, int N, int K) { return M > 0 && N > 0 && M % pt::BM == 0 && N % pt::BN == 0 && K % pt::BK == 0 && K >= 2 * pt::BK; }

static int pt_group_default() { return 4; }

// C (M, ldc) = A B^T (+ bias); epi 5 = main loop only (measurement)
bool gemm_pt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int ldc, int epi, int group,
             hipStream_t st) {
  if (!pt_shape_ok(M, N, K) || ldc < N || ldc % 8) return false;
  PtArgs e{};
  e.stagger = -1;
  e.C = (__bf16*)C;
  e.bias = (const __bf16*)bias;
  e.ldc = ldc;
  e.group = group ? group : pt_group_default();
  // epi: 0 plain, 5 main loop only; +10 = one tile per workgroup, +20 = persistent (default: env),
  // +30 = one tile per workgroup without the start stagger
  const int persist = (epi >= 20 && epi < 30) ? 1 : (epi >= 10 ? 0 : -1);
  if (epi >= 30) e.stagger = 0;
  if (epi == 40 || epi == 41) {  // measurement: per-workgroup timestamps into bias (as int64 buffer)
    e.stamps = (unsigned long long*)bias;
    e.bias = nullptr;
    e.skip_odd = epi == 41;
    epi = 30;
  }
  if (epi % 10 == 5) pt_launch<5>(A, B, M, N, K, e, st, persist);
  else pt_launch<0>(A, B, M, N, K, e, st, persist);
  return true;
}

// QKV projection + rotary into the attention storage layout (q pre-scaled); cs = (n + 1, 32, 2) fp32
bool gemm_pt_qkv_rope(const void* A, const void* W, void* q, void* k, void* v, const float* cs, int M, int K, int H, int T,
                      int S, int n, int col_major, float qscale, hipStream_t st, int persist) {
  const int N = 3 * H * 64;
  if (!pt_shape_ok(M, N, K) || M % n) return false;
  int logS = 0;
  while ((1 << logS) < S) ++logS;
  PtArgs e{};
  e.stagger = -1;
  e.q = (__bf16*)q;
  e.k = (__bf16*)k;
  e.v = (__bf16*)v;
  e.cs = cs;
  e.T = T;
  e.Tp = (T + 31) / 32 * 32;
  e.S = S;
  e.logS = logS;
  e.n = n;
  e.Np = e.Tp + S * S;
  e.H = H;
  e.col_major = col_major;
  e.qscale = qscale;
  e.group = pt_group_default();
  // whole-line stores pair rows 8 apart inside a 16-row sub-tile: one sample's positions when n % 16 == 0
  pt_launch<1>(A, W, M, N, K, e, st, persist, n % 16 == 0);
  return true;
}

// FF-out dgrad + GEGLU backward: du = dy (M, K) . W2 with w2t = W2^T (F, K); h (M, 2F) -> dh (M, 2F) and
// part (M / 64, 2F) partial bias grads
bool gemm_pt_geglu_bwd(const void* dy, const void* w2t, const void* h, void* dh, float* part, int M, int F, int K, hipStream_t st,
                       int persist) {
  if (!pt_shape_ok(M, F, K)) return false;
  PtArgs e{};
  e.stagger = -1;
  e.h = (const __bf16*)h;
  e.dh = (__bf16*)dh;
  e.part = part;
  e.F = F;
  e.group = pt_group_default();
  pt_launch<2>(dy, w2t, M, F, K, e, st, persist);
  return true;
}

// FF-in GEMM + GEGLU forward: x (M, K) . W1i^T where W1i (2F, K) holds W1's rows interleaved per
// 64-row group ([32 value rows | the 32 matching gate rows]) and b1i the same permutation of b1 ->
// a (M, 2F) in the original [value | gate] order and u = value * gelu(gate) (M, F)
bool gemm_pt_geglu_fwd(const void* x, const void* w1i, const void* b1i, void* a, void* u, int M, int F, int K, hipStream_t st,
                       int persist) {
  if (!pt_shape_ok(M, 2 * F, K) || F % 32) return false;
  PtArgs e{};
  e.stagger = -1;
  e.bias = (const __bf16*)b1i;
  e.a = (__bf16*)a;
  e.u = (__bf16*)u;
  e.F = F;
  e.group = pt_group_default();
  pt_launch<3>(x, w1i, M, 2 * F, K, e, st, persist);
  return true;
}

// device probe of the v_permlane16_swap lane convention the epilogues rely on: out[0:64] = x, out[64:128] = y
// after swap16(x = lane, y = 100 + lane)
__global__ void permlane16_probe_kernel(unsigned* out) {
  unsigned x = threadIdx.x, y = 100 + threadIdx.x;
  pt::swap16(x, y);
  out[threadIdx.x] = x;
  out[64 + threadIdx.x] = y;
}
void permlane16_probe(unsigned* out, hipStream_t st) { hipLaunchKernelGGL(permlane16_probe_kernel, dim3(1), dim3(64), 0, st, out); }

}  // namespace dalle
