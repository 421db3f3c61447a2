// bf16 GEMM on CDNA4 MFMA with fused epilogues (SURVEY K9/K10 epilogue targets).
//
//   C[M, N] = A[M, K] . B[N, K]^T     (both operands K-contiguous: "NT"; fp32 accumulate)
//
// Workgroup tile 256 x 256 x 64, 8 waves (2 along M x 4 along N, 128 x 64 outputs per wave, 32
// v_mfma_f32_16x16x32_bf16 accumulators). Operands stream global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: one 1 KiB piece = 8 rows x 128 B per wave-instruction), double
// buffered. The LDS image is lane-linear (the DMA writes base + 16*lane), so the XOR swizzle that
// makes the fragment reads bank-conflict-free is applied to the per-lane SOURCE address:
// physical 16-byte chunk c of row r holds logical chunk c ^ swz(r), swz(r) = (r >> 1) & 7 -- the 16
// rows x 1 chunk read by each ds_read_b128 lane group then land on 16 distinct bank slots.
// Workgroups walk the output tiles in an XCD-aware, column-grouped order (B column panels stay in
// one XCD's L2 while its A row panels stream).
//
// Epilogues (template EPI): 0 = bf16 store (+bias); further epilogues fuse the GEGLU forward /
// backward into the FF GEMMs (see gemm_epilogue).
//
// Measured and rejected (profiles/r2_gemm_persistent_vs_8ph_vs_hipblaslt.jsonl): a persistent form
// (one workgroup per CU walking the tiles, the next tile's first K-tile DMA issued before the current
// tile's epilogue, which staged through the other buffer in two 64-row halves) was 1-7 % SLOWER than
// this one-tile-per-workgroup kernel on every training shape and on both fused epilogues: keeping the
// loop-invariant fragment / DMA offsets live across the epilogue pushed it past 256 VGPRs (40-56
// spilled, reloaded once per tile), and the exposed prologue was not the bottleneck.
#include "common.h"

#include <cstdlib>

namespace dalle {

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int GBM = 256, GBN = 256, GBK = 64;
constexpr int G_THREADS = 512;

__device__ __forceinline__ int gswz(int r) { return (r >> 1) & 7; }

// one operand tile (256 rows x 64 k) of buffer `buf` into LDS via 4 DMA pieces per wave
__device__ __forceinline__ void gemm_stage(const __bf16* __restrict__ src, int ld, int row0, int k0, __bf16* lds_tile,
                                           int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;           // 0..31, rows 8*piece .. 8*piece+7
    const int row = piece * 8 + (lane >> 3);  // this lane's row in the tile
    const int lchunk = (lane & 7) ^ gswz(row);  // logical chunk that lands in physical chunk (lane & 7)
    const __bf16* g = src + (size_t)(row0 + row) * ld + k0 + lchunk * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)(lds_tile + piece * 512), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 gemm_frag(const __bf16* tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(tile + row * 64 + ((chunk ^ gswz(row)) << 3));
}

// XCD-aware tile order: linear id -> XCD slot; within an XCD, tiles sweep M inside groups of
// `group` column panels (group > 0), or sweep N inside groups of -group row panels (group < 0)
__device__ __forceinline__ void gemm_tile_of(int& tm, int& tn, int tiles_m, int tiles_n, int group = 4) {
  const int nwg = tiles_m * tiles_n;
  int id = blockIdx.x;
  if ((nwg & 7) == 0) id = (id & 7) * (nwg >> 3) + (id >> 3);  // bijective when nwg % 8 == 0
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

template <int EPI, int VAR>
__global__ __launch_bounds__(G_THREADS, 1) void gemm_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                               __bf16* __restrict__ C, const __bf16* __restrict__ bias,
                                                               int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * GBM * GBK];  // [buf][A | B] 128 KiB
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  gemm_tile_of(tm, tn, M / GBM, N / GBN);
  const int row0 = tm * GBM, col0 = tn * GBN;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  gemm_stage(A, K, row0, 0, smem, wave, lane);
  gemm_stage(B, K, col0, 0, smem + GBM * GBK, wave, lane);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) {
      __bf16* nb = smem + (buf ^ 1) * (2 * GBM * GBK);
      gemm_stage(A, K, row0, (t + 1) * GBK, nb, wave, lane);
      gemm_stage(B, K, col0, (t + 1) * GBK, nb + GBM * GBK, wave, lane);
    }
    const __bf16* As = smem + buf * (2 * GBM * GBK);
    const __bf16* Bs = As + GBM * GBK;
    if (VAR == 0) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a[8], b[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = gemm_frag(As, wm * 128 + i * 16 + fr, kk * 4 + fq);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = gemm_frag(Bs, wn * 64 + j * 16 + fr, kk * 4 + fq);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // all fragments of the K-step first (24 ds_read_b128 in flight), then 64 MFMAs at raised priority
      bf16x8 a[2][8], b[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[kk][j] = gemm_frag(Bs, wn * 64 + j * 16 + fr, kk * 4 + fq);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[kk][i] = gemm_frag(As, wm * 128 + i * 16 + fr, kk * 4 + fq);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- epilogue: stage the wave's 128 x 64 tile (bf16) through LDS, then 16-byte row stores ----
  __bf16* ep = smem + wave * (128 * 64);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 16 + fr;  // column within the wave tile
    float bv = 0.f;
    if (bias != nullptr) bv = (float)bias[col0 + wn * 64 + c];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + fq * 4 + r;
        // row-major [128][64] image with the 16-byte chunk XOR-swizzled by row (conflict-free reads below)
        ep[row * 64 + (((c >> 3) ^ (row & 7)) << 3) + (c & 7)] = (__bf16)(acc[i][j][r] + bv);
      }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __bf16* Cw = C + (size_t)(row0 + wm * 128) * N + col0 + wn * 64;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 64 + lane;  // 128 rows x 8 chunks
    const int row = idx >> 3, ch = idx & 7;
    const s16x8 v = *reinterpret_cast<const s16x8*>(ep + row * 64 + ((ch ^ (row & 7)) << 3));
    *reinterpret_cast<s16x8*>(Cw + (size_t)row * N + ch * 8) = v;
  }
}


// Epilogue parameters of the QKV projection with the 3-axis rotary fused in (EPI 1): the GEMM writes
// q (rotated, pre-scaled), k, v (rotated) straight into the padded attention storage layout
// (B*H, Np, 64) instead of a (M, 3*H*64) tensor -- the separate rotary pass disappears.
struct RopeEpi {
  __bf16* q;
  __bf16* k;
  __bf16* v;
  const float* cosT;
  const float* sinT;
  int T, Tp, S, logS, n, Np, H, col_major;
  float qscale;
  // EPI 2 (GEGLU backward fused into the FF-out dgrad GEMM, see gemm_geglu_bwd): h = the FF-in
  // pre-activation [value | gate] (M, 2F), dh its gradient, part = per-128-row partial bias grads
  const __bf16* gh;
  __bf16* gdh;
  float* gpart;
  int F;
  // EPI 3 / 4 (weight gradients, MN-major operands): fp32 tile stored into slab blockIdx.y of fout
  // (3) or accumulated into fout (4)
  float* fout;
  // non-temporal epilogue output stores (former switch GEMM_NT_STORE=1): -5 % on the plain-store kernel at
  // the large shapes, no gain on the fused epilogues or the full step (profiles/r2_gemm_epilogue_cost.jsonl)
  int nt = 0;
  int drain = 0;  // s_waitcnt vmcnt(0) after the epilogue (gemm_pt.hip former switch GEMM_DRAIN)
  int cpol = 0;  // cache policy of the output stores (common.h cstore16; gemm_pt.hip former switch GEMM_CPOL)
  int stagger = 0, first_wave = 0;  // start-time stagger of the first wave (common.h stagger_start)
};

// 16-byte epilogue store, non-temporal when the launch asks for it (wave-uniform branch)
__device__ __forceinline__ void epi_store16(s16x8* dst, const s16x8& v, int nt) {
  if (nt) __builtin_nontemporal_store(v, dst);
  else *dst = v;
}

static int gemm_nt_store_default() { return 0; }

__device__ __forceinline__ int rope_epi_seq2st(const RopeEpi& e, int p) {
  if (p < e.T) return p;
  const int kk = p - e.T;
  const int kst = e.col_major ? ((kk & (e.S - 1)) << e.logS) + (kk >> e.logS) : kk;
  return e.Tp + kst;
}

// ------------------------------------------------------------------------------------------------
// Phase-pipelined variant (cdna_hip_programming.md, "256^2 8-phase template", re-derived here):
// each K-tile runs as 4 phases, one per 64 x 32 quadrant of the wave's 128 x 64 output (16 MFMAs
// each). The tile buffers are split into half-tiles (A rows 0-127 / 128-255, B rows 0-127 / 128-255:
// a wave only ever reads ITS A half and B half), and every phase issues the LDS-DMA of one half-tile
// of the NEXT K-tile into the other buffer, in consumption order (A0, B0, B1, A1). A counted
// vmcnt(4) before each phase's barrier keeps two half-tiles in flight across barriers while retiring
// exactly the half the next phase reads; a restaged half was last read >= 4 phases earlier (WAR).
//   phase 0: read A[q rows 0-63] + B[cols 0-31] -> MFMA quadrant (0,0)
//   phase 1: read B[cols 32-63]                 -> MFMA quadrant (0,1)
//   phase 2: read A[q rows 64-127]              -> MFMA quadrant (1,1)
//   phase 3: (registers only)                   -> MFMA quadrant (1,0)
// ------------------------------------------------------------------------------------------------
constexpr int HALF = 128 * GBK;  // elements of one half-tile image

// Half-tile image of 128 operand rows: the rows one PHASE reads across all 8 waves. For A (blk = 64)
// the "lo" half holds tile rows 0-63 and 128-191 (rows 0-63 of both wave rows), "hi" the other 128;
// for B (blk = 32) "lo" holds columns {0-31, 64-95, 128-159, 192-223} (the first 32 of each wave's
// 64), "hi" the rest. Image row hr <-> tile row (hr / blk) * 2 blk + off + hr % blk.
__device__ __forceinline__ void stage_half(const __bf16* __restrict__ src, int ld, int row0, int k0, __bf16* lds_half,
                                           int wave, int lane, int blk, int off) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;           // 0..15: image rows 8*piece .. 8*piece+7
    const int hr = piece * 8 + (lane >> 3);
    const int row = (hr / blk) * 2 * blk + off + (hr % blk);
    const int lchunk = (lane & 7) ^ gswz(hr);
    const __bf16* g = src + (size_t)(row0 + row) * ld + k0 + lchunk * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)(lds_half + piece * 512), 16, 0, 0);
  }
}

// ---- MN-major operands (weight gradients: dW[N, K] = G^T X with G (tokens, N), X (tokens, K) both
// row-major, the reduction running over tokens = the slow axis of both) ----
// A half-tile image is 64 tokens x 128 columns (256 B rows). Fragments are read with
// ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses token row q, columns 4p..4p+3 and
// receives its own column's 4 consecutive tokens, i.e. exactly an MFMA operand fragment (M / N index
// on the lane, tokens along K). The 16-byte chunk index is XOR-swizzled by token row so the 4 rows x
// 2 chunks of a 16-lane group, and the two groups of a half-wave (rows 8 apart), hit 16 distinct
// 16-byte bank groups.
__device__ __forceinline__ int mn_swz(int t) { return ((t & 3) << 1) | (((t >> 3) & 1) << 3); }

// In MN mode a half-tile is 128 CONTIGUOUS tile columns (off = 0 or 128: 256 B per token row), so
// the waves' output columns interleave accordingly (see the EPI 3 / 4 store): wave (wm, wn) owns
// rows {wm*64 + 0..63, 128 + wm*64 + 0..63} and columns {wn*32 + 0..31, 128 + wn*32 + 0..31}.
__device__ __forceinline__ void stage_half_mn(const __bf16* __restrict__ src, int ld, int col0, int t0, __bf16* lds_half,
                                              int wave, int lane, int off) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;           // 0..15: token rows 4*piece .. 4*piece+3
    const int tr = piece * 4 + (lane >> 4);   // this lane's token row in the image
    const int lchunk = (lane & 15) ^ mn_swz(tr);
    const __bf16* g = src + (size_t)(t0 + tr) * ld + col0 + off + lchunk * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)(lds_half + piece * 512), 16, 0, 0);
  }
}

typedef __attribute__((ext_vector_type(4))) short s16x4_t;

__device__ __forceinline__ bf16x8 frag_mn(const __bf16* img, int c_img, int kk, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int t1 = kk * 32 + g * 8 + q, t2 = t1 + 4;
  const int chunk = (c_img >> 3) + (p >> 1), sub = (p & 1) * 4;
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(img + t1 * 128 + ((chunk ^ mn_swz(t1)) << 3) + sub));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(img + t2 * 128 + ((chunk ^ mn_swz(t2)) << 3) + sub));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// Shared epilogue of the phased kernels: stage each wave's 128 x 64 accumulator tile (bf16) through
// LDS, then EPI 0 = 16-byte row stores (+bias), EPI 1 = rotary + scatter into the attention storage.
// All LDS operand reads and DMA must be retired by the caller (the whole 128 KiB is reused).
// (wm, wn) = the wave's 128 x 64 block of the tile; ep = its private 16 KB of LDS
template <int EPI>
__device__ __forceinline__ void gemm_store_epilogue_w(f32x4_t (&acc)[8][4], __bf16* ep, __bf16* __restrict__ C,
                                                      const __bf16* __restrict__ bias, int N, int row0, int col0, int wm,
                                                      int wn, int lane, const RopeEpi& rope) {
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (EPI == 5) {  // measurement only: main loop without the epilogue (results kept live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) t += acc[i][j][r];
    if (N < 0) C[lane] = (__bf16)t;
    return;
  }
  // EPI 2: all 32 [value | gate] pre-activation loads of a lane (16 rows x 2 halves) are issued before
  // any math instead of the 8 a partially unrolled loop keeps in flight (the epilogue does not overlap
  // this workgroup's MFMA work, so its HBM latency is exposed once per tile)
  s16x8 hv[2][8], hg[2][8];
  const int gcol = col0 + wn * 64 + (lane & 7) * 8;
  auto load_h = [&](int half) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const size_t r = (size_t)(row0 + wm * 128 + (half * 8 + k) * 8 + (lane >> 3));
      hv[half][k] = *reinterpret_cast<const s16x8*>(rope.gh + r * 2 * rope.F + gcol);
      hg[half][k] = *reinterpret_cast<const s16x8*>(rope.gh + r * 2 * rope.F + rope.F + gcol);
    }
  };
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = j * 16 + fr;
    float bv = 0.f;
    if (bias != nullptr) bv = (float)bias[col0 + wn * 64 + c];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + fq * 4 + r;
        ep[row * 64 + (((c >> 3) ^ (row & 7)) << 3) + (c & 7)] = (__bf16)(acc[i][j][r] + bv);
      }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (EPI == 0 || EPI == 6 || EPI == 7) {  // 6: measurement only, LDS staging without the global stores
    const __amdgpu_buffer_rsrc_t oc = uniform_rsrc(C);
    __bf16* Cw = C + (size_t)(row0 + wm * 128) * N + col0 + wn * 64;
    int t = 0;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, ch = idx & 7;
      const s16x8 v = *reinterpret_cast<const s16x8*>(ep + row * 64 + ((ch ^ (row & 7)) << 3));
      if (EPI == 0) {
        if (rope.cpol) cstore16(C, oc, (uint32_t)(((size_t)(row0 + wm * 128 + row) * N + col0 + wn * 64 + ch * 8) * 2),
                                __builtin_bit_cast(u32x4_vs, v), rope.cpol);
        else epi_store16(reinterpret_cast<s16x8*>(Cw + (size_t)row * N + ch * 8), v, rope.nt);
      } else if (EPI == 7) {  // non-temporal stores
        __builtin_nontemporal_store(v, reinterpret_cast<s16x8*>(Cw + (size_t)row * N + ch * 8));
      } else {
        t += v[0];
      }
    }
    if (EPI == 6 && N < 0) C[lane] = (__bf16)(float)t;
  } else if (EPI == 2) {
    // GEGLU backward: the staged tile is du = dy . W2 (bf16, as the unfused path rounds it) for F-columns
    // [c0, c0 + 64); each lane owns one 8-column chunk of 16 rows: da_value = du * gelu(gate),
    // da_gate = du * value * gelu'(gate) straight into dh, and the chunk's column sums of the propagated
    // (bf16) values -- the FF-in bias gradient -- reduced over the 8 lanes sharing it (fixed xor tree)
    // into one partial row per 128-row wave block.
    const int F = rope.F;
    const int c = gcol;
    const __amdgpu_buffer_rsrc_t od = uniform_rsrc(rope.gdh);
    float sv[8] = {}, sg[8] = {};
    load_h(0);
    load_h(1);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int row = it * 8 + (lane >> 3), ch = lane & 7;
      const size_t r = (size_t)(row0 + wm * 128 + row);
      float d[8], a[8], gg[8], da[8], dg[8];
      unpack8(*reinterpret_cast<const s16x8*>(ep + row * 64 + ((ch ^ (row & 7)) << 3)), d);
      unpack8(hv[it >> 3][it & 7], a);
      unpack8(hg[it >> 3][it & 7], gg);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float ge, gr;
        gelu_and_grad(gg[i], ge, gr);
        da[i] = d[i] * ge;
        dg[i] = d[i] * a[i] * gr;
      }
      const s16x8 pa = pack8(da), pg = pack8(dg);
      if (rope.cpol) {
        cstore16(rope.gdh, od, (uint32_t)((r * 2 * F + c) * 2), __builtin_bit_cast(u32x4_vs, pa), rope.cpol);
        cstore16(rope.gdh, od, (uint32_t)((r * 2 * F + F + c) * 2), __builtin_bit_cast(u32x4_vs, pg), rope.cpol);
      } else {
        epi_store16(reinterpret_cast<s16x8*>(rope.gdh + r * 2 * F + c), pa, rope.nt);
        epi_store16(reinterpret_cast<s16x8*>(rope.gdh + r * 2 * F + F + c), pg, rope.nt);
      }
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
      float* pr = rope.gpart + (size_t)((row0 >> 7) + wm) * 2 * F;
#pragma unroll
      for (int i = 0; i < 8; ++i) { pr[c + i] = sv[i]; pr[F + c + i] = sg[i]; }
    }
  } else {
    // the wave's 64 columns are exactly one (part, head): rotate each 8-column chunk of each row and
    // scatter the row to its storage slot
    const int HD = rope.H * 64;
    const int c0 = col0 + wn * 64;
    const int part = c0 / HD, h = (c0 - part * HD) >> 6;
    __bf16* dstT = part == 0 ? rope.q : (part == 1 ? rope.k : rope.v);
    const float sc = part == 0 ? rope.qscale : 1.0f;
    const __amdgpu_buffer_rsrc_t oq = uniform_rsrc(dstT);
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 64 + lane;
      const int row = idx >> 3, ch = idx & 7;
      const int r = row0 + wm * 128 + row;
      const int b = r / rope.n, p = r - b * rope.n;
      float x[8], cs[8], sn[8];
      unpack8(*reinterpret_cast<const s16x8*>(ep + row * 64 + ((ch ^ (row & 7)) << 3)), x);
      const float* cp = rope.cosT + (size_t)p * 64 + ch * 8;
      const float* sp = rope.sinT + (size_t)p * 64 + ch * 8;
      *reinterpret_cast<f32x4*>(cs) = *reinterpret_cast<const f32x4*>(cp);
      *reinterpret_cast<f32x4*>(cs + 4) = *reinterpret_cast<const f32x4*>(cp + 4);
      *reinterpret_cast<f32x4*>(sn) = *reinterpret_cast<const f32x4*>(sp);
      *reinterpret_cast<f32x4*>(sn + 4) = *reinterpret_cast<const f32x4*>(sp + 4);
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const float a0 = x[i], a1 = x[i + 1];
        x[i] = (a0 * cs[i] + a1 * sn[i]) * sc;
        x[i + 1] = (a1 * cs[i + 1] + a0 * sn[i + 1]) * sc;
      }
      const int srow = rope_epi_seq2st(rope, p);
      const size_t o = ((size_t)(b * rope.H + h) * rope.Np + srow) * 64 + ch * 8;
      if (rope.cpol) cstore16(dstT, oq, (uint32_t)(o * 2), __builtin_bit_cast(u32x4_vs, pack8(x)), rope.cpol);
      else epi_store16(reinterpret_cast<s16x8*>(dstT + o), pack8(x), rope.nt);
    }
  }
}

template <int EPI>
__device__ __forceinline__ void gemm_store_epilogue(f32x4_t (&acc)[8][4], __bf16* smem, __bf16* __restrict__ C,
                                                    const __bf16* __restrict__ bias, int N, int row0, int col0, int wave,
                                                    int lane, const RopeEpi& rope) {
  gemm_store_epilogue_w<EPI>(acc, smem + wave * (128 * 64), C, bias, N, row0, col0, wave >> 2, wave & 3, lane, rope);
}

template <int EPI, int OPT>
__global__ __launch_bounds__(G_THREADS, 1) void gemm_nt_phased_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                                      __bf16* __restrict__ C, const __bf16* __restrict__ bias,
                                                                      int M, int N, int K, RopeEpi rope) {
  // [buf][A0 | A1 | B0 | B1] half-tile images, 128 KiB in ONE array (a second __shared__ object can
  // make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 4 * HALF];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  gemm_tile_of(tm, tn, M / GBM, N / GBN);
  const int row0 = tm * GBM, col0 = tn * GBN;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // half-tile images per buffer, in consumption order: 0 A-lo (phase 0), 1 B-lo (phase 0),
  // 2 B-hi (phase 1), 3 A-hi (phase 2)
  auto slot = [&](int buf, int which) { return smem + (buf * 4 + which) * HALF; };
  auto stage = [&](int t, int p) {
    const int buf = t & 1, k0 = t * GBK;
    if (p == 0) stage_half(A, K, row0, k0, slot(buf, 0), wave, lane, 64, 0);
    else if (p == 1) stage_half(B, K, col0, k0, slot(buf, 1), wave, lane, 32, 0);
    else if (p == 2) stage_half(B, K, col0, k0, slot(buf, 2), wave, lane, 32, 32);
    else stage_half(A, K, row0, k0, slot(buf, 3), wave, lane, 64, 64);
  };

  const int nk = K / GBK;
  for (int p = 0; p < 4; ++p) stage(0, p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");

  bf16x8 a[4][2], b0[2][2], b1[2][2];  // [m-tile][kk], [n-tile][kk]
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const __bf16* Alo = slot(buf, 0);
    const __bf16* Blo = slot(buf, 1);
    const __bf16* Bhi = slot(buf, 2);
    const __bf16* Ahi = slot(buf, 3);
    const bool more = t + 1 < nk;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // 1) fragment reads of this phase (data retired one phase earlier)
      if (p == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0[j][kk] = gemm_frag(Blo, wn * 32 + j * 16 + fr, kk * 4 + fq);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a[i][kk] = gemm_frag(Alo, wm * 64 + i * 16 + fr, kk * 4 + fq);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1[j][kk] = gemm_frag(Bhi, wn * 32 + j * 16 + fr, kk * 4 + fq);
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a[i][kk] = gemm_frag(Ahi, wm * 64 + i * 16 + fr, kk * 4 + fq);
      }
      // 2) LDS-DMA of one half-tile of the next K-tile, then retire all but the two youngest halves
      if (more) {
        stage(t + 1, p);
        // phase 3 reads nothing from LDS, so phase 2 need not retire anything (OPT & 1)
        if (!((OPT & 1) && p == 2)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // a compiler-visible barrier: the builtin s_barrier does not order memory operations, and a
      // ds_read of the next phase hoisted above it would race with other waves' DMA retirement
      asm volatile("s_barrier" ::: "memory");
      // 3) the quadrant's 16 MFMAs
      if (!(OPT & 2)) __builtin_amdgcn_s_setprio(1);
      const int mi0 = (p >= 2) ? 4 : 0;
      const bool right = (p == 1 || p == 2);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x4_t& c = acc[mi0 + i][(right ? 2 : 0) + j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], right ? b1[j][kk] : b0[j][kk], c, 0, 0, 0);
          }
      if (!(OPT & 2)) __builtin_amdgcn_s_setprio(0);
      if (OPT & 4) asm volatile("s_barrier" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  gemm_store_epilogue<EPI>(acc, smem, C, bias, N, row0, col0, wave, lane, rope);
}

// ------------------------------------------------------------------------------------------------
// 8-phase template (cdna_hip_programming.md §5 "The 256^2 8-phase template", T3+T4+T5), re-derived:
// the same 256x256x64 tile, half-tile images and quadrant order as gemm_nt_phased_kernel, but
//   * each phase is {ds_read subtile ; 1 half-tile LDS-DMA ; s_barrier ; lgkmcnt(0) ; 16 MFMA ;
//     s_barrier} and the two wave rows run STAGGERED by one barrier (wm == 1 enters one barrier
//     late), so on every SIMD one wave issues MFMAs while its partner reads LDS / issues DMA;
//   * three half-tiles stay in flight: the counted vmcnt(6) runs once per K-tile (phase 4), never 0
//     in the steady state. Staging order per K-tile t (consumption order is A-lo B-lo | B-hi | A-hi):
//       phase 1: A-hi(t+1) -> buf^1   (A-hi of buf^1 last read 2 phases ago)
//       phase 2: B-lo(t+2) -> buf     (B-lo read in phase 1, retired by its lgkmcnt(8) before phase 1's
//                                      first barrier, so 1 phase later is safe for both wave rows)
//       phase 3: A-lo(t+2) -> buf     (read in phase 1, 2 phases ago)
//       phase 4: B-hi(t+2) -> buf     (read in phase 2, 2 phases ago); then vmcnt(6) retires A-hi(t+1),
//                                      the last half of K-tile t+1, before phase 4's first barrier
//     so K-tile t+1 is complete for every wave before any wave's phase-5 reads (RAW), even for the
//     lagging wave row.
// ------------------------------------------------------------------------------------------------
// MN = 1: MN-major operands (see stage_half_mn): A = G (tokens, M), B = X (tokens, N), K = tokens per
// split; blockIdx.y selects the split (tokens [y K, (y + 1) K)).
template <int EPI, int OPT, int MN = 0>
__global__ __launch_bounds__(G_THREADS, 1) void gemm_nt_8ph_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                                   __bf16* __restrict__ C, const __bf16* __restrict__ bias,
                                                                   int M, int N, int K, RopeEpi rope, int group) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 4 * HALF];  // [buf][A-lo | B-lo | B-hi | A-hi]
  stagger_start(rope.stagger, rope.first_wave);
  constexpr bool STAGGER = !(OPT & 1);
  if (MN) {
    A += (size_t)blockIdx.y * K * M;
    B += (size_t)blockIdx.y * K * N;
  }
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  gemm_tile_of(tm, tn, M / GBM, N / GBN, group);
  const int row0 = tm * GBM, col0 = tn * GBN;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto slot = [&](int buf, int which) { return smem + (buf * 4 + which) * HALF; };
  // which: 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi
  auto stage = [&](int t, int which) {
    const int buf = t & 1, k0 = t * GBK;
    if constexpr (MN) {
      if (which == 0) stage_half_mn(A, M, row0, k0, slot(buf, 0), wave, lane, 0);
      else if (which == 1) stage_half_mn(B, N, col0, k0, slot(buf, 1), wave, lane, 0);
      else if (which == 2) stage_half_mn(B, N, col0, k0, slot(buf, 2), wave, lane, 128);
      else stage_half_mn(A, M, row0, k0, slot(buf, 3), wave, lane, 128);
    } else {
      if (which == 0) stage_half(A, K, row0, k0, slot(buf, 0), wave, lane, 64, 0);
      else if (which == 1) stage_half(B, K, col0, k0, slot(buf, 1), wave, lane, 32, 0);
      else if (which == 2) stage_half(B, K, col0, k0, slot(buf, 2), wave, lane, 32, 32);
      else stage_half(A, K, row0, k0, slot(buf, 3), wave, lane, 64, 64);
    }
  };
  // operand fragment: image rows (NT) / image columns (MN) r0 .. r0+15, k-half kk
  auto frag = [&](const __bf16* img, int r0, int kk) {
    if constexpr (MN) return frag_mn(img, r0, kk, lane);
    else return gemm_frag(img, r0 + fr, kk * 4 + fq);
  };

  const int nk = K / GBK;
  stage(0, 1); stage(0, 0); stage(0, 2); stage(0, 3);
  if (nk > 1) {
    stage(1, 1); stage(1, 0); stage(1, 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_barrier" ::: "memory");
  if (STAGGER && wm == 1) asm volatile("s_barrier" ::: "memory");

  bf16x8 a[4][2], b0[2][2], b1[2][2];  // [m-tile][kk], [n-tile][kk]
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const __bf16* Alo = slot(buf, 0);
    const __bf16* Blo = slot(buf, 1);
    const __bf16* Bhi = slot(buf, 2);
    const __bf16* Ahi = slot(buf, 3);
    const bool s1 = t + 1 < nk, s2 = t + 2 < nk;

    // ---- phase 1: B-lo then A-lo -> quadrant (lo, lo)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b0[j][kk] = frag(Blo, wn * 32 + j * 16, kk);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) a[i][kk] = frag(Alo, wm * 64 + i * 16, kk);
    if (s1) stage(t + 1, 3);
    // the B reads (issued first: 4 fragments, 8 tr-reads in MN mode) have retired
    if constexpr (MN) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b0[j][kk], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");

    // ---- phase 2: B-hi -> quadrant (lo, hi)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b1[j][kk] = frag(Bhi, wn * 32 + j * 16, kk);
    if (s2) stage(t + 2, 1);
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
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b1[j][kk], acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");

    // ---- phase 3: A-hi -> quadrant (hi, hi)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) a[i][kk] = frag(Ahi, wm * 64 + i * 16, kk);
    if (s2) stage(t + 2, 0);
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
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b1[j][kk], acc[4 + i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");

    // ---- phase 4: registers only -> quadrant (hi, lo); retire K-tile t+1
    if (s2) {
      stage(t + 2, 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b0[j][kk], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");
  }
  if (STAGGER && wm == 0) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (EPI == 3 || EPI == 4) {
    // fp32 tile straight from the accumulators: 16 lanes store 16 consecutive floats of a row
    float* Cf = rope.fout + (EPI == 3 ? (size_t)blockIdx.y * M * N : 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = (i < 4 ? wm * 64 + i * 16 : 128 + wm * 64 + (i - 4) * 16) + fq * 4 + r;
          const int cc = (j < 2 ? wn * 32 + j * 16 : 128 + wn * 32 + (j - 2) * 16) + fr;
          float* dst = Cf + (size_t)(row0 + rr) * N + col0 + cc;
          if (EPI == 3) *dst = acc[i][j][r];
          else *dst += acc[i][j][r];
        }
  } else {
    gemm_store_epilogue<EPI>(acc, smem, C, bias, N, row0, col0, wave, lane, rope);
  }
  if (rope.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// zero the storage rows that have no sequence position (text padding [T, Tp) and the last image slot)
__global__ void rope_pad_zero_kernel(__bf16* q, __bf16* k, __bf16* v, int Tp, int T, int Np, int BH) {
  const int bh = blockIdx.x, t = threadIdx.x;  // 256 threads: (pad row, 8-chunk)
  const int npad = Tp - T + 1;
  const int pr = t >> 3, ch = t & 7;
  if (pr >= npad) return;
  const int srow = pr < Tp - T ? T + pr : Np - 1;
  const size_t off = ((size_t)bh * Np + srow) * 64 + ch * 8;
  const s16x8 z = {};
  *reinterpret_cast<s16x8*>(q + off) = z;
  *reinterpret_cast<s16x8*>(k + off) = z;
  *reinterpret_cast<s16x8*>(v + off) = z;
}

void rope_pad_zero(void* q, void* k, void* v, int Tp, int T, int Np, int BH, hipStream_t st) {
  hipLaunchKernelGGL(rope_pad_zero_kernel, dim3(BH), dim3(256), 0, st, (__bf16*)q, (__bf16*)k, (__bf16*)v, Tp, T, Np, BH);
}

int gemm_stagger_ticks(int ntiles, int K);
int gemm_cpol();
int gemm_drain();
bool gemm_nt(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int epi, hipStream_t st) {
  if (M % GBM || N % GBN || K % GBK) return false;
  const int nwg = (M / GBM) * (N / GBN);
  switch (epi) {
    case 0:
      hipLaunchKernelGGL((gemm_nt_kernel<0, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                         (__bf16*)C, (const __bf16*)bias, M, N, K);
      return true;
#define PHASED_CASE(o)                                                                                          \
  case 200 + o:                                                                                                \
    hipLaunchKernelGGL((gemm_nt_phased_kernel<0, o>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A,      \
                       (const __bf16*)B, (__bf16*)C, (const __bf16*)bias, M, N, K, RopeEpi{});                  \
    return true;
    PHASED_CASE(0) PHASED_CASE(1) PHASED_CASE(2) PHASED_CASE(3) PHASED_CASE(4) PHASED_CASE(5) PHASED_CASE(6) PHASED_CASE(7)
#undef PHASED_CASE
    case 100:
      hipLaunchKernelGGL((gemm_nt_kernel<0, 1>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                         (__bf16*)C, (const __bf16*)bias, M, N, K);
      return true;
    default:
      // 8-phase template; variant 3xx picks the tile order: 300 -> column groups of 4, 301..332 ->
      // column groups of (variant - 300), 400 + g -> row groups of g
      if (epi >= 300 && epi < 333) {
        const int group = epi == 300 ? 4 : epi - 300;
        RopeEpi e{};
        e.cpol = (size_t)M * N * 2 < (1ull << 32) ? gemm_cpol() : 0;  // buffer stores: 32-bit byte offsets
        e.drain = gemm_drain();
        hipLaunchKernelGGL((gemm_nt_8ph_kernel<0, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                           (__bf16*)C, (const __bf16*)bias, M, N, K, e, group);
        return true;
      }
      if (epi == 390) {  // measurement: the 8-phase kernel with the first-wave start stagger
        RopeEpi e{};
        e.stagger = gemm_stagger_ticks(nwg, K);
        e.first_wave = 256;
        hipLaunchKernelGGL((gemm_nt_8ph_kernel<0, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                           (__bf16*)C, (const __bf16*)bias, M, N, K, e, 4);
        return true;
      }
      if (epi == 350 || epi == 360 || epi == 370) {  // measurement: no epilogue / staging only / nt stores
        if (epi == 370)
          hipLaunchKernelGGL((gemm_nt_8ph_kernel<7, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                             (__bf16*)C, (const __bf16*)bias, M, N, K, RopeEpi{}, 4);
        else if (epi == 350)
          hipLaunchKernelGGL((gemm_nt_8ph_kernel<5, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                             (__bf16*)C, (const __bf16*)bias, M, N, K, RopeEpi{}, 4);
        else
          hipLaunchKernelGGL((gemm_nt_8ph_kernel<6, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                             (__bf16*)C, (const __bf16*)bias, M, N, K, RopeEpi{}, 4);
        return true;
      }
      if (epi > 400 && epi < 433) {
        hipLaunchKernelGGL((gemm_nt_8ph_kernel<0, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)B,
                           (__bf16*)C, (const __bf16*)bias, M, N, K, RopeEpi{}, -(epi - 400));
        return true;
      }
      return false;
  }
}


// ------------------------------------------------------------------------------------------------
// Two co-resident workgroups per CU (round 4; first built and measured in round 2 for plain stores,
// profiles/r2_gemm_2wg_variant.hip.txt). A workgroup is 4 waves (2 x 2, each the 8-phase kernel's 128 x 64
// output block) on a 256 x 128 tile, K-step 32, operands through a 3-slot LDS ring (24 KB per slot, 72 KB
// per workgroup), so two workgroups fit on a CU (<= 256 VGPRs at 2 waves per SIMD, 144 KB of LDS) and one's
// epilogue runs beside the other's MFMAs. Its simple main loop is ~25 % slower than the 8-phase one on plain
// products (hence rejected there), but the GEGLU-backward epilogue (512 KB of HBM traffic per 256 x 256 of
// output, serialised after the main loop in the one-workgroup-per-CU kernels) is what this structure hides.
// LDS image: rows of 32 bf16 (64 B, 4 chunks of 16 B); physical chunk = logical ^ g((row >> 2) & 3),
// g = {0, 2, 3, 1}: conflict-free for the ds_read_b128 lane groups of a 16-row fragment read.
// ------------------------------------------------------------------------------------------------
constexpr int W2_BM = 256, W2_BN = 128, W2_BK = 32;
constexpr int W2_SLOT = (W2_BM + W2_BN) * W2_BK;  // elements per ring slot (A rows, then B rows)

__device__ __forceinline__ int w2_swz(int r) {
  const int q = (r >> 2) & 3;
  return (0x1320 >> (4 * q)) & 3;  // g = {0, 2, 3, 1}
}

// one K-step of A (256 rows) and B (128 rows) into a ring slot: 24 pieces of 16 rows x 64 B, 6 per wave
__device__ __forceinline__ void w2_stage(const __bf16* __restrict__ A, const __bf16* __restrict__ B, int K, int row0,
                                         int col0, int k0, __bf16* slot, int wave, int lane) {
  const int pr = lane >> 2, pc = lane & 3;  // row within the piece, physical chunk
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int piece = wave * 6 + i;  // 0..15: A rows 16 piece.., 16..23: B rows 16 (piece - 16)..
    const int r = piece * 16 + pr;   // image row (A rows 0-255, then B rows 256-383)
    const int lc = pc ^ w2_swz(r);
    const __bf16* g = piece < 16 ? A + (size_t)(row0 + r) * K + k0 + lc * 8
                                 : B + (size_t)(col0 + r - W2_BM) * K + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)(slot + piece * 512), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 w2_frag(const __bf16* slot, int r, int fq) {
  return *reinterpret_cast<const bf16x8*>(slot + r * W2_BK + ((fq ^ w2_swz(r)) << 3));
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_2wg_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                             __bf16* __restrict__ C, const __bf16* __restrict__ bias, int M,
                                                             int N, int K, RopeEpi rope, int group) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[3 * W2_SLOT];  // 72 KB, one array (see the 8-phase kernel)
  // the two co-resident workgroups of a CU start in phase and would stay there (equal tiles), so their
  // epilogues would coincide: first_wave < 0 delays the second slot's first workgroups ([-fw, -2 fw)) by
  // `stagger` ticks; first_wave > 0 is the 4-phase start of stagger_start
  if (rope.stagger > 0) {
    if (rope.first_wave < 0) {
      const int w0 = -rope.first_wave;
      if ((int)blockIdx.x >= w0 && (int)blockIdx.x < 2 * w0) {
        const unsigned long long until = __builtin_amdgcn_s_memrealtime() + (unsigned long long)rope.stagger;
        while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(4);
      }
    } else {
      stagger_start(rope.stagger, rope.first_wave);
    }
  }
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  gemm_tile_of(tm, tn, M / W2_BM, N / W2_BN, group);
  const int row0 = tm * W2_BM, col0 = tn * W2_BN;
  const int fq = lane >> 4, fr = lane & 15;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / W2_BK;
  w2_stage(A, B, K, row0, col0, 0, smem, wave, lane);
  if (nk > 1) w2_stage(A, B, K, row0, col0, W2_BK, smem + W2_SLOT, wave, lane);
  int slot = 0;  // ring slot of K-step t
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (t + 2 < nk) {
      const int s2 = slot == 0 ? 2 : slot - 1;  // (t + 2) % 3 = the slot read at t - 1
      w2_stage(A, B, K, row0, col0, (t + 2) * W2_BK, smem + s2 * W2_SLOT, wave, lane);
    }
    const __bf16* S = smem + slot * W2_SLOT;
    bf16x8 a[8], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = w2_frag(S, W2_BM + wn * 64 + j * 16 + fr, fq);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = w2_frag(S, wm * 128 + i * 16 + fr, fq);
    // first half of the MFMAs as soon as B and the first four A fragments are in (the other four
    // A reads land under them)
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 4; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    slot = slot == 2 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  gemm_store_epilogue_w<EPI>(acc, smem + wave * (128 * 64), C, bias, N, row0, col0, wm, wn, lane, rope);
  if (rope.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// former switch GEGLU_BWD_2WG=1: the FF-out dgrad + GEGLU backward on the two-workgroup kernel (gemm_set_geglu_bwd_2wg)
static int g_geglu_bwd_2wg = 0;
void gemm_set_geglu_bwd_2wg(int v) { g_geglu_bwd_2wg = v; }
// former switch 2WG_STAGGER=<ticks>[,<first_wave>] (10 ns ticks; first_wave < 0: delay the second slot's first
// workgroups, > 0: the 4-phase stagger_start over the first first_wave workgroups)
static int g_2wg_stagger[2] = {0, -256};
static void w2_stagger(RopeEpi& e) {
  e.stagger = g_2wg_stagger[0];
  e.first_wave = g_2wg_stagger[1];
}
void gemm_set_2wg_stagger(int ticks, int first_wave) {
  g_2wg_stagger[0] = ticks;
  g_2wg_stagger[1] = first_wave;
}

// plain C = A B^T on the two-workgroup kernel (tests / benchmarks)
bool gemm_2wg(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, hipStream_t st) {
  if (M % W2_BM || N % W2_BN || K % W2_BK || K < 2 * W2_BK) return false;
  RopeEpi e{};
  w2_stagger(e);
  const int nwg = (M / W2_BM) * (N / W2_BN);
  hipLaunchKernelGGL((gemm_nt_2wg_kernel<0>), dim3(nwg), dim3(256), 0, st, (const __bf16*)A, (const __bf16*)B, (__bf16*)C,
                     (const __bf16*)bias, M, N, K, e, 4);
  return true;
}

// FF-out dgrad with the GEGLU backward in the epilogue: du = dy (M, K) . W2^T where w2t = W2^T (F, K)
// bf16, then dh (M, 2F) = GEGLU'(h, du) and part ((M / 128), 2F) = partial FF-in bias grads. The
// (M, F) du intermediate never exists.
int gemm_stagger_ticks(int ntiles, int K);
int gemm_cpol();
int gemm_drain();
bool gemm_geglu_bwd(const void* dy, const void* w2t, const void* h, void* dh, float* part, int M, int F, int K,
                    hipStream_t st, int stagger) {
  if (M % GBM || F % GBN || K % GBK) return false;
  RopeEpi e{};
  e.nt = gemm_nt_store_default();
  e.stagger = stagger < 0 ? gemm_stagger_ticks((M / GBM) * (F / GBN), K) : stagger;
  e.first_wave = 256;
  e.gh = (const __bf16*)h;
  e.gdh = (__bf16*)dh;
  e.gpart = part;
  e.F = F;
  e.cpol = (size_t)M * F * 4 < (1ull << 32) ? gemm_cpol() : 0;  // buffer stores: 32-bit byte offsets
  e.drain = gemm_drain();
  if (g_geglu_bwd_2wg && F % W2_BN == 0 && K % W2_BK == 0 && K >= 2 * W2_BK) {
    const int nwg2 = (M / W2_BM) * (F / W2_BN);
    w2_stagger(e);
    hipLaunchKernelGGL((gemm_nt_2wg_kernel<2>), dim3(nwg2), dim3(256), 0, st, (const __bf16*)dy, (const __bf16*)w2t,
                       (__bf16*)nullptr, (const __bf16*)nullptr, M, F, K, e, 4);
    return true;
  }
  const int nwg = (M / GBM) * (F / GBN);
  hipLaunchKernelGGL((gemm_nt_8ph_kernel<2, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)dy, (const __bf16*)w2t,
                     (__bf16*)nullptr, (const __bf16*)nullptr, M, F, K, e, 4);
  return true;
}

// QKV projection + rotary into the attention storage layout (q pre-scaled); M = B*n rows
bool gemm_qkv_rope(const void* A, const void* W, void* q, void* k, void* v, const float* cosT, const float* sinT, int M, int K,
                   int H, int T, int S, int n, int col_major, float qscale, hipStream_t st) {
  const int N = 3 * H * 64;
  if (M % GBM || N % GBN || K % GBK || M % n) return false;
  int logS = 0;
  while ((1 << logS) < S) ++logS;
  const int Tp = (T + 31) / 32 * 32;
  RopeEpi e{(__bf16*)q, (__bf16*)k, (__bf16*)v, cosT, sinT, T, Tp, S, logS, n, Tp + S * S, H, col_major, qscale};
  e.nt = gemm_nt_store_default();
  e.cpol = (size_t)M * N * 4 < (1ull << 32) ? gemm_cpol() : 0;  // buffer stores: 32-bit byte offsets
  e.drain = gemm_drain();
  const int nwg = (M / GBM) * (N / GBN);
  // 8-phase staggered template: 1073 vs 1042 TF for the phased kernel at M=61440, N=3072, K=1024
  // (profiles/r1_gemm_8phase.jsonl)
  hipLaunchKernelGGL((gemm_nt_8ph_kernel<1, 0>), dim3(nwg), dim3(G_THREADS), 0, st, (const __bf16*)A, (const __bf16*)W,
                     (__bf16*)nullptr, (const __bf16*)nullptr, M, N, K, e, 4);
  const int BH = (M / n) * H;
  hipLaunchKernelGGL(rope_pad_zero_kernel, dim3(BH), dim3(256), 0, st, (__bf16*)q, (__bf16*)k, (__bf16*)v, Tp, T, Tp + S * S, BH);
  return true;
}

}  // namespace dalle

