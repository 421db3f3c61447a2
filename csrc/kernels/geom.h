// Launch geometry structs shared by the HIP kernels and the (host-compiled) bindings.
#pragma once
#include <stdint.h>
namespace dalle {
struct AttnGeom {
  int T;        // text positions incl. BOS (257)
  int Tp;       // padded text rows (288)
  int S;        // image side (32)
  int logS;     // log2(S)
  int I;        // S*S
  int Np;       // Tp + I
  int n;        // unpadded sequence length (1280)
  int K;        // conv window
  int H;        // heads
  int pattern;  // 0 full, 1 axial_row, 2 axial_col, 3 conv_like
};
struct RopeGeom {
  int T, Tp, S, logS, n, Np, H, col_major;
};
struct DecodeGeom {
  int T;        // text positions incl. BOS
  int S;        // image side
  int n;        // cache length (seq_len)
  int H;        // heads
  int K;        // conv window
  int pattern;  // 0 full, 1 axial_row, 2 axial_col, 3 conv_like
};
struct ShiftGeom {
  int n;      // sequence length
  int T;      // text_len (BOS + text)
  int S;      // image side
  int shift;  // 0 = plain LayerNorm
};
// VQGAN decoder 3x3 convolution (conv.hip): bf16 tensors passed as void pointers (host-compiled header)
struct ConvArgs {
  const void* x;       // [N, Hs, Ws, Cin] NHWC (Hs = H / 2 when ups)
  const void* w;       // [Cout, 9 * Cin] tap-major, channel-contiguous
  const float* bias;   // [Cout] or nullptr
  const void* res;     // [N, H, W, Cout] or nullptr
  void* y;             // [N, H, W, Cout]
  const float* mean;   // [N, 32] GroupNorm statistics (gn)
  const float* rstd;   // [N, 32]
  const float* gamma;  // [Cin]
  const float* beta;   // [Cin]
  int N, H, W, Cin, Cout, ups, gn;
};

// Destination of a column-reduced parameter gradient (see column_sum_kernel)
struct GradSink {
  float* out0;        // columns [0, split)
  float* out1;        // columns [split, width) (nullptr: dropped)
  const float* mul1;  // optional per-column multiplier for out1
  int split;
  int accumulate;     // 1: dst += v (the fp32 grad arena), 0: dst = v
};

// Decode-step skinny GEMM (skinny.hip): Y (M <= 64, N) = X (M, K) . W (N, K)^T + fused epilogue.
// bf16 operands are passed as void pointers (this header is also compiled by the host compiler).
struct SkinnyArgs {
  const void* X;
  const void* W;
  const void* bias;  // bf16, may be null
  int M, N, K, ldx;  // N: output columns (F for GEGLU: W holds 2F rows)
  int KS;            // cross-workgroup split-K factor (must equal skinny_ks(M, N, K, G))
  int steps;         // 128-wide K chunks per wave (set by skinny_gemm)
  float* ws;         // KS * (N / 16) * ceil16(M) * 16 * (1 or 2) floats
  int* cnt;          // >= N / 16 zero-initialised counters (self-resetting)
  void* out;         // EPI 0 (bf16 or fp32), EPI 1 (bf16)
  int out_f32;
  float* resid;        // EPI 2: resid += scale * (y + bias), fp32 (M, N)
  const float* scale;
  void* q;           // EPI 3: rotary q (pre-scaled) -> q (M*H, 64); k, v -> caches (M*H, n, 64) at *pos
  void* kc;
  void* vc;
  const float* cosT;
  const float* sinT;
  const int* pos;
  int H, n;
  float qscale;
  int dbg;  // benchmark-only: bit 0 skips the X loads, bit 1 the W loads
  // EPI 5 (split-K slabs + LayerNorm tail): the slabs (a.out) are stored write-through, every workgroup
  // takes a ticket on *cnt, and the last M arrivers each finish one row: resid += scale * (sum + bias),
  // then the decode LayerNorm + cached token shift of that row (ln_w / ln_b, LN history `hist` (M, n, N)
  // bf16 at *pos, shifted row to `y` (M, N) bf16); T / S: text length / image side, shift: 0 = plain LN
  const float* ln_w;
  const float* ln_b;
  void* hist;
  void* y;
  int T, S, shift;
  unsigned* err;  // set to 1 if a tail's wait for the other workgroups gave up (bounded spin)
};

// Fused decode sampler (sample.hip): top-k / top-p / temperature / Gumbel-max + token bookkeeping.
struct SampleArgs {
  const float* logits;  // (B, V) fp32
  int B, V;
  int top_k;            // <= 0 or >= V: off
  float top_p;          // >= 1: off
  float temperature;    // <= 1e-10: greedy
  const int64_t* seed;  // device scalar
  const int* pos;       // device scalar: the position this step ran
  const int64_t* text;  // (B, T) caption ids (BOS first)
  int T, img_len;
  int64_t vt;           // text vocabulary size (image token id offset)
  int64_t* codes;       // (B, img_len), may be null
  int64_t* tok;         // (B,) next input token, may be null
  int64_t* sampled;     // (B,) the raw sample, may be null
};

}  // namespace dalle
