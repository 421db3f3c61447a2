// Launch geometry structs shared by the HIP kernels and the (host-compiled) bindings.
#pragma once
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
// Destination of a column-reduced parameter gradient (see column_sum_kernel)
struct GradSink {
  float* out0;        // columns [0, split)
  float* out1;        // columns [split, width) (nullptr: dropped)
  const float* mul1;  // optional per-column multiplier for out1
  int split;
  int accumulate;     // 1: dst += v (the fp32 grad arena), 0: dst = v
};
}  // namespace dalle
