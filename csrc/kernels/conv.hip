// VQGAN decoder on CDNA4 (reference: taming-transformers Decoder, run by
// inference/run_inference.py:122-123 through VQGanVAE.decode). Activations are NHWC bf16.
//
// * conv3x3_kernel: 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on MFMA
//     Y[p, co] = sum_{tap, ci} X'[shift_tap(p), ci] * W[co, tap, ci]   (+ bias, + residual)
//   M = pixels, N = Cout, K = 9 * Cin. Workgroup tile 128 pixels x 128 channels, K-step 64 (one tap,
//   64 input channels), 4 waves of 64 x 64 (4 x 4 v_mfma_f32_16x16x32_bf16 per 32-deep half step).
//   The A tile is GATHERED: each row is the 128-byte channel slice of the tap-shifted pixel (zero
//   outside the image), and the ResNet block's GroupNorm + SiLU is applied to it in registers on its
//   way to LDS (per-channel scale / shift of this image from an LDS table), so the normalised
//   activation never exists in memory. The 2x nearest upsampling in front of the Upsample conv is
//   folded into the same gather (source pixel = shifted pixel / 2). Register-staged double buffer
//   (next K-step's global loads in flight during the MFMAs), XOR-swizzled LDS rows, bf16 epilogue
//   through LDS with the bias and the ResNet residual added on the way out.
// * gn_stats: GroupNorm (32 groups) mean / rstd per (image, group): per-workgroup partial sums over a
//   pixel range, reduced in a fixed order in double (deterministic).
// * gn_apply: GroupNorm without activation into bf16 (the attention block's input).
// * conv_out_kernel: the final GroupNorm + SiLU + 3x3 conv to 3 channels (VALU; N = 3 is far too
//   narrow for MFMA tiles; 16 x 16 output tiles over an LDS halo of activations computed once per pixel)
//   fused with clamp(-1, 1) -> (x + 1) / 2 and the NCHW fp32 image store.
// * softmax_rows: row softmax of the attention block's scores (fp32 in, bf16 probabilities out).
#include "common.h"
#include "geom.h"

namespace dalle {

constexpr int CV_BM = 128, CV_BN = 128, CV_BK = 64, CV_THREADS = 256;
constexpr int GN_GROUPS = 32;


__device__ __forceinline__ int cv_idx(int row, int col) { return row * 64 + ((((col >> 3) ^ (row & 7)) << 3) | (col & 7)); }

__device__ __forceinline__ float silu(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * LOG2E)); }

__global__ __launch_bounds__(CV_THREADS, 2) void conv3x3_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * CV_BM * CV_BK];  // [buf][A | B], 64 KiB
  __shared__ float gsc[1024], gsh[1024];                                      // GN scale / shift per channel
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const __bf16* __restrict__ X = (const __bf16*)a.x;
  const __bf16* __restrict__ Wt = (const __bf16*)a.w;
  const __bf16* __restrict__ Res = (const __bf16*)a.res;
  __bf16* __restrict__ Y = (__bf16*)a.y;
  const int HW = a.H * a.W;
  const int tiles_n = a.Cout / CV_BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int m0 = tm * CV_BM, n0 = tn * CV_BN;
  const int img = m0 / HW;  // a tile never spans two images (HW % 128 == 0)
  if (a.gn) {
    for (int c = tid; c < a.Cin; c += CV_THREADS) {
      const int g = c / (a.Cin / GN_GROUPS);
      const float sc = a.rstd[img * GN_GROUPS + g] * a.gamma[c];
      gsc[c] = sc;
      gsh[c] = a.beta[c] - a.mean[img * GN_GROUPS + g] * sc;
    }
  }
  // this thread's 4 gathered rows (pixels) and the chunk (8 channels) it moves
  const int lrow = tid >> 3, lch = tid & 7;
  int py[4], px[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rem = m0 + lrow + 32 * i - img * HW;
    py[i] = rem / a.W;
    px[i] = rem - py[i] * a.W;
  }
  const int Hs = a.ups ? a.H >> 1 : a.H, Ws = a.ups ? a.W >> 1 : a.W;
  const int cchunks = a.Cin / CV_BK;
  const int nk = 9 * cchunks;
  s16x8 ra[4], rb[4];
  bool va[4];
  auto load = [&](int s) {
    const int tap = s / cchunks, c0 = (s - tap * cchunks) * CV_BK;
    const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int yy = py[i] + dy, xx = px[i] + dx;
      va[i] = yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      if (a.ups) { yy >>= 1; xx >>= 1; }
      const size_t off = (((size_t)img * Hs + (va[i] ? yy : 0)) * Ws + (va[i] ? xx : 0)) * a.Cin + c0 + lch * 8;
      ra[i] = *reinterpret_cast<const s16x8*>(X + off);
      rb[i] = *reinterpret_cast<const s16x8*>(Wt + (size_t)(n0 + lrow + 32 * i) * (9 * a.Cin) + tap * a.Cin + c0 + lch * 8);
    }
  };
  auto store = [&](int s, int buf) {
    const int c0 = (s - (s / cchunks) * cchunks) * CV_BK + lch * 8;
    __bf16* As = smem + buf * (2 * CV_BM * CV_BK);
    __bf16* Bs = As + CV_BM * CV_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = lrow + 32 * i;
      s16x8 v = ra[i];
      if (a.gn) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = silu(fmaf(f[j], gsc[c0 + j], gsh[c0 + j]));
        v = pack8(f);
      }
      if (!va[i]) v = s16x8{};  // zero padding of the (normalised) conv input
      *reinterpret_cast<s16x8*>(As + cv_idx(row, lch * 8)) = v;
      *reinterpret_cast<s16x8*>(Bs + cv_idx(row, lch * 8)) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // GN table
  load(0);
  store(0, 0);
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load(s + 1);
    const __bf16* As = smem + buf * (2 * CV_BM * CV_BK);
    const __bf16* Bs = As + CV_BM * CV_BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(As + cv_idx(wm * 64 + i * 16 + fr, (kk * 4 + fq) * 8));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(Bs + cv_idx(wn * 64 + j * 16 + fr, (kk * 4 + fq) * 8));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nk) store(s + 1, buf ^ 1);
    __syncthreads();
  }

  // epilogue: the 128 x 128 tile as bf16 through LDS (rows of 256 B, 16-byte chunks swizzled by row),
  // then 16-byte stores of whole channel runs with bias + residual
  __bf16* ep = smem;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = wn * 64 + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + fq * 4 + r;
        ep[row * 128 + ((((c >> 3) ^ (row & 15)) << 3) | (c & 7))] = (__bf16)acc[i][j][r];
      }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * CV_THREADS + tid;  // 128 rows x 16 chunks
    const int row = idx >> 4, ch = idx & 15;
    float f[8];
    unpack8(*reinterpret_cast<const s16x8*>(ep + row * 128 + ((ch ^ (row & 15)) << 3)), f);
    const int co = n0 + ch * 8;
    if (a.bias != nullptr) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(a.bias + co), b1 = *reinterpret_cast<const f32x4*>(a.bias + co + 4);
      f[0] += b0[0]; f[1] += b0[1]; f[2] += b0[2]; f[3] += b0[3];
      f[4] += b1[0]; f[5] += b1[1]; f[6] += b1[2]; f[7] += b1[3];
    }
    const size_t o = (size_t)(m0 + row) * a.Cout + co;
    if (Res != nullptr) {
      float r8[8];
      unpack8(*reinterpret_cast<const s16x8*>(Res + o), r8);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += r8[j];
    }
    *reinterpret_cast<s16x8*>(Y + o) = pack8(f);
  }
}

// ---------------------------------------------------------------------------------------------
// GroupNorm statistics: grid (N, GN_CHUNKS); thread t owns channel chunk t % (C / 8) (8 channels) of
// every (256 / (C / 8))-th pixel of the workgroup's pixel range and keeps per-CHANNEL partial sums;
// the workgroup then folds them into per-group partials (any channels-per-group that divides C).
constexpr int GN_CHUNKS = 64;

__global__ __launch_bounds__(256) void gn_partial_kernel(const __bf16* __restrict__ x, float* __restrict__ part, int HW, int C) {
  __shared__ float red[256 * 16];
  const int n = blockIdx.x, chunk = blockIdx.y, tid = threadIdx.x;
  const int cpr = C / 8;        // 16-byte chunks per pixel (<= 256)
  const int ppass = 256 / cpr;  // pixels per pass
  const int cc = tid % cpr, pr = tid / cpr;
  const int per = (HW + GN_CHUNKS - 1) / GN_CHUNKS;
  const int p0 = chunk * per, p1 = min(HW, p0 + per);
  float s[8] = {}, q[8] = {};
  if (pr < ppass) {
    for (int p = p0 + pr; p < p1; p += ppass) {
      float f[8];
      unpack8(*reinterpret_cast<const s16x8*>(x + ((size_t)n * HW + p) * C + cc * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += f[j]; q[j] += f[j] * f[j]; }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid * 16 + j] = s[j]; red[tid * 16 + 8 + j] = q[j]; }
  __syncthreads();
  if (tid < GN_GROUPS) {
    const int g = tid, cg = C / GN_GROUPS;
    double S = 0.0, Q = 0.0;
    for (int r = 0; r < ppass; ++r)
      for (int c = g * cg; c < (g + 1) * cg; ++c) {
        const int t = r * cpr + (c >> 3);
        S += red[t * 16 + (c & 7)];
        Q += red[t * 16 + 8 + (c & 7)];
      }
    part[(((size_t)n * GN_CHUNKS + chunk) * GN_GROUPS + g) * 2] = (float)S;
    part[(((size_t)n * GN_CHUNKS + chunk) * GN_GROUPS + g) * 2 + 1] = (float)Q;
  }
}

__global__ void gn_finalize_kernel(const float* __restrict__ part, float* __restrict__ mean, float* __restrict__ rstd, int N,
                                   int HW, int C, float eps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (n, g)
  if (i >= N * GN_GROUPS) return;
  const int n = i / GN_GROUPS, g = i - n * GN_GROUPS;
  double S = 0.0, Q = 0.0;
  for (int c = 0; c < GN_CHUNKS; ++c) {
    S += part[(((size_t)n * GN_CHUNKS + c) * GN_GROUPS + g) * 2];
    Q += part[(((size_t)n * GN_CHUNKS + c) * GN_GROUPS + g) * 2 + 1];
  }
  const double cnt = (double)HW * (C / GN_GROUPS);
  const double mu = S / cnt;
  double var = Q / cnt - mu * mu;
  var = var > 0.0 ? var : 0.0;
  mean[i] = (float)mu;
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

// y = GN(x) (affine, no activation), bf16 NHWC
__global__ __launch_bounds__(256) void gn_apply_kernel(const __bf16* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, __bf16* __restrict__ y, long total8, int HW,
                                                       int C, int act) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total8) return;
  const int cpr = C / 8;
  const long pix = i / cpr;
  const int c0 = (int)(i - pix * cpr) * 8;
  const int n = (int)(pix / HW);
  float f[8];
  unpack8(*reinterpret_cast<const s16x8*>(x + i * 8), f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j, g = c / (C / GN_GROUPS);
    f[j] = (f[j] - mean[n * GN_GROUPS + g]) * rstd[n * GN_GROUPS + g] * gamma[c] + beta[c];
    if (act) f[j] = silu(f[j]);
  }
  *reinterpret_cast<s16x8*>(y + i * 8) = pack8(f);
}

// final GN + SiLU + 3x3 conv (Cin -> 3) + clamp / rescale -> NCHW fp32 image. One workgroup per 16 x 16 output
// tile: the activations SiLU(GN(x)) of the 18 x 18 input halo are computed ONCE per pixel into LDS (fp32, 32
// channels at a time; zero outside the image: the conv pads its post-SiLU input) and every thread accumulates
// its pixel's 9 taps x 32 channels x 3 outputs from there, the weights (fp32) and the image's GN scale / shift
// also in LDS. (The former one-thread-per-pixel form recomputed every activation for each of the 9 taps and
// gathered a 256-B pixel row per lane per tap: 9.3 ms at batch 64, 256 x 256, 128 channels.)
constexpr int CO_T = 16, CO_CC = 32, CO_HALO = CO_T + 2, CO_LD = CO_CC + 4;
__global__ __launch_bounds__(256) void conv_out_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float* __restrict__ img, int H, int W,
                                                       int C) {
  __shared__ __attribute__((aligned(16))) float wl[3 * 9 * 128];
  __shared__ float sc[128], sh[128];
  __shared__ __attribute__((aligned(16))) float act[CO_HALO * CO_HALO * CO_LD];  // 46.7 KB
  const int n = blockIdx.z, tid = threadIdx.x;
  const int ty0 = blockIdx.y * CO_T, tx0 = blockIdx.x * CO_T;
  for (int i = tid; i < 27 * C; i += 256) wl[i] = (float)w[i];
  for (int c = tid; c < C; c += 256) {
    const int g = c / (C / GN_GROUPS);
    sc[c] = rstd[n * GN_GROUPS + g] * gamma[c];
    sh[c] = beta[c] - mean[n * GN_GROUPS + g] * sc[c];
  }
  const int ty = tid >> 4, tx = tid & 15;
  float o0 = bias[0], o1 = bias[1], o2 = bias[2], p0 = 0.f, p1 = 0.f, p2 = 0.f;
  for (int c0 = 0; c0 < C; c0 += CO_CC) {
    __syncthreads();  // the tables are written / the previous chunk's activations are consumed
    for (int e = tid; e < CO_HALO * CO_HALO * (CO_CC / 8); e += 256) {
      const int pix = e >> 2, part = e & 3;
      const int hy = pix / CO_HALO, hx = pix - hy * CO_HALO;
      const int sy = ty0 + hy - 1, sx = tx0 + hx - 1;
      float v[8];
      if (sy >= 0 && sy < H && sx >= 0 && sx < W) {
        float f[8];
        unpack8(*reinterpret_cast<const s16x8*>(x + (((size_t)n * H + sy) * W + sx) * C + c0 + part * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = c0 + part * 8 + j;
          v[j] = silu(fmaf(f[j], sc[c], sh[c]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
      float* d = act + pix * CO_LD + part * 8;
      *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(d + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    __syncthreads();
#pragma unroll 3
    for (int tap = 0; tap < 9; ++tap) {
      const float* a = act + ((ty + tap / 3) * CO_HALO + tx + tap % 3) * CO_LD;
      const float* w0 = wl + (0 * 9 + tap) * C + c0;
      const float* w1 = wl + (1 * 9 + tap) * C + c0;
      const float* w2 = wl + (2 * 9 + tap) * C + c0;
#pragma unroll
      for (int c = 0; c < CO_CC; c += 4) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(a + c);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(w0 + c);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(w1 + c);
        const f32x4 b2 = *reinterpret_cast<const f32x4*>(w2 + c);
#pragma unroll
        for (int q = 0; q < 4; q += 2) {  // two accumulator sets: six independent FMA chains
          o0 = fmaf(av[q], b0[q], o0);
          o1 = fmaf(av[q], b1[q], o1);
          o2 = fmaf(av[q], b2[q], o2);
          p0 = fmaf(av[q + 1], b0[q + 1], p0);
          p1 = fmaf(av[q + 1], b1[q + 1], p1);
          p2 = fmaf(av[q + 1], b2[q + 1], p2);
        }
      }
    }
  }
  o0 += p0;
  o1 += p1;
  o2 += p2;
  const int yy = ty0 + ty, xx = tx0 + tx;
  if (yy >= H || xx >= W) return;
  const size_t plane = (size_t)H * W;
  float* out = img + (size_t)n * 3 * plane + (size_t)yy * W + xx;
  out[0] = (fminf(fmaxf(o0, -1.f), 1.f) + 1.f) * 0.5f;
  out[plane] = (fminf(fmaxf(o1, -1.f), 1.f) + 1.f) * 0.5f;
  out[2 * plane] = (fminf(fmaxf(o2, -1.f), 1.f) + 1.f) * 0.5f;
}

// row softmax: s (R, L) fp32 * scale -> p bf16. One workgroup per row.
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ s, __bf16* __restrict__ p, int L, float scale) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const float* sr = s + row * L;
  float m = NEG_BIG;
  for (int i = threadIdx.x; i < L; i += 256) m = fmaxf(m, sr[i] * scale);
  m = wave_max(m);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float z = 0.f;
  for (int i = threadIdx.x; i < L; i += 256) z += __builtin_amdgcn_exp2f((sr[i] * scale - m) * LOG2E);
  z = wave_sum(z);
  __syncthreads();
  if (l == 0) red[4 + w] = z;
  __syncthreads();
  const float inv = 1.0f / (red[4] + red[5] + red[6] + red[7]);
  for (int i = threadIdx.x; i < L; i += 256) p[row * L + i] = (__bf16)(__builtin_amdgcn_exp2f((sr[i] * scale - m) * LOG2E) * inv);
}

bool conv3x3(const ConvArgs& a, hipStream_t st) {
  if (a.Cin % CV_BK || a.Cout % CV_BN || (a.H * a.W) % CV_BM || a.Cin > 1024) return false;
  if (a.ups && ((a.H & 1) || (a.W & 1))) return false;
  const int tiles = (a.N * a.H * a.W / CV_BM) * (a.Cout / CV_BN);
  hipLaunchKernelGGL(conv3x3_kernel, dim3(tiles), dim3(CV_THREADS), 0, st, a);
  return true;
}

bool gn_stats(const void* x, float* part, float* mean, float* rstd, int N, int HW, int C, float eps, hipStream_t st) {
  if (C % GN_GROUPS || C % 8 || C / 8 > 256) return false;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(N, GN_CHUNKS), dim3(256), 0, st, (const __bf16*)x, part, HW, C);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((N * GN_GROUPS + 255) / 256), dim3(256), 0, st, part, mean, rstd, N, HW, C, eps);
  return true;
}

size_t gn_part_floats(int N) { return (size_t)N * GN_CHUNKS * GN_GROUPS * 2; }

void gn_apply(const void* x, const float* mean, const float* rstd, const float* gamma, const float* beta, void* y, int N, int HW,
              int C, hipStream_t st, int act) {
  const long total8 = (long)N * HW * C / 8;
  hipLaunchKernelGGL(gn_apply_kernel, dim3((total8 + 255) / 256), dim3(256), 0, st, (const __bf16*)x, mean, rstd, gamma, beta,
                     (__bf16*)y, total8, HW, C, act);
}

bool conv_out(const void* x, const void* w, const float* bias, const float* mean, const float* rstd, const float* gamma,
              const float* beta, float* img, int N, int H, int W, int C, hipStream_t st) {
  if (C > 128 || C % CO_CC) return false;  // C % 32: the GroupNorm's 32 groups and whole 32-channel chunks
  hipLaunchKernelGGL(conv_out_kernel, dim3((W + CO_T - 1) / CO_T, (H + CO_T - 1) / CO_T, N), dim3(256), 0, st, (const __bf16*)x,
                     (const __bf16*)w, bias, mean, rstd, gamma, beta, img, H, W, C);
  return true;
}

void softmax_rows(const float* s, void* p, long R, int L, float scale, hipStream_t st) {
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(R), dim3(256), 0, st, s, (__bf16*)p, L, scale);
}

}  // namespace dalle
