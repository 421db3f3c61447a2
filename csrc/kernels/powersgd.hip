// PowerSGD rank-r gradient compression helpers (BASELINE config 3).
//
// The two skinny products P = M Q and Q = M^T P stay on hipBLASLt; this file holds the two pieces
// that are not GEMMs:
//   * psgd_orthonormalize: modified Gram-Schmidt on the columns of EVERY P factor of a step in one
//     launch (one workgroup per matrix; P is row-major n x r, r <= 8). Replaces one rocSOLVER QR
//     launch chain per matrix. Columns whose norm collapses are zeroed (their rank-1 term vanishes),
//     never divided by ~0.
//   * psgd_reconstruct: the rank-r outer product fused with the error-feedback update,
//       A = P Q^T;   grad = A;   E = M_e - A     (E holds M_e on entry)
//     one pass over the n x m matrix (read E, write E and grad) instead of materialising A.
#include "common.h"

namespace dalle {

constexpr int PSGD_MAX_R = 8;
constexpr int PSGD_THREADS = 256;

// one workgroup per matrix: rows [row_off[b], row_off[b] + rows[b]) of the flat P buffer
__global__ __launch_bounds__(PSGD_THREADS) void psgd_orthonormalize_kernel(float* __restrict__ P, const long* __restrict__ off,
                                                                          const int* __restrict__ rows, int r, float eps) {
  __shared__ float red[8];
  const int b = blockIdx.x;
  float* M = P + off[b];
  const int n = rows[b];
  for (int j = 0; j < r; ++j) {
    // subtract the projections on the already-orthonormal columns 0..j-1 (modified Gram-Schmidt)
    for (int k = 0; k < j; ++k) {
      float d = 0.f;
      for (int i = threadIdx.x; i < n; i += PSGD_THREADS) d += M[(long)i * r + j] * M[(long)i * r + k];
      d = block_sum_256(d, red);
      for (int i = threadIdx.x; i < n; i += PSGD_THREADS) M[(long)i * r + j] -= d * M[(long)i * r + k];
      __syncthreads();
    }
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += PSGD_THREADS) {
      const float v = M[(long)i * r + j];
      s += v * v;
    }
    s = block_sum_256(s, red);
    const float inv = s > eps * eps ? rsqrtf(s) : 0.f;
    for (int i = threadIdx.x; i < n; i += PSGD_THREADS) M[(long)i * r + j] *= inv;
    __syncthreads();
  }
}

// grad (n x m, fp32) = P Q^T; E -= P Q^T. Each thread: 4 consecutive columns of one row.
template <int R>
__global__ __launch_bounds__(PSGD_THREADS) void psgd_reconstruct_kernel(float* __restrict__ grad, float* __restrict__ E,
                                                                       const float* __restrict__ P, const float* __restrict__ Q,
                                                                       long n, int m) {
  const int per_row = m >> 2;
  const long gid = (long)blockIdx.x * PSGD_THREADS + threadIdx.x;
  if (gid >= n * per_row) return;
  const long i = gid / per_row;
  const int j0 = (int)(gid - i * per_row) * 4;
  float p[R];
#pragma unroll
  for (int t = 0; t < R; ++t) p[t] = P[i * R + t];
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float* q = Q + (long)(j0 + c) * R;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < R; ++t) s += p[t] * q[t];
    a[c] = s;
  }
  const long idx = i * m + j0;
  f32x4 e = *reinterpret_cast<const f32x4*>(E + idx);
  *reinterpret_cast<f32x4*>(grad + idx) = a;
  *reinterpret_cast<f32x4*>(E + idx) = e - a;
}

void psgd_orthonormalize(float* P, const long* off, const int* rows, int nmat, int r, float eps, hipStream_t st) {
  hipLaunchKernelGGL(psgd_orthonormalize_kernel, dim3(nmat), dim3(PSGD_THREADS), 0, st, P, off, rows, r, eps);
}

bool psgd_reconstruct(float* grad, float* E, const float* P, const float* Q, long n, int m, int r, hipStream_t st) {
  if (m % 4) return false;
  const long t = n * (m / 4);
  const dim3 grid((unsigned)((t + PSGD_THREADS - 1) / PSGD_THREADS));
  switch (r) {
#define PSGD_CASE(R)                                                                                                    \
  case R:                                                                                                               \
    hipLaunchKernelGGL(psgd_reconstruct_kernel<R>, grid, dim3(PSGD_THREADS), 0, st, grad, E, P, Q, n, m);               \
    return true;
    PSGD_CASE(1) PSGD_CASE(2) PSGD_CASE(4) PSGD_CASE(8)
#undef PSGD_CASE
    default:
      return false;
  }
}

}  // namespace dalle
