// Uniform 8-bit quantisation for collaborative averaging (reference: hivemind's
// Uniform8BitQuantization, chosen at task.py:125-126 for tensors >= 2^16+1 elements):
//   mean, std -> scale = 6 std / 256 -> q = clamp(rint((x - mean) / scale) + 128, 0, 255)
//   codebook[b] = mean of the original values that fell into bin b; dequant = codebook[q].
//
// Passes (all bandwidth-bound; one launch each, no host sync):
//   1. block partials of sum(x) (fp64) and max|x|       -> finalize: mean, maxabs, fixed-point shift
//   2. block partials of sum((x - mean)^2) (fp64)        -> finalize: scale
//   3. quantise + per-block bin histograms in LDS        -> finalize: codebook
// The bin sums use INT64 fixed point (value * 2^shift, shift chosen from max|x| and n so the total
// cannot overflow): integer addition is associative, so the LDS atomics and the cross-block sums
// give bit-identical codebooks on every run and every peer -- float atomics would not.
#include "common.h"

namespace dalle {

constexpr int Q_THREADS = 256;
constexpr int Q_BLOCKS = 1024;  // partial rows (grid-stride over the tensor)

__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < Q_THREADS / 64; ++i) t += red[i];
  __syncthreads();
  return t;  // valid on thread 0
}

__global__ __launch_bounds__(Q_THREADS) void uq8_sum_kernel(const float* __restrict__ x, long n, double* __restrict__ part,
                                                            float* __restrict__ pmax) {
  __shared__ double red[Q_THREADS / 64];
  __shared__ float redm[Q_THREADS / 64];
  double s = 0.0;
  float m = 0.f;
  for (long i = (long)blockIdx.x * Q_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * Q_THREADS) {
    const float v = x[i];
    s += v;
    m = fmaxf(m, fabsf(v));
  }
  const double t = block_sum_d(s, red);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) redm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = 0.f;
    for (int i = 0; i < Q_THREADS / 64; ++i) mm = fmaxf(mm, redm[i]);
    part[blockIdx.x] = t;
    pmax[blockIdx.x] = mm;
  }
}

__global__ __launch_bounds__(Q_THREADS) void uq8_var_kernel(const float* __restrict__ x, long n, const double* __restrict__ stats,
                                                            double* __restrict__ part) {
  __shared__ double red[Q_THREADS / 64];
  const double mean = stats[0];
  double s = 0.0;
  for (long i = (long)blockIdx.x * Q_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * Q_THREADS) {
    const double d = (double)x[i] - mean;
    s += d * d;
  }
  const double t = block_sum_d(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// stats layout (double): [0] mean, [1] scale, [2] 2^shift, [3] max|x|
__global__ void uq8_finalize_mean_kernel(const double* __restrict__ part, const float* __restrict__ pmax, int nb, long n,
                                         double* __restrict__ stats) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  float m = 0.f;
  for (int i = 0; i < nb; ++i) { s += part[i]; m = fmaxf(m, pmax[i]); }  // fixed order
  stats[0] = s / (double)n;
  stats[3] = m;
  // fixed-point shift: n * (max|x| * 2^shift) < 2^62
  const double lim = 4.611686018427388e18 / ((double)n * ((double)m + 1e-30));
  int sh = (int)floor(log2(lim));
  sh = sh > 60 ? 60 : (sh < -60 ? -60 : sh);
  stats[2] = ldexp(1.0, sh);
}

__global__ void uq8_finalize_scale_kernel(const double* __restrict__ part, int nb, long n, double* __restrict__ stats) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) s += part[i];
  const double stdv = sqrt(s / (double)(n > 1 ? n - 1 : 1));
  double scale = 6.0 * stdv / 256.0;
  stats[1] = scale > 1e-30 ? scale : 1e-30;
}

__global__ __launch_bounds__(Q_THREADS) void uq8_quantize_kernel(const float* __restrict__ x, long n,
                                                                 const double* __restrict__ stats, uint8_t* __restrict__ q,
                                                                 long long* __restrict__ psum, unsigned* __restrict__ pcnt) {
  __shared__ long long hs[256];
  __shared__ unsigned hc[256];
  hs[threadIdx.x] = 0;
  hc[threadIdx.x] = 0;
  __syncthreads();
  const float mean = (float)stats[0];
  const float inv = (float)(1.0 / stats[1]);
  const double fx = stats[2];
  for (long i = (long)blockIdx.x * Q_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * Q_THREADS) {
    const float v = x[i];
    float r = rintf((v - mean) * inv) + 128.f;
    r = fminf(fmaxf(r, 0.f), 255.f);
    const int b = (int)r;
    q[i] = (uint8_t)b;
    atomicAdd(reinterpret_cast<unsigned long long*>(&hs[b]), (unsigned long long)llrint((double)v * fx));
    atomicAdd(&hc[b], 1u);
  }
  __syncthreads();
  psum[(size_t)blockIdx.x * 256 + threadIdx.x] = hs[threadIdx.x];
  pcnt[(size_t)blockIdx.x * 256 + threadIdx.x] = hc[threadIdx.x];
}

__global__ void uq8_codebook_kernel(const long long* __restrict__ psum, const unsigned* __restrict__ pcnt, int nb,
                                    const double* __restrict__ stats, float* __restrict__ codebook) {
  const int b = threadIdx.x;  // 256 threads
  long long s = 0;
  unsigned long long c = 0;
  for (int i = 0; i < nb; ++i) { s += psum[(size_t)i * 256 + b]; c += pcnt[(size_t)i * 256 + b]; }
  codebook[b] = c ? (float)((double)s / stats[2] / (double)c) : 0.f;
}

// out [+]= weight * codebook[q]
__global__ void uq8_dequant_kernel(const uint8_t* __restrict__ q, const float* __restrict__ codebook, float* __restrict__ out,
                                   long n, float weight, int accumulate) {
  __shared__ float cb[256];
  cb[threadIdx.x] = codebook[threadIdx.x];
  __syncthreads();
  for (long i = (long)blockIdx.x * Q_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * Q_THREADS) {
    const float v = weight * cb[q[i]];
    out[i] = accumulate ? out[i] + v : v;
  }
}

// ---------------------------------------------------------------------------------------------
// Segmented form (the butterfly's per-tensor parts, hivemind compresses every part of every tensor
// separately): ONE launch quantises all parts, one workgroup per part. A part is at most a few
// hundred KB, so its three passes (sum/max, variance, quantise + histogram) re-read it from L2;
// the codebook is written by the same workgroup. Same fixed-point bin sums as above, so the result
// is deterministic and identical on every peer.
//   part s: x[x_off[s] : x_off[s] + len[s]]  ->  q[q_off[s] : q_off[s] + len[s]], codebook[256 s : 256 s + 256]
__global__ __launch_bounds__(Q_THREADS) void uq8_seg_compress_kernel(const float* __restrict__ x, const long* __restrict__ x_off,
                                                                     const long* __restrict__ q_off, const int* __restrict__ len,
                                                                     uint8_t* __restrict__ q, float* __restrict__ codebook) {
  __shared__ double red[Q_THREADS / 64];
  __shared__ float redm[Q_THREADS / 64];
  __shared__ double bc[3];  // mean, 1/scale, 2^shift
  __shared__ long long hs[256];
  __shared__ unsigned hc[256];
  const int s = blockIdx.x;
  const float* __restrict__ xs = x + x_off[s];
  uint8_t* __restrict__ qs = q + q_off[s];
  const int n = len[s];
  double sum = 0.0;
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += Q_THREADS) {
    const float v = xs[i];
    sum += v;
    m = fmaxf(m, fabsf(v));
  }
  const double t = block_sum_d(sum, red);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) redm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = 0.f;
    for (int i = 0; i < Q_THREADS / 64; ++i) mm = fmaxf(mm, redm[i]);
    bc[0] = t / (double)(n > 0 ? n : 1);
    const double lim = 4.611686018427388e18 / ((double)(n > 0 ? n : 1) * ((double)mm + 1e-30));
    int sh = (int)floor(log2(lim));
    sh = sh > 60 ? 60 : (sh < -60 ? -60 : sh);
    bc[2] = ldexp(1.0, sh);
  }
  hs[threadIdx.x] = 0;
  hc[threadIdx.x] = 0;
  __syncthreads();
  const double mean = bc[0];
  double v2 = 0.0;
  for (int i = threadIdx.x; i < n; i += Q_THREADS) {
    const double d = (double)xs[i] - mean;
    v2 += d * d;
  }
  const double t2 = block_sum_d(v2, red);
  if (threadIdx.x == 0) {
    const double stdv = sqrt(t2 / (double)(n > 1 ? n - 1 : 1));
    double scale = 6.0 * stdv / 256.0;
    bc[1] = 1.0 / (scale > 1e-30 ? scale : 1e-30);
  }
  __syncthreads();
  const float meanf = (float)mean;
  const float inv = (float)bc[1];
  const double fx = bc[2];
  for (int i = threadIdx.x; i < n; i += Q_THREADS) {
    const float v = xs[i];
    float r = rintf((v - meanf) * inv) + 128.f;
    r = fminf(fmaxf(r, 0.f), 255.f);
    const int b = (int)r;
    qs[i] = (uint8_t)b;
    atomicAdd(reinterpret_cast<unsigned long long*>(&hs[b]), (unsigned long long)llrint((double)v * fx));
    atomicAdd(&hc[b], 1u);
  }
  __syncthreads();
  const unsigned c = hc[threadIdx.x];
  codebook[(size_t)s * 256 + threadIdx.x] = c ? (float)((double)hs[threadIdx.x] / fx / (double)c) : 0.f;
}

// out[out_off[s] + i] [+]= weight * codebook[256 s + q[q_off[s] + i]]
__global__ __launch_bounds__(Q_THREADS) void uq8_seg_dequant_kernel(const uint8_t* __restrict__ q, const long* __restrict__ q_off,
                                                                    const float* __restrict__ codebook,
                                                                    const long* __restrict__ out_off, const int* __restrict__ len,
                                                                    float* __restrict__ out, float weight, int accumulate) {
  __shared__ float cb[256];
  const int s = blockIdx.x;
  cb[threadIdx.x] = codebook[(size_t)s * 256 + threadIdx.x];
  __syncthreads();
  const uint8_t* __restrict__ qs = q + q_off[s];
  float* __restrict__ os = out + out_off[s];
  const int n = len[s];
  for (int i = threadIdx.x; i < n; i += Q_THREADS) {
    const float v = weight * cb[qs[i]];
    os[i] = accumulate ? os[i] + v : v;
  }
}

void uq8_seg_compress(const float* x, const long* x_off, const long* q_off, const int* len, int nseg, uint8_t* q,
                      float* codebook, hipStream_t st) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(uq8_seg_compress_kernel, dim3(nseg), dim3(Q_THREADS), 0, st, x, x_off, q_off, len, q, codebook);
}

void uq8_seg_dequant(const uint8_t* q, const long* q_off, const float* codebook, const long* out_off, const int* len, int nseg,
                     float* out, float weight, int accumulate, hipStream_t st) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(uq8_seg_dequant_kernel, dim3(nseg), dim3(Q_THREADS), 0, st, q, q_off, codebook, out_off, len, out, weight,
                     accumulate);
}

void uq8_compress(const float* x, long n, uint8_t* q, float* codebook, void* ws, hipStream_t st) {
  // ws: [Q_BLOCKS doubles | Q_BLOCKS floats | 4 doubles | Q_BLOCKS*256 int64 | Q_BLOCKS*256 uint32]
  double* part = reinterpret_cast<double*>(ws);
  float* pmax = reinterpret_cast<float*>(part + Q_BLOCKS);
  double* stats = reinterpret_cast<double*>(pmax + Q_BLOCKS);
  long long* psum = reinterpret_cast<long long*>(stats + 4);
  unsigned* pcnt = reinterpret_cast<unsigned*>(psum + (size_t)Q_BLOCKS * 256);
  long blocks = (n + Q_THREADS - 1) / Q_THREADS;
  const int nb = (int)(blocks < Q_BLOCKS ? (blocks > 0 ? blocks : 1) : Q_BLOCKS);
  hipLaunchKernelGGL(uq8_sum_kernel, dim3(nb), dim3(Q_THREADS), 0, st, x, n, part, pmax);
  hipLaunchKernelGGL(uq8_finalize_mean_kernel, dim3(1), dim3(64), 0, st, part, pmax, nb, n, stats);
  hipLaunchKernelGGL(uq8_var_kernel, dim3(nb), dim3(Q_THREADS), 0, st, x, n, stats, part);
  hipLaunchKernelGGL(uq8_finalize_scale_kernel, dim3(1), dim3(64), 0, st, part, nb, n, stats);
  hipLaunchKernelGGL(uq8_quantize_kernel, dim3(nb), dim3(Q_THREADS), 0, st, x, n, stats, q, psum, pcnt);
  hipLaunchKernelGGL(uq8_codebook_kernel, dim3(1), dim3(256), 0, st, psum, pcnt, nb, stats, codebook);
}

size_t uq8_workspace_bytes() {
  return Q_BLOCKS * sizeof(double) + Q_BLOCKS * sizeof(float) + 4 * sizeof(double) +
         (size_t)Q_BLOCKS * 256 * (sizeof(long long) + sizeof(unsigned));
}

void uq8_dequant(const uint8_t* q, const float* codebook, float* out, long n, float weight, int accumulate, hipStream_t st) {
  long blocks = (n + Q_THREADS - 1) / Q_THREADS;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(uq8_dequant_kernel, dim3(blocks), dim3(Q_THREADS), 0, st, q, codebook, out, n, weight, accumulate);
}

}  // namespace dalle
