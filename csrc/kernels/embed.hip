// Token embedding of the tied DALL-E table (SURVEY K1 + K2; reference: dalle_pytorch DALLE.forward
// text remap / BOS / SharedEmbedding, task.py:82).
//
// Forward (one workgroup per sequence position, 16-byte row copies):
//   position 0          -> id 0 (BOS)
//   positions 1..Ttxt   -> text id; a 0 becomes the unique per-position pad id pad_base + (p - 1)
//   positions Ttxt+1..  -> Vt + image code
// The rows are gathered from the fp32 head weight straight into the fp32 residual stream, and the
// token ids are written out for the backward. An id outside the table is clamped and flagged.
//
// Backward: the gradient of every table row is the sum of the rows of d(tokens) that gathered it.
// Deterministic without float atomics: the ids are sorted (stable), runs of equal ids are split into
// chunks of at most EMB_CHUNK rows; pass 1 sums each chunk in sorted order into a partial row, pass 2
// adds a run's partials, again in order, into the (arena) gradient of the table row. A long run (the
// eos/pad id of short captions) is spread over many workgroups instead of serialising in one.
#include "common.h"

namespace dalle {

constexpr int EMB_THREADS = 256;
constexpr int EMB_CHUNK = 64;

__global__ __launch_bounds__(EMB_THREADS) void embed_fwd_kernel(const int64_t* __restrict__ text, const int64_t* __restrict__ image,
                                                                const float* __restrict__ table, float* __restrict__ out,
                                                                int* __restrict__ ids, int* __restrict__ bad, int n, int Ttxt,
                                                                int Timg, int d, int pad_base, int Vt, int V) {
  const int row = blockIdx.x;
  const int b = row / n, p = row - b * n;
  long id;
  if (p == 0) {
    id = 0;
  } else if (p <= Ttxt) {
    const long t = text[(size_t)b * Ttxt + p - 1];
    id = t == 0 ? (long)pad_base + p - 1 : t;
  } else {
    id = (long)Vt + image[(size_t)b * Timg + (p - Ttxt - 1)];
  }
  if (id < 0 || id >= V) {
    if (threadIdx.x == 0) atomicOr(bad, 1);
    id = id < 0 ? 0 : V - 1;
  }
  if (threadIdx.x == 0) ids[row] = (int)id;
  const f32x4* src = reinterpret_cast<const f32x4*>(table + (size_t)id * d);
  f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)row * d);
  for (int c = threadIdx.x; c < d / 4; c += EMB_THREADS) dst[c] = src[c];
}

// pass 1: sorted position r starts a chunk iff (r - head[r]) % EMB_CHUNK == 0 (head = first sorted
// position of r's run); the chunk's rows are summed in sorted order into partial[r]
__global__ __launch_bounds__(EMB_THREADS) void embed_bwd_chunk_kernel(const float* __restrict__ dout, const int* __restrict__ order,
                                                                      const int* __restrict__ head, float* __restrict__ partial,
                                                                      int N, int d) {
  const int r = blockIdx.x;
  const int h = head[r];
  if ((r - h) % EMB_CHUNK != 0) return;
  for (int c = threadIdx.x; c < d / 4; c += EMB_THREADS) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = r; i < N && i < r + EMB_CHUNK && head[i] == h; ++i) {
      const f32x4 v = reinterpret_cast<const f32x4*>(dout + (size_t)order[i] * d)[c];
      acc += v;
    }
    reinterpret_cast<f32x4*>(partial + (size_t)r * d)[c] = acc;
  }
}

// pass 2: the run starting at sorted position r adds its chunk partials (in order) into grad[id]
__global__ __launch_bounds__(EMB_THREADS) void embed_bwd_run_kernel(const float* __restrict__ partial, const int* __restrict__ sorted_ids,
                                                                    const int* __restrict__ head, float* __restrict__ grad, int N,
                                                                    int d) {
  const int r = blockIdx.x;
  if (head[r] != r) return;
  const int id = sorted_ids[r];
  for (int c = threadIdx.x; c < d / 4; c += EMB_THREADS) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = r; i < N && head[i] == r; i += EMB_CHUNK) acc += reinterpret_cast<const f32x4*>(partial + (size_t)i * d)[c];
    f32x4* g = reinterpret_cast<f32x4*>(grad + (size_t)id * d) + c;
    *g = *g + acc;
  }
}

void embed_fwd(const int64_t* text, const int64_t* image, const float* table, float* out, int* ids, int* bad, int B, int n,
               int Ttxt, int Timg, int d, int pad_base, int Vt, int V, hipStream_t st) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(B * n), dim3(EMB_THREADS), 0, st, text, image, table, out, ids, bad, n, Ttxt, Timg,
                     d, pad_base, Vt, V);
}

void embed_bwd(const float* dout, const int* order, const int* sorted_ids, const int* head, float* partial, float* grad, int N,
               int d, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_chunk_kernel, dim3(N), dim3(EMB_THREADS), 0, st, dout, order, head, partial, N, d);
  hipLaunchKernelGGL(embed_bwd_run_kernel, dim3(N), dim3(EMB_THREADS), 0, st, partial, sorted_ids, head, grad, N, d);
}

}  // namespace dalle
