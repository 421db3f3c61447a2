// Fused decode-step sampler: top-k + nucleus (top-p) filtering, temperature, Gumbel-max
// sampling and the device-side token bookkeeping of the hipGraph decode step, in ONE launch -- it
// replaces ~20 small library kernels per position (radix top-k, sort, softmax, cumsum, rand, log,
// argmax, scatter/gather/where). Semantics follow dalle_amd.models.generation.filter_logits:
//   * top-k: keep logits >= the k-th largest (ties kept);
//   * top-p on the softmax of the kept logits, sorted descending: keep while the EXCLUSIVE cumulative
//     probability <= p (the token that crosses p stays);
//   * sample argmax(l / T - log(-log u)) over the kept set (T <= 1e-10: greedy argmax).
// One workgroup (1024 threads) per batch row, the row's logits (V <= 8192) live in registers:
//   * k-th largest on order-preserving uint32 keys, bit by bit from the top (32 block counts, no atomics:
//     exact and order independent);
//   * top-p only: the survivors are compacted (index order) into LDS as 64-bit (key, ~index) words,
//     bitonic-sorted descending, and a fixed-order block scan of exp(l - max) finds the cut;
//   * the uniforms come from a counter-based hash of (seed, position, row, token) -- replay-safe inside
//     a captured graph (the position is read from device memory) and deterministic for a seed.
// Finally thread 0 writes the image code of this position and the next input token (the next caption
// token during prefill, else the sample shifted into the image vocabulary).
#include "common.h"
#include "geom.h"

namespace dalle {

constexpr int SMP_THREADS = 1024;                     // 16 waves: the top-k select's per-step work is per lane
constexpr int SMP_VPT = 8;                            // logits per thread
constexpr int SMP_NW = SMP_THREADS / 64;
constexpr int SMP_VMAX = SMP_THREADS * SMP_VPT;       // 8192 = the image vocabulary

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float gumbel(uint64_t seed, int pos, int row, int idx) {
  const uint64_t ctr = ((uint64_t)(uint32_t)pos << 40) | ((uint64_t)(uint32_t)row << 16) | (uint32_t)idx;
  const uint64_t h = mix64(seed ^ mix64(ctr + 0x9e3779b97f4a7c15ull));
  const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1), 24 bits
  return -__logf(-__logf(u));
}

// Exclusive scan over the SMP_THREADS threads of the block in a fixed order (wave shuffles + the wave totals);
// returns this thread's exclusive prefix and the block total. `red` holds >= SMP_NW floats of LDS.
__device__ __forceinline__ float block_excl_scan(float v, float* red, float& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  __syncthreads();
  if (lane == 63) red[wave] = inc;
  __syncthreads();
  float before = 0.f, tot = 0.f;
  for (int w = 0; w < SMP_NW; ++w) {
    if (w < wave) before += red[w];
    tot += red[w];
  }
  total = tot;
  return before + inc - v;
}

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(SMP_THREADS) void sample_kernel(SampleArgs a) {
  __shared__ uint64_t srt[SMP_VMAX];  // top-p: (key << 32 | ~index), 64 KB
  __shared__ int cntb[2][SMP_NW];
  __shared__ float redf[SMP_NW];
  __shared__ int redi[SMP_NW];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* lr = a.logits + (size_t)row * a.V;

  uint32_t key[SMP_VPT];
  {
    // unconditional (clamped) loads: all 32 in flight at once (a guarded load per slot compiled to 32 serial
    // load -> vmcnt(0) round trips, ~7 us per row)
    float lv[SMP_VPT];
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) lv[i] = lr[min(i * SMP_THREADS + tid, a.V - 1)];  // coalesced
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) key[i] = i * SMP_THREADS + tid < a.V ? order_key(lv[i]) : 0u;
  }

  // ---- top-k threshold: the k-th largest key, bit by bit from the top ----
  // t = the largest key with #{key >= t} >= k (exact; ties kept), one block count per bit. No atomics: the former
  // radix histograms' LDS atomics serialised on the few exponent bins that logits share. (Two bits per step --
  // three candidate counts per barrier -- measured slower at 256 and at 1024 threads.)
  uint32_t kth = 0u;
  if (a.top_k > 0 && a.top_k < a.V) {
    uint32_t t = 0u;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = t | (1u << bit);
      int c = 0;  // the wave's count: one compare-to-mask and a scalar popcount per slot, no cross-lane shuffles
#pragma unroll
      for (int i = 0; i < SMP_VPT; ++i) c += __popcll(__ballot(key[i] >= cand));  // padding keys are 0 < cand
      if (lane == 0) cntb[bit & 1][wave] = c;  // two buffers: one barrier per bit suffices
      __syncthreads();
      int tot = 0;
#pragma unroll
      for (int w = 0; w < SMP_NW; ++w) tot += cntb[bit & 1][w];
      if (tot >= a.top_k) t = cand;
    }
    kth = t;
  }

  // ---- top-p: compact the survivors, sort descending, cut at the exclusive-cumsum crossing ----
  const bool nucleus = a.top_p < 1.0f;
  int n_keep = 0;
  if (nucleus) {
    int mine = 0;
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) mine += (i * SMP_THREADS + tid < a.V && key[i] >= kth) ? 1 : 0;
    // slots by an exclusive scan of the per-thread counts (any fixed order: the sort imposes the final one)
    float ftot;
    int w = (int)block_excl_scan((float)mine, redf, ftot);
    const int cnt = (int)ftot;
    int P = 1;
    while (P < cnt) P <<= 1;
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) {
      const int idx = i * SMP_THREADS + tid;
      if (idx < a.V && key[i] >= kth) srt[w++] = ((uint64_t)key[i] << 32) | (uint32_t)(~idx);
    }
    for (int j = cnt + tid; j < P; j += SMP_THREADS) srt[j] = 0ull;  // pads sort last
    __syncthreads();
    // bitonic sort, descending
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = tid; t < P / 2; t += SMP_THREADS) {
          const int lo = 2 * t - (t & (j - 1)), hi = lo + j;
          const bool desc = (lo & k) == 0;
          const uint64_t x = srt[lo], y = srt[hi];
          if ((x < y) == desc) { srt[lo] = y; srt[hi] = x; }
        }
        __syncthreads();
      }
    }
    // probabilities of the sorted survivors; each thread owns a contiguous chunk (fixed order)
    const float mx = key_float((uint32_t)(srt[0] >> 32));
    const int chunk = (cnt + SMP_THREADS - 1) / SMP_THREADS;
    const int c0 = min(cnt, tid * chunk), c1 = min(cnt, c0 + chunk);
    float part = 0.f;
    for (int j = c0; j < c1; ++j) part += __expf(key_float((uint32_t)(srt[j] >> 32)) - mx);
    float psum;
    float run = block_excl_scan(part, redf, psum);
    const float limit = a.top_p * psum;
    // kept = #{j : exclusive_cum(j) <= limit}; monotone, so each chunk counts its own
    int kept = 0;
    for (int j = c0; j < c1; ++j) {
      if (run <= limit) ++kept;
      run += __expf(key_float((uint32_t)(srt[j] >> 32)) - mx);
    }
    kept = wave_sum_int(kept);
    __syncthreads();
    if (lane == 0) redi[wave] = kept;
    __syncthreads();
    n_keep = 0;
    for (int w = 0; w < SMP_NW; ++w) n_keep += redi[w];
    n_keep = max(n_keep, 1);
  }

  // ---- Gumbel-max sample (argmax, ties -> smallest index) ----
  const int pos = *a.pos;
  const uint64_t seed = (uint64_t)*a.seed;
  const bool greedy = !(a.temperature > 1e-10f);
  const float invt = greedy ? 1.0f : 1.0f / a.temperature;
  float best = -INFINITY;
  int besti = 0x7fffffff;
  auto consider = [&](float l, int idx) {
    const float s = greedy ? l : l * invt + gumbel(seed, pos, row, idx);
    if (s > best || (s == best && idx < besti)) { best = s; besti = idx; }
  };
  if (nucleus) {
    for (int j = tid; j < n_keep; j += SMP_THREADS) {
      const uint64_t e = srt[j];
      consider(key_float((uint32_t)(e >> 32)), (int)(~(uint32_t)e));
    }
  } else if (kth != 0u && !greedy) {
    // top-k: the kept (key, index) pairs compacted per wave (ballot + prefix popcount) into the wave's region of
    // the sort buffer, then each lane draws the Gumbel noise of ~1 pair instead of the wave running the hash and
    // logs for every slot in which any lane kept a logit (divergent: ~11 us per row)
    uint64_t* wbuf = srt + wave * (SMP_VMAX / SMP_NW);
    const uint64_t lt = (1ull << lane) - 1ull;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) {
      const int idx = i * SMP_THREADS + tid;
      const bool kept = idx < a.V && key[i] >= kth;
      const uint64_t m = __ballot(kept);
      if (kept) wbuf[cnt + __popcll(m & lt)] = ((uint64_t)key[i] << 32) | (uint32_t)idx;
      cnt += __popcll(m);
    }
    __syncthreads();  // the wave's pairs are in LDS before its lanes read each other's
    for (int j = lane; j < cnt; j += 64) {
      const uint64_t e = wbuf[j];
      consider(key_float((uint32_t)(e >> 32)), (int)(uint32_t)e);
    }
  } else {
#pragma unroll
    for (int i = 0; i < SMP_VPT; ++i) {
      const int idx = i * SMP_THREADS + tid;
      if (idx < a.V && key[i] >= kth) consider(key_float(key[i]), idx);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
  }
  __syncthreads();  // every thread has read redi (n_keep) before it is reused
  if (lane == 0) { redf[wave] = best; redi[wave] = besti; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < SMP_NW; ++w)
      if (redf[w] > best || (redf[w] == best && redi[w] < besti)) { best = redf[w]; besti = redi[w]; }
    const int64_t nxt = besti;
    if (a.sampled) a.sampled[row] = nxt;
    if (a.codes) {
      const int ci = min(max(pos - (a.T - 1), 0), a.img_len - 1);
      a.codes[(size_t)row * a.img_len + ci] = nxt;
    }
    if (a.tok) {
      a.tok[row] = (pos + 1 < a.T) ? a.text[(size_t)row * a.T + min(pos + 1, a.T - 1)] : nxt + a.vt;
    }
  }
}

bool sample_step(const SampleArgs& a, hipStream_t st) {
  if (a.B < 1 || a.V < 1 || a.V > SMP_VMAX) return false;
  hipLaunchKernelGGL(sample_kernel, dim3(a.B), dim3(SMP_THREADS), 0, st, a);
  return true;
}

}  // namespace dalle
