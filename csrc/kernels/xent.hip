// Fused softmax cross-entropy with the gradient produced in the same pass.
// logits (R, V) bf16 (one split of the text/image vocabulary), labels (R) int64 (already offset into
// this split). Per row: loss = logsumexp(l) - l[label]; dlogits = (softmax(l) - onehot) * gscale
// written IN PLACE over the logits (bf16), so the backward pass is two GEMMs with no extra
// elementwise kernel. One 256-thread workgroup per row; online max/sum over 16-byte loads.
#include "common.h"

namespace dalle {

__global__ __launch_bounds__(256) void xent_fwd_bwd_kernel(__bf16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss, int V, float gscale) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  __bf16* lrow = logits + row * (long)V;
  const int tid = threadIdx.x;
  // rows of an odd-length vocabulary are not 16-B aligned: scalar head, vector body, scalar tail
  const int head = (int)((8 - ((row * (long)V) & 7)) & 7) < V ? (int)((8 - ((row * (long)V) & 7)) & 7) : V;
  __bf16* lr = lrow + head;
  const int Vb = V - head;
  const int nvec = Vb / 8;
  float m = NEG_BIG, s = 0.f;
  if (tid < head) {
    const float f = bf2f(reinterpret_cast<const bf16_raw*>(lrow)[tid]);
    s = 1.0f;
    m = f;
  }
  for (int i = tid; i < nvec; i += 256) {
    float f[8];
    unpack8(*reinterpret_cast<const s16x8*>(lr + 8 * i), f);
    float mx = f[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, f[j]);
    const float mn = fmaxf(m, mx);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
    m = mn;
    s = acc;
  }
  for (int i = nvec * 8 + tid; i < Vb; i += 256) {
    const float f = bf2f(reinterpret_cast<const bf16_raw*>(lr)[i]);
    const float mn = fmaxf(m, f);
    s = s * __expf(m - mn) + __expf(f - mn);
    m = mn;
  }
  // block reduce (max, sum)
  float wm = wave_max(m);
  float ws = wave_sum(s * __expf(m - wm));
  const int w = tid >> 6, l = tid & 63;
  if (l == 0) { red[w] = wm; red[4 + w] = ws; }
  __syncthreads();
  float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float Ssum = red[4] * __expf(red[0] - M) + red[5] * __expf(red[1] - M) + red[6] * __expf(red[2] - M) +
               red[7] * __expf(red[3] - M);
  const float lse = M + __logf(Ssum);
  const int64_t lab = labels[row];
  __syncthreads();
  if (tid == 0) {
    const float xl = bf2f(reinterpret_cast<const bf16_raw*>(lrow)[lab]);
    loss[row] = lse - xl;
  }
  __syncthreads();
  if (tid < head) {
    bf16_raw* p = reinterpret_cast<bf16_raw*>(lrow) + tid;
    float g = __expf(bf2f(*p) - lse);
    if (tid == lab) g -= 1.0f;
    *p = f2bf(g * gscale);
  }
  const int64_t labb = lab - head;
  for (int i = tid; i < nvec; i += 256) {
    float f[8];
    s16x8* p = reinterpret_cast<s16x8*>(lr + 8 * i);
    unpack8(*p, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = __expf(f[j] - lse);
      if (8 * i + j == labb) g -= 1.0f;
      f[j] = g * gscale;
    }
    *p = pack8(f);
  }
  for (int i = nvec * 8 + tid; i < Vb; i += 256) {
    bf16_raw* p = reinterpret_cast<bf16_raw*>(lr) + i;
    float g = __expf(bf2f(*p) - lse);
    if (i == labb) g -= 1.0f;
    *p = f2bf(g * gscale);
  }
}

void xent_fwd_bwd(void* logits, const int64_t* labels, float* loss, long R, int V, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(xent_fwd_bwd_kernel, dim3(R), dim3(256), 0, st, (__bf16*)logits, labels, loss, V, gscale);
}

// Same per-row math, XENT_RB consecutive rows per workgroup, plus the COLUMN sums of the produced
// dlogits (the head-bias gradient): a V-float accumulator in LDS (<= 40960 columns = 160 KiB) that each
// row adds into (within a row every column belongs to one thread; rows are separated by barriers), then
// one partial row per workgroup, reduced over workgroups in a fixed order by column_sum -- so the
// separate column-reduction pass over the logits disappears, deterministically.
constexpr int XENT_RB = 16;
constexpr int XENT_T = 1024;  // 16 waves: one workgroup per CU when the vocabulary fills the LDS
constexpr int XENT_MAXV = 35000;  // the padded accumulator (9/8 V floats + 32) must fit the 160 KiB per workgroup
// column c of the LDS accumulator lives at c + c/8: a lane adds 8 consecutive columns, so unpadded the
// 64 lanes of a wave would hit banks 8 apart (8-way conflicts, 23M per dispatch measured); with one pad
// float per 8 columns consecutive lanes are 9 floats apart -- conflict-free
__host__ __device__ __forceinline__ int xpad(int c) { return c + (c >> 3); }

__global__ __launch_bounds__(XENT_T) void xent_colsum_kernel(__bf16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                          float* __restrict__ loss, float* __restrict__ part, long R, int V,
                                                          float gscale) {
  extern __shared__ float colacc[];  // xpad(V) floats (+32 for the reductions)
  float* red = colacc + ((xpad(V) + 3) & ~3);
  const int tid = threadIdx.x;
  for (int c = tid; c < V; c += XENT_T) colacc[xpad(c)] = 0.f;
  const long r0 = (long)blockIdx.x * XENT_RB;
  for (long row = r0; row < r0 + XENT_RB && row < R; ++row) {
    __bf16* lrow = logits + row * (long)V;
    const int hd = (int)((8 - ((row * (long)V) & 7)) & 7);
    const int head = hd < V ? hd : V;
    __bf16* lr = lrow + head;
    const int Vb = V - head;
    const int nvec = Vb / 8;
    float m = NEG_BIG, s = 0.f;
    if (tid < head) {
      m = bf2f(reinterpret_cast<const bf16_raw*>(lrow)[tid]);
      s = 1.0f;
    }
    for (int i = tid; i < nvec; i += XENT_T) {
      float f[8];
      unpack8(*reinterpret_cast<const s16x8*>(lr + 8 * i), f);
      float mx = f[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx = fmaxf(mx, f[j]);
      const float mn = fmaxf(m, mx);
      float acc = s * __expf(m - mn);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
      m = mn;
      s = acc;
    }
    for (int i = nvec * 8 + tid; i < Vb; i += XENT_T) {
      const float f = bf2f(reinterpret_cast<const bf16_raw*>(lr)[i]);
      const float mn = fmaxf(m, f);
      s = s * __expf(m - mn) + __expf(f - mn);
      m = mn;
    }
    const float wm = wave_max(m);
    const float ws = wave_sum(s * __expf(m - wm));
    const int w = tid >> 6, l = tid & 63;
    constexpr int NW = XENT_T / 64;
    __syncthreads();  // the previous row's users of `red` are done
    if (l == 0) { red[w] = wm; red[NW + w] = ws; }
    __syncthreads();
    float M = red[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) M = fmaxf(M, red[k]);
    float Ssum = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) Ssum += red[NW + k] * __expf(red[k] - M);
    const float lse = M + __logf(Ssum);
    const int64_t lab = labels[row];
    if (tid == 0) loss[row] = lse - bf2f(reinterpret_cast<const bf16_raw*>(lrow)[lab]);
    __syncthreads();  // the label logit is read before it is overwritten
    if (tid < head) {
      bf16_raw* p = reinterpret_cast<bf16_raw*>(lrow) + tid;
      float g = __expf(bf2f(*p) - lse);
      if (tid == lab) g -= 1.0f;
      const bf16_raw q = f2bf(g * gscale);
      *p = q;
      colacc[xpad(tid)] += bf2f(q);
    }
    const int64_t labb = lab - head;
    for (int i = tid; i < nvec; i += XENT_T) {
      float f[8];
      s16x8* p = reinterpret_cast<s16x8*>(lr + 8 * i);
      unpack8(*p, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g = __expf(f[j] - lse);
        if (8 * i + j == labb) g -= 1.0f;
        f[j] = g * gscale;
      }
      const s16x8 q = pack8(f);
      *p = q;
      unpack8(q, f);  // the bias gradient sums the bf16 values the GEMMs consume
#pragma unroll
      for (int j = 0; j < 8; ++j) colacc[xpad(head + 8 * i + j)] += f[j];
    }
    for (int i = nvec * 8 + tid; i < Vb; i += XENT_T) {
      bf16_raw* p = reinterpret_cast<bf16_raw*>(lr) + i;
      float g = __expf(bf2f(*p) - lse);
      if (i == labb) g -= 1.0f;
      const bf16_raw q = f2bf(g * gscale);
      *p = q;
      colacc[xpad(head + i)] += bf2f(q);
    }
    __syncthreads();  // the next row may map a column to another thread
  }
  float* prow = part + (size_t)blockIdx.x * V;
  for (int c = tid; c < V; c += XENT_T) prow[c] = colacc[xpad(c)];
}

// Register-resident form: a row is spread over the W waves of one workgroup (image vocabulary: W = 4, 4
// x 16 B per lane; text: W = 16, 8 x 8 B per lane), so it is read from HBM exactly once -- max, sum of
// exponentials and the gradient all come from registers -- and each lane keeps the column sums of its
// own columns in registers (no LDS accumulator: the LDS form above fits one workgroup, one row in flight,
// per CU at the text vocabulary; this one keeps several rows per CU in flight). Every wave owns fixed
// columns, so the workgroup's partial row is written without a combine. Fixed-order reductions
// throughout: deterministic.
template <int NV, int W, int E>
__global__ __launch_bounds__(64 * W) void xent_reg_kernel(__bf16* __restrict__ logits, const int64_t* __restrict__ labels,
                                                          float* __restrict__ loss, float* __restrict__ part, long R, int V,
                                                          float gscale) {
  typedef short vecE __attribute__((ext_vector_type(E)));
  __shared__ float xs[2][W];  // per-wave row max / sum of exponentials
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  float acc[NV][E];
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < E; ++e) acc[j][e] = 0.f;
  for (long row = blockIdx.x; row < R; row += gridDim.x) {
    const bf16_raw* lr = reinterpret_cast<const bf16_raw*>(logits) + row * (long)V;
    vecE d[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = ((j * W + wave) * 64 + lane) * E;
      d[j] = c < V ? *reinterpret_cast<const vecE*>(lr + c) : vecE{};
    }
    const int lab = (int)labels[row];
    float m = NEG_BIG;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = ((j * W + wave) * 64 + lane) * E;
      if (c < V) {
#pragma unroll
        for (int e = 0; e < E; ++e) m = fmaxf(m, bf2f((bf16_raw)d[j][e]));
      }
    }
    m = wave_max(m);
    if (lane == 0) xs[0][wave] = m;
    __syncthreads();
    m = xs[0][0];
#pragma unroll
    for (int k = 1; k < W; ++k) m = fmaxf(m, xs[0][k]);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = ((j * W + wave) * 64 + lane) * E;
      if (c < V) {
#pragma unroll
        for (int e = 0; e < E; ++e) s += __expf(bf2f((bf16_raw)d[j][e]) - m);
      }
    }
    s = wave_sum(s);
    if (lane == 0) xs[1][wave] = s;  // a different slot than the max: no wave can overwrite what another still reads
    __syncthreads();
    s = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) s += xs[1][k];
    const float lse = m + __logf(s);
    bf16_raw* lw = reinterpret_cast<bf16_raw*>(logits) + row * (long)V;
    float xl = 0.f;
    bool own = false;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = ((j * W + wave) * 64 + lane) * E;
      if (c < V) {
        vecE q;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float f = bf2f((bf16_raw)d[j][e]);
          const bool hit = c + e == lab;
          const float g = __expf(f - lse) - (hit ? 1.0f : 0.0f);
          xl = hit ? f : xl;
          own |= hit;
          q[e] = (short)f2bf(g * gscale);
          acc[j][e] += bf2f((bf16_raw)q[e]);  // the bias gradient sums the bf16 values the GEMMs consume
        }
        *reinterpret_cast<vecE*>(lw + c) = q;
      }
    }
    if (own) loss[row] = lse - xl;
  }
  float* prow = part + (size_t)blockIdx.x * V;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = ((j * W + wave) * 64 + lane) * E;
    if (c < V) {
#pragma unroll
      for (int e = 0; e < E; ++e) prow[c + e] = acc[j][e];
    }
  }
}

// which form runs: 2 = register-resident, 4 waves (V <= 8192, 16-B rows), 1 = register-resident, 16
// waves (V <= 32768, 8-B rows), 0 = the LDS-accumulator kernel (wider vocabularies).
static int xent_form(int V) {
  if (V % 8 == 0 && V <= 4 * 4 * 64 * 8) return 2;
  if (V % 4 == 0 && V <= 8 * 16 * 64 * 4) return 1;
  return 0;
}

long xent_colsum_blocks(long R, int V) {
  const int form = xent_form(V);
  if (form == 0) return (R + XENT_RB - 1) / XENT_RB;
  const long cap = form == 2 ? 1024 : 512;  // 4 / 2 workgroups per CU; partial rows are 4 V bytes each
  return R < cap ? R : cap;
}

bool xent_colsum(void* logits, const int64_t* labels, float* loss, float* part, long R, int V, float gscale, hipStream_t st) {
  const int form = xent_form(V);
  if (form == 2) {
    hipLaunchKernelGGL((xent_reg_kernel<4, 4, 8>), dim3(xent_colsum_blocks(R, V)), dim3(256), 0, st, (__bf16*)logits, labels,
                       loss, part, R, V, gscale);
    return true;
  }
  if (form == 1) {
    hipLaunchKernelGGL((xent_reg_kernel<8, 16, 4>), dim3(xent_colsum_blocks(R, V)), dim3(1024), 0, st, (__bf16*)logits, labels,
                       loss, part, R, V, gscale);
    return true;
  }
  if (V > XENT_MAXV) return false;
  const long nblk = (R + XENT_RB - 1) / XENT_RB;
  const size_t lds = (size_t)(((xpad(V) + 3) & ~3) + 2 * (XENT_T / 64)) * sizeof(float);
  static bool attr = false;
  if (!attr) {  // dynamic LDS beyond the default cap needs an explicit per-kernel limit
    (void)hipFuncSetAttribute((const void*)xent_colsum_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(xent_colsum_kernel, dim3(nblk), dim3(XENT_T), lds, st, (__bf16*)logits, labels, loss, part, R, V, gscale);
  return true;
}

}  // namespace dalle
