// Hand-scheduled assembly GEMMs (csrc/asm/gen_gemm.py): C[M, N] = A[M, K] . B[N, K]^T, bf16 operands,
// fp32 accumulation. M, N multiples of 256, K a multiple of 128 and >= 256; rows of A / B / C are lda / ldb /
// ldc elements apart. Returns false (launches nothing) for unsupported shapes.
#pragma once
#include <hip/hip_runtime.h>

namespace dalle {

bool asm_gemm_nt(const char* kernel, const void* A, const void* B, void* C, const void* aux0, const void* aux1,
                 const void* aux2, int M, int N, int K, int lda, int ldb, int ldc, int ld_aux, int flags, hipStream_t st);
int asm_gemm_grid(int num_tiles);
// QKV projection + 3-axis rotary into the attention storage qkv (3, B H, Np, 64) bf16: h (M = B n, 1024), w (3 H 64,
// 1024), cs3 (3, n + 1, 32, 2) fp32 (cos, sin) per pair for q (pre-scaled) / k / v (all rotated). n % 256 == 0.
bool asm_qkv_rope(bool col, const void* h, const void* w, void* qkv, const float* cs3, int M, int N, int K, int lda, int ldb,
                  int n, int T, int Tp, int Np, int H, int logS, hipStream_t st);
// Weight-gradient form: part[s] (M x N fp32) = A[s Kc : (s + 1) Kc, :]^T . B[s Kc : (s + 1) Kc, :] for s < splits,
// Kc = Ktot / splits; A (Ktot x M) and B (Ktot x N) bf16 token-major with row pitches lda / ldb. M, N multiples
// of 256, Kc a multiple of 128 and >= 256. Returns false (launches nothing) for unsupported shapes.
bool asm_gemm_tn(const void* A, const void* B, void* part, int M, int N, int Ktot, int lda, int ldb, int splits, hipStream_t st);

}  // namespace dalle
