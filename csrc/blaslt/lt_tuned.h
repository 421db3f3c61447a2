// Strided-batched bf16 x bf16 -> fp32 GEMM on hipBLASLt with a measured solution per problem (lt_tuned.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <tuple>

namespace dalle {

struct LtProblem {
  int opA = 0, opB = 0;                  // hipblasOperation_t of X1, X2
  long m = 0, n = 0, k = 0, batch = 1;   // C (m x n, column-major) = op(X1) (m x k) . op(X2) (k x n)
  long lda = 0, ldb = 0, ldc = 0;        // leading dims of the stored X1, X2, C
  long sa = 0, sb = 0, sc = 0;           // batch strides (elements)
  bool operator<(const LtProblem& o) const {
    return std::tie(opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc) <
           std::tie(o.opA, o.opB, o.m, o.n, o.k, o.batch, o.lda, o.ldb, o.ldc, o.sa, o.sb, o.sc);
  }
};

size_t lt_max_workspace();
int lt_count(const LtProblem& p);
size_t lt_ws_bytes(const LtProblem& p, int i);
bool lt_tuned(const LtProblem& p);
int lt_chosen(const LtProblem& p);
void lt_choose(const LtProblem& p, int i);
std::string lt_solution_name(const LtProblem& p, int i);
void lt_run_idx(const LtProblem& p, int i, const void* X1, const void* X2, float* C, void* ws, hipStream_t st);

}  // namespace dalle
