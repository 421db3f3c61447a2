// Launchers of the hand-scheduled assembly GEMMs (csrc/asm/gen_gemm.py). The code object is embedded in
// this translation unit (gemm_hsaco.inc, generated at build time) and loaded once per device with
// hipModuleLoadData; kernels are launched with hipModuleLaunchKernel on the caller's stream.
#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>

#include "asm_gemm.h"
#include "gemm_hsaco.inc"

namespace dalle {
namespace {

struct Module {
  hipModule_t mod = nullptr;
  std::unordered_map<std::string, hipFunction_t> fns;
};

std::mutex g_mu;
std::array<Module, 64> g_mods;

hipFunction_t get_function(const char* name) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= (int)g_mods.size()) throw std::runtime_error("asm_gemm: no device");
  std::lock_guard<std::mutex> lk(g_mu);
  Module& m = g_mods[dev];
  if (m.mod == nullptr) {
    hipError_t e = hipModuleLoadData(&m.mod, kGemmHsaco);
    if (e != hipSuccess) throw std::runtime_error(std::string("asm_gemm: hipModuleLoadData: ") + hipGetErrorString(e));
  }
  auto it = m.fns.find(name);
  if (it != m.fns.end()) return it->second;
  hipFunction_t f = nullptr;
  hipError_t e = hipModuleGetFunction(&f, m.mod, name);
  if (e != hipSuccess) throw std::runtime_error(std::string("asm_gemm: no kernel ") + name);
  m.fns[name] = f;
  return f;
}

// kernel argument block (must match gen_gemm.py: 6 pointers then 16 int32)
struct alignas(8) GemmArgs {
  const void* a;
  const void* b;
  void* c;
  const void* aux0;
  const void* aux1;
  const void* aux2;
  int32_t m, n, k, lda, ldb, ldc, tiles_n, num_tiles, grid, ld_aux, flags, pad;
  int32_t e0, e1, e2, e3;  // kernel-specific (the QKV + rotary kernel's attention geometry)
};
static_assert(sizeof(GemmArgs) == 112, "kernarg block size");

int g_num_cus = 0;

}  // namespace

int asm_gemm_grid(int num_tiles) {
  if (g_num_cus == 0) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = cus > 0 ? cus : 256;
  }
  int g = num_tiles < g_num_cus ? num_tiles : g_num_cus;
  return (g + 7) / 8 * 8;  // the kernel's XCD tile map needs a multiple of 8 workgroups
}

bool asm_gemm_nt(const char* kernel, const void* A, const void* B, void* C, const void* aux0, const void* aux1,
                 const void* aux2, int M, int N, int K, int lda, int ldb, int ldc, int ld_aux, int flags, hipStream_t st) {
  if (M <= 0 || N <= 0 || M % 256 || N % 256 || K % 128 || K < 256) return false;
  GemmArgs args;
  std::memset(&args, 0, sizeof(args));
  args.a = A; args.b = B; args.c = C; args.aux0 = aux0; args.aux1 = aux1; args.aux2 = aux2;
  args.m = M; args.n = N; args.k = K; args.lda = lda; args.ldb = ldb; args.ldc = ldc;
  args.tiles_n = N / 256;
  args.num_tiles = (M / 256) * (N / 256);
  args.grid = asm_gemm_grid(args.num_tiles);
  args.ld_aux = ld_aux; args.flags = flags;
  size_t size = sizeof(args);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  hipFunction_t f = get_function(kernel);
  return hipModuleLaunchKernel(f, args.grid, 1, 1, 256, 1, 1, 0, st, nullptr, extra) == hipSuccess;
}

bool asm_qkv_rope(bool col, const void* h, const void* w, void* qkv, const float* cs3, int M, int N, int K, int lda, int ldb,
                  int n, int T, int Tp, int Np, int H, int logS, hipStream_t st) {
  if (M <= 0 || M % 256 || N % 256 || K < 1024 || K % 128 || n % 256 || M % n || (H * 64) % 256 || N != 3 * H * 64) return false;
  GemmArgs args;
  std::memset(&args, 0, sizeof(args));
  args.a = h; args.b = w; args.c = qkv; args.aux0 = cs3;
  args.m = M; args.n = N; args.k = K; args.lda = lda; args.ldb = ldb;
  args.tiles_n = N / 256;
  args.num_tiles = (M / 256) * (N / 256);
  args.grid = asm_gemm_grid(args.num_tiles);
  args.ld_aux = n; args.flags = T; args.pad = Tp; args.e0 = Np; args.e1 = H; args.e2 = logS;
  size_t size = sizeof(args);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  hipFunction_t f = get_function(col ? "dalle_gemm_nt_qkv_col" : "dalle_gemm_nt_qkv_row");
  return hipModuleLaunchKernel(f, args.grid, 1, 1, 256, 1, 1, 0, st, nullptr, extra) == hipSuccess;
}

bool asm_gemm_tn(const void* A, const void* B, void* part, int M, int N, int Ktot, int lda, int ldb, int splits, hipStream_t st) {
  if (M <= 0 || N <= 0 || M % 256 || N % 256 || splits <= 0 || Ktot % splits) return false;
  const int Kc = Ktot / splits;
  if (Kc % 128 || Kc < 256 || lda < M || ldb < N || lda >= (1 << 23) || ldb >= (1 << 23)) return false;
  GemmArgs args;
  std::memset(&args, 0, sizeof(args));
  args.a = A; args.b = B; args.c = part;
  args.m = M; args.n = N; args.k = Kc; args.lda = lda; args.ldb = ldb; args.ldc = N;
  args.tiles_n = N / 256;
  args.num_tiles = (M / 256) * (N / 256) * splits;  // work units (tile, split)
  args.grid = args.num_tiles;                       // one unit per workgroup
  size_t size = sizeof(args);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  hipFunction_t f = get_function("dalle_gemm_tn_wgrad");
  return hipModuleLaunchKernel(f, args.grid, 1, 1, 256, 1, 1, 0, st, nullptr, extra) == hipSuccess;
}

}  // namespace dalle
