// PyTorch bindings for the dalle_amd HIP kernels (module dalle_amd._C).
// Every op checks device, dtype, contiguity and the shapes its kernel's grid assumes BEFORE launching
// (a mis-sized launch of a hand-written kernel can fault the GPU).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include "kernels/geom.h"
#include "asm/asm_gemm.h"

namespace dalle {

void attn_fwd(const void*, const void*, const void*, void*, float*, const AttnGeom&, int, hipStream_t);
void attn_bwd(const void*, const void*, const void*, const void*, const void*, const float*, float*, void*, void*,
              void*, const AttnGeom&, int, hipStream_t, const float*, const float*, void*, float, const float* rotf = nullptr,
              int rot_nl = 0, int rot_np = 0, float rot_img_text_pos = 0.f, float rot_text_axial = 0.f);
void rope_fwd(const void*, const float*, const float*, void*, void*, void*, const RopeGeom&, int, float, hipStream_t);
void rope_bwd(const void*, const void*, const void*, const float*, const float*, void*, const RopeGeom&, int, float, hipStream_t);
bool ln_shift_fwd(const float*, const float*, const float*, void*, float*, float*, const ShiftGeom&, int, int, float, hipStream_t,
                  const void* = nullptr, const float* = nullptr, float* = nullptr);
bool ln_shift_bwd(const float*, const float*, const void*, const float*, const float*, const float*, float*, float*,
                  const GradSink&, const ShiftGeom&, int, int, hipStream_t, const void* = nullptr, const float* = nullptr,
                  void* = nullptr, float* = nullptr, const GradSink* = nullptr);
void geglu_fwd(const void*, void*, long, int, hipStream_t);
void geglu_bwd(const void*, const void*, void*, long, int, hipStream_t);
void geglu_bwd_bias(const void*, const void*, void*, float*, const GradSink&, long, int, hipStream_t);
void scale_residual(const float*, const void*, const float*, float*, long, int, hipStream_t);
void scale_residual_bwd(const float*, const void*, const float*, void*, float*, const GradSink&, long, int, hipStream_t);
void nonfinite(const float*, long, int*, hipStream_t);
void zero_if_flag(float*, long, const int*, hipStream_t);
bool gemm_nt(const void*, const void*, void*, const void*, int, int, int, int, hipStream_t);
void uq8_compress(const float*, long, uint8_t*, float*, void*, hipStream_t);
size_t uq8_workspace_bytes();
void uq8_dequant(const uint8_t*, const float*, float*, long, float, int, hipStream_t);
void uq8_seg_compress(const float*, const long*, const long*, const int*, int, uint8_t*, float*, hipStream_t);
void uq8_seg_dequant(const uint8_t*, const long*, const float*, const long*, const int*, int, float*, float, int, hipStream_t);
bool skinny_gemm(int, SkinnyArgs, hipStream_t);
int skinny_ks(int, int, int, int);
void skinny_force_config(int, int, int, int);
std::vector<int> skinny_shape_info(int, int, int, int);
bool gemm_qkv_rope(const void*, const void*, void*, void*, void*, const float*, const float*, int, int, int, int, int, int, int,
                   float, hipStream_t);
void splitk_accum(const float*, float*, long, int, int, hipStream_t);
void psgd_orthonormalize(float*, const long*, const int*, int, int, float, hipStream_t);
bool psgd_reconstruct(float*, float*, const float*, const float*, long, int, int, hipStream_t);
void xent_fwd_bwd(void*, const int64_t*, float*, long, int, float, hipStream_t);
void embed_fwd(const int64_t*, const int64_t*, const float*, float*, int*, int*, int, int, int, int, int, int, int, int,
               hipStream_t);
bool xent_colsum(void*, const int64_t*, float*, float*, long, int, float, hipStream_t);
void transpose_cast_bf16(const float* w, void* wt, int R, int C, hipStream_t st);
void transpose_bf16(const void* x, void* xt, int R, int C, hipStream_t st);
bool conv3x3(const ConvArgs&, hipStream_t);
bool gn_stats(const void*, float*, float*, float*, int, int, int, float, hipStream_t);
size_t gn_part_floats(int);
void gn_apply(const void*, const float*, const float*, const float*, const float*, void*, int, int, int, hipStream_t, int);
bool conv_out(const void*, const void*, const float*, const float*, const float*, const float*, const float*, float*, int, int,
              int, int, hipStream_t);
void softmax_rows(const float*, void*, long, int, float, hipStream_t);
long xent_colsum_blocks(long, int);
void embed_bwd(const float*, const int*, const int*, const int*, float*, float*, int, int, hipStream_t);
void decode_ln_shift(float*, const float*, const float*, void*, void*, const int*, const DecodeGeom&, int, int, int, hipStream_t,
                     const float*, const void*, const float*, int);
void residual_from_partials(float*, const float*, const void*, const float*, int, int, int, hipStream_t);
void prefill_rope(const void*, const float*, const float*, void*, void*, void*, int, int, int, int, float, hipStream_t);
void prefill_ln_shift(const float*, const float*, const float*, void*, void*, int, int, int, int, float, int, hipStream_t);
void prefill_softmax(const float*, const bool*, void*, long, int, hipStream_t);
void prefill_residual(float*, const void*, const float*, long, int, hipStream_t);
void decode_attn_part(const float*, int, const float*, const float*, float, void*, void*, void*, const int*, const DecodeGeom&, int,
                      hipStream_t, const int*);
bool skinny_partials(SkinnyArgs, hipStream_t);
bool skinny_partials_ln(SkinnyArgs, hipStream_t);
bool skinny_partials_ln_ok(int, int, int);
int skinny_partials_ks(int, int, int);
void decode_rope(const void*, const float*, const float*, void*, void*, void*, const int*, const DecodeGeom&, int, float,
                 hipStream_t);
void decode_attn(const void*, void*, void*, void*, const int*, const DecodeGeom&, int, hipStream_t, const int*);
void vq_embed(const int64_t*, const float*, float*, int, int, int, hipStream_t);
bool sample_step(const SampleArgs&, hipStream_t);
bool gemm_geglu_bwd(const void*, const void*, const void*, void*, float*, int, int, int, hipStream_t, int);
void column_sum(const float*, int, int, const GradSink&, hipStream_t);
bool gemm_pt(const void*, const void*, void*, const void*, int, int, int, int, int, int, hipStream_t);
void gemm_set_cpol(int);
void gemm_set_pt_overlap(int, int);
void gemm_set_geglu_bwd_2wg(int);
void gemm_set_2wg_stagger(int, int);
bool gemm_2wg(const void*, const void*, void*, const void*, int, int, int, hipStream_t);
void gemm_set_drain(int);
bool gemm_pt_qkv_rope(const void*, const void*, void*, void*, void*, const float*, int, int, int, int, int, int, int, float,
                      hipStream_t, int);
bool gemm_pt_geglu_bwd(const void*, const void*, const void*, void*, float*, int, int, int, hipStream_t, int);
bool gemm_pt_geglu_fwd(const void*, const void*, const void*, void*, void*, int, int, int, hipStream_t, int);
void permlane16_probe(unsigned*, hipStream_t);
void rope_pad_zero(void*, void*, void*, int, int, int, int, hipStream_t);
void lamb_grad_norm(const float*, long, float*, float, float*, float*, hipStream_t);
void lamb_step(float*, const float*, uint8_t*, uint8_t*, float*, float*, float*, float*, const float*, const float*,
               const int*, const int*, const long*, const long*, const int*, const float*, const float*, const float*, float*,
               float*, float*, float*, int, long, float, float, float, float, int, hipStream_t);
}  // namespace dalle

using torch::Tensor;

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

#define DALLE_CAT2(a, b) a##b
#define DALLE_CAT(a, b) DALLE_CAT2(a, b)
// every op's first device check also makes that tensor's GPU the current device for the rest of the op,
// so cur_stream() and the kernel launches bind to the operand's device (a serving thread whose current
// device is still GPU 0 must not launch on GPU 0's stream against GPU N's memory)
#define CHECK_CUDA(x)                                                  \
  TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor");              \
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA DALLE_CAT(_dev_guard_, __COUNTER__)((x).device())
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " has wrong dtype")
#define CHECK_IN(x, dt) CHECK_CUDA(x); CHECK_CONTIG(x); CHECK_DT(x, dt)

// ---------------------------------------------------------------------------------------------
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  TORCH_CHECK((1 << l) == v, "image side must be a power of two");
  return l;
}

static dalle::AttnGeom make_attn_geom(int T, int S, int n, int K, int H, int pattern) {
  dalle::AttnGeom g;
  g.T = T;
  g.Tp = (T + 31) / 32 * 32;
  g.S = S;
  g.logS = ilog2(S);
  g.I = S * S;
  g.Np = g.Tp + g.I;
  g.n = n;
  g.K = K;
  g.H = H;
  g.pattern = pattern;
  TORCH_CHECK(g.I % 32 == 0, "image grid must be a multiple of 32 tokens");
  TORCH_CHECK(n == T + g.I - 1, "sequence length must be text_len + image_seq_len - 1");
  return g;
}

// ---------------------------------------------------------------------------------------------
std::vector<Tensor> ln_shift_fwd(Tensor x, Tensor w, Tensor b, int64_t T, int64_t S, bool shift, double eps) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(w, torch::kFloat32); CHECK_IN(b, torch::kFloat32);
  TORCH_CHECK(x.dim() == 3, "x must be (B, n, D)");
  const int B = x.size(0), n = x.size(1), D = x.size(2);
  TORCH_CHECK(w.numel() == D && b.numel() == D);
  if (shift) TORCH_CHECK(n >= T && n - T <= S * S && D % 4 == 0, "token shift geometry mismatch");
  auto y = torch::empty({B, n, D}, x.options().dtype(torch::kBFloat16));
  auto mean = torch::empty({B * n}, x.options());
  auto rstd = torch::empty({B * n}, x.options());
  dalle::ShiftGeom g{n, (int)T, (int)S, shift ? 1 : 0};
  bool ok = dalle::ln_shift_fwd(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr(),
                                mean.data_ptr<float>(), rstd.data_ptr<float>(), g, B * n, D, (float)eps, cur_stream());
  TORCH_CHECK(ok, "ln_shift: unsupported hidden size ", D);
  return {y, mean, rstd};
}

// Sublayer boundary, forward: x = res + scale_prev * y_prev (returned) and LN(+shift)(x) in one pass.
std::vector<Tensor> ln_shift_fwd_res(Tensor res, Tensor yprev, Tensor sprev, Tensor w, Tensor b, int64_t T, int64_t S, bool shift,
                                     double eps) {
  CHECK_IN(res, torch::kFloat32); CHECK_IN(yprev, torch::kBFloat16); CHECK_IN(sprev, torch::kFloat32);
  CHECK_IN(w, torch::kFloat32); CHECK_IN(b, torch::kFloat32);
  TORCH_CHECK(res.dim() == 3, "res must be (B, n, D)");
  const int B = res.size(0), n = res.size(1), D = res.size(2);
  TORCH_CHECK(yprev.numel() == res.numel() && sprev.numel() == D && w.numel() == D && b.numel() == D,
              "ln_shift_fwd_res: shape mismatch");
  if (shift) TORCH_CHECK(n >= T && n - T <= S * S && D % 4 == 0, "token shift geometry mismatch");
  auto x = torch::empty_like(res);
  auto y = torch::empty({B, n, D}, res.options().dtype(torch::kBFloat16));
  auto mean = torch::empty({B * n}, res.options());
  auto rstd = torch::empty({B * n}, res.options());
  dalle::ShiftGeom g{n, (int)T, (int)S, shift ? 1 : 0};
  bool ok = dalle::ln_shift_fwd(res.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr(), mean.data_ptr<float>(),
                                rstd.data_ptr<float>(), g, B * n, D, (float)eps, cur_stream(), yprev.data_ptr(),
                                sprev.data_ptr<float>(), x.data_ptr<float>());
  TORCH_CHECK(ok, "ln_shift: unsupported hidden size ", D);
  return {x, y, mean, rstd};
}

// grad sink: an fp32 contiguous buffer of `n` floats that the kernel ACCUMULATES into (a .grad view
// of the flat arena); returns its pointer or nullptr when absent
static float* sink_ptr(const c10::optional<Tensor>& t, long n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous() && t->numel() == n, what,
              ": grad sink must be a contiguous fp32 CUDA tensor of ", n, " elements");
  return t->data_ptr<float>();
}

// LN(+shift) backward. resid (optional, fp32 like x): residual-stream grad added into dx.
// gw/gb (optional, together): accumulate dweight/dbias into them and return undefined (None) for both.
std::vector<Tensor> ln_shift_bwd(Tensor x, Tensor w, Tensor dy, Tensor mean, Tensor rstd, int64_t T, int64_t S, bool shift,
                                 c10::optional<Tensor> resid, c10::optional<Tensor> gw, c10::optional<Tensor> gb) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(w, torch::kFloat32); CHECK_IN(dy, torch::kBFloat16);
  CHECK_IN(mean, torch::kFloat32); CHECK_IN(rstd, torch::kFloat32);
  const int B = x.size(0), n = x.size(1), D = x.size(2);
  TORCH_CHECK(dy.sizes() == x.sizes() && mean.numel() == B * n && rstd.numel() == B * n);
  const float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    CHECK_IN((*resid), torch::kFloat32);
    TORCH_CHECK(resid->sizes() == x.sizes(), "ln_shift_bwd: residual grad shape mismatch");
    rp = resid->data_ptr<float>();
  }
  float* pw = sink_ptr(gw, D, "ln_shift_bwd dweight");
  float* pb = sink_ptr(gb, D, "ln_shift_bwd dbias");
  TORCH_CHECK((pw == nullptr) == (pb == nullptr), "ln_shift_bwd: give both weight and bias grad sinks or neither");
  auto dx = torch::empty_like(x);
  auto part = torch::empty({512, 2 * D}, x.options());  // per-block partial [dw | db] rows
  Tensor dwdb;
  dalle::GradSink sink;
  if (pw) {
    sink = dalle::GradSink{pw, pb, nullptr, D, 1};
  } else {
    dwdb = torch::empty({2 * D}, x.options());
    sink = dalle::GradSink{dwdb.data_ptr<float>(), dwdb.data_ptr<float>() + D, nullptr, D, 0};
  }
  dalle::ShiftGeom g{n, (int)T, (int)S, shift ? 1 : 0};
  bool ok = dalle::ln_shift_bwd(x.data_ptr<float>(), w.data_ptr<float>(), dy.data_ptr(), mean.data_ptr<float>(),
                                rstd.data_ptr<float>(), rp, dx.data_ptr<float>(), part.data_ptr<float>(), sink, g, B * n, D,
                                cur_stream());
  TORCH_CHECK(ok, "ln_shift: unsupported hidden size ", D);
  if (pw) return {dx, Tensor(), Tensor()};
  return {dx, dwdb.slice(0, 0, D), dwdb.slice(0, D, 2 * D)};
}

// ---------------------------------------------------------------------------------------------
static dalle::RopeGeom make_rope_geom(int T, int S, int n, int H, bool col_major) {
  dalle::RopeGeom g;
  g.T = T;
  g.Tp = (T + 31) / 32 * 32;
  g.S = S;
  g.logS = ilog2(S);
  g.n = n;
  g.Np = g.Tp + S * S;
  g.H = H;
  g.col_major = col_major ? 1 : 0;
  TORCH_CHECK(n == T + S * S - 1, "rope: sequence length mismatch");
  return g;
}

std::vector<Tensor> rope_fwd(Tensor qkv, Tensor cosT, Tensor sinT, int64_t T, int64_t S, int64_t H, bool col_major, double qscale) {
  CHECK_IN(qkv, torch::kBFloat16); CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  const int B = qkv.size(0), n = qkv.size(1);
  TORCH_CHECK(qkv.size(2) == 3 * H * 64, "rope: dim_head must be 64");
  TORCH_CHECK(cosT.size(0) >= n && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes());
  auto g = make_rope_geom(T, S, n, H, col_major);
  auto opts = qkv.options();
  auto q = torch::empty({B * H, g.Np, 64}, opts);
  auto k = torch::empty({B * H, g.Np, 64}, opts);
  auto v = torch::empty({B * H, g.Np, 64}, opts);
  dalle::rope_fwd(qkv.data_ptr(), cosT.data_ptr<float>(), sinT.data_ptr<float>(), q.data_ptr(), k.data_ptr(), v.data_ptr(), g,
                  B * H, (float)qscale, cur_stream());
  return {q, k, v};
}

Tensor rope_bwd(Tensor dq, Tensor dk, Tensor dv, Tensor cosT, Tensor sinT, int64_t B, int64_t T, int64_t S, int64_t H, int64_t n,
                bool col_major, double qscale) {
  CHECK_IN(dq, torch::kBFloat16); CHECK_IN(dk, torch::kBFloat16); CHECK_IN(dv, torch::kBFloat16);
  CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  auto g = make_rope_geom(T, S, n, H, col_major);
  TORCH_CHECK(dq.size(0) == B * H && dq.size(1) == g.Np && dq.size(2) == 64);
  TORCH_CHECK(dk.sizes() == dq.sizes() && dv.sizes() == dq.sizes());
  auto dqkv = torch::empty({B, n, 3 * H * 64}, dq.options());
  dalle::rope_bwd(dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), cosT.data_ptr<float>(), sinT.data_ptr<float>(), dqkv.data_ptr(),
                  g, B, (float)qscale, cur_stream());
  return dqkv;
}

// Sublayer boundary, backward: LN(+shift) backward of this sublayer (dx = resid + LN'(dy), dweight/dbias
// into gw/gb) fused with the previous sublayer's LayerScale-residual backward (dy_prev = bf16(sprev * dx),
// dscale_prev / dbias_prev into gsp / gbp). All four grad sinks are required (the flat-arena path).
std::vector<Tensor> ln_shift_bwd_sr(Tensor x, Tensor w, Tensor dy, Tensor mean, Tensor rstd, int64_t T, int64_t S, bool shift,
                                    Tensor resid, Tensor yprev, Tensor sprev, Tensor gw, Tensor gb, Tensor gsp, Tensor gbp) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(w, torch::kFloat32); CHECK_IN(dy, torch::kBFloat16);
  CHECK_IN(mean, torch::kFloat32); CHECK_IN(rstd, torch::kFloat32); CHECK_IN(resid, torch::kFloat32);
  CHECK_IN(yprev, torch::kBFloat16); CHECK_IN(sprev, torch::kFloat32);
  const int B = x.size(0), n = x.size(1), D = x.size(2);
  TORCH_CHECK(dy.sizes() == x.sizes() && resid.sizes() == x.sizes() && yprev.numel() == x.numel() && sprev.numel() == D &&
              mean.numel() == B * n && rstd.numel() == B * n, "ln_shift_bwd_sr: shape mismatch");
  float* pw = sink_ptr(gw, D, "ln_shift_bwd_sr dweight");
  float* pb = sink_ptr(gb, D, "ln_shift_bwd_sr dbias");
  float* ps = sink_ptr(gsp, D, "ln_shift_bwd_sr dscale_prev");
  float* pbp = sink_ptr(gbp, D, "ln_shift_bwd_sr dbias_prev");
  auto dx = torch::empty_like(x);
  auto dyp = torch::empty(x.sizes(), dy.options());
  auto part = torch::empty({2, 512, 2 * D}, x.options());  // per-block partial rows [dw | db] and [g*y_prev | g]
  const dalle::GradSink sink{pw, pb, nullptr, D, 1};
  const dalle::GradSink sink2{ps, pbp, sprev.data_ptr<float>(), D, 1};  // dbias_prev = sprev * sum(g)
  dalle::ShiftGeom g{n, (int)T, (int)S, shift ? 1 : 0};
  bool ok = dalle::ln_shift_bwd(x.data_ptr<float>(), w.data_ptr<float>(), dy.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                resid.data_ptr<float>(), dx.data_ptr<float>(), part.data_ptr<float>(), sink, g, B * n, D, cur_stream(),
                                yprev.data_ptr(), sprev.data_ptr<float>(), dyp.data_ptr(), part.data_ptr<float>() + 512 * 2 * D,
                                &sink2);
  TORCH_CHECK(ok, "ln_shift: unsupported hidden size ", D);
  return {dx, dyp};
}

// ---------------------------------------------------------------------------------------------
std::vector<Tensor> attn_fwd(Tensor q, Tensor k, Tensor v, int64_t B, int64_t T, int64_t S, int64_t n, int64_t K, int64_t H,
                             int64_t pattern) {
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(k, torch::kBFloat16); CHECK_IN(v, torch::kBFloat16);
  auto g = make_attn_geom(T, S, n, K, H, pattern);
  TORCH_CHECK(q.size(0) == B * H && q.size(1) == g.Np && q.size(2) == 64, "attn: q must be (B*H, Np, 64)");
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes());
  TORCH_CHECK(pattern >= 0 && pattern <= 3);
  auto out = torch::empty({B, n, H * 64}, q.options());
  auto lse = torch::empty({B * H, g.Np}, q.options().dtype(torch::kFloat32));
  dalle::attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), g, B * H, cur_stream());
  return {out, lse};
}

std::vector<Tensor> attn_bwd(Tensor q, Tensor k, Tensor v, Tensor out, Tensor dout, Tensor lse, int64_t B, int64_t T, int64_t S,
                             int64_t n, int64_t K, int64_t H, int64_t pattern) {
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(k, torch::kBFloat16); CHECK_IN(v, torch::kBFloat16);
  CHECK_IN(out, torch::kBFloat16); CHECK_IN(dout, torch::kBFloat16); CHECK_IN(lse, torch::kFloat32);
  auto g = make_attn_geom(T, S, n, K, H, pattern);
  TORCH_CHECK(q.size(0) == B * H && q.size(1) == g.Np && q.size(2) == 64);
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes());
  TORCH_CHECK(out.size(0) == B && out.size(1) == n && out.size(2) == H * 64 && dout.sizes() == out.sizes());
  TORCH_CHECK(lse.numel() == B * H * g.Np);
  auto delta = torch::empty({B * H, g.Np}, lse.options());
  auto dq = torch::empty_like(q);
  auto dk = torch::empty_like(q);
  auto dv = torch::empty_like(q);
  dalle::attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                  delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), g, B * H,
                  cur_stream(), nullptr, nullptr, nullptr, 0.f);
  return {dq, dk, dv};
}

// Attention backward with the rotary backward fused into its epilogues: returns dqkv (B, n, 3*H*64)
// directly (no (B*H, Np, 64) dq / dk / dv intermediates, no rope_bwd pass).
// rotf (optional): the rotary frequencies of rotary.rotary_freq_split ((64,) fp32 on the device) with their axis
// split (n_lang, n_pix) and fixed positions -- given, the axial S = 32 backward runs as the fused one-workgroup-
// per-head kernel, which computes the rotary angles in-kernel instead of reading the tables
Tensor attn_bwd_rope(Tensor q, Tensor k, Tensor v, Tensor out, Tensor dout, Tensor lse, Tensor cosT, Tensor sinT, int64_t B,
                     int64_t T, int64_t S, int64_t n, int64_t K, int64_t H, int64_t pattern, double qscale,
                     c10::optional<Tensor> rotf, int64_t n_lang, int64_t n_pix, double img_text_pos, double text_axial) {
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(k, torch::kBFloat16); CHECK_IN(v, torch::kBFloat16);
  CHECK_IN(out, torch::kBFloat16); CHECK_IN(dout, torch::kBFloat16); CHECK_IN(lse, torch::kFloat32);
  CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  auto g = make_attn_geom(T, S, n, K, H, pattern);
  TORCH_CHECK(q.size(0) == B * H && q.size(1) == g.Np && q.size(2) == 64);
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes());
  TORCH_CHECK(out.size(0) == B && out.size(1) == n && out.size(2) == H * 64 && dout.sizes() == out.sizes());
  TORCH_CHECK(lse.numel() == B * H * g.Np);
  TORCH_CHECK(cosT.dim() == 2 && cosT.size(0) >= n && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes(),
              "attn_bwd_rope: rotary tables must be (>= n, 64)");
  auto delta = torch::empty({B * H, g.Np}, lse.options());
  auto dqkv = torch::empty({B, n, 3 * H * 64}, q.options());
  const float* rf = nullptr;
  if (rotf.has_value() && rotf->defined()) {
    CHECK_IN((*rotf), torch::kFloat32);
    TORCH_CHECK(rotf->numel() == 64 && n_lang >= 0 && n_pix >= 0 && n_lang + 2 * n_pix <= 32, "attn_bwd_rope: rotf (64,) + axis split");
    rf = rotf->data_ptr<float>();
  }
  dalle::attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                  delta.data_ptr<float>(), nullptr, nullptr, nullptr, g, B * H, cur_stream(),
                  cosT.data_ptr<float>(), sinT.data_ptr<float>(), dqkv.data_ptr(), (float)qscale, rf, (int)n_lang, (int)n_pix,
                  (float)img_text_pos, (float)text_axial);
  return dqkv;
}

// ---------------------------------------------------------------------------------------------
Tensor geglu_fwd(Tensor h) {
  CHECK_IN(h, torch::kBFloat16);
  const long F2 = h.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "geglu: hidden must be a multiple of 16");
  const long M = h.numel() / F2;
  auto sizes = h.sizes().vec();
  sizes.back() = F2 / 2;
  auto out = torch::empty(sizes, h.options());
  dalle::geglu_fwd(h.data_ptr(), out.data_ptr(), M, F2 / 2, cur_stream());
  return out;
}

Tensor geglu_bwd(Tensor h, Tensor dout) {
  CHECK_IN(h, torch::kBFloat16); CHECK_IN(dout, torch::kBFloat16);
  const long F2 = h.size(-1);
  const long M = h.numel() / F2;
  TORCH_CHECK(dout.numel() == M * F2 / 2);
  auto dh = torch::empty_like(h);
  dalle::geglu_bwd(h.data_ptr(), dout.data_ptr(), dh.data_ptr(), M, F2 / 2, cur_stream());
  return dh;
}

// GEGLU backward + FF-in bias grad (column sums of dh) in one pass: returns {dh, dbias(2F, fp32)}, or
// {dh, undefined} after accumulating dbias into the optional sink `gb`
std::vector<Tensor> geglu_bwd_bias(Tensor h, Tensor dout, c10::optional<Tensor> gb) {
  CHECK_IN(h, torch::kBFloat16); CHECK_IN(dout, torch::kBFloat16);
  const long F2 = h.size(-1);
  const long M = h.numel() / F2;
  TORCH_CHECK(F2 % 16 == 0 && dout.numel() == M * F2 / 2);
  auto dh = torch::empty_like(h);
  auto part = torch::empty({512, F2}, h.options().dtype(torch::kFloat32));  // GEGLU_ROW_BLOCKS partial rows
  float* pb = sink_ptr(gb, F2, "geglu_bwd_bias dbias");
  Tensor db;
  if (!pb) {
    db = torch::empty({F2}, h.options().dtype(torch::kFloat32));
    pb = db.data_ptr<float>();
  }
  dalle::geglu_bwd_bias(h.data_ptr(), dout.data_ptr(), dh.data_ptr(), part.data_ptr<float>(),
                        dalle::GradSink{pb, nullptr, nullptr, (int)F2, db.defined() ? 0 : 1}, M, F2 / 2, cur_stream());
  return {dh, db};
}

// FF-out dgrad GEMM with the GEGLU backward + FF-in bias grad in its epilogue (csrc/kernels/gemm.hip
// EPI 2): dy (M, K) bf16, w2t = W2^T (F, K) bf16, h = FF-in pre-activation (M, 2F) -> (dh, dbias).
std::vector<Tensor> ff_dgrad_geglu(Tensor dy, Tensor w2t, Tensor h, c10::optional<Tensor> gb, int64_t stagger) {
  CHECK_IN(dy, torch::kBFloat16); CHECK_IN(w2t, torch::kBFloat16); CHECK_IN(h, torch::kBFloat16);
  TORCH_CHECK(dy.dim() == 2 && w2t.dim() == 2 && h.dim() == 2, "ff_dgrad_geglu: 2-D operands");
  const long M = dy.size(0), K = dy.size(1), F = w2t.size(0);
  TORCH_CHECK(w2t.size(1) == K && h.size(0) == M && h.size(1) == 2 * F, "ff_dgrad_geglu: shape mismatch");
  TORCH_CHECK(M % 256 == 0 && F % 256 == 0 && K % 64 == 0, "ff_dgrad_geglu: M, F multiples of 256 and K of 64");
  auto dh = torch::empty_like(h);
  auto part = torch::empty({M / 128, 2 * F}, h.options().dtype(torch::kFloat32));
  float* pb = sink_ptr(gb, 2 * F, "ff_dgrad_geglu dbias");
  Tensor db;
  if (!pb) {
    db = torch::empty({2 * F}, h.options().dtype(torch::kFloat32));
    pb = db.data_ptr<float>();
  }
  TORCH_CHECK(dalle::gemm_geglu_bwd(dy.data_ptr(), w2t.data_ptr(), h.data_ptr(), dh.data_ptr(), part.data_ptr<float>(), M, F, K,
                                    cur_stream(), (int)stagger), "ff_dgrad_geglu: unsupported shape");
  dalle::column_sum(part.data_ptr<float>(), M / 128, 2 * F, dalle::GradSink{pb, nullptr, nullptr, (int)(2 * F), db.defined() ? 0 : 1},
                    cur_stream());
  return {dh, db};
}

// Row-strided operands of the assembly kernels: the kernels form a tile's base address in 64-bit scalar math but
// a lane's offset inside the tile as 32-bit (row < 256) x (stride * 2 bytes), and a buffer resource's num_records
// from 256 rows of stride: keep every operand's last byte under 2^40 and its row stride under 2^20 elements.
static void check_asm_operand(const Tensor& t, const char* what) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, what, ": 2-D with unit column stride");
  TORCH_CHECK(t.stride(0) >= t.size(1) && t.stride(0) < (1 << 20), what, ": row stride out of range");
  TORCH_CHECK((int64_t)t.size(0) * t.stride(0) * 2 < (1ll << 40), what, ": operand exceeds 2^40 bytes");
}

// The same on the assembly kernel (csrc/asm/gen_gemm.py kernel_geglu_bwd): K a multiple of 128 and >= 1024 (the
// unrolled successor K-steps), M and F multiples of 256
std::vector<Tensor> asm_ff_dgrad_geglu(Tensor dy, Tensor w2t, Tensor h, c10::optional<Tensor> gb) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == torch::kBFloat16 && w2t.scalar_type() == torch::kBFloat16, "asm_ff_dgrad_geglu: bf16");
  CHECK_IN(h, torch::kBFloat16);
  TORCH_CHECK(dy.dim() == 2 && w2t.dim() == 2 && h.dim() == 2 && dy.stride(1) == 1 && w2t.stride(1) == 1, "asm_ff_dgrad_geglu: 2-D, K-contiguous");
  const long M = dy.size(0), K = dy.size(1), F = w2t.size(0);
  TORCH_CHECK(w2t.size(1) == K && h.size(0) == M && h.size(1) == 2 * F, "asm_ff_dgrad_geglu: shape mismatch");
  TORCH_CHECK(K >= 1024 && K % 128 == 0 && M % 256 == 0 && F % 256 == 0,
              "asm_ff_dgrad_geglu: K a multiple of 128 (>= 1024), M and F multiples of 256");
  check_asm_operand(dy, "asm_ff_dgrad_geglu dy");
  check_asm_operand(w2t, "asm_ff_dgrad_geglu w2t");
  TORCH_CHECK(h.is_contiguous(), "asm_ff_dgrad_geglu: h contiguous");
  check_asm_operand(h, "asm_ff_dgrad_geglu h");
  auto dh = torch::empty_like(h);
  auto part = torch::empty({M / 128, 2 * F}, h.options().dtype(torch::kFloat32));
  float* pb = sink_ptr(gb, 2 * F, "asm_ff_dgrad_geglu dbias");
  Tensor db;
  if (!pb) {
    db = torch::empty({2 * F}, h.options().dtype(torch::kFloat32));
    pb = db.data_ptr<float>();
  }
  TORCH_CHECK(dalle::asm_gemm_nt("dalle_gemm_nt_geglu_bwd", dy.data_ptr(), w2t.data_ptr(), dh.data_ptr(), h.data_ptr(), part.data_ptr(),
                                 nullptr, (int)M, (int)F, (int)K, (int)dy.stride(0), (int)w2t.stride(0), (int)(2 * F), (int)F, 0,
                                 cur_stream()), "asm_ff_dgrad_geglu: launch failed");
  dalle::column_sum(part.data_ptr<float>(), M / 128, 2 * F, dalle::GradSink{pb, nullptr, nullptr, (int)(2 * F), db.defined() ? 0 : 1},
                    cur_stream());
  return {dh, db};
}

void scale_residual_(Tensor x, Tensor y, Tensor scale) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(y, torch::kBFloat16); CHECK_IN(scale, torch::kFloat32);
  const long D = x.size(-1);
  TORCH_CHECK(D % 8 == 0 && y.numel() == x.numel() && scale.numel() == D);
  dalle::scale_residual(x.data_ptr<float>(), y.data_ptr(), scale.data_ptr<float>(), x.data_ptr<float>(), x.numel() / D, D,
                        cur_stream());
}

Tensor transpose_bf16(Tensor w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kFloat32 && w.dim() == 2 && w.is_contiguous(),
              "transpose_bf16: contiguous fp32 matrix expected");
  TORCH_CHECK(w.size(0) < (1L << 31) && w.size(1) < (1L << 31), "transpose_bf16: matrix too large");
  auto wt = torch::empty({w.size(1), w.size(0)}, w.options().dtype(torch::kBFloat16));
  if (w.numel()) dalle::transpose_cast_bf16(w.data_ptr<float>(), wt.data_ptr(), (int)w.size(0), (int)w.size(1), cur_stream());
  return wt;
}

Tensor transpose_act_bf16(Tensor x) {
  CHECK_IN(x, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 2, "transpose_act_bf16: bf16 matrix expected");
  TORCH_CHECK(x.size(0) % 64 == 0 && x.size(1) % 64 == 0, "transpose_act_bf16: both dims must be multiples of 64");
  TORCH_CHECK(x.size(0) < (1L << 31) && x.size(1) < (1L << 31), "transpose_act_bf16: matrix too large");
  auto xt = torch::empty({x.size(1), x.size(0)}, x.options());
  if (x.numel()) dalle::transpose_bf16(x.data_ptr(), xt.data_ptr(), (int)x.size(0), (int)x.size(1), cur_stream());
  return xt;
}

void scale_residual_out(Tensor x, Tensor y, Tensor scale, Tensor out) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(y, torch::kBFloat16); CHECK_IN(scale, torch::kFloat32); CHECK_IN(out, torch::kFloat32);
  const long D = x.size(-1);
  TORCH_CHECK(D % 8 == 0 && y.numel() == x.numel() && out.numel() == x.numel() && scale.numel() == D);
  dalle::scale_residual(x.data_ptr<float>(), y.data_ptr(), scale.data_ptr<float>(), out.data_ptr<float>(), x.numel() / D, D,
                        cur_stream());
}

// LayerScale(+residual) backward: dy = bf16(scale * g) and the column sums (sum g*y, sum g).
// Without sinks returns {dy, dscale, gsum}. With the optional sinks it accumulates dscale into
// `gscale` and scale * gsum (the bias grad of a GEMM whose output was y) into `gbias` (if given),
// returning {dy, undefined, undefined}.
std::vector<Tensor> scale_residual_bwd(Tensor g, Tensor y, Tensor scale, c10::optional<Tensor> gscale,
                                       c10::optional<Tensor> gbias) {
  CHECK_IN(g, torch::kFloat32); CHECK_IN(y, torch::kBFloat16); CHECK_IN(scale, torch::kFloat32);
  const long D = g.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 2048 && y.numel() == g.numel() && scale.numel() == D);
  float* ps = sink_ptr(gscale, D, "scale_residual_bwd dscale");
  float* pb = sink_ptr(gbias, D, "scale_residual_bwd dbias");
  TORCH_CHECK(ps || !pb, "scale_residual_bwd: a bias sink needs a scale sink");
  auto dy = torch::empty(g.sizes(), y.options());
  auto ws = torch::empty({(512 + (ps ? 0 : 1)) * 2 * D}, g.options());  // 512 partial rows (+ the reduced row)
  float* red = ws.data_ptr<float>() + 512 * 2 * D;
  dalle::GradSink sink = ps ? dalle::GradSink{ps, pb, scale.data_ptr<float>(), (int)D, 1}
                            : dalle::GradSink{red, red + D, nullptr, (int)D, 0};
  dalle::scale_residual_bwd(g.data_ptr<float>(), y.data_ptr(), scale.data_ptr<float>(), dy.data_ptr(), ws.data_ptr<float>(), sink,
                            g.numel() / D, D, cur_stream());
  if (ps) return {dy, Tensor(), Tensor()};
  return {dy, ws.slice(0, 512 * 2 * D, 512 * 2 * D + D), ws.slice(0, 512 * 2 * D + D, 513 * 2 * D)};
}

// acc [+]= part.sum(0) for a (s, ...) fp32 split-K partial buffer
void splitk_accum_(Tensor acc, Tensor part, bool accumulate) {
  CHECK_IN(acc, torch::kFloat32); CHECK_IN(part, torch::kFloat32);
  const long n = acc.numel();
  TORCH_CHECK(part.dim() >= 1 && part.numel() == part.size(0) * n && n % 4 == 0, "splitk_accum: shape mismatch");
  dalle::splitk_accum(part.data_ptr<float>(), acc.data_ptr<float>(), n, (int)part.size(0), accumulate ? 1 : 0, cur_stream());
}

// C = A . B^T (+ bias): A (M, K), B (N, K) bf16, both K-contiguous; M, N multiples of 256, K of 64
Tensor gemm_nt(Tensor A, Tensor B, c10::optional<Tensor> bias, int64_t variant) {
  CHECK_IN(A, torch::kBFloat16); CHECK_IN(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt: A (M, K) and B (N, K)");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 64 == 0, "gemm_nt: M, N multiples of 256 and K of 64");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_IN((*bias), torch::kBFloat16);
    TORCH_CHECK(bias->numel() == N);
    bp = bias->data_ptr();
  }
  auto C = torch::empty({M, N}, A.options());
  TORCH_CHECK(dalle::gemm_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), bp, M, N, K, (int)variant, cur_stream()));
  return C;
}

// ---- hand-scheduled assembly GEMMs (csrc/asm/gen_gemm.py): C = A . B^T (+ fp32 bias) ----
// A (M, K), B (N, K) bf16 (row strides free, K-contiguous); M, N multiples of 256, K of 128, K >= 256
// out (M, N) fp32 (+)= A^T B: A (Ktot, M), B (Ktot, N) bf16 token-major (unit column stride); the reduction over
// the Ktot tokens runs as `splits` K-ranges on the assembly TN kernel, whose fp32 partial slabs splitk_accum folds
// into out in a fixed order (deterministic)
void asm_wgrad_(Tensor out, Tensor A, Tensor B, int64_t splits, bool accumulate) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "asm_wgrad: bf16 cuda");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0), "asm_wgrad: A (Ktot, M), B (Ktot, N)");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "asm_wgrad: unit column stride");
  CHECK_IN(out, torch::kFloat32);
  const int Ktot = A.size(0), M = A.size(1), N = B.size(1);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N, "asm_wgrad: out (M, N)");
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && splits > 0 && Ktot % splits == 0 && (Ktot / splits) % 128 == 0 &&
                  Ktot / splits >= 256, "asm_wgrad: M, N multiples of 256, Ktot / splits a multiple of 128 (>= 256)");
  TORCH_CHECK((int64_t)Ktot * A.stride(0) * 2 < (1ll << 40) && (int64_t)Ktot * B.stride(0) * 2 < (1ll << 40) &&
                  A.stride(0) < (1 << 23) && B.stride(0) < (1 << 23), "asm_wgrad: strides");
  Tensor part = torch::empty({splits, M, N}, out.options());
  TORCH_CHECK(dalle::asm_gemm_tn(A.data_ptr(), B.data_ptr(), part.data_ptr(), M, N, Ktot, (int)A.stride(0), (int)B.stride(0),
                                 (int)splits, cur_stream()),
              "asm_wgrad: launch failed");
  dalle::splitk_accum(part.data_ptr<float>(), out.data_ptr<float>(), (long)M * N, (int)splits, accumulate ? 1 : 0, cur_stream());
}

// QKV + rotary on the assembly kernel: h (M, d) bf16, w (3 H 64, d) bf16 (d a multiple of 128, >= 1024), cs3 (3, n + 1, 32, 2) fp32 (q's
// (cos, sin) pre-scaled, k's and v's plain: all three rotated) -> q, k, v (B H, Np, 64) storage views (padding rows zeroed)
std::vector<Tensor> asm_qkv_rope(Tensor h, Tensor w, Tensor cs3, int64_t T, int64_t S, int64_t H, int64_t n, bool col_major) {
  CHECK_IN(h, torch::kBFloat16); CHECK_IN(w, torch::kBFloat16); CHECK_IN(cs3, torch::kFloat32);
  TORCH_CHECK(h.dim() == 2 && w.dim() == 2 && w.size(0) == 3 * H * 64 && w.size(1) == h.size(1), "asm_qkv_rope: shapes");
  const int M = h.size(0), K = h.size(1);
  check_asm_operand(h, "asm_qkv_rope h");
  check_asm_operand(w, "asm_qkv_rope w");
  TORCH_CHECK(cs3.dim() == 4 && cs3.size(0) == 3 && cs3.size(1) >= n + 1 && cs3.size(2) == 32 && cs3.size(3) == 2,
              "asm_qkv_rope: cs3 (3, n + 1, 32, 2)");
  auto g = make_attn_geom(T, S, n, 1, H, 0);
  const int B = M / n;
  auto qkv = torch::empty({3, B * H, g.Np, 64}, h.options());
  TORCH_CHECK(dalle::asm_qkv_rope(col_major, h.data_ptr(), w.data_ptr(), qkv.data_ptr(), cs3.data_ptr<float>(), M, (int)w.size(0), K,
                                  (int)h.stride(0), (int)w.stride(0), (int)n, (int)T, g.Tp, g.Np, (int)H, ilog2((int)S), cur_stream()),
              "asm_qkv_rope: unsupported shape");
  auto q = qkv[0], k = qkv[1], v = qkv[2];
  dalle::rope_pad_zero(q.data_ptr(), k.data_ptr(), v.data_ptr(), g.Tp, T, g.Np, B * H, cur_stream());
  return {q, k, v};
}

// FF-in GEMM + GEGLU on the assembly kernel: x (M, d) bf16, w1p (2F, d) bf16 (d a multiple of 128, >= 1024) = W1 with its rows in the
// interleaved [value 8 | gate 8] order (hip_ops.ff_in_perm), b1p (2F,) fp32 in the same order ->
// a (M, 2F) bf16 pre-activation in the ORIGINAL [value | gate] order, u (M, F) = value * gelu(gate)
std::vector<Tensor> asm_ff_in_geglu(Tensor x, Tensor w1p, Tensor b1p) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && w1p.scalar_type() == torch::kBFloat16, "asm_ff_in_geglu: bf16");
  TORCH_CHECK(x.dim() == 2 && w1p.dim() == 2 && x.size(1) == w1p.size(1) && x.stride(1) == 1 && w1p.stride(1) == 1,
              "asm_ff_in_geglu: x (M, K), w1p (2F, K), K-contiguous");
  CHECK_IN(b1p, torch::kFloat32);
  const int M = x.size(0), N = w1p.size(0), K = x.size(1);
  TORCH_CHECK(K >= 1024 && K % 128 == 0 && M % 256 == 0 && N % 256 == 0 && b1p.numel() == N,
              "asm_ff_in_geglu: K a multiple of 128 (>= 1024), M and 2F multiples of 256");
  check_asm_operand(x, "asm_ff_in_geglu x");
  check_asm_operand(w1p, "asm_ff_in_geglu w1p");
  auto a = torch::empty({M, N}, x.options());
  auto u = torch::empty({M, N / 2}, x.options());
  TORCH_CHECK(dalle::asm_gemm_nt("dalle_gemm_nt_geglu", x.data_ptr(), w1p.data_ptr(), a.data_ptr(), b1p.data_ptr(), u.data_ptr(), nullptr,
                                 M, N, K, (int)x.stride(0), (int)w1p.stride(0), N, N / 2, 0, cur_stream()),
              "asm_ff_in_geglu: launch failed");
  return {a, u};
}

Tensor asm_gemm(Tensor A, Tensor B, c10::optional<Tensor> bias, c10::optional<Tensor> out) {
  TORCH_CHECK(A.is_cuda() && A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "asm_gemm: bf16 cuda");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "asm_gemm: A (M, K) and B (N, K)");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "asm_gemm: K-contiguous operands");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K >= 256, "asm_gemm: M, N multiples of 256, K of 128 (>= 256)");
  check_asm_operand(A, "asm_gemm A");
  check_asm_operand(B, "asm_gemm B");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_IN((*bias), torch::kFloat32);
    TORCH_CHECK(bias->numel() == N, "asm_gemm: bias (N,) fp32");
    bp = bias->data_ptr();
  }
  Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == torch::kBFloat16 && C.dim() == 2 && C.size(0) == M && C.size(1) == N && C.stride(1) == 1,
                "asm_gemm: out (M, N) bf16");
  } else {
    C = torch::empty({M, N}, A.options());
  }
  TORCH_CHECK(dalle::asm_gemm_nt(bp ? "dalle_gemm_nt_bias" : "dalle_gemm_nt_plain", A.data_ptr(), B.data_ptr(), C.data_ptr(), bp,
                                 nullptr, nullptr, M, N, K, (int)A.stride(0), (int)B.stride(0), (int)C.stride(0), 0, 0, cur_stream()),
              "asm_gemm: launch failed");
  return C;
}

// ---- persistent GEMM family (csrc/kernels/gemm_pt.hip): transposed accumulators, register-direct epilogues ----
// C (M, N) = A (M, K) . B (N, K)^T (+ bias); variant 5 = main loop only (measurement)
Tensor gemm_pt(Tensor A, Tensor B, c10::optional<Tensor> bias, int64_t variant, int64_t group) {
  CHECK_IN(A, torch::kBFloat16); CHECK_IN(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_pt: A (M, K) and B (N, K)");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && K >= 128, "gemm_pt: M, N multiples of 256, K of 64 (>= 128)");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    if (variant == 40 || variant == 41) {  // measurement: per-workgroup timestamps (int64, 5 per tile)
      CHECK_IN((*bias), torch::kLong);
      TORCH_CHECK(bias->numel() >= (int64_t)(M / 256) * (N / 256) * 5, "gemm_pt: stamps (tiles * 5,)");
    } else {
      CHECK_IN((*bias), torch::kBFloat16);
      TORCH_CHECK(bias->numel() == N, "gemm_pt: bias (N,)");
    }
    bp = bias->data_ptr();
  }
  TORCH_CHECK(variant != 40 && variant != 41 || bp != nullptr, "gemm_pt: stamp variants need the stamp buffer");
  auto C = torch::empty({M, N}, A.options());
  TORCH_CHECK(dalle::gemm_pt(A.data_ptr(), B.data_ptr(), C.data_ptr(), bp, M, N, K, N, (int)variant, (int)group, cur_stream()),
              "gemm_pt: unsupported shape");
  return C;
}

// QKV projection + rotary (persistent kernel): cs = (n + 1, 32, 2) fp32 (cos, sin) per rotary pair
std::vector<Tensor> qkv_rope_pt(Tensor h, Tensor w, Tensor cs, int64_t T, int64_t S, int64_t H, int64_t n, bool col_major,
                                double qscale, int64_t persist) {
  CHECK_IN(h, torch::kBFloat16); CHECK_IN(w, torch::kBFloat16); CHECK_IN(cs, torch::kFloat32);
  TORCH_CHECK(h.dim() == 2 && w.dim() == 2 && w.size(0) == 3 * H * 64 && w.size(1) == h.size(1), "qkv_rope_pt: shapes");
  const int M = h.size(0), K = h.size(1);
  TORCH_CHECK(M % n == 0 && M % 256 == 0 && (3 * H * 64) % 256 == 0 && K % 64 == 0 && K >= 128, "qkv_rope_pt: tile multiples");
  TORCH_CHECK(cs.dim() == 3 && cs.size(0) >= n && cs.size(1) == 32 && cs.size(2) == 2, "qkv_rope_pt: cs (n + 1, 32, 2)");
  auto g = make_attn_geom(T, S, n, 1, H, 0);
  const int B = M / n;
  auto opts = h.options();
  auto q = torch::empty({B * H, g.Np, 64}, opts);
  auto k = torch::empty({B * H, g.Np, 64}, opts);
  auto v = torch::empty({B * H, g.Np, 64}, opts);
  TORCH_CHECK(dalle::gemm_pt_qkv_rope(h.data_ptr(), w.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cs.data_ptr<float>(), M,
                                      K, H, T, S, n, col_major ? 1 : 0, (float)qscale, cur_stream(), (int)persist),
              "qkv_rope_pt: unsupported shape");
  dalle::rope_pad_zero(q.data_ptr(), k.data_ptr(), v.data_ptr(), g.Tp, T, g.Np, B * H, cur_stream());
  return {q, k, v};
}

// FF-out dgrad + GEGLU backward (persistent kernel): dy (M, K), w2t = W2^T (F, K), h (M, 2F) -> (dh, dbias)
std::vector<Tensor> ff_dgrad_geglu_pt(Tensor dy, Tensor w2t, Tensor h, c10::optional<Tensor> gb, int64_t persist) {
  CHECK_IN(dy, torch::kBFloat16); CHECK_IN(w2t, torch::kBFloat16); CHECK_IN(h, torch::kBFloat16);
  TORCH_CHECK(dy.dim() == 2 && w2t.dim() == 2 && h.dim() == 2, "ff_dgrad_geglu_pt: 2-D operands");
  const long M = dy.size(0), K = dy.size(1), F = w2t.size(0);
  TORCH_CHECK(w2t.size(1) == K && h.size(0) == M && h.size(1) == 2 * F, "ff_dgrad_geglu_pt: shape mismatch");
  TORCH_CHECK(M % 256 == 0 && F % 256 == 0 && K % 64 == 0 && K >= 128, "ff_dgrad_geglu_pt: M, F multiples of 256, K of 64");
  auto dh = torch::empty_like(h);
  auto part = torch::empty({M / 64, 2 * F}, h.options().dtype(torch::kFloat32));
  float* pb = sink_ptr(gb, 2 * F, "ff_dgrad_geglu_pt dbias");
  Tensor db;
  if (!pb) {
    db = torch::empty({2 * F}, h.options().dtype(torch::kFloat32));
    pb = db.data_ptr<float>();
  }
  TORCH_CHECK(dalle::gemm_pt_geglu_bwd(dy.data_ptr(), w2t.data_ptr(), h.data_ptr(), dh.data_ptr(), part.data_ptr<float>(), M, F, K,
                                       cur_stream(), (int)persist), "ff_dgrad_geglu_pt: unsupported shape");
  dalle::column_sum(part.data_ptr<float>(), M / 64, 2 * F, dalle::GradSink{pb, nullptr, nullptr, (int)(2 * F), db.defined() ? 0 : 1},
                    cur_stream());
  return {dh, db};
}

// FF-in GEMM + GEGLU forward (persistent kernel): x (M, K), w1i / b1i = W1 / b1 rows interleaved per 64-row
// group ([32 value | 32 gate]) -> a (M, 2F) pre-activation in the original [value | gate] order, u (M, F)
std::vector<Tensor> ff_in_geglu_pt(Tensor x, Tensor w1i, c10::optional<Tensor> b1i, int64_t persist) {
  CHECK_IN(x, torch::kBFloat16); CHECK_IN(w1i, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && w1i.dim() == 2 && x.size(1) == w1i.size(1), "ff_in_geglu_pt: x (M, K), w1i (2F, K)");
  const int M = x.size(0), K = x.size(1), F2 = w1i.size(0);
  TORCH_CHECK(M % 256 == 0 && F2 % 256 == 0 && K % 64 == 0 && K >= 128, "ff_in_geglu_pt: M, 2F multiples of 256, K of 64");
  const void* bp = nullptr;
  if (b1i.has_value() && b1i->defined()) {
    CHECK_IN((*b1i), torch::kBFloat16);
    TORCH_CHECK(b1i->numel() == F2, "ff_in_geglu_pt: bias (2F,)");
    bp = b1i->data_ptr();
  }
  auto a = torch::empty({M, F2}, x.options());
  auto u = torch::empty({M, F2 / 2}, x.options());
  TORCH_CHECK(dalle::gemm_pt_geglu_fwd(x.data_ptr(), w1i.data_ptr(), bp, a.data_ptr(), u.data_ptr(), M, F2 / 2, K, cur_stream(),
                                       (int)persist),
              "ff_in_geglu_pt: unsupported shape");
  return {a, u};
}

Tensor permlane16_probe() {
  auto out = torch::empty({128}, torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA));
  CHECK_CUDA(out);
  dalle::permlane16_probe((unsigned*)out.data_ptr<int>(), cur_stream());
  return out;
}

// ---- decode-step skinny GEMMs (M <= 64): one launch each, epilogue fused ----
static dalle::SkinnyArgs skinny_prep(const Tensor& X, const Tensor& W, const c10::optional<Tensor>& bias, int64_t nout,
                                     int nb, const Tensor& cnt, Tensor& ws) {
  CHECK_CUDA(X); CHECK_DT(X, torch::kBFloat16); CHECK_IN(W, torch::kBFloat16); CHECK_IN(cnt, torch::kInt32);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1 && W.dim() == 2 && X.size(1) == W.size(1), "skinny: X (M, K), W (N, K)");
  const int M = X.size(0), K = X.size(1);
  TORCH_CHECK(M >= 1 && M <= 64, "skinny: 1 <= M <= 64");
  TORCH_CHECK(nout % 16 == 0 && W.size(0) == nout * nb && K % 128 == 0, "skinny: N % 16, K % 128");
  TORCH_CHECK(cnt.numel() >= nout / 16, "skinny: counter buffer too small");
  TORCH_CHECK(X.stride(0) % 8 == 0, "skinny: X rows must be 16-byte aligned");
  dalle::SkinnyArgs a{};
  a.X = X.data_ptr();
  a.W = W.data_ptr();
  a.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_IN((*bias), torch::kBFloat16);
    TORCH_CHECK(bias->numel() == nout * nb, "skinny: bias size");
    a.bias = bias->data_ptr();
  }
  a.M = M; a.N = nout; a.K = K; a.ldx = X.stride(0);
  a.KS = dalle::skinny_ks(M, nout, K, nb);
  const int mpad = M <= 16 ? 16 : (M <= 32 ? 32 : 64);
  if (a.KS > 1) ws = torch::empty({(int64_t)a.KS * nout * mpad * nb}, X.options().dtype(torch::kFloat32));
  a.ws = a.KS > 1 ? ws.data_ptr<float>() : nullptr;
  a.cnt = cnt.data_ptr<int>();
  return a;
}

Tensor skinny_linear(Tensor X, Tensor W, c10::optional<Tensor> bias, bool out_f32, Tensor cnt) {
  Tensor ws;
  auto a = skinny_prep(X, W, bias, W.size(0), 1, cnt, ws);
  auto out = torch::empty({X.size(0), W.size(0)}, X.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  a.out = out.data_ptr();
  a.out_f32 = out_f32;
  TORCH_CHECK(dalle::skinny_gemm(0, a, cur_stream()), "skinny_linear: unsupported shape");
  return out;
}

// split-K partial slabs (KS, M, N) fp32 of Y = X W^T for a consumer that sums them (no bias)
Tensor skinny_partials(Tensor X, Tensor W) {
  CHECK_CUDA(X); CHECK_DT(X, torch::kBFloat16); CHECK_IN(W, torch::kBFloat16);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1 && W.dim() == 2 && X.size(1) == W.size(1), "skinny_partials: X (M, K), W (N, K)");
  const int M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && N % 16 == 0 && K % 128 == 0 && X.stride(0) % 8 == 0, "skinny_partials: shapes");
  const int KS = dalle::skinny_partials_ks(M, N, K);
  auto part = torch::empty({KS, M, N}, X.options().dtype(torch::kFloat32));
  dalle::SkinnyArgs a{};
  a.X = X.data_ptr(); a.W = W.data_ptr(); a.M = M; a.N = N; a.K = K; a.ldx = X.stride(0); a.KS = KS;
  a.out = part.data_ptr();
  TORCH_CHECK(dalle::skinny_partials(a, cur_stream()), "skinny_partials: unsupported shape");
  return part;
}

// The residual projection's split-K slabs with the NEXT LayerNorm in the same launch (skinny EPI 5): x +=
// scale * (X W^T + bias), then y = shift(LN(x)) with the LN history row at *pos -- decode_ln_shift_ folded
// into the projection's last workgroups. cnt: this launch site's ticket word (int32, zeroed once per
// generate call), err: set to 1 if a tail gave up waiting.
void skinny_partials_ln_(Tensor X, Tensor W, c10::optional<Tensor> bias, Tensor scale, Tensor x, Tensor ln_w, Tensor ln_b,
                         Tensor hist, Tensor y, Tensor pos, int64_t T, int64_t S, bool shift, Tensor cnt, Tensor err) {
  CHECK_CUDA(X); CHECK_DT(X, torch::kBFloat16); CHECK_IN(W, torch::kBFloat16);
  CHECK_IN(scale, torch::kFloat32); CHECK_IN(x, torch::kFloat32); CHECK_IN(ln_w, torch::kFloat32); CHECK_IN(ln_b, torch::kFloat32);
  CHECK_IN(hist, torch::kBFloat16); CHECK_IN(y, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  CHECK_CUDA(cnt); CHECK_DT(cnt, torch::kInt32); CHECK_CUDA(err); CHECK_DT(err, torch::kInt32);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1 && W.dim() == 2 && X.size(1) == W.size(1), "skinny_partials_ln_: X (M, K), W (N, K)");
  const int M = X.size(0), K = X.size(1), N = W.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && N % 16 == 0 && K % 128 == 0 && X.stride(0) % 8 == 0, "skinny_partials_ln_: shapes");
  TORCH_CHECK(dalle::skinny_partials_ln_ok(M, N, K), "skinny_partials_ln_: no tail tiling for this shape");
  TORCH_CHECK(x.numel() == (int64_t)M * N && y.numel() == (int64_t)M * N && scale.numel() == N && ln_w.numel() == N &&
              ln_b.numel() == N, "skinny_partials_ln_: row / parameter sizes");
  TORCH_CHECK(hist.dim() == 3 && hist.size(0) == M && hist.size(2) == N, "skinny_partials_ln_: hist (M, n, N)");
  TORCH_CHECK(cnt.numel() >= 1 && err.numel() >= 1, "skinny_partials_ln_: counter / error words");
  const int KS = dalle::skinny_partials_ks(M, N, K);
  auto part = torch::empty({KS, M, N}, X.options().dtype(torch::kFloat32));
  dalle::SkinnyArgs a{};
  a.X = X.data_ptr(); a.W = W.data_ptr(); a.M = M; a.N = N; a.K = K; a.ldx = X.stride(0); a.KS = KS;
  a.out = part.data_ptr();
  a.bias = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_IN((*bias), torch::kBFloat16);
    TORCH_CHECK(bias->numel() == N, "skinny_partials_ln_: bias size");
    a.bias = bias->data_ptr();
  }
  a.scale = scale.data_ptr<float>();
  a.resid = x.data_ptr<float>();
  a.ln_w = ln_w.data_ptr<float>(); a.ln_b = ln_b.data_ptr<float>();
  a.hist = hist.data_ptr(); a.y = y.data_ptr();
  a.pos = pos.data_ptr<int>(); a.n = hist.size(1);
  a.T = T; a.S = S; a.shift = shift ? 1 : 0;
  a.cnt = cnt.data_ptr<int>();
  a.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  TORCH_CHECK(dalle::skinny_partials_ln(a, cur_stream()), "skinny_partials_ln_: unsupported shape");
}

Tensor skinny_geglu(Tensor X, Tensor W, c10::optional<Tensor> bias, Tensor cnt) {
  TORCH_CHECK(W.size(0) % 2 == 0, "skinny_geglu: W holds the value and gate halves");
  Tensor ws;
  auto a = skinny_prep(X, W, bias, W.size(0) / 2, 2, cnt, ws);
  auto out = torch::empty({X.size(0), W.size(0) / 2}, X.options().dtype(torch::kBFloat16));
  a.out = out.data_ptr();
  TORCH_CHECK(dalle::skinny_gemm(1, a, cur_stream()), "skinny_geglu: unsupported shape");
  return out;
}

void skinny_residual_(Tensor resid, Tensor X, Tensor W, c10::optional<Tensor> bias, Tensor scale, Tensor cnt) {
  CHECK_IN(resid, torch::kFloat32); CHECK_IN(scale, torch::kFloat32);
  Tensor ws;
  auto a = skinny_prep(X, W, bias, W.size(0), 1, cnt, ws);
  TORCH_CHECK(resid.dim() == 2 && resid.size(0) == X.size(0) && resid.size(1) == W.size(0), "skinny_residual_: resid (M, N)");
  TORCH_CHECK(scale.numel() == W.size(0), "skinny_residual_: scale (N,)");
  a.resid = resid.data_ptr<float>();
  a.scale = scale.data_ptr<float>();
  TORCH_CHECK(dalle::skinny_gemm(2, a, cur_stream()), "skinny_residual_: unsupported shape");
}

void skinny_qkv_rope_(Tensor X, Tensor W, Tensor cosT, Tensor sinT, Tensor q, Tensor kc, Tensor vc, Tensor pos, int64_t H,
                      double qscale, Tensor cnt) {
  CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32); CHECK_IN(q, torch::kBFloat16);
  CHECK_IN(kc, torch::kBFloat16); CHECK_IN(vc, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  TORCH_CHECK(W.size(0) == 3 * H * 64, "skinny_qkv_rope_: W (3*H*64, K)");
  const int M = X.size(0);
  TORCH_CHECK(q.numel() == (int64_t)M * H * 64, "skinny_qkv_rope_: q (M*H, 64)");
  TORCH_CHECK(kc.dim() == 3 && kc.size(0) == M * H && kc.size(2) == 64 && vc.sizes() == kc.sizes(),
              "skinny_qkv_rope_: caches (M*H, n, 64)");
  TORCH_CHECK(cosT.size(0) >= kc.size(1) && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes(), "skinny_qkv_rope_: tables");
  Tensor ws;
  auto a = skinny_prep(X, W, c10::nullopt, W.size(0), 1, cnt, ws);
  a.q = q.data_ptr(); a.kc = kc.data_ptr(); a.vc = vc.data_ptr();
  a.cosT = cosT.data_ptr<float>(); a.sinT = sinT.data_ptr<float>();
  a.pos = pos.data_ptr<int>();
  a.H = H; a.n = kc.size(1); a.qscale = (float)qscale;
  TORCH_CHECK(dalle::skinny_gemm(3, a, cur_stream()), "skinny_qkv_rope_: unsupported shape");
}

// QKV projection with the rotary fused into the GEMM epilogue: h (B*n, K) . Wqkv (3*H*64, K)^T ->
// q (pre-scaled), k, v in the padded attention storage layout (B*H, Np, 64); padding rows zeroed.
std::vector<Tensor> qkv_rope(Tensor h, Tensor w, Tensor cosT, Tensor sinT, int64_t T, int64_t S, int64_t H, int64_t n,
                             bool col_major, double qscale) {
  CHECK_IN(h, torch::kBFloat16); CHECK_IN(w, torch::kBFloat16); CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  TORCH_CHECK(h.dim() == 2 && w.dim() == 2 && w.size(0) == 3 * H * 64 && w.size(1) == h.size(1), "qkv_rope: shapes");
  const int M = h.size(0), K = h.size(1);
  TORCH_CHECK(M % n == 0 && M % 256 == 0 && (3 * H * 64) % 256 == 0 && K % 64 == 0, "qkv_rope: tile multiples");
  TORCH_CHECK(cosT.size(0) >= n && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes());
  auto g = make_attn_geom(T, S, n, 1, H, 0);
  const int B = M / n;
  auto opts = h.options();
  auto q = torch::empty({B * H, g.Np, 64}, opts);
  auto k = torch::empty({B * H, g.Np, 64}, opts);
  auto v = torch::empty({B * H, g.Np, 64}, opts);
  TORCH_CHECK(dalle::gemm_qkv_rope(h.data_ptr(), w.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cosT.data_ptr<float>(),
                                   sinT.data_ptr<float>(), M, K, H, T, S, n, col_major ? 1 : 0, (float)qscale, cur_stream()));
  return {q, k, v};
}

// Uniform 8-bit quantisation (collaborative averaging compression): x fp32 -> (q uint8, codebook[256] fp32)
std::vector<Tensor> uq8_compress(Tensor x) {
  CHECK_IN(x, torch::kFloat32);
  const long n = x.numel();
  TORCH_CHECK(n > 0, "uq8_compress: empty tensor");
  auto q = torch::empty({n}, x.options().dtype(torch::kUInt8));
  auto cb = torch::empty({256}, x.options());
  auto ws = torch::empty({(long)dalle::uq8_workspace_bytes()}, x.options().dtype(torch::kUInt8));
  dalle::uq8_compress(x.data_ptr<float>(), n, q.data_ptr<uint8_t>(), cb.data_ptr<float>(), ws.data_ptr(), cur_stream());
  return {q, cb};
}

// out [+]= weight * codebook[q]
void uq8_dequant_(Tensor q, Tensor codebook, Tensor out, double weight, bool accumulate) {
  CHECK_IN(q, torch::kUInt8); CHECK_IN(codebook, torch::kFloat32); CHECK_IN(out, torch::kFloat32);
  TORCH_CHECK(codebook.numel() == 256 && out.numel() == q.numel());
  dalle::uq8_dequant(q.data_ptr<uint8_t>(), codebook.data_ptr<float>(), out.data_ptr<float>(), q.numel(), (float)weight,
                     accumulate ? 1 : 0, cur_stream());
}

// Segmented uniform 8-bit (one codebook per part, one launch for all parts). The part tables are
// device tensors built once per averaging plan; their extents were checked on the host when the
// plan was built (x_end = max(x_off + len), q_end = max(q_off + len)) and are re-checked here
// against the buffers, so no part can read or write outside them.
void uq8_seg_compress(Tensor x, Tensor x_off, Tensor q_off, Tensor len, Tensor q, Tensor codebook, int64_t x_end,
                      int64_t q_end) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(x_off, torch::kInt64); CHECK_IN(q_off, torch::kInt64);
  CHECK_IN(len, torch::kInt32); CHECK_IN(q, torch::kUInt8); CHECK_IN(codebook, torch::kFloat32);
  const long nseg = len.numel();
  TORCH_CHECK(x_off.numel() == nseg && q_off.numel() == nseg && codebook.numel() == nseg * 256, "uq8_seg_compress: table sizes");
  TORCH_CHECK(x_end <= x.numel() && q_end <= q.numel(), "uq8_seg_compress: parts exceed the buffers");
  dalle::uq8_seg_compress(x.data_ptr<float>(), x_off.data_ptr<int64_t>(), q_off.data_ptr<int64_t>(), len.data_ptr<int>(),
                          (int)nseg, q.data_ptr<uint8_t>(), codebook.data_ptr<float>(), cur_stream());
}

void uq8_seg_dequant_(Tensor q, Tensor q_off, Tensor codebook, Tensor out_off, Tensor len, Tensor out, double weight,
                      bool accumulate, int64_t q_end, int64_t out_end) {
  CHECK_IN(q, torch::kUInt8); CHECK_IN(q_off, torch::kInt64); CHECK_IN(codebook, torch::kFloat32);
  CHECK_IN(out_off, torch::kInt64); CHECK_IN(len, torch::kInt32); CHECK_IN(out, torch::kFloat32);
  const long nseg = len.numel();
  TORCH_CHECK(q_off.numel() == nseg && out_off.numel() == nseg && codebook.numel() == nseg * 256, "uq8_seg_dequant: table sizes");
  TORCH_CHECK(q_end <= q.numel() && out_end <= out.numel(), "uq8_seg_dequant: parts exceed the buffers");
  dalle::uq8_seg_dequant(q.data_ptr<uint8_t>(), q_off.data_ptr<int64_t>(), codebook.data_ptr<float>(), out_off.data_ptr<int64_t>(),
                         len.data_ptr<int>(), (int)nseg, out.data_ptr<float>(), (float)weight, accumulate ? 1 : 0, cur_stream());
}

// Zero x if it holds a NaN/Inf; returns the device flag (no host sync).
Tensor zero_if_nonfinite_(Tensor x) {
  CHECK_IN(x, torch::kFloat32);
  auto flag = torch::zeros({1}, x.options().dtype(torch::kInt32));
  dalle::nonfinite(x.data_ptr<float>(), x.numel(), flag.data_ptr<int>(), cur_stream());
  dalle::zero_if_flag(x.data_ptr<float>(), x.numel(), flag.data_ptr<int>(), cur_stream());
  return flag;
}

Tensor nonfinite(Tensor x) {
  CHECK_IN(x, torch::kFloat32);
  auto flag = torch::zeros({1}, x.options().dtype(torch::kInt32));
  dalle::nonfinite(x.data_ptr<float>(), x.numel(), flag.data_ptr<int>(), cur_stream());
  return flag;
}

// K1 + K2: token ids (BOS, unique pad ids, offset image codes) and the gather of their rows of the
// fp32 table into the fp32 residual stream. Returns {tokens (B, n, d), ids (B*n) int32, bad flag}.
std::vector<Tensor> embed_fwd(Tensor text, Tensor image, Tensor table, int64_t pad_base, int64_t Vt) {
  CHECK_IN(text, torch::kInt64); CHECK_IN(image, torch::kInt64); CHECK_IN(table, torch::kFloat32);
  TORCH_CHECK(text.dim() == 2 && image.dim() == 2 && table.dim() == 2, "embed_fwd: text (B, T), image (B, I), table (V, d)");
  const int B = text.size(0), Ttxt = text.size(1), Timg = image.size(1), V = table.size(0), d = table.size(1);
  TORCH_CHECK(image.size(0) == B || Timg == 0, "embed_fwd: batch mismatch");
  TORCH_CHECK(d % 4 == 0, "embed_fwd: d must be a multiple of 4");
  TORCH_CHECK(pad_base >= 0 && pad_base + Ttxt <= V && Vt >= 0 && Vt <= V, "embed_fwd: id ranges exceed the table");
  const int n = Timg > 0 ? Ttxt + Timg : Ttxt + 1;  // BOS + text + image, the last image token dropped
  auto out = torch::empty({B, n, d}, table.options());
  auto ids = torch::empty({(long)B * n}, table.options().dtype(torch::kInt32));
  auto bad = torch::zeros({1}, table.options().dtype(torch::kInt32));
  if (B * n > 0)
    dalle::embed_fwd(text.data_ptr<int64_t>(), image.data_ptr<int64_t>(), table.data_ptr<float>(), out.data_ptr<float>(),
                     ids.data_ptr<int>(), bad.data_ptr<int>(), B, n, Ttxt, Timg, d, (int)pad_base, (int)Vt, V, cur_stream());
  return {out, ids, bad};
}

// grad[sorted_ids[r]] += sum of dout rows order[...] over each run of equal ids (deterministic order).
// order / sorted_ids / head come from a stable sort of the forward's ids (values < N, < V, < N).
void embed_bwd_(Tensor dout, Tensor order, Tensor sorted_ids, Tensor head, Tensor grad) {
  CHECK_IN(dout, torch::kFloat32); CHECK_IN(order, torch::kInt32); CHECK_IN(sorted_ids, torch::kInt32);
  CHECK_IN(head, torch::kInt32); CHECK_IN(grad, torch::kFloat32);
  TORCH_CHECK(dout.dim() == 2 && grad.dim() == 2 && dout.size(1) == grad.size(1) && dout.size(1) % 4 == 0, "embed_bwd: shapes");
  const long N = dout.size(0);
  TORCH_CHECK(order.numel() == N && sorted_ids.numel() == N && head.numel() == N, "embed_bwd: table sizes");
  if (N == 0) return;
  auto partial = torch::empty_like(dout);
  dalle::embed_bwd(dout.data_ptr<float>(), order.data_ptr<int>(), sorted_ids.data_ptr<int>(), head.data_ptr<int>(),
                   partial.data_ptr<float>(), grad.data_ptr<float>(), (int)N, (int)dout.size(1), cur_stream());
}

// Cross entropy + in-place dlogits + their column sums accumulated into `dbias` (fp32, += ) through
// per-workgroup partial rows and the fixed-order column_sum reducer. Returns the per-row losses.
Tensor xent_colsum_(Tensor logits, Tensor labels, double gscale, Tensor dbias) {
  CHECK_IN(logits, torch::kBFloat16); CHECK_IN(labels, torch::kInt64); CHECK_IN(dbias, torch::kFloat32);
  TORCH_CHECK(logits.dim() == 2 && labels.numel() == logits.size(0) && dbias.numel() == logits.size(1), "xent_colsum: shapes");
  const long R = logits.size(0);
  const int V = logits.size(1);
  auto loss = torch::empty({R}, logits.options().dtype(torch::kFloat32));
  if (R == 0) return loss;
  auto part = torch::empty({dalle::xent_colsum_blocks(R, V), V}, logits.options().dtype(torch::kFloat32));
  TORCH_CHECK(dalle::xent_colsum(logits.data_ptr(), labels.data_ptr<int64_t>(), loss.data_ptr<float>(), part.data_ptr<float>(),
                                 R, V, (float)gscale, cur_stream()), "xent_colsum: vocabulary split too wide for LDS");
  dalle::GradSink sink{dbias.data_ptr<float>(), nullptr, nullptr, V, 1};
  dalle::column_sum(part.data_ptr<float>(), (int)part.size(0), V, sink, cur_stream());
  return loss;
}

// ---------------------------------------------------------------------------------------------
// VQGAN decoder (K20): NHWC bf16 activations
static const float* opt_f32(const c10::optional<Tensor>& t, long n, const char* what) {
  if (!t.has_value()) return nullptr;
  CHECK_IN((*t), torch::kFloat32);
  TORCH_CHECK(t->numel() == n, what, ": wrong size");
  return t->data_ptr<float>();
}

// y (N, H, W, Cout) = conv3x3(silu(GN(x)) or x, upsampled 2x if ups) + bias (+ res)
Tensor conv3x3(Tensor x, Tensor w, c10::optional<Tensor> bias, c10::optional<Tensor> res, c10::optional<Tensor> mean,
               c10::optional<Tensor> rstd, c10::optional<Tensor> gamma, c10::optional<Tensor> beta, bool ups) {
  CHECK_IN(x, torch::kBFloat16); CHECK_IN(w, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "conv3x3: x (N, H, W, Cin) NHWC, w (Cout, 9 * Cin)");
  const int N = x.size(0), Hs = x.size(1), Ws = x.size(2), Cin = x.size(3), Cout = w.size(0);
  TORCH_CHECK(w.size(1) == 9 * Cin, "conv3x3: weight / input channels mismatch");
  const int H = ups ? 2 * Hs : Hs, W = ups ? 2 * Ws : Ws;
  auto y = torch::empty({N, H, W, Cout}, x.options());
  dalle::ConvArgs a{};
  a.x = x.data_ptr();
  a.w = w.data_ptr();
  a.bias = opt_f32(bias, Cout, "conv3x3 bias");
  if (res.has_value()) {
    CHECK_IN((*res), torch::kBFloat16);
    TORCH_CHECK(res->numel() == (long)N * H * W * Cout, "conv3x3: residual shape");
    a.res = res->data_ptr();
  }
  a.gn = mean.has_value() ? 1 : 0;
  if (a.gn) {
    a.mean = opt_f32(mean, (long)N * 32, "conv3x3 mean");
    a.rstd = opt_f32(rstd, (long)N * 32, "conv3x3 rstd");
    a.gamma = opt_f32(gamma, Cin, "conv3x3 gamma");
    a.beta = opt_f32(beta, Cin, "conv3x3 beta");
    TORCH_CHECK(a.rstd && a.gamma && a.beta, "conv3x3: GroupNorm needs mean, rstd, gamma, beta");
  }
  a.y = y.data_ptr();
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ups = ups ? 1 : 0;
  TORCH_CHECK(dalle::conv3x3(a, cur_stream()), "conv3x3: unsupported shape (Cin % 64, Cout % 128, H*W % 128, Cin <= 1024)");
  return y;
}

std::vector<Tensor> gn_stats(Tensor x, double eps) {
  CHECK_IN(x, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4, "gn_stats: x (N, H, W, C)");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto opts = x.options().dtype(torch::kFloat32);
  auto part = torch::empty({(long)dalle::gn_part_floats(N)}, opts);
  auto mean = torch::empty({N, 32}, opts), rstd = torch::empty({N, 32}, opts);
  TORCH_CHECK(dalle::gn_stats(x.data_ptr(), part.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), N, HW, C,
                              (float)eps, cur_stream()), "gn_stats: unsupported channel count");
  return {mean, rstd};
}

Tensor gn_apply(Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor beta, bool silu) {
  CHECK_IN(x, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 32 == 0 && x.size(3) % 8 == 0, "gn_apply: x (N, H, W, C)");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  const float* m = opt_f32(mean, (long)N * 32, "gn_apply mean");
  const float* r = opt_f32(rstd, (long)N * 32, "gn_apply rstd");
  const float* g = opt_f32(gamma, C, "gn_apply gamma");
  const float* b = opt_f32(beta, C, "gn_apply beta");
  auto y = torch::empty_like(x);
  dalle::gn_apply(x.data_ptr(), m, r, g, b, y.data_ptr(), N, HW, C, cur_stream(), silu ? 1 : 0);
  return y;
}

// final GN + SiLU + conv3x3 (C -> 3) + clamp / (x + 1) / 2: NCHW fp32 images; w (3, 9 * C) bf16
Tensor conv_out(Tensor x, Tensor w, Tensor bias, Tensor mean, Tensor rstd, Tensor gamma, Tensor beta) {
  CHECK_IN(x, torch::kBFloat16); CHECK_IN(w, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2 && w.size(0) == 3 && w.size(1) == 9 * x.size(3), "conv_out: shapes");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  auto img = torch::empty({N, 3, H, W}, x.options().dtype(torch::kFloat32));
  TORCH_CHECK(dalle::conv_out(x.data_ptr(), w.data_ptr(), opt_f32(bias, 3, "conv_out bias"), opt_f32(mean, (long)N * 32, "mean"),
                              opt_f32(rstd, (long)N * 32, "rstd"), opt_f32(gamma, C, "gamma"), opt_f32(beta, C, "beta"),
                              img.data_ptr<float>(), N, H, W, C, cur_stream()), "conv_out: C must be <= 128 and a multiple of 32");
  return img;
}

Tensor softmax_rows(Tensor s, double scale) {
  CHECK_IN(s, torch::kFloat32);
  const int L = s.size(-1);
  const long R = s.numel() / L;
  auto p = torch::empty(s.sizes(), s.options().dtype(torch::kBFloat16));
  if (R > 0) dalle::softmax_rows(s.data_ptr<float>(), p.data_ptr(), R, L, (float)scale, cur_stream());
  return p;
}

Tensor xent_fwd_bwd_(Tensor logits, Tensor labels, double gscale) {
  CHECK_IN(logits, torch::kBFloat16); CHECK_IN(labels, torch::kInt64);
  TORCH_CHECK(logits.dim() == 2 && labels.numel() == logits.size(0));
  auto loss = torch::empty({logits.size(0)}, logits.options().dtype(torch::kFloat32));
  dalle::xent_fwd_bwd(logits.data_ptr(), labels.data_ptr<int64_t>(), loss.data_ptr<float>(), logits.size(0), logits.size(1),
                      (float)gscale, cur_stream());
  return loss;
}

// ---------------------------------------------------------------------------------------------
// decode (KV-cache) path: all positions come from the device scalar `pos` (hipGraph-capturable)
static dalle::DecodeGeom make_decode_geom(int T, int S, int n, int H, int K, int pattern) {
  dalle::DecodeGeom g{T, S, n, H, K, pattern};
  TORCH_CHECK(n <= 2048, "decode attention supports up to 2048 cached positions");
  TORCH_CHECK(pattern >= 0 && pattern <= 3);
  return g;
}

// pending: (part (KS, B, D) fp32, bias (D) bf16 or None, scale (D) fp32) applied to x before the LN
void decode_ln_shift_(Tensor x, Tensor w, Tensor b, Tensor hist, Tensor y, Tensor pos, int64_t T, int64_t S, bool shift,
                      c10::optional<Tensor> part, c10::optional<Tensor> pbias, c10::optional<Tensor> pscale) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(w, torch::kFloat32); CHECK_IN(b, torch::kFloat32);
  CHECK_IN(hist, torch::kBFloat16); CHECK_IN(y, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  const int B = x.size(0), D = x.size(-1);
  TORCH_CHECK(x.numel() == (long)B * D && hist.size(0) == B && hist.size(2) == D && y.numel() == (long)B * D);
  TORCH_CHECK(D == 256 || D == 512 || D == 1024 || D == 2048, "decode_ln_shift: unsupported hidden size");
  auto g = make_decode_geom(T, S, hist.size(1), 1, 1, 0);
  const float* pp = nullptr;
  const void* pb = nullptr;
  const float* ps = nullptr;
  int KS = 0;
  if (part.has_value() && part->defined()) {
    CHECK_IN((*part), torch::kFloat32); TORCH_CHECK(pscale.has_value() && pscale->defined(), "decode_ln_shift: pending needs a scale");
    CHECK_IN((*pscale), torch::kFloat32);
    TORCH_CHECK(part->dim() == 3 && part->size(1) == B && part->size(2) == D && pscale->numel() == D, "decode_ln_shift: pending shapes");
    pp = part->data_ptr<float>();
    ps = pscale->data_ptr<float>();
    KS = part->size(0);
    TORCH_CHECK(KS >= 1 && KS <= 16, "decode_ln_shift: at most 16 pending slabs");
    if (pbias.has_value() && pbias->defined()) {
      CHECK_IN((*pbias), torch::kBFloat16); TORCH_CHECK(pbias->numel() == D);
      pb = pbias->data_ptr();
    }
  }
  dalle::decode_ln_shift(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), hist.data_ptr(), y.data_ptr(),
                         pos.data_ptr<int>(), g, B, D, shift ? 1 : 0, cur_stream(), pp, pb, ps, KS);
}

void residual_from_partials_(Tensor x, Tensor part, c10::optional<Tensor> pbias, Tensor pscale) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(part, torch::kFloat32); CHECK_IN(pscale, torch::kFloat32);
  const int B = x.size(0), D = x.size(-1);
  TORCH_CHECK(x.numel() == (long)B * D && D % 4 == 0 && part.dim() == 3 && part.size(1) == B && part.size(2) == D &&
              pscale.numel() == D, "residual_from_partials: shapes");
  const void* pb = nullptr;
  if (pbias.has_value() && pbias->defined()) {
    CHECK_IN((*pbias), torch::kBFloat16); TORCH_CHECK(pbias->numel() == D);
    pb = pbias->data_ptr();
  }
  dalle::residual_from_partials(x.data_ptr<float>(), part.data_ptr<float>(), pb, pscale.data_ptr<float>(), part.size(0), B, D,
                                cur_stream());
}

// attention of the new token whose q / k / v are still split-K partials of the QKV projection
// text_shared: optional int32 device flag, 1 = every batch row has the same caption (text keys read from row 0's cache)
static const int* shared_flag(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_CUDA((*t)); CHECK_DT((*t), torch::kInt32);
  TORCH_CHECK(t->numel() == 1, "text_shared: one int32 flag");
  return t->data_ptr<int>();
}

void decode_attn_part_(Tensor part, Tensor cosT, Tensor sinT, double qscale, Tensor kc, Tensor vc, Tensor out, Tensor pos,
                       int64_t T, int64_t S, int64_t H, int64_t K, int64_t pattern, c10::optional<Tensor> text_shared) {
  CHECK_IN(part, torch::kFloat32); CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  CHECK_IN(kc, torch::kBFloat16); CHECK_IN(vc, torch::kBFloat16); CHECK_IN(out, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  const int BH = kc.size(0), B = BH / H;
  TORCH_CHECK(BH % H == 0 && out.numel() == (long)BH * 64 && vc.sizes() == kc.sizes() && kc.size(2) == 64);
  TORCH_CHECK(part.dim() == 3 && part.size(1) == B && part.size(2) == 3 * H * 64, "decode_attn_part: part (KS, B, 3*H*64)");
  TORCH_CHECK(kc.size(1) == T + S * S - 1, "decode cache must hold the full sequence");
  TORCH_CHECK(cosT.size(0) >= kc.size(1) && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes());
  auto g = make_decode_geom(T, S, kc.size(1), H, K, pattern);
  dalle::decode_attn_part(part.data_ptr<float>(), part.size(0), cosT.data_ptr<float>(), sinT.data_ptr<float>(), (float)qscale,
                          kc.data_ptr(), vc.data_ptr(), out.data_ptr(), pos.data_ptr<int>(), g, B, cur_stream(),
                          shared_flag(text_shared));
}

// caption prefill: qkv (B, P, 3*H*64) bf16 -> q (B*H, P, 64) rotated + pre-scaled, k / v rotated into cache rows 0..P-1
void prefill_rope_(Tensor qkv, Tensor cosT, Tensor sinT, Tensor q, Tensor kc, Tensor vc, int64_t H, double qscale) {
  CHECK_IN(qkv, torch::kBFloat16); CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(kc, torch::kBFloat16); CHECK_IN(vc, torch::kBFloat16);
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == 3 * H * 64, "prefill_rope: qkv (B, P, 3*H*64)");
  const int B = qkv.size(0), P = qkv.size(1);
  TORCH_CHECK(q.numel() == (long)B * H * P * 64 && kc.dim() == 3 && kc.size(0) == B * H && kc.size(2) == 64 &&
              kc.size(1) >= P && vc.sizes() == kc.sizes() && cosT.size(0) >= P && cosT.size(1) == 64 &&
              sinT.sizes() == cosT.sizes(), "prefill_rope: shapes");
  dalle::prefill_rope(qkv.data_ptr(), cosT.data_ptr<float>(), sinT.data_ptr<float>(), q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                      B, P, H, kc.size(1), (float)qscale, cur_stream());
}

// caption prefill: LN + text shift of x (B, P, D) fp32 -> hist[:, :P] (B, n, D) bf16 (unshifted) and out (B, P, D) bf16
void prefill_ln_shift_(Tensor x, Tensor w, Tensor b, Tensor hist, Tensor out, bool shift, double eps) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(w, torch::kFloat32); CHECK_IN(b, torch::kFloat32);
  CHECK_IN(hist, torch::kBFloat16); CHECK_IN(out, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 3, "prefill_ln_shift: x (B, P, D)");
  const int B = x.size(0), P = x.size(1), D = x.size(2);
  TORCH_CHECK(D == 256 || D == 512 || D == 1024 || D == 2048, "prefill_ln_shift: unsupported hidden size");
  TORCH_CHECK(w.numel() == D && b.numel() == D && out.sizes() == x.sizes() && hist.dim() == 3 && hist.size(0) == B &&
              hist.size(1) >= P && hist.size(2) == D, "prefill_ln_shift: shapes");
  dalle::prefill_ln_shift(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), hist.data_ptr(), out.data_ptr(), B, P,
                          hist.size(1), D, (float)eps, shift ? 1 : 0, cur_stream());
}

// caption prefill: masked row softmax of fp32 scores (R, P, P) -> bf16, mask (>= P, >= P) bool, row i of a (P, P) block
// reads mask row i
void prefill_softmax_(Tensor sc, Tensor mask, Tensor out) {
  CHECK_IN(sc, torch::kFloat32); CHECK_IN(out, torch::kBFloat16); CHECK_CUDA(mask);
  TORCH_CHECK(mask.scalar_type() == torch::kBool, "prefill_softmax: mask must be bool");
  TORCH_CHECK(sc.dim() == 3 && sc.size(1) == sc.size(2) && out.sizes() == sc.sizes(), "prefill_softmax: sc / out (R, P, P)");
  const int P = sc.size(2);
  TORCH_CHECK(P <= 512, "prefill_softmax: at most 512 keys");
  TORCH_CHECK(mask.dim() == 2 && mask.size(0) == P && mask.size(1) == P && mask.is_contiguous(), "prefill_softmax: mask (P, P) contiguous");
  dalle::prefill_softmax(sc.data_ptr<float>(), mask.data_ptr<bool>(), out.data_ptr(), (long)sc.size(0) * P, P, cur_stream());
}

// caption prefill: x += scale * y (x fp32, y bf16, same shape (.., D); scale (D,) fp32)
void prefill_residual_(Tensor x, Tensor y, Tensor scale) {
  CHECK_IN(x, torch::kFloat32); CHECK_IN(y, torch::kBFloat16); CHECK_IN(scale, torch::kFloat32);
  const int D = x.size(-1);
  TORCH_CHECK(y.sizes() == x.sizes() && scale.numel() == D && D % 4 == 0, "prefill_residual: shapes");
  dalle::prefill_residual(x.data_ptr<float>(), y.data_ptr(), scale.data_ptr<float>(), x.numel(), D, cur_stream());
}

void decode_rope_(Tensor qkv, Tensor cosT, Tensor sinT, Tensor q, Tensor kc, Tensor vc, Tensor pos, int64_t H, double qscale) {
  CHECK_IN(qkv, torch::kBFloat16); CHECK_IN(cosT, torch::kFloat32); CHECK_IN(sinT, torch::kFloat32);
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(kc, torch::kBFloat16); CHECK_IN(vc, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  const int B = qkv.size(0);
  TORCH_CHECK(qkv.numel() == (long)B * 3 * H * 64 && q.numel() == (long)B * H * 64);
  TORCH_CHECK(kc.size(0) == B * H && kc.size(2) == 64 && vc.sizes() == kc.sizes() && cosT.size(0) >= kc.size(1));
  auto g = make_decode_geom(1, 1, kc.size(1), H, 1, 0);
  dalle::decode_rope(qkv.data_ptr(), cosT.data_ptr<float>(), sinT.data_ptr<float>(), q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                     pos.data_ptr<int>(), g, B, (float)qscale, cur_stream());
}

void decode_attn_(Tensor q, Tensor kc, Tensor vc, Tensor out, Tensor pos, int64_t T, int64_t S, int64_t H, int64_t K,
                  int64_t pattern, c10::optional<Tensor> text_shared) {
  CHECK_IN(q, torch::kBFloat16); CHECK_IN(kc, torch::kBFloat16); CHECK_IN(vc, torch::kBFloat16);
  CHECK_IN(out, torch::kBFloat16); CHECK_IN(pos, torch::kInt32);
  const int BH = kc.size(0);
  TORCH_CHECK(BH % H == 0 && q.numel() == (long)BH * 64 && out.numel() == (long)BH * 64 && vc.sizes() == kc.sizes());
  TORCH_CHECK(kc.size(1) == T + S * S - 1, "decode cache must hold the full sequence");
  auto g = make_decode_geom(T, S, kc.size(1), H, K, pattern);
  dalle::decode_attn(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), out.data_ptr(), pos.data_ptr<int>(), g, BH / H, cur_stream(),
                     shared_flag(text_shared));
}

// Fused sampler. Returns the raw samples (B,); with text/codes/tok given it also does the decode-step
// bookkeeping at device position *pos (codes[:, pos - T + 1] = sample, tok = next input token).
Tensor sample_step(Tensor logits, int64_t top_k, double top_p, double temperature, Tensor seed, Tensor pos,
                   c10::optional<Tensor> text, c10::optional<Tensor> codes, c10::optional<Tensor> tok, int64_t vt) {
  CHECK_IN(logits, torch::kFloat32); CHECK_IN(seed, torch::kInt64); CHECK_IN(pos, torch::kInt32);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) >= 1 && logits.size(1) <= 8192, "sample: logits must be (B, V <= 8192)");
  TORCH_CHECK(seed.numel() == 1 && pos.numel() == 1, "sample: seed / pos are device scalars");
  const int B = logits.size(0);
  dalle::SampleArgs a{};
  a.logits = logits.data_ptr<float>();
  a.B = B;
  a.V = logits.size(1);
  a.top_k = (int)top_k;
  a.top_p = (float)top_p;
  a.temperature = (float)temperature;
  a.seed = seed.data_ptr<int64_t>();
  a.pos = pos.data_ptr<int>();
  a.vt = vt;
  const bool book = text.has_value();
  TORCH_CHECK(book == codes.has_value() && book == tok.has_value(), "sample: give text, codes and tok together");
  if (book) {
    CHECK_IN((*text), torch::kInt64); CHECK_IN((*codes), torch::kInt64); CHECK_IN((*tok), torch::kInt64);
    TORCH_CHECK(text->dim() == 2 && text->size(0) == B && codes->dim() == 2 && codes->size(0) == B && tok->numel() == B,
                "sample: text (B, T), codes (B, image_len), tok (B,)");
    a.text = text->data_ptr<int64_t>();
    a.T = text->size(1);
    a.codes = codes->data_ptr<int64_t>();
    a.img_len = codes->size(1);
    a.tok = tok->data_ptr<int64_t>();
  }
  auto out = torch::empty({B}, logits.options().dtype(torch::kInt64));
  a.sampled = out.data_ptr<int64_t>();
  TORCH_CHECK(dalle::sample_step(a, cur_stream()), "sample: unsupported shape");
  return out;
}

Tensor vq_embed(Tensor idx, Tensor codebook, int64_t side) {
  CHECK_IN(idx, torch::kInt64); CHECK_IN(codebook, torch::kFloat32);
  const int B = idx.size(0), HW = idx.size(1), C = codebook.size(1);
  TORCH_CHECK(HW == side * side);
  auto z = torch::empty({B, C, side, side}, codebook.options());
  dalle::vq_embed(idx.data_ptr<int64_t>(), codebook.data_ptr<float>(), z.data_ptr<float>(), HW, C, B, cur_stream());
  return z;
}

// ---------------------------------------------------------------------------------------------
void lamb_grad_norm(Tensor g, Tensor partial, double max_norm, Tensor coef, Tensor norm) {
  CHECK_IN(g, torch::kFloat32); CHECK_IN(partial, torch::kFloat32);
  TORCH_CHECK(g.numel() % 4096 == 0 && partial.numel() >= g.numel() / 4096);
  dalle::lamb_grad_norm(g.data_ptr<float>(), g.numel(), partial.data_ptr<float>(), (float)max_norm, coef.data_ptr<float>(),
                        norm.data_ptr<float>(), cur_stream());
}

// bslot[blk]: the block's slot in its mode's compact state array (8-bit: q1/q2 rows of 4096 +
// absmax; fp32: m32/v32 rows). The table is built and range-checked on the host by the engine
// (dalle_amd/optim/fused.py); here the array sizes are checked against the slot counts it reports.
void lamb_step(Tensor p, Tensor g, Tensor q1, Tensor q2, Tensor absmax1, Tensor absmax2, Tensor m32, Tensor v32,
               Tensor code1, Tensor code2, Tensor block_tensor, Tensor bslot, Tensor tstart, Tensor tsize, Tensor tmode,
               Tensor twd, Tensor tlr, Tensor coef, Tensor partial, Tensor trust, Tensor wnorm, Tensor snorm, int64_t n8_blocks,
               int64_t n32_blocks, double beta1, double beta2, double eps, double clamp_value, bool use_clip) {
  CHECK_IN(p, torch::kFloat32); CHECK_IN(g, torch::kFloat32);
  CHECK_IN(q1, torch::kUInt8); CHECK_IN(q2, torch::kUInt8);
  CHECK_IN(absmax1, torch::kFloat32); CHECK_IN(absmax2, torch::kFloat32);
  CHECK_IN(m32, torch::kFloat32); CHECK_IN(v32, torch::kFloat32);
  CHECK_IN(block_tensor, torch::kInt32); CHECK_IN(bslot, torch::kInt32);
  CHECK_IN(tstart, torch::kInt64); CHECK_IN(tsize, torch::kInt64);
  const long n = p.numel();
  const long nb = n / 4096;
  TORCH_CHECK(n % 4096 == 0 && g.numel() == n, "lamb_step: arena sizes");
  TORCH_CHECK(q1.numel() == n8_blocks * 4096 && q2.numel() == n8_blocks * 4096 && absmax1.numel() == n8_blocks &&
                  absmax2.numel() == n8_blocks, "lamb_step: 8-bit state sizes");
  TORCH_CHECK(m32.numel() == n32_blocks * 4096 && v32.numel() == n32_blocks * 4096, "lamb_step: fp32 state sizes");
  TORCH_CHECK(n8_blocks + n32_blocks == nb, "lamb_step: every block needs exactly one state slot");
  TORCH_CHECK(block_tensor.numel() == nb && bslot.numel() == nb && partial.numel() >= 2 * nb);
  TORCH_CHECK(code1.numel() == 256 && code2.numel() == 256);
  const int nt = tstart.numel();
  TORCH_CHECK(tsize.numel() == nt && tmode.numel() == nt && twd.numel() == nt && tlr.numel() == nt && trust.numel() == nt);
  // 1-element placeholders keep the pointers valid when one mode has no tensors
  dalle::lamb_step(p.data_ptr<float>(), g.data_ptr<float>(), q1.data_ptr<uint8_t>(), q2.data_ptr<uint8_t>(),
                   absmax1.data_ptr<float>(), absmax2.data_ptr<float>(), m32.data_ptr<float>(), v32.data_ptr<float>(),
                   code1.data_ptr<float>(), code2.data_ptr<float>(), block_tensor.data_ptr<int>(), bslot.data_ptr<int>(),
                   (const long*)tstart.data_ptr<int64_t>(), (const long*)tsize.data_ptr<int64_t>(), tmode.data_ptr<int>(),
                   twd.data_ptr<float>(), tlr.data_ptr<float>(), coef.data_ptr<float>(), partial.data_ptr<float>(),
                   trust.data_ptr<float>(), wnorm.data_ptr<float>(), snorm.data_ptr<float>(), nt, n, (float)beta1, (float)beta2,
                   (float)eps, (float)clamp_value, use_clip ? 1 : 0, cur_stream());
}

// ---------------------------------------------------------------------------------------------
// PowerSGD: in-place column orthonormalisation of every P factor (flat buffer, one launch) and the
// fused rank-r reconstruction + error-feedback update
void psgd_orthonormalize_(Tensor P, Tensor offsets, Tensor rows, int64_t r, double eps) {
  CHECK_IN(P, torch::kFloat32); CHECK_IN(offsets, torch::kInt64); CHECK_IN(rows, torch::kInt32);
  TORCH_CHECK(r >= 1 && r <= 8, "psgd: rank must be in [1, 8]");
  TORCH_CHECK(offsets.numel() == rows.numel() && offsets.device() == P.device() && rows.device() == P.device());
  const int nmat = rows.numel();
  if (nmat == 0) return;
  // host-side bounds check of the layout the kernel walks (tiny tensors)
  auto oc = offsets.cpu(), rc = rows.cpu();
  const long* o = oc.data_ptr<int64_t>();
  const int* rr = rc.data_ptr<int>();
  for (int i = 0; i < nmat; ++i)
    TORCH_CHECK(o[i] >= 0 && rr[i] >= 0 && o[i] + (long)rr[i] * r <= P.numel(), "psgd_orthonormalize: matrix ", i, " out of bounds");
  dalle::psgd_orthonormalize(P.data_ptr<float>(), offsets.data_ptr<int64_t>(), rows.data_ptr<int>(), nmat, (int)r, (float)eps,
                             cur_stream());
}

void psgd_reconstruct_(Tensor grad, Tensor E, Tensor P, Tensor Q) {
  CHECK_IN(grad, torch::kFloat32); CHECK_IN(E, torch::kFloat32); CHECK_IN(P, torch::kFloat32); CHECK_IN(Q, torch::kFloat32);
  TORCH_CHECK(E.dim() == 2 && P.dim() == 2 && Q.dim() == 2, "psgd_reconstruct: E (n, m), P (n, r), Q (m, r)");
  const long n = E.size(0);
  const int m = E.size(1), r = P.size(1);
  TORCH_CHECK(P.size(0) == n && Q.size(0) == m && Q.size(1) == r && grad.numel() == E.numel());
  TORCH_CHECK(dalle::psgd_reconstruct(grad.data_ptr<float>(), E.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(), n, m, r,
                                      cur_stream()),
              "psgd_reconstruct: needs m % 4 == 0 and rank in {1, 2, 4, 8}");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dalle_amd HIP/CDNA4 kernels (gfx950)";
  m.def("ln_shift_fwd", &ln_shift_fwd);
  m.def("ln_shift_fwd_res", &ln_shift_fwd_res);
  m.def("ln_shift_bwd_sr", &ln_shift_bwd_sr);
  m.def("ln_shift_bwd", &ln_shift_bwd, py::arg("x"), py::arg("w"), py::arg("dy"), py::arg("mean"), py::arg("rstd"),
        py::arg("T"), py::arg("S"), py::arg("shift"), py::arg("resid") = py::none(), py::arg("gw") = py::none(),
        py::arg("gb") = py::none());
  m.def("rope_fwd", &rope_fwd);
  m.def("rope_bwd", &rope_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_bwd_rope", &attn_bwd_rope, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("out"), py::arg("dout"),
        py::arg("lse"), py::arg("cosT"), py::arg("sinT"), py::arg("B"), py::arg("T"), py::arg("S"), py::arg("n"), py::arg("K"),
        py::arg("H"), py::arg("pattern"), py::arg("qscale"), py::arg("rotf") = py::none(), py::arg("n_lang") = 0,
        py::arg("n_pix") = 0, py::arg("img_text_pos") = 0.0, py::arg("text_axial") = 0.0);
  m.def("geglu_fwd", &geglu_fwd);
  m.def("geglu_bwd", &geglu_bwd);
  m.def("geglu_bwd_bias", &geglu_bwd_bias, py::arg("h"), py::arg("dout"), py::arg("gb") = py::none());
  m.def("ff_dgrad_geglu", &ff_dgrad_geglu, py::arg("dy"), py::arg("w2t"), py::arg("h"), py::arg("gb") = py::none(),
        py::arg("stagger") = -1);
  m.def("scale_residual_", &scale_residual_);
  m.def("scale_residual_out", &scale_residual_out);
  m.def("transpose_bf16", &transpose_bf16, "fp32 (R, C) -> bf16 (C, R) in one pass");
  m.def("transpose_act_bf16", &transpose_act_bf16, "bf16 (R, C) -> bf16 (C, R), 64 x 64 LDS tiles (R, C multiples of 64)");
  m.def("scale_residual_bwd", &scale_residual_bwd, py::arg("g"), py::arg("y"), py::arg("scale"),
        py::arg("gscale") = py::none(), py::arg("gbias") = py::none());
  m.def("nonfinite", &nonfinite);
  m.def("splitk_accum_", &splitk_accum_);
  m.def("psgd_orthonormalize_", &psgd_orthonormalize_);
  m.def("psgd_reconstruct_", &psgd_reconstruct_);
  m.def("qkv_rope", &qkv_rope);
  m.def("uq8_compress", &uq8_compress);
  m.def("uq8_dequant_", &uq8_dequant_);
  m.def("uq8_seg_compress", &uq8_seg_compress);
  m.def("zero_if_nonfinite_", &zero_if_nonfinite_);
  m.def("uq8_seg_dequant_", &uq8_seg_dequant_);
  m.def("gemm_nt", &gemm_nt, py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("variant") = 0);
  m.def("gemm_set_cpol", [](int64_t c) { dalle::gemm_set_cpol((int)c); }, py::arg("cpol"),
        "cache policy of the hand-written GEMMs' output stores: 0 plain, 1 sc0, 2 nt, 16 sc1, 17 sc0 sc1");
  m.def("gemm_set_geglu_bwd_2wg", [](int64_t v) { dalle::gemm_set_geglu_bwd_2wg((int)v); }, py::arg("v"),
        "1: FF-out dgrad + GEGLU backward on the two-workgroups-per-CU kernel");
  m.def("gemm_set_2wg_stagger", [](int64_t ticks, int64_t first_wave) { dalle::gemm_set_2wg_stagger((int)ticks, (int)first_wave); },
        py::arg("ticks"), py::arg("first_wave") = -256,
        "two-workgroup GEMM start stagger: 10 ns ticks; first_wave < 0 delays workgroups [-fw, -2 fw), > 0 is 4-phase");
  m.def("gemm_2wg", [](Tensor A, Tensor B) {
    CHECK_IN(A, torch::kBFloat16); CHECK_IN(B, torch::kBFloat16);
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_2wg: A (M, K), B (N, K)");
    auto C = torch::empty({A.size(0), B.size(0)}, A.options());
    TORCH_CHECK(dalle::gemm_2wg(A.data_ptr(), B.data_ptr(), C.data_ptr(), nullptr, (int)A.size(0), (int)B.size(0), (int)A.size(1),
                                cur_stream()), "gemm_2wg: M % 256, N % 128, K % 32 (K >= 64)");
    return C;
  });
  m.def("gemm_set_pt_overlap", [](int64_t v, int64_t stagger) { dalle::gemm_set_pt_overlap((int)v, (int)stagger); },
        py::arg("overlap"), py::arg("stagger_pct") = 0,
        "persistent plain GEMM: epilogue stores beside the next tile's first K-step; start stagger in % of a tile");
  m.def("gemm_set_drain", [](int64_t d) { dalle::gemm_set_drain((int)d); }, py::arg("drain"),
        "1: hand-written GEMM workgroups wait for their output stores before ending");
  m.def("asm_gemm", &asm_gemm, py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("out") = py::none());
  m.def("asm_qkv_rope", &asm_qkv_rope, py::arg("h"), py::arg("w"), py::arg("cs3"), py::arg("T"), py::arg("S"), py::arg("H"),
        py::arg("n"), py::arg("col_major"));
  m.def("asm_ff_in_geglu", &asm_ff_in_geglu, py::arg("x"), py::arg("w1p"), py::arg("b1p"));
  m.def("asm_ff_dgrad_geglu", &asm_ff_dgrad_geglu, py::arg("dy"), py::arg("w2t"), py::arg("h"), py::arg("gb") = py::none());
  m.def("asm_wgrad_", &asm_wgrad_, py::arg("out"), py::arg("A"), py::arg("B"), py::arg("splits"), py::arg("accumulate"));
  m.def("gemm_pt", &gemm_pt, py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("variant") = 0, py::arg("group") = 0);
  m.def("qkv_rope_pt", &qkv_rope_pt, py::arg("h"), py::arg("w"), py::arg("cs"), py::arg("T"), py::arg("S"), py::arg("H"),
        py::arg("n"), py::arg("col_major"), py::arg("qscale"), py::arg("persist") = -1);
  m.def("ff_dgrad_geglu_pt", &ff_dgrad_geglu_pt, py::arg("dy"), py::arg("w2t"), py::arg("h"), py::arg("gb") = py::none(),
        py::arg("persist") = -1);
  m.def("ff_in_geglu_pt", &ff_in_geglu_pt, py::arg("x"), py::arg("w1i"), py::arg("b1i") = py::none(), py::arg("persist") = -1);
  m.def("permlane16_probe", &permlane16_probe);
  m.def("xent_fwd_bwd_", &xent_fwd_bwd_);
  m.def("embed_fwd", &embed_fwd);
  m.def("xent_colsum_", &xent_colsum_);
  m.def("conv3x3", &conv3x3, py::arg("x"), py::arg("w"), py::arg("bias") = py::none(), py::arg("res") = py::none(),
        py::arg("mean") = py::none(), py::arg("rstd") = py::none(), py::arg("gamma") = py::none(), py::arg("beta") = py::none(),
        py::arg("ups") = false);
  m.def("gn_stats", &gn_stats);
  m.def("gn_apply", &gn_apply, py::arg("x"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("beta"),
        py::arg("silu") = false);
  m.def("conv_out", &conv_out);
  m.def("softmax_rows", &softmax_rows);
  m.def("embed_bwd_", &embed_bwd_);
  m.def("decode_ln_shift_", &decode_ln_shift_, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("hist"), py::arg("y"),
        py::arg("pos"), py::arg("T"), py::arg("S"), py::arg("shift"), py::arg("part") = py::none(),
        py::arg("pbias") = py::none(), py::arg("pscale") = py::none());
  m.def("decode_rope_", &decode_rope_);
  m.def("prefill_rope_", &prefill_rope_);
  m.def("prefill_ln_shift_", &prefill_ln_shift_);
  m.def("prefill_softmax_", &prefill_softmax_);
  m.def("prefill_residual_", &prefill_residual_);
  m.def("decode_attn_", &decode_attn_, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("out"), py::arg("pos"), py::arg("T"),
        py::arg("S"), py::arg("H"), py::arg("K"), py::arg("pattern"), py::arg("text_shared") = py::none());
  m.def("skinny_linear", &skinny_linear);
  m.def("skinny_partials", &skinny_partials);
  m.def("skinny_partials_ln_", &skinny_partials_ln_, py::arg("X"), py::arg("W"), py::arg("bias"), py::arg("scale"), py::arg("x"),
        py::arg("ln_w"), py::arg("ln_b"), py::arg("hist"), py::arg("y"), py::arg("pos"), py::arg("T"), py::arg("S"),
        py::arg("shift"), py::arg("cnt"), py::arg("err"));
  m.def("skinny_partials_ln_ok", [](int64_t M, int64_t N, int64_t K) { return dalle::skinny_partials_ln_ok(M, N, K); });
  m.def("residual_from_partials_", &residual_from_partials_, py::arg("x"), py::arg("part"), py::arg("pbias"), py::arg("pscale"));
  m.def("decode_attn_part_", &decode_attn_part_, py::arg("part"), py::arg("cosT"), py::arg("sinT"), py::arg("qscale"), py::arg("kc"),
        py::arg("vc"), py::arg("out"), py::arg("pos"), py::arg("T"), py::arg("S"), py::arg("H"), py::arg("K"), py::arg("pattern"),
        py::arg("text_shared") = py::none());
  m.def("skinny_force_config", &dalle::skinny_force_config);
  m.def("skinny_shape_info", &dalle::skinny_shape_info);
  m.def("skinny_geglu", &skinny_geglu);
  m.def("skinny_residual_", &skinny_residual_);
  m.def("skinny_qkv_rope_", &skinny_qkv_rope_);
  m.def("vq_embed", &vq_embed);
  m.def("sample_step", &sample_step, py::arg("logits"), py::arg("top_k"), py::arg("top_p"), py::arg("temperature"),
        py::arg("seed"), py::arg("pos"), py::arg("text") = py::none(), py::arg("codes") = py::none(),
        py::arg("tok") = py::none(), py::arg("vt") = 0);
  m.def("lamb_grad_norm", &lamb_grad_norm);
  m.def("lamb_step", &lamb_step);
}
