// PyTorch bindings for the deeperspeed_amd HIP kernels (module `_hip_ops`).
//
// Thin layer: validates shapes/dtypes on the host (a wrong shape never reaches
// a kernel), allocates outputs with the caching allocator and launches on the
// current HIP stream. All device code lives in kernels/*.hip.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <ATen/Parallel.h>

#include <cstring>
#include <optional>
#include <vector>

#include "include/launchers.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

inline int dcode(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return dsa::kCodeF32;
    case at::kBFloat16: return dsa::kCodeBF16;
    case at::kHalf: return dsa::kCodeF16;
    default: TORCH_CHECK(false, "deeperspeed_amd kernels support fp32/bf16/fp16, got ", t.scalar_type());
  }
  return -1;
}

inline void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ----------------------------------------------------------------------------- optim
void adam_flat(Tensor w, Tensor g, Tensor m, Tensor v, OptT out, double lr, double beta1, double beta2, double eps,
               double wd, double bc1, double bc2, double grad_scale, bool adamw) {
  check_dev(w, "w"); check_dev(g, "g"); check_dev(m, "exp_avg"); check_dev(v, "exp_avg_sq");
  const int64_t n = w.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam_flat: size mismatch");
  TORCH_CHECK(m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat, "adam states must be fp32");
  TORCH_CHECK(aligned16(w.data_ptr()) && aligned16(m.data_ptr()) && aligned16(v.data_ptr()),
              "adam_flat: w/m/v must be 16-byte aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr()) & (g.element_size() * 4 - 1)) == 0,
              "adam_flat: grad must be aligned to 4 elements");
  void* optr = nullptr;
  int ot = dsa::kCodeBF16;
  if (out.has_value()) {
    check_dev(*out, "out");
    TORCH_CHECK(out->numel() == n, "adam_flat: out size mismatch");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(out->data_ptr()) & (out->element_size() * 4 - 1)) == 0,
                "adam_flat: out must be aligned to 4 elements");
    optr = out->data_ptr();
    ot = dcode(*out);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  dsa::AdamArgs a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                  (float)grad_scale, adamw ? 1 : 0};
  dsa::launch_adam_flat(w.data_ptr(), dcode(w), g.data_ptr(), dcode(g), m.data_ptr<float>(), v.data_ptr<float>(),
                        optr, ot, n, a, cur_stream());
}

// Compact master: hi = bf16 model weights (updated in place), res = int16 residual.
void adam_compact(Tensor hi, Tensor res, Tensor g, Tensor m, Tensor v, double lr, double beta1, double beta2,
                  double eps, double wd, double bc1, double bc2, double grad_scale, bool adamw) {
  check_dev(hi, "hi"); check_dev(res, "res"); check_dev(g, "g"); check_dev(m, "exp_avg"); check_dev(v, "exp_avg_sq");
  const int64_t n = hi.numel();
  TORCH_CHECK(hi.scalar_type() == at::kBFloat16 && res.scalar_type() == at::kShort, "adam_compact: bf16 hi, int16 res");
  TORCH_CHECK(res.numel() == n && g.numel() == n && m.numel() == n && v.numel() == n, "adam_compact: size mismatch");
  TORCH_CHECK(m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat, "adam states must be fp32");
  for (const Tensor* t : {&hi, &res, &g, &m, &v})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & (t->element_size() * 4 - 1)) == 0,
                "adam_compact: operands must be aligned to 4 elements");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(hi.device());
  dsa::AdamArgs a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                  (float)grad_scale, adamw ? 1 : 0};
  dsa::launch_adam_compact(hi.data_ptr(), res.data_ptr(), g.data_ptr(), dcode(g), m.data_ptr<float>(),
                           v.data_ptr<float>(), n, a, cur_stream());
}

// meta: device int64 table built by ops/adam.py (see optim.hip adam_multi_kernel)
void adam_multi(Tensor meta, int64_t T, int64_t total_chunks, int64_t chunk, int64_t wt, int64_t gt, int64_t ot,
                double lr, double beta1, double beta2, double eps, double wd, double bc1, double bc2,
                double grad_scale, bool adamw) {
  check_dev(meta, "meta");
  TORCH_CHECK(meta.scalar_type() == at::kLong && meta.numel() == 7 * T + 1, "adam_multi: bad meta table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(meta.device());
  dsa::AdamArgs a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                  (float)grad_scale, adamw ? 1 : 0};
  dsa::launch_adam_multi(meta.data_ptr<int64_t>(), (int)T, total_chunks, chunk, (int)wt, (int)gt, (int)ot, a,
                         cur_stream());
}

// out[0] += sum(x^2) in fp32. workspace >= 1024 floats.
// out[0] += sum of squares of every tensor listed in meta (see launch_sumsq_multi); partial holds
// total_chunks floats.
void sumsq_multi(Tensor meta, int64_t nt, int64_t total_chunks, int64_t chunk, int64_t xt, Tensor partial,
                 Tensor out) {
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == at::kLong && meta.numel() == 3 * nt + 1, "sumsq_multi: meta");
  TORCH_CHECK(partial.is_cuda() && partial.scalar_type() == at::kFloat && partial.numel() >= total_chunks,
              "sumsq_multi: partial");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() >= 1, "sumsq_multi: out");
  TORCH_CHECK(xt >= 0 && xt <= 2, "sumsq_multi: dtype code");
  dsa::launch_sumsq_multi(meta.data_ptr<int64_t>(), (int)nt, total_chunks, chunk, (int)xt, partial.data_ptr<float>(),
                          out.data_ptr<float>(), cur_stream());
}

void sumsq_accum(Tensor x, Tensor workspace, Tensor out) {
  check_dev(x, "x");
  TORCH_CHECK(workspace.numel() >= 1024 && workspace.scalar_type() == at::kFloat, "sumsq: workspace");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "sumsq: out must be fp32");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, "sumsq: x must be 16-byte aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  dsa::launch_sumsq_accum(x.data_ptr(), dcode(x), x.numel(), workspace.data_ptr<float>(), out.data_ptr<float>(),
                          cur_stream());
}

void scale_copy(Tensor x, Tensor y, OptT scale_t, double scale, bool accumulate) {
  check_dev(x, "x"); check_dev(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "scale_copy: size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & (x.element_size() * 4 - 1)) == 0 &&
                  (reinterpret_cast<uintptr_t>(y.data_ptr()) & (y.element_size() * 4 - 1)) == 0,
              "scale_copy: tensors must be aligned to 4 elements");
  const float* sp = nullptr;
  if (scale_t.has_value()) {
    TORCH_CHECK(scale_t->scalar_type() == at::kFloat && scale_t->is_cuda(), "scale tensor must be fp32 GPU");
    sp = scale_t->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  dsa::launch_scale_copy(x.data_ptr(), dcode(x), y.data_ptr(), dcode(y), x.numel(), sp, (float)scale,
                         cur_stream(), accumulate ? 1 : 0);
}

void lamb(Tensor w, Tensor g, Tensor m, Tensor v, Tensor upd, OptT out, double lr, double beta1, double beta2,
          double eps, double wd, double bc1, double bc2, double grad_scale, double max_coeff, double min_coeff,
          bool adamw, Tensor workspace, Tensor coeff_out) {
  check_dev(w, "w"); check_dev(g, "g"); check_dev(m, "m"); check_dev(v, "v"); check_dev(upd, "upd");
  const int64_t n = w.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && upd.numel() == n, "lamb: size mismatch");
  TORCH_CHECK(workspace.numel() >= 2048 && coeff_out.numel() >= 1, "lamb: workspace");
  void* optr = nullptr;
  int ot = dsa::kCodeBF16;
  if (out.has_value()) { optr = out->data_ptr(); ot = dcode(*out); TORCH_CHECK(out->numel() == n); }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  dsa::LambArgs a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                  (float)grad_scale, (float)max_coeff, (float)min_coeff, adamw ? 1 : 0};
  dsa::launch_lamb(w.data_ptr(), dcode(w), g.data_ptr(), dcode(g), m.data_ptr<float>(), v.data_ptr<float>(),
                   upd.data_ptr<float>(), optr, ot, n, a, workspace.data_ptr<float>(), coeff_out.data_ptr<float>(),
                   cur_stream());
}

// multi-tensor LAMB over a meta table (layout of adam_multi); partial >= 2*total_chunks, coeff >= T
void lamb_multi(Tensor meta, int64_t T, int64_t total_chunks, int64_t chunk, int64_t wt, int64_t gt, int64_t ot,
                double lr, double beta1, double beta2, double eps, double wd, double bc1, double bc2,
                double grad_scale, double max_coeff, double min_coeff, bool adamw, Tensor partial, Tensor coeff,
                OptT scale, OptT lr_dev) {
  check_dev(meta, "meta"); check_dev(partial, "partial"); check_dev(coeff, "coeff");
  if (lr_dev.has_value()) {
    check_dev(*lr_dev, "lr_dev");
    TORCH_CHECK(lr_dev->scalar_type() == at::kFloat && lr_dev->numel() == 1, "lamb_multi: lr_dev must be one fp32");
  }
  if (scale.has_value()) {
    check_dev(*scale, "scale");
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1, "lamb_multi: scale must be one fp32");
  }
  TORCH_CHECK(meta.scalar_type() == at::kLong && meta.numel() == 7 * T + 1, "lamb_multi: bad meta table");
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.numel() >= 2 * total_chunks, "lamb_multi: partial");
  TORCH_CHECK(coeff.scalar_type() == at::kFloat && coeff.numel() >= T, "lamb_multi: coeff");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(meta.device());
  dsa::LambArgs a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2,
                  (float)grad_scale, (float)max_coeff, (float)min_coeff, adamw ? 1 : 0,
                  scale.has_value() ? scale->data_ptr<float>() : nullptr,
                  lr_dev.has_value() ? lr_dev->data_ptr<float>() : nullptr};
  dsa::launch_lamb_multi(meta.data_ptr<int64_t>(), (int)T, total_chunks, chunk, (int)wt, (int)gt, (int)ot, a,
                         partial.data_ptr<float>(), coeff.data_ptr<float>(), cur_stream());
}

// A caller-provided output buffer (layer-stacked slabs, ops/wgrad_batch.py) or a fresh one like `like`.
static Tensor out_or_new(const OptT& out, at::IntArrayRef sizes, const at::TensorOptions& opt, const char* what) {
  if (!out.has_value()) return at::empty(sizes, opt);
  TORCH_CHECK(out->sizes() == sizes && out->scalar_type() == opt.dtype().toScalarType() && out->is_contiguous() &&
                  out->device() == opt.device() && reinterpret_cast<uintptr_t>(out->data_ptr()) % 16 == 0,
              what, ": out must be a contiguous 16-byte aligned tensor of the result's shape and dtype");
  return *out;
}
static Tensor out_or_empty(const OptT& out, const Tensor& like, const char* what) {
  return out_or_new(out, like.sizes(), like.options(), what);
}

// ----------------------------------------------------------------------------- layer norm
// Returns (y, mean, rstd, sum) where sum = x + res (+bias) when res is given (else undefined).
std::vector<Tensor> ln_fwd(Tensor x, Tensor gamma, OptT beta, double eps, OptT res, OptT bias, OptT y_out) {
  check_dev(x, "x"); check_dev(gamma, "gamma");
  const int64_t H = x.size(-1);
  const int64_t rows = x.numel() / H;
  const int dt = dcode(x);
  TORCH_CHECK(gamma.numel() == H && gamma.scalar_type() == x.scalar_type(), "ln_fwd: gamma must match x");
  TORCH_CHECK(H % (dt == dsa::kCodeF32 ? 4 : 8) == 0, "ln_fwd: hidden must be a multiple of 16 bytes");
  TORCH_CHECK(H <= dsa::ln_max_hidden(dt), "ln_fwd: hidden too large");
  if (beta.has_value()) TORCH_CHECK(beta->numel() == H && beta->scalar_type() == x.scalar_type(), "ln_fwd: beta");
  Tensor sum;
  if (res.has_value()) {
    check_dev(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(), "ln_fwd: res mismatch");
    sum = at::empty_like(x);
    if (bias.has_value()) TORCH_CHECK(bias->numel() == H && bias->scalar_type() == x.scalar_type());
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = out_or_empty(y_out, x, "ln_fwd");
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rows}, f32), rstd = at::empty({rows}, f32);
  dsa::launch_ln_fwd(x.data_ptr(), res.has_value() ? res->data_ptr() : nullptr,
                     (res.has_value() && bias.has_value()) ? bias->data_ptr() : nullptr,
                     res.has_value() ? sum.data_ptr() : nullptr, gamma.data_ptr(),
                     beta.has_value() ? beta->data_ptr() : nullptr, y.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), rows, (int)H, (float)eps, dt, cur_stream());
  return {y, mean, rstd, sum};
}

// Returns (dx, dgamma, dbeta)
// dgamma_acc / dbeta_acc: existing gradient buffers the parameter gradients are accumulated into
// (the engine's bound p.grad views) instead of fresh tensors for autograd to add
std::vector<Tensor> ln_bwd(Tensor dy, Tensor x, Tensor gamma, Tensor mean, Tensor rstd, bool has_beta, OptT dres,
                           OptT dgamma_acc, OptT dbeta_acc) {
  check_dev(dy, "dy"); check_dev(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "ln_bwd: dy/x mismatch");
  const int64_t H = x.size(-1);
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "ln_bwd: stats size");
  if (dres.has_value()) TORCH_CHECK(dres->sizes() == x.sizes() && dres->is_contiguous(), "ln_bwd: dres");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor dx = at::empty_like(x);
  const bool acc = dgamma_acc.has_value();
  if (acc) {
    TORCH_CHECK(dgamma_acc->sizes() == gamma.sizes() && dgamma_acc->scalar_type() == gamma.scalar_type() &&
                dgamma_acc->is_contiguous(), "ln_bwd: dgamma_acc must match gamma");
    TORCH_CHECK(!has_beta || (dbeta_acc.has_value() && dbeta_acc->sizes() == gamma.sizes() &&
                              dbeta_acc->scalar_type() == gamma.scalar_type() && dbeta_acc->is_contiguous()),
                "ln_bwd: dbeta_acc must match gamma");
  }
  Tensor dgamma = acc ? *dgamma_acc : at::empty_like(gamma);
  Tensor dbeta = has_beta ? (acc ? *dbeta_acc : at::empty_like(gamma)) : Tensor();
  const int grid = dsa::ln_bwd_grid(rows);
  Tensor partial = at::empty({2 * (int64_t)grid * H}, x.options().dtype(at::kFloat));
  dsa::launch_ln_bwd(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                     dres.has_value() ? dres->data_ptr() : nullptr, dx.data_ptr(), dgamma.data_ptr(),
                     has_beta ? dbeta.data_ptr() : nullptr, partial.data_ptr<float>(), rows, (int)H, dcode(x),
                     cur_stream(), acc ? 1 : 0);
  return {dx, dgamma, dbeta};
}

// ----------------------------------------------------------------------------- bias + gelu
// out (+)= part.sum(0) for part [S, ...] 16-bit contiguous; out of part's dtype or fp32, numel = part[0].numel()
Tensor sum_slices(Tensor part, Tensor out, bool accumulate) {
  check_dev(part, "sum_slices"); check_dev(out, "sum_slices");
  TORCH_CHECK(part.is_contiguous() && out.is_contiguous() && part.dim() >= 2, "sum_slices: contiguous part [S, ...]");
  const int64_t n = part.numel() / part.size(0);
  TORCH_CHECK(out.numel() == n && n % 8 == 0, "sum_slices: out must hold one slice (numel % 8 == 0)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  if (part.scalar_type() == at::kFloat) {  // fp32 partials, any out dtype
    dsa::launch_sum_slices_f32(part.data_ptr<float>(), (int)part.size(0), n, out.data_ptr(), accumulate ? 1 : 0,
                               dcode(out), cur_stream());
    return out;
  }
  TORCH_CHECK(part.scalar_type() == at::kBFloat16 || part.scalar_type() == at::kHalf, "sum_slices: partial dtype");
  TORCH_CHECK(out.scalar_type() == part.scalar_type() || out.scalar_type() == at::kFloat, "sum_slices: out dtype");
  dsa::launch_sum_slices(part.data_ptr(), (int)part.size(0), n, out.data_ptr(), out.scalar_type() == at::kFloat,
                         accumulate ? 1 : 0, dcode(part), cur_stream());
  return out;
}

Tensor add3(Tensor a, Tensor b, OptT c) {
  check_dev(a, "add3"); check_dev(b, "add3");
  TORCH_CHECK(a.sizes() == b.sizes() && a.scalar_type() == b.scalar_type() && a.is_contiguous() && b.is_contiguous(),
              "add3: a and b must match and be contiguous");
  if (c.has_value())
    TORCH_CHECK(c->sizes() == a.sizes() && c->scalar_type() == a.scalar_type() && c->is_contiguous(), "add3: c");
  const int vn = a.scalar_type() == at::kFloat ? 4 : 8;
  TORCH_CHECK(a.numel() % vn == 0, "add3: numel must be a multiple of 16 bytes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  Tensor y = at::empty_like(a);
  dsa::launch_add3(a.data_ptr(), b.data_ptr(), c.has_value() ? c->data_ptr() : nullptr, y.data_ptr(), a.numel(),
                   dcode(a), cur_stream());
  return y;
}

Tensor bias_gelu_fwd(Tensor x, OptT b, bool approx, OptT out) {
  check_dev(x, "x");
  const int64_t C = x.size(-1);
  const int dt = dcode(x);
  TORCH_CHECK(C % (dt == dsa::kCodeF32 ? 4 : 8) == 0, "bias_gelu: last dim must be a multiple of 16 bytes");
  if (b.has_value()) TORCH_CHECK(b->numel() == C && b->scalar_type() == x.scalar_type(), "bias_gelu: bias");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = out_or_empty(out, x, "bias_gelu_fwd");
  dsa::launch_bias_gelu_fwd(x.data_ptr(), b.has_value() ? b->data_ptr() : nullptr, y.data_ptr(), x.numel() / C,
                            (int)C, approx ? 1 : 0, dt, cur_stream());
  return y;
}

// Returns (dx, dbias)
// db_acc: a bound bias gradient the column sums are accumulated into (returned as db)
std::vector<Tensor> bias_gelu_bwd(Tensor dy, Tensor x, OptT b, bool approx, OptT dx_out, OptT db_acc) {
  check_dev(dy, "dy"); check_dev(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "bias_gelu_bwd: mismatch");
  const int64_t C = x.size(-1);
  const int64_t rows = x.numel() / C;
  const int dt = dcode(x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor dx = out_or_empty(dx_out, x, "bias_gelu_bwd");
  Tensor db, partial;
  if (b.has_value()) {
    if (db_acc.has_value())
      TORCH_CHECK(db_acc->sizes() == b->sizes() && db_acc->scalar_type() == b->scalar_type() && db_acc->is_contiguous(),
                  "bias_gelu_bwd: db_acc must match the bias");
    db = db_acc.has_value() ? *db_acc : at::empty_like(*b);
    partial = at::empty({(int64_t)dsa::bias_gelu_row_chunks(rows, (int)C, dt) * C}, x.options().dtype(at::kFloat));
  }
  dsa::launch_bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), b.has_value() ? b->data_ptr() : nullptr, dx.data_ptr(),
                            b.has_value() ? db.data_ptr() : nullptr,
                            b.has_value() ? partial.data_ptr<float>() : nullptr, rows, (int)C, approx ? 1 : 0, dt,
                            cur_stream(), db_acc.has_value() ? 1 : 0);
  return {dx, db};
}

// Sum over all leading dims -> [C]
// out[C] (+)= column sums of x [..., C]; a fresh out when none is given
Tensor colsum(Tensor x, OptT out_opt, bool accumulate) {
  check_dev(x, "x");
  const int64_t C = x.size(-1);
  const int64_t rows = x.numel() / C;
  const int dt = dcode(x);
  TORCH_CHECK(C % (dt == dsa::kCodeF32 ? 4 : 8) == 0, "colsum: last dim must be a multiple of 16 bytes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor out;
  if (out_opt.has_value()) {
    out = *out_opt;
    check_dev(out, "colsum out");
    TORCH_CHECK(out.numel() == C && out.is_contiguous() && out.scalar_type() == x.scalar_type(),
                "colsum: out must be a contiguous [C] tensor of x's dtype");
  } else {
    TORCH_CHECK(!accumulate, "colsum: accumulate needs out");
    out = at::empty({C}, x.options());
  }
  Tensor partial =
      at::empty({(int64_t)dsa::bias_gelu_row_chunks(rows, (int)C, dt) * C}, x.options().dtype(at::kFloat));
  dsa::launch_colsum(x.data_ptr(), out.data_ptr(), partial.data_ptr<float>(), rows, (int)C, accumulate ? 1 : 0, dt,
                     cur_stream());
  return out;
}

// y = x^T for a 2-D 16-bit x [R, C] (unit column stride, any 16-byte aligned row stride).
// With colsum_out ([C], x's dtype) the column sums of x are also written (accum: added) there.
Tensor transpose2d(Tensor x, OptT colsum_out, bool accum, OptT out) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "transpose2d: x must be a 2-D GPU tensor, unit column stride");
  const int dt = dcode(x);
  TORCH_CHECK(dt != dsa::kCodeF32, "transpose2d: 16-bit dtypes only");
  const int64_t R = x.size(0), C = x.size(1), ldx = x.stride(0);
  TORCH_CHECK(dsa::transpose_supported(R, C), "transpose2d: rows must be a multiple of 128 and cols of 64");
  TORCH_CHECK(aligned16(x.data_ptr()) && ldx % 8 == 0, "transpose2d: rows must be 16-byte aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y;
  if (out.has_value()) {  // caller-owned destination (a persistent prefetch buffer)
    check_dev(*out, "out");
    TORCH_CHECK(out->dim() == 2 && out->size(0) == C && out->size(1) == R && out->is_contiguous() &&
                    out->scalar_type() == x.scalar_type() && aligned16(out->data_ptr()),
                "transpose2d: out must be a contiguous [C, R] tensor of x's dtype, 16-byte aligned");
    y = *out;
  } else {
    y = at::empty({C, R}, x.options());
  }
  Tensor partial;
  void* cptr = nullptr;
  if (colsum_out.has_value()) {
    check_dev(*colsum_out, "colsum_out");
    TORCH_CHECK(colsum_out->numel() == C && colsum_out->scalar_type() == x.scalar_type(),
                "transpose2d: colsum_out must be [C] in x's dtype");
    partial = at::empty({dsa::transpose_partial_rows(R) * C}, x.options().dtype(at::kFloat));
    cptr = colsum_out->data_ptr();
  }
  dsa::launch_transpose(x.data_ptr(), y.data_ptr(), partial.defined() ? partial.data_ptr<float>() : nullptr, cptr,
                        accum ? 1 : 0, R, (int)C, ldx, dt, cur_stream());
  return y;
}

// [L, R, C] -> [L, C, R] for a contiguous 16-bit stack (R % 128 == 0, C % 64 == 0) in one launch:
// the per-step W^T of every weight of a stack (ops/wgrad_batch.py stacked_wt)
Tensor transpose_batched(Tensor x, Tensor out) {
  check_dev(x, "x");
  check_dev(out, "out");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous() && aligned16(x.data_ptr()), "transpose_batched: contiguous [L, R, C] x");
  const int dt = dcode(x);
  TORCH_CHECK(dt != dsa::kCodeF32, "transpose_batched: 16-bit dtypes only");
  const int64_t L = x.size(0), R = x.size(1), C = x.size(2);
  TORCH_CHECK(dsa::transpose_supported(R, C), "transpose_batched: rows must be a multiple of 128 and cols of 64");
  TORCH_CHECK(out.dim() == 3 && out.size(0) == L && out.size(1) == C && out.size(2) == R && out.is_contiguous() &&
                  out.scalar_type() == x.scalar_type() && aligned16(out.data_ptr()),
              "transpose_batched: out must be a contiguous [L, C, R] tensor of x's dtype");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  if (L > 0) dsa::launch_transpose_batched(x.data_ptr(), out.data_ptr(), (int)L, R, (int)C, C, dt, cur_stream());
  return out;
}

// gelu(x + b)^T for x [R, C] contiguous 16-bit (R % 128 == 0, C % 64 == 0): the activation
// recompute's fc1 output handed straight to fc2's weight gradient in the layout it wants.
Tensor bias_gelu_fwd_t(Tensor x, OptT b, bool approx) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && aligned16(x.data_ptr()), "bias_gelu_fwd_t: x must be contiguous 2-D");
  const int dt = dcode(x);
  TORCH_CHECK(dt != dsa::kCodeF32, "bias_gelu_fwd_t: 16-bit dtypes only");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(dsa::transpose_supported(R, C), "bias_gelu_fwd_t: rows must be a multiple of 128 and cols of 64");
  if (b.has_value()) TORCH_CHECK(b->numel() == C && b->scalar_type() == x.scalar_type() && b->is_contiguous(),
                                 "bias_gelu_fwd_t: bias");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor yt = at::empty({C, R}, x.options());
  dsa::launch_bias_gelu_fwd_t(x.data_ptr(), b.has_value() ? b->data_ptr() : nullptr, yt.data_ptr(), R, (int)C,
                              approx ? 1 : 0, dt, cur_stream());
  return yt;
}

// Returns (dx, dx^T, dbias): dx = dy * gelu'(x + b) for contiguous 2-D dy, x [R, C].
std::vector<Tensor> bias_gelu_bwd_t(Tensor dy, Tensor x, OptT b, bool approx) {
  check_dev(dy, "dy"); check_dev(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type() && x.dim() == 2 && x.is_contiguous() &&
              dy.is_contiguous() && aligned16(x.data_ptr()) && aligned16(dy.data_ptr()), "bias_gelu_bwd_t: operands");
  const int dt = dcode(x);
  TORCH_CHECK(dt != dsa::kCodeF32, "bias_gelu_bwd_t: 16-bit dtypes only");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(dsa::transpose_supported(R, C), "bias_gelu_bwd_t: rows must be a multiple of 128 and cols of 64");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor dx = at::empty_like(x), dxt = at::empty({C, R}, x.options());
  Tensor db, partial;
  if (b.has_value()) {
    TORCH_CHECK(b->numel() == C && b->scalar_type() == x.scalar_type() && b->is_contiguous(), "bias_gelu_bwd_t: bias");
    db = at::empty_like(*b);
    partial = at::empty({dsa::transpose_partial_rows(R) * C}, x.options().dtype(at::kFloat));
  }
  dsa::launch_bias_gelu_bwd_t(dy.data_ptr(), x.data_ptr(), b.has_value() ? b->data_ptr() : nullptr, dx.data_ptr(),
                              dxt.data_ptr(), partial.defined() ? partial.data_ptr<float>() : nullptr,
                              b.has_value() ? db.data_ptr() : nullptr, R, (int)C, approx ? 1 : 0, dt, cur_stream());
  return {dx, dxt, db};
}

// BERT head layout moves (16-bit, head dim % 8 == 0)
std::vector<Tensor> heads_split(Tensor qkv, int64_t NH) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) % (3 * NH) == 0 && qkv.element_size() == 2, "heads_split: qkv [B,S,3*NH*HD] 16-bit");
  const int64_t B = qkv.size(0), S = qkv.size(1), HD = qkv.size(2) / (3 * NH);
  TORCH_CHECK(HD % 8 == 0 && aligned16(qkv.data_ptr()), "heads_split: head dim % 8, 16-byte aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  auto o = qkv.options();
  Tensor q = at::empty({B, NH, S, HD}, o), k = at::empty({B, NH, S, HD}, o), v = at::empty({B, NH, S, HD}, o);
  dsa::launch_heads_split(qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), (int)B, (int)S, (int)NH, (int)HD,
                          cur_stream());
  return {q, k, v};
}

Tensor heads_merge(Tensor q, Tensor k, Tensor v) {
  check_dev(q, "q"); check_dev(k, "k"); check_dev(v, "v");
  TORCH_CHECK(q.dim() == 4 && q.sizes() == k.sizes() && q.sizes() == v.sizes() && q.element_size() == 2,
              "heads_merge: q,k,v [B,NH,S,HD] 16-bit");
  const int64_t B = q.size(0), NH = q.size(1), S = q.size(2), HD = q.size(3);
  TORCH_CHECK(HD % 8 == 0, "heads_merge: head dim % 8");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor qkv = at::empty({B, S, 3 * NH * HD}, q.options());
  dsa::launch_heads_merge(q.data_ptr(), k.data_ptr(), v.data_ptr(), qkv.data_ptr(), (int)B, (int)S, (int)NH, (int)HD,
                          cur_stream());
  return qkv;
}

// x [A,P,Q,D] -> contiguous [A,Q,P,D]
Tensor swap12(Tensor x) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.element_size() == 2 && x.size(3) % 8 == 0 && aligned16(x.data_ptr()),
              "swap12: 4-D 16-bit, last dim % 8");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({x.size(0), x.size(2), x.size(1), x.size(3)}, x.options());
  dsa::launch_swap12(x.data_ptr(), y.data_ptr(), x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                     cur_stream());
  return y;
}

// ----------------------------------------------------------------------------- attention elementwise
// qkv [B,S,NH*3*HD] (NeoX per-head q|k|v) -> q,k,v [B,NH,S,HD]; cs [S, ROT/2, 2] fp32
std::vector<Tensor> rotary_split_fwd(Tensor qkv, Tensor cs, int64_t NH, int64_t HD, int64_t ROT, double qscale) {
  check_dev(qkv, "qkv"); check_dev(cs, "cos_sin");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) == NH * 3 * HD, "rotary_split: qkv must be [B,S,NH*3*HD]");
  TORCH_CHECK(HD % 8 == 0 && ROT % 2 == 0 && ROT <= HD, "rotary_split: HD % 8 == 0, ROT even and <= HD");
  TORCH_CHECK(qkv.scalar_type() != at::kFloat, "rotary_split: 16-bit inputs only");
  const int64_t B = qkv.size(0), S = qkv.size(1);
  TORCH_CHECK(cs.scalar_type() == at::kFloat && cs.numel() >= S * (ROT / 2) * 2, "rotary_split: cos/sin table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  auto opts = qkv.options();
  Tensor q = at::empty({B, NH, S, HD}, opts), k = at::empty({B, NH, S, HD}, opts), v = at::empty({B, NH, S, HD}, opts);
  dsa::launch_rotary_split_fwd(qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cs.data_ptr<float>(),
                               (int)B, (int)S, (int)NH, (int)HD, (int)ROT, (float)qscale, dcode(qkv), cur_stream());
  return {q, k, v};
}

Tensor rotary_split_bwd(Tensor dq, Tensor dk, Tensor dv, Tensor cs, int64_t ROT, double qscale) {
  check_dev(dq, "dq"); check_dev(dk, "dk"); check_dev(dv, "dv");
  TORCH_CHECK(dq.dim() == 4 && dq.sizes() == dk.sizes() && dq.sizes() == dv.sizes(), "rotary_split_bwd: shapes");
  const int64_t B = dq.size(0), NH = dq.size(1), S = dq.size(2), HD = dq.size(3);
  TORCH_CHECK(HD % 8 == 0, "rotary_split_bwd: HD % 8");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dq.device());
  Tensor dqkv = at::empty({B, S, NH * 3 * HD}, dq.options());
  dsa::launch_rotary_split_bwd(dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dqkv.data_ptr(), cs.data_ptr<float>(),
                               (int)B, (int)S, (int)NH, (int)HD, (int)ROT, (float)qscale, dcode(dq), cur_stream());
  return dqkv;
}

// scores [..., Sq, C] -> probs. mask: optional additive [Bm, 1|.., Sq, C] broadcast over heads.
Tensor softmax_fwd(Tensor x, OptT mask, double scale, bool causal, int64_t heads) {
  check_dev(x, "scores");
  TORCH_CHECK(x.scalar_type() != at::kFloat, "softmax: 16-bit inputs only");
  const int64_t C = x.size(-1), Sq = x.size(-2);
  const int64_t R = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= dsa::softmax_max_cols(), "softmax: key length must be a multiple of 8 and <= ",
              dsa::softmax_max_cols());
  if (mask.has_value()) {
    check_dev(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == x.scalar_type() && mask->size(-1) == C &&
                (mask->size(-2) == Sq || mask->size(-2) == 1) && mask->is_contiguous(),
                "softmax: mask must be [B,1,Sq|1,C] in the score dtype");
    TORCH_CHECK(mask->numel() / (mask->size(-2) * C) * heads * Sq * C == x.numel(), "softmax: mask batch mismatch");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty_like(x);
  dsa::launch_softmax_fwd(x.data_ptr(), y.data_ptr(), mask.has_value() ? mask->data_ptr() : nullptr, R, (int)C,
                          (int)Sq, (int)heads, (float)scale, causal ? 1 : 0,
                          mask.has_value() ? (int)mask->size(-2) : 1, dcode(x), cur_stream());
  return y;
}

Tensor softmax_bwd(Tensor dy, Tensor y, double scale) {
  check_dev(dy, "dy"); check_dev(y, "y");
  TORCH_CHECK(dy.sizes() == y.sizes() && dy.scalar_type() == y.scalar_type(), "softmax_bwd: mismatch");
  const int64_t C = y.size(-1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  Tensor dx = at::empty_like(y);
  dsa::launch_softmax_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), y.numel() / C, (int)C, (float)scale, dcode(y),
                          cur_stream());
  return dx;
}

// 1-bit compression. worker: m, err fp32 [n] (n % 8 == 0) -> (packed uint8 [n/8], scale [1]);
// err is updated in place with the new compression error.
std::vector<Tensor> onebit_worker_compress(Tensor m, Tensor err, Tensor ws) {
  check_dev(m, "m"); check_dev(err, "err");
  TORCH_CHECK(m.scalar_type() == at::kFloat && err.scalar_type() == at::kFloat && m.numel() == err.numel() &&
              m.numel() % 8 == 0, "onebit: fp32 m/err of equal length, multiple of 8");
  TORCH_CHECK(ws.numel() >= 1024 && ws.scalar_type() == at::kFloat, "onebit: workspace");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(m.device());
  Tensor packed = at::empty({m.numel() / 8}, m.options().dtype(at::kByte));
  Tensor scale = at::empty({1}, m.options());
  dsa::launch_onebit_worker(m.data_ptr<float>(), err.data_ptr<float>(), m.numel(), packed.data_ptr<uint8_t>(),
                            scale.data_ptr<float>(), ws.data_ptr<float>(), cur_stream());
  return {packed, scale};
}

// server: signs uint8 [P * nbytes], scales fp32 [P], server_err fp32 [nbytes*8] (updated)
std::vector<Tensor> onebit_server_compress(Tensor signs, Tensor scales, Tensor server_err, Tensor ws) {
  check_dev(signs, "signs"); check_dev(scales, "scales"); check_dev(server_err, "server_err");
  const int64_t P = scales.numel();
  const int64_t nbytes = server_err.numel() / 8;
  TORCH_CHECK(signs.scalar_type() == at::kByte && signs.numel() == P * nbytes && server_err.numel() % 8 == 0,
              "onebit_server: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(signs.device());
  Tensor packed = at::empty({nbytes}, signs.options());
  Tensor scale = at::empty({1}, scales.options());
  dsa::launch_onebit_server(signs.data_ptr<uint8_t>(), scales.data_ptr<float>(), (int)P, nbytes,
                            server_err.data_ptr<float>(), packed.data_ptr<uint8_t>(), scale.data_ptr<float>(),
                            ws.data_ptr<float>(), cur_stream());
  return {packed, scale};
}

// unpack: signs uint8 [P * nbytes_per], scales fp32 [P] -> out fp32 [P * nbytes_per * 8]
void onebit_unpack(Tensor signs, Tensor scales, Tensor out) {
  check_dev(signs, "signs"); check_dev(out, "out");
  const int64_t P = scales.numel();
  TORCH_CHECK(signs.numel() % P == 0 && out.numel() == signs.numel() * 8 && out.scalar_type() == at::kFloat &&
              (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0, "onebit_unpack: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(signs.device());
  dsa::launch_onebit_unpack(signs.data_ptr<uint8_t>(), scales.data_ptr<float>(), (int)P, signs.numel() / P,
                            out.data_ptr<float>(), cur_stream());
}

// ----------------------------------------------------------------------------- block-sparse attention
// A 16-bit [Z,H,R,K] operand of the sparse products, unit stride along K (returns false) or
// along R (returns true), every other stride and the base 16-byte aligned (sparse_attn.hip
// stages 16-byte chunks along the unit-stride dim).  The Python side normalises anything else.
static bool sparse_mat(const Tensor& x, const char* name, int64_t* st) {
  TORCH_CHECK(x.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() != at::kFloat, "sparse ", name, ": 16-bit [Z,H,R,K]");
  for (int d = 0; d < 4; ++d) st[d] = x.size(d) == 1 ? 0 : x.stride(d);
  const bool t = x.stride(3) != 1 || x.size(3) == 1;
  const int u = t ? 2 : 3;
  TORCH_CHECK(x.stride(u) == 1 || x.size(u) == 1, "sparse ", name, ": needs a unit-stride last or second-last dim");
  st[u] = 1;
  bool ok = x.size(u) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0;
  for (int d = 0; d < 4; ++d)
    if (d != u) ok = ok && st[d] % 8 == 0;
  TORCH_CHECK(ok, "sparse ", name, ": unit-stride extent, strides and base must be multiples of 8 elements");
  return t;
}

// sdd: C[z][n] = alpha * A[rows of r] . B[rows of c]^T; A [Z,H,Mr,K], B [Z,H,Nr,K] (views)
Tensor sparse_sdd(Tensor A, Tensor B, Tensor nz, int64_t blk, double alpha) {
  int64_t sa[4], sb[4];
  const bool at = sparse_mat(A, "A", sa), bt = sparse_mat(B, "B", sb);
  check_dev(nz, "nz");
  TORCH_CHECK(A.size(0) == B.size(0) && A.size(1) == B.size(1) && A.size(3) == B.size(3) &&
              A.scalar_type() == B.scalar_type(), "sparse_sdd: A/B must match in Z, H, K and dtype");
  TORCH_CHECK((blk == 16 || blk == 32 || blk == 64 || blk == 128) && A.size(2) % blk == 0 && B.size(2) % blk == 0,
              "sparse_sdd: block in {16,32,64,128} dividing the rows");
  TORCH_CHECK(nz.scalar_type() == at::kInt && nz.dim() == 2 && nz.size(1) == 3 && nz.is_contiguous(),
              "sparse_sdd: nz int32 [nnz,3]");
  const int64_t nnz = nz.size(0);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  Tensor C = at::empty({A.size(0), nnz, blk, blk}, A.options());
  dsa::launch_sparse_sdd(A.data_ptr(), sa, at, B.data_ptr(), sb, bt, C.data_ptr(), nz.data_ptr<int>(), (int)nnz,
                         (int)A.size(0), (int)A.size(3), (int)blk, (float)alpha, dcode(A), cur_stream());
  return C;
}

// dsd: C[z,h, rows of r, :] = sum over the row's blocks of S_eff . D[rows of col, :]; S [Z,nnz,blk,blk]
// contiguous; seg int32 [nseg,4] = (h*nbr + r, first, end, partial slot | -1) covering every row,
// fin int32 [nfin,4] = (h*nbr + r, slot0, nslots, 0) for split rows; perm (optional) = walk of
// layout^T (S_eff = stored block perm[p] transposed); D [Z,H,Kd,N] and the preallocated
// C [Z,H,nbr*blk,N] are views of either orientation.
void sparse_dsd(Tensor S, Tensor seg, Tensor fin, int64_t nslots, Tensor cols, OptT perm, Tensor D, Tensor C,
                int64_t H, int64_t nbr, int64_t blk) {
  check_dev(S, "S"); check_dev(seg, "seg"); check_dev(fin, "fin"); check_dev(cols, "cols");
  int64_t sd[4], sc[4];
  const bool dtr = sparse_mat(D, "D", sd), ctr = sparse_mat(C, "C", sc);
  TORCH_CHECK(S.dim() == 4 && S.is_contiguous() && S.size(2) == blk && S.size(3) == blk &&
              S.scalar_type() == D.scalar_type() && C.scalar_type() == D.scalar_type(), "sparse_dsd: S");
  TORCH_CHECK((blk == 16 || blk == 32 || blk == 64 || blk == 128) && D.size(0) == S.size(0) && D.size(1) == H &&
              D.size(2) % blk == 0 && C.size(0) == S.size(0) && C.size(1) == H && C.size(2) == nbr * blk &&
              C.size(3) == D.size(3), "sparse_dsd: shapes");
  TORCH_CHECK(seg.scalar_type() == at::kInt && seg.dim() == 2 && seg.size(1) == 4 && fin.scalar_type() == at::kInt &&
              fin.dim() == 2 && fin.size(1) == 4 && cols.scalar_type() == at::kInt && cols.numel() == S.size(1),
              "sparse_dsd: LUTs");
  if (perm.has_value()) {
    check_dev(*perm, "perm");
    TORCH_CHECK(perm->scalar_type() == at::kInt && perm->numel() == S.size(1), "sparse_dsd: perm int32 [nnz]");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  const int64_t N = D.size(3), Np = (N + 63) / 64 * 64;
  Tensor ws;
  if (nslots > 0) ws = at::empty({S.size(0), nslots, blk, Np}, S.options().dtype(at::kFloat));
  dsa::launch_sparse_dsd(S.data_ptr(), seg.data_ptr<int>(), (int)seg.size(0), fin.data_ptr<int>(), (int)fin.size(0),
                         cols.data_ptr<int>(), perm.has_value() ? perm->data_ptr<int>() : nullptr, D.data_ptr(), sd,
                         dtr, C.data_ptr(), sc, ctr, nslots > 0 ? ws.data_ptr<float>() : nullptr, (int)nslots,
                         (int)S.size(1), (int)S.size(0), (int)nbr, (int)N, (int)blk, dcode(S), cur_stream());
}

// softmax over the non-zero blocks of each row, x -> y (may alias); max_row = longest row (elements)
void sparse_softmax_fwd(Tensor x, Tensor y, Tensor rowptr, Tensor cols, int64_t H, int64_t nbr, int64_t max_row,
                        double scale, OptT rpe, OptT kpm, OptT attn, bool kpm_mul, bool attn_mul, bool causal) {
  check_dev(x, "x"); check_dev(y, "y");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && y.is_contiguous() && x.sizes() == y.sizes() &&
              x.scalar_type() == y.scalar_type() && x.size(2) % 16 == 0, "sparse softmax: x/y [Z,nnz,blk,blk]");
  const int64_t blk = x.size(2), S = nbr * blk;
  int64_t rsz = 0, rsh = 0, rsr = 0, ksz = 0, asr = 0;
  if (rpe.has_value()) {
    TORCH_CHECK(rpe->dim() == 4 && rpe->size(2) == S && rpe->size(3) == S && rpe->stride(3) == 1 &&
                rpe->scalar_type() == x.scalar_type(), "sparse softmax: rpe [Z|1,H|1,S,S]");
    rsz = rpe->size(0) == 1 ? 0 : rpe->stride(0);
    rsh = rpe->size(1) == 1 ? 0 : rpe->stride(1);
    rsr = rpe->stride(2);
  }
  if (kpm.has_value()) {
    TORCH_CHECK(kpm->dim() == 2 && kpm->size(1) == S && kpm->stride(1) == 1 && kpm->scalar_type() == x.scalar_type(),
                "sparse softmax: key padding mask [Z,S]");
    ksz = kpm->size(0) == 1 ? 0 : kpm->stride(0);
  }
  if (attn.has_value()) {
    TORCH_CHECK(attn->dim() == 2 && attn->size(0) == S && attn->size(1) == S && attn->stride(1) == 1 &&
                attn->scalar_type() == x.scalar_type(), "sparse softmax: attn mask [S,S]");
    asr = attn->stride(0);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  dsa::launch_sparse_softmax_fwd(x.data_ptr(), y.data_ptr(), rowptr.data_ptr<int>(), cols.data_ptr<int>(),
                                 (int)x.size(1), (int)x.size(0), (int)H, (int)nbr, (int)blk, (int)max_row,
                                 rpe.has_value() ? rpe->data_ptr() : nullptr, rsz, rsh, rsr,
                                 kpm.has_value() ? kpm->data_ptr() : nullptr, ksz,
                                 attn.has_value() ? attn->data_ptr() : nullptr, asr, kpm_mul ? 1 : 0,
                                 attn_mul ? 1 : 0, (float)scale, causal ? 1 : 0, dcode(x), cur_stream());
}

void sparse_softmax_bwd(Tensor y, Tensor dy, Tensor dx, Tensor rowptr, int64_t H, int64_t nbr, int64_t max_row,
                        double scale) {
  check_dev(y, "y"); check_dev(dy, "dy"); check_dev(dx, "dx");
  TORCH_CHECK(y.sizes() == dy.sizes() && y.sizes() == dx.sizes() && y.scalar_type() == dy.scalar_type() &&
              dx.scalar_type() == y.scalar_type() && y.is_contiguous() && dy.is_contiguous() && dx.is_contiguous() &&
              y.size(2) % 16 == 0, "sparse softmax bwd: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  dsa::launch_sparse_softmax_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), rowptr.data_ptr<int>(), (int)y.size(1),
                                 (int)y.size(0), (int)H, (int)nbr, (int)y.size(2), (int)max_row, (float)scale,
                                 dcode(y), cur_stream());
}

// ----------------------------------------------------------------------------- dropout
// optional device RNG state int64 [seed, step] (graph-replayable dropout, dropout.hip rng_apply)
static const int64_t* rng_ptr(const OptT& rng, const Tensor& like) {
  if (!rng.has_value()) return nullptr;
  TORCH_CHECK(rng->scalar_type() == at::kLong && rng->numel() == 2 && rng->is_contiguous() &&
              rng->device() == like.device(), "rng must be a contiguous int64 [seed, step] on the tensor's device");
  return rng->data_ptr<int64_t>();
}

std::vector<Tensor> dropout_fwd(Tensor x, double p, int64_t seed, int64_t offset, OptT rng) {
  check_dev(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty_like(x);
  Tensor mask = at::empty(x.sizes(), x.options().dtype(at::kByte));
  dsa::launch_dropout_fwd(x.data_ptr(), y.data_ptr(), mask.data_ptr<uint8_t>(), x.numel(), (float)p, (uint64_t)seed,
                          (uint64_t)offset, dcode(x), cur_stream(), rng_ptr(rng, x));
  return {y, mask};
}

// y = res + dropout(x + bias); x/res [rows, C], bias [C]
std::vector<Tensor> bias_dropout_residual(Tensor x, Tensor bias, Tensor res, double p, int64_t seed, int64_t offset,
                                          OptT rng) {
  check_dev(x, "x"); check_dev(bias, "bias"); check_dev(res, "res");
  const int64_t C = x.size(-1);
  TORCH_CHECK(bias.numel() == C && res.sizes() == x.sizes() && x.scalar_type() == res.scalar_type() &&
              bias.scalar_type() == x.scalar_type(), "bias_dropout_residual: shapes/dtypes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty_like(x);
  Tensor mask = at::empty(x.sizes(), x.options().dtype(at::kByte));
  dsa::launch_bias_dropout_residual(x.data_ptr(), bias.data_ptr(), res.data_ptr(), y.data_ptr(),
                                    mask.data_ptr<uint8_t>(), x.numel() / C, (int)C, (float)p, (uint64_t)seed,
                                    (uint64_t)offset, dcode(x), cur_stream(), rng_ptr(rng, x));
  return {y, mask};
}

// (y, out, mask, mean, rstd): out = res + dropout(x + bias), y = LayerNorm(out) in one pass
std::vector<Tensor> bdr_ln_fwd(Tensor x, Tensor bias, Tensor res, Tensor gamma, OptT beta, double p, double eps,
                               int64_t seed, int64_t offset, OptT rng, OptT y_out) {
  check_dev(x, "x"); check_dev(bias, "bias"); check_dev(res, "res"); check_dev(gamma, "gamma");
  const int64_t H = x.size(-1), rows = x.numel() / H;
  const int dt = dcode(x);
  TORCH_CHECK(dsa::bdr_ln_supported((int)H, dt), "bdr_ln_fwd: 16-bit rows of <= 1024 elements (multiple of 8)");
  TORCH_CHECK(x.is_contiguous() && res.is_contiguous() && res.sizes() == x.sizes() &&
                  res.scalar_type() == x.scalar_type(), "bdr_ln_fwd: contiguous x / res of one shape and dtype");
  TORCH_CHECK(bias.numel() == H && bias.is_contiguous() && bias.scalar_type() == x.scalar_type(), "bdr_ln_fwd: bias");
  TORCH_CHECK(gamma.numel() == H && gamma.is_contiguous() && gamma.scalar_type() == x.scalar_type(),
              "bdr_ln_fwd: gamma");
  if (beta.has_value())
    TORCH_CHECK(beta->numel() == H && beta->is_contiguous() && beta->scalar_type() == x.scalar_type(),
                "bdr_ln_fwd: beta");
  for (const Tensor* t : {&x, &res, &bias, &gamma})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "bdr_ln_fwd: 16-byte aligned tensors");
  if (beta.has_value()) TORCH_CHECK(reinterpret_cast<uintptr_t>(beta->data_ptr()) % 16 == 0, "bdr_ln_fwd: beta align");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor out = at::empty_like(x), y = out_or_empty(y_out, x, "bdr_ln_fwd");
  Tensor mask = at::empty(x.sizes(), x.options().dtype(at::kByte));
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({rows}, f32), rstd = at::empty({rows}, f32);
  dsa::launch_bdr_ln_fwd(x.data_ptr(), bias.data_ptr(), res.data_ptr(), out.data_ptr(), mask.data_ptr<uint8_t>(),
                         gamma.data_ptr(), beta.has_value() ? beta->data_ptr() : nullptr, y.data_ptr(),
                         mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)H, (float)p, (float)eps,
                         (uint64_t)seed, (uint64_t)offset, dt, cur_stream(), rng_ptr(rng, x));
  return {y, out, mask, mean, rstd};
}

// (dtot, dxb, dgamma, dbeta, dbias) of bdr_ln_fwd: dtot = d(out) (the residual input's gradient),
// dxb = the branch input's.  *_acc: bound gradient buffers accumulated into (returned as is).
std::vector<Tensor> bdr_ln_bwd(Tensor dy, Tensor out, Tensor gamma, Tensor mean, Tensor rstd, bool has_beta,
                               OptT dres, Tensor mask, double p, OptT dgamma_acc, OptT dbeta_acc, OptT dbias_acc,
                               OptT dxb_out) {
  check_dev(dy, "dy"); check_dev(out, "out"); check_dev(mask, "mask");
  const int64_t H = out.size(-1), rows = out.numel() / H;
  const int dt = dcode(out);
  TORCH_CHECK(dsa::bdr_ln_supported((int)H, dt), "bdr_ln_bwd: 16-bit rows of <= 1024 elements");
  TORCH_CHECK(dy.is_contiguous() && dy.sizes() == out.sizes() && dy.scalar_type() == out.scalar_type() &&
                  out.is_contiguous(), "bdr_ln_bwd: contiguous dy / out of one shape");
  TORCH_CHECK(mask.is_contiguous() && mask.numel() == out.numel() && mask.scalar_type() == at::kByte,
              "bdr_ln_bwd: uint8 mask of out's size");
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "bdr_ln_bwd: stats size");
  if (dres.has_value())
    TORCH_CHECK(dres->sizes() == out.sizes() && dres->is_contiguous() && dres->scalar_type() == out.scalar_type(),
                "bdr_ln_bwd: dres");
  auto like_gamma = [&](const OptT& t, const char* what) {
    TORCH_CHECK(t->numel() == H && t->is_contiguous() && t->scalar_type() == gamma.scalar_type(), what);
  };
  const bool acc = dgamma_acc.has_value();
  if (acc) {
    like_gamma(dgamma_acc, "bdr_ln_bwd: dgamma_acc");
    TORCH_CHECK(!has_beta || dbeta_acc.has_value(), "bdr_ln_bwd: dbeta_acc");
    if (has_beta) like_gamma(dbeta_acc, "bdr_ln_bwd: dbeta_acc");
  }
  if (dbias_acc.has_value()) like_gamma(dbias_acc, "bdr_ln_bwd: dbias_acc");
  for (const Tensor* t : {&dy, &out, &gamma})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "bdr_ln_bwd: 16-byte aligned tensors");
  if (dres.has_value()) TORCH_CHECK(reinterpret_cast<uintptr_t>(dres->data_ptr()) % 16 == 0, "bdr_ln_bwd: dres align");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(mask.data_ptr()) % 8 == 0, "bdr_ln_bwd: mask align");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  Tensor dtot = at::empty_like(out), dxb = out_or_empty(dxb_out, out, "bdr_ln_bwd");
  Tensor dgamma = acc ? *dgamma_acc : at::empty_like(gamma);
  Tensor dbeta = has_beta ? (acc ? *dbeta_acc : at::empty_like(gamma)) : Tensor();
  Tensor dbias = dbias_acc.has_value() ? *dbias_acc : at::empty_like(gamma);
  const int grid = dsa::bdr_ln_bwd_grid(rows);
  Tensor partial = at::empty({3 * (int64_t)grid * H}, out.options().dtype(at::kFloat));
  dsa::launch_bdr_ln_bwd(dy.data_ptr(), out.data_ptr(), gamma.data_ptr(), mean.data_ptr<float>(),
                         rstd.data_ptr<float>(), dres.has_value() ? dres->data_ptr() : nullptr,
                         mask.data_ptr<uint8_t>(), dtot.data_ptr(), dxb.data_ptr(), dgamma.data_ptr(),
                         has_beta ? dbeta.data_ptr() : nullptr, dbias.data_ptr(), partial.data_ptr<float>(), rows,
                         (int)H, (float)p, acc ? 1 : 0, dbias_acc.has_value() ? 1 : 0, dt, cur_stream());
  return {dtot, dxb, dgamma, dbeta, dbias};
}

// (dx, db) for a bias + dropout + residual block: dx = dy * mask / (1 - p), db = column sums of dx
std::vector<Tensor> dropout_bwd_db(Tensor dy, Tensor mask, double p) {
  check_dev(dy, "dropout_bwd_db"); check_dev(mask, "dropout_bwd_db");
  TORCH_CHECK(dy.is_contiguous() && mask.is_contiguous() && mask.numel() == dy.numel() &&
                  mask.scalar_type() == at::kByte, "dropout_bwd_db: contiguous dy and uint8 mask of its size");
  const int64_t C = dy.size(-1), rows = dy.numel() / C;
  const int dt = dcode(dy);
  const int vn = dt == dsa::kCodeF32 ? 4 : 8;
  TORCH_CHECK(C % vn == 0 && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(mask.data_ptr()) % 8 == 0, "dropout_bwd_db: 16-byte rows");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  int cb, rc, pr;
  dsa::dropout_bwd_colsum_dims(rows, (int)C, dt, &cb, &rc, &pr);
  Tensor dx = at::empty_like(dy);
  Tensor db = at::empty({C}, dy.options());
  Tensor partial = at::empty({(int64_t)pr * C}, dy.options().dtype(at::kFloat));
  dsa::launch_dropout_bwd_colsum(dy.data_ptr(), mask.data_ptr<uint8_t>(), dx.data_ptr(), db.data_ptr(),
                                 partial.data_ptr<float>(), rows, (int)C, (float)p, dt, cur_stream());
  return {dx, db};
}

Tensor dropout_bwd(Tensor dy, Tensor mask, double p) {
  check_dev(dy, "dy"); check_dev(mask, "mask");
  TORCH_CHECK(mask.numel() == dy.numel() && mask.scalar_type() == at::kByte, "dropout_bwd: mask");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = at::empty_like(dy);
  dsa::launch_dropout_bwd(dy.data_ptr(), mask.data_ptr<uint8_t>(), dx.data_ptr(), dy.numel(), (float)p, dcode(dy),
                          cur_stream());
  return dx;
}

// Fused softmax cross-entropy. logits [R, V] 16-bit, labels [R] int64 (<0 = ignored)
// -> (per-row loss fp32 [R], lse fp32 [R])
std::vector<Tensor> xent_fwd(Tensor logits, Tensor labels) {
  check_dev(logits, "logits"); check_dev(labels, "labels");
  TORCH_CHECK(logits.dim() == 2 && logits.scalar_type() != at::kFloat, "xent: 16-bit [rows, vocab] logits");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0), "xent: int64 labels per row");
  TORCH_CHECK(logits.size(1) % 8 == 0, "xent: vocab must be a multiple of 8");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  const int64_t R = logits.size(0);
  Tensor loss = at::empty({R}, logits.options().dtype(at::kFloat));
  Tensor lse = at::empty({R}, logits.options().dtype(at::kFloat));
  dsa::launch_xent_fwd(logits.data_ptr(), labels.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                       R, (int)logits.size(1), dcode(logits), cur_stream());
  return {loss, lse};
}

// dloss: fp32 [R] per-row upstream grads, or a single element broadcast to every row
// inplace: dlogits overwrite the logits (each element is read once, by the thread that writes it)
Tensor xent_bwd(Tensor logits, Tensor labels, Tensor lse, Tensor dloss, bool inplace) {
  check_dev(logits, "logits"); check_dev(dloss, "dloss");
  TORCH_CHECK(dloss.scalar_type() == at::kFloat && (dloss.numel() == 1 || dloss.numel() == logits.size(0)),
              "xent_bwd: dloss");
  TORCH_CHECK(!inplace || logits.is_contiguous(), "xent_bwd: in-place needs contiguous logits");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  Tensor dx = inplace ? logits : at::empty_like(logits);
  dsa::launch_xent_bwd(logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), dloss.data_ptr<float>(),
                       dloss.numel() == 1 ? 0 : 1, dx.data_ptr(), logits.size(0), (int)logits.size(1), dcode(logits),
                       cur_stream());
  return dx;
}

// Fused attention. q,k,v [B, H, S, D] contiguous 16-bit -> (o, lse [B,H,S] fp32) with o [B,H,S,D], or
// [B,S,H,D] when out_bshd (token-major: viewed as [B,S,H*D] by the output projection, no transpose).
std::vector<Tensor> flash_attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, double scale, bool out_bshd) {
  check_dev(q, "q"); check_dev(k, "k"); check_dev(v, "v");
  TORCH_CHECK(q.dim() == 4 && q.sizes() == k.sizes() && q.sizes() == v.sizes(), "flash_attn: q/k/v shape mismatch");
  TORCH_CHECK(q.scalar_type() != at::kFloat && q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(),
              "flash_attn: 16-bit q/k/v of one dtype");
  TORCH_CHECK(q.is_contiguous() && k.is_contiguous() && v.is_contiguous(), "flash_attn: contiguous inputs");
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  TORCH_CHECK(dsa::flash_supported((int)D), "flash_attn: head dim must be 64, 96 or 128");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor o = out_bshd ? at::empty({B, S, H, D}, q.options()) : at::empty_like(q);
  Tensor lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  dsa::launch_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), (int)(B * H),
                        (int)S, (int)D, causal, (float)scale, dcode(q), cur_stream(), out_bshd ? (int)H : 0);
  return {o, lse};
}

// dout and o in the layout flash_attn_fwd produced (o_bshd: [B,S,H,D]); dq, dk, dv [B,H,S,D].
std::vector<Tensor> flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal,
                                   double scale, bool o_bshd) {
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  for (auto* t : {&q, &k, &v}) {
    check_dev(*t, "flash_attn_bwd");
    TORCH_CHECK(t->sizes() == q.sizes() && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "flash_attn_bwd: q/k/v must match");
  }
  const std::vector<int64_t> oshape = o_bshd ? std::vector<int64_t>{B, S, H, D} : std::vector<int64_t>{B, H, S, D};
  for (auto* t : {&dout, &o}) {
    check_dev(*t, "flash_attn_bwd");
    TORCH_CHECK(t->sizes() == at::IntArrayRef(oshape) && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "flash_attn_bwd: dout/o must be contiguous in the forward's output layout");
  }
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == q.numel() / q.size(3),
              "flash_attn_bwd: lse");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  Tensor delta = at::empty_like(lse);
  dsa::launch_flash_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                        delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), (int)(B * H), (int)S,
                        (int)D, causal, (float)scale, dcode(q), cur_stream(), o_bshd ? (int)H : 0);
  return {dq, dk, dv};
}

// Encoder (non-causal) flash attention with an optional additive per-key bias kbias [B, S] fp32
// (the [B,1,1,S] padding mask) and in-kernel attention dropout p_drop, whose keep mask is a hash
// of (seed, b*H+h, query, key) regenerated by the backward.  S % 8 == 0, head dim 64 or 128.
static void check_ex(const Tensor& q, const c10::optional<Tensor>& kbias, double p_drop, const char* what) {
  const int64_t B = q.size(0), S = q.size(2), D = q.size(3);
  TORCH_CHECK(S % 8 == 0 && (D == 64 || D == 128), what, ": S % 8 == 0 and head dim 64 or 128");
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, what, ": dropout probability in [0, 1)");
  TORCH_CHECK(kbias.has_value() || p_drop > 0.0, what, ": needs a key bias or dropout (use flash_attn_fwd)");
  if (kbias.has_value()) {
    check_dev(*kbias, what);
    TORCH_CHECK(kbias->scalar_type() == at::kFloat && kbias->is_contiguous() && kbias->numel() == B * S, what,
                ": kbias must be contiguous fp32 [B, S]");
  }
}

std::vector<Tensor> flash_attn_fwd_ex(Tensor q, Tensor k, Tensor v, c10::optional<Tensor> kbias, double scale,
                                      double p_drop, int64_t seed, bool out_bshd) {
  check_dev(q, "q"); check_dev(k, "k"); check_dev(v, "v");
  TORCH_CHECK(q.dim() == 4 && q.sizes() == k.sizes() && q.sizes() == v.sizes(), "flash_attn_ex: q/k/v shape mismatch");
  TORCH_CHECK(q.scalar_type() != at::kFloat && q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(),
              "flash_attn_ex: 16-bit q/k/v of one dtype");
  TORCH_CHECK(q.is_contiguous() && k.is_contiguous() && v.is_contiguous(), "flash_attn_ex: contiguous inputs");
  check_ex(q, kbias, p_drop, "flash_attn_fwd_ex");
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor o = out_bshd ? at::empty({B, S, H, D}, q.options()) : at::empty_like(q);
  Tensor lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  dsa::launch_flash_fwd_ex(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), (int)(B * H),
                           (int)S, (int)D, (float)scale, kbias ? kbias->data_ptr<float>() : nullptr, (int)H,
                           (float)p_drop, (uint64_t)seed, dcode(q), cur_stream(), out_bshd ? (int)H : 0);
  return {o, lse};
}

std::vector<Tensor> flash_attn_bwd_ex(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse,
                                      c10::optional<Tensor> kbias, double scale, double p_drop, int64_t seed,
                                      bool o_bshd) {
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  for (auto* t : {&q, &k, &v}) {
    check_dev(*t, "flash_attn_bwd_ex");
    TORCH_CHECK(t->sizes() == q.sizes() && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "flash_attn_bwd_ex: q/k/v must match");
  }
  const std::vector<int64_t> oshape = o_bshd ? std::vector<int64_t>{B, S, H, D} : std::vector<int64_t>{B, H, S, D};
  for (auto* t : {&dout, &o}) {
    check_dev(*t, "flash_attn_bwd_ex");
    TORCH_CHECK(t->sizes() == at::IntArrayRef(oshape) && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "flash_attn_bwd_ex: dout/o must be contiguous in the forward's output layout");
  }
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * S,
              "flash_attn_bwd_ex: lse");
  check_ex(q, kbias, p_drop, "flash_attn_bwd_ex");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  Tensor delta = at::empty_like(lse);
  dsa::launch_flash_bwd_ex(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                           lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                           (int)(B * H), (int)S, (int)D, (float)scale, kbias ? kbias->data_ptr<float>() : nullptr,
                           (int)H, (float)p_drop, (uint64_t)seed, dcode(q), cur_stream(), o_bshd ? (int)H : 0);
  return {dq, dk, dv};
}

// The same encoder attention reading q, k, v straight from the fused QKV projection output
// qkv [B, S, 3, H, D] (contiguous) and writing o [B, S, H, D]; the backward writes dqkv in the
// qkv layout, so no head split / merge copies are needed around the kernels.
static void check_qkv(const Tensor& qkv, const char* what) {
  check_dev(qkv, what);
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.is_contiguous() && qkv.scalar_type() != at::kFloat, what,
              ": qkv must be a contiguous 16-bit [B, S, 3, H, D] tensor");
}

std::vector<Tensor> flash_attn_qkv_fwd(Tensor qkv, c10::optional<Tensor> kbias, double scale, double p_drop,
                                       int64_t seed, OptT rng, OptT o_out) {
  check_qkv(qkv, "flash_attn_qkv_fwd");
  const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(3), D = qkv.size(4);
  TORCH_CHECK(S % 8 == 0 && (D == 64 || D == 128), "flash_attn_qkv_fwd: S % 8 == 0 and head dim 64 or 128");
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "flash_attn_qkv_fwd: dropout probability in [0, 1)");
  if (kbias.has_value()) {
    check_dev(*kbias, "flash_attn_qkv_fwd");
    TORCH_CHECK(kbias->scalar_type() == at::kFloat && kbias->is_contiguous() && kbias->numel() == B * S,
                "flash_attn_qkv_fwd: kbias must be contiguous fp32 [B, S]");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  Tensor o = out_or_new(o_out, {B, S, H, D}, qkv.options(), "flash_attn_qkv_fwd");
  Tensor lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  const char* base = static_cast<const char*>(qkv.data_ptr());
  const int64_t hd = H * D * qkv.element_size();
  dsa::launch_flash_fwd_ex(base, base + hd, base + 2 * hd, o.data_ptr(), lse.data_ptr<float>(), (int)(B * H), (int)S,
                           (int)D, (float)scale, kbias ? kbias->data_ptr<float>() : nullptr, (int)H, (float)p_drop,
                           (uint64_t)seed, dcode(qkv), cur_stream(), (int)H, (int)H, 3 * H * D, rng_ptr(rng, qkv));
  return {o, lse};
}

Tensor flash_attn_qkv_bwd(Tensor dout, Tensor qkv, Tensor o, Tensor lse, c10::optional<Tensor> kbias, double scale,
                          double p_drop, int64_t seed, OptT rng, OptT dqkv_out) {
  check_qkv(qkv, "flash_attn_qkv_bwd");
  const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(3), D = qkv.size(4);
  for (auto* t : {&dout, &o}) {
    check_dev(*t, "flash_attn_qkv_bwd");
    TORCH_CHECK(t->sizes() == at::IntArrayRef({B, S, H, D}) && t->scalar_type() == qkv.scalar_type() &&
                    t->is_contiguous(), "flash_attn_qkv_bwd: dout/o must be contiguous [B, S, H, D]");
  }
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * S,
              "flash_attn_qkv_bwd: lse");
  if (kbias.has_value()) {
    check_dev(*kbias, "flash_attn_qkv_bwd");
    TORCH_CHECK(kbias->scalar_type() == at::kFloat && kbias->is_contiguous() && kbias->numel() == B * S,
                "flash_attn_qkv_bwd: kbias");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  Tensor dqkv = out_or_empty(dqkv_out, qkv, "flash_attn_qkv_bwd");
  Tensor delta = at::empty_like(lse);
  const char* base = static_cast<const char*>(qkv.data_ptr());
  char* dbase = static_cast<char*>(dqkv.data_ptr());
  const int64_t hd = H * D * qkv.element_size();
  dsa::launch_flash_bwd_ex(dout.data_ptr(), base, base + hd, base + 2 * hd, o.data_ptr(), lse.data_ptr<float>(),
                           delta.data_ptr<float>(), dbase, dbase + hd, dbase + 2 * hd, (int)(B * H), (int)S, (int)D,
                           (float)scale, kbias ? kbias->data_ptr<float>() : nullptr, (int)H, (float)p_drop,
                           (uint64_t)seed, dcode(qkv), cur_stream(), (int)H, (int)H, 3 * H * D, rng_ptr(rng, qkv));
  return dqkv;
}

// Block-sparse flash attention.  q,k,v [B, H, S, D] (S % 64 == 0); LUT tensors int32 on the
// device (see flash_attn.hip): rowptr [Hl * S/64 + 1], cols / masks [nnz]; the transposed LUT
// colptr / rows / masks_t for the backward.  `shift` = min(6, log2(layout block)).
static void check_lut(const Tensor& ptr, const Tensor& idx, const Tensor& msk, int64_t Hl, int64_t ntiles,
                      const char* what) {
  check_dev(ptr, what); check_dev(idx, what); check_dev(msk, what);
  TORCH_CHECK(ptr.scalar_type() == at::kInt && idx.scalar_type() == at::kInt && msk.scalar_type() == at::kInt &&
                  ptr.is_contiguous() && idx.is_contiguous() && msk.is_contiguous(),
              what, ": int32 contiguous LUT tensors");
  TORCH_CHECK(ptr.numel() == Hl * ntiles + 1, what, ": pointer array must hold Hl * S/64 + 1 entries");
  TORCH_CHECK(idx.numel() == 4 * msk.numel(), what, ": four gathered 16-blocks per mask entry");
}

// Score biases of the fused sparse kernels: kbias [B, S] fp32 (key padding, additive), ebias a
// 16-bit [B|1, H|1, S, S] view in q's dtype (relative position embedding + attention mask) whose
// batch / head strides may be 0.  Returns (kbias ptr, ebias ptr, ez, eh, er).
struct SBias {
  const float* kb = nullptr;
  const void* eb = nullptr;
  int64_t ez = 0, eh = 0, er = 0;
};
static SBias sparse_bias(const OptT& kbias, const OptT& ebias, const Tensor& q) {
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2);
  SBias b;
  if (kbias.has_value()) {
    check_dev(*kbias, "sparse_flash kbias");
    TORCH_CHECK(kbias->scalar_type() == at::kFloat && kbias->is_contiguous() && kbias->dim() == 2 &&
                    kbias->size(0) == B && kbias->size(1) == S, "sparse_flash: kbias must be contiguous fp32 [B, S]");
    b.kb = kbias->data_ptr<float>();
  }
  if (ebias.has_value()) {
    const Tensor& e = *ebias;
    check_dev(e, "sparse_flash ebias");
    TORCH_CHECK(e.scalar_type() == q.scalar_type() && e.dim() == 4 && (e.size(0) == B || e.size(0) == 1) &&
                    (e.size(1) == H || e.size(1) == 1) && e.size(2) == S && e.size(3) == S && e.stride(3) == 1 &&
                    e.stride(2) % 4 == 0, "sparse_flash: ebias must be [B|1, H|1, S, S] in q's dtype, unit key stride");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(e.data_ptr()) % 8 == 0, "sparse_flash: ebias must be 8-byte aligned");
    b.eb = e.data_ptr();
    b.ez = e.size(0) == 1 ? 0 : e.stride(0);
    b.eh = e.size(1) == 1 ? 0 : e.stride(1);
    b.er = e.stride(2);
  }
  return b;
}

std::vector<Tensor> sparse_flash_fwd(Tensor q, Tensor k, Tensor v, Tensor rowptr, Tensor cols, Tensor masks,
                                     int64_t Hl, bool causal, double scale, int64_t shift, bool out_bshd,
                                     OptT kbias, OptT ebias) {
  check_dev(q, "q"); check_dev(k, "k"); check_dev(v, "v");
  TORCH_CHECK(q.dim() == 4 && q.sizes() == k.sizes() && q.sizes() == v.sizes(), "sparse_flash: q/k/v shape mismatch");
  TORCH_CHECK(q.scalar_type() != at::kFloat && q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(),
              "sparse_flash: 16-bit q/k/v of one dtype");
  TORCH_CHECK(q.is_contiguous() && k.is_contiguous() && v.is_contiguous(), "sparse_flash: contiguous inputs");
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  TORCH_CHECK(dsa::flash_supported((int)D), "sparse_flash: head dim must be 64, 96 or 128");
  TORCH_CHECK(S % 64 == 0 && S > 0, "sparse_flash: sequence length must be a multiple of 64");
  TORCH_CHECK(Hl == 1 || Hl == H, "sparse_flash: layout heads must be 1 or H");
  TORCH_CHECK(shift >= 0 && shift <= 6, "sparse_flash: shift in [0, 6]");
  check_lut(rowptr, cols, masks, Hl, S / 64, "sparse_flash rowptr/cols/masks");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor o = out_bshd ? at::empty({B, S, H, D}, q.options()) : at::empty_like(q);
  Tensor lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  const SBias sb = sparse_bias(kbias, ebias, q);
  dsa::launch_sparse_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                               rowptr.data_ptr<int>(), cols.data_ptr<int>(),
                               reinterpret_cast<const uint32_t*>(masks.data_ptr<int>()), (int)(B * H), (int)H, (int)Hl,
                               (int)S, (int)D, causal, (float)scale, (int)shift, dcode(q), cur_stream(),
                               out_bshd ? (int)H : 0, sb.kb, sb.eb, sb.ez, sb.eh, sb.er);
  return {o, lse};
}

// tasks int32 [Hl, ntask, 4] = (key tile or -1, entry begin, entry end, partial slot or -1) over
// rows / masks_t (the transposed LUT); fin int32 [Hl, nfin, 4] = (key tile or -1, first slot, chunks, 0);
// nslot = partial slots per (batch, head).
std::vector<Tensor> sparse_flash_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor rowptr,
                                     Tensor cols, Tensor masks, Tensor rows, Tensor masks_t, Tensor tasks, Tensor fin,
                                     Tensor kgroups, int64_t nslot, int64_t Hl, bool causal, double scale,
                                     int64_t shift, bool o_bshd, OptT kbias, OptT ebias) {
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  for (auto* t : {&q, &k, &v}) {
    check_dev(*t, "sparse_flash_bwd");
    TORCH_CHECK(t->sizes() == q.sizes() && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "sparse_flash_bwd: q/k/v must match");
  }
  const std::vector<int64_t> oshape = o_bshd ? std::vector<int64_t>{B, S, H, D} : std::vector<int64_t>{B, H, S, D};
  for (auto* t : {&dout, &o}) {
    check_dev(*t, "sparse_flash_bwd");
    TORCH_CHECK(t->sizes() == at::IntArrayRef(oshape) && t->scalar_type() == q.scalar_type() && t->is_contiguous(),
                "sparse_flash_bwd: dout/o must be contiguous in the forward's output layout");
  }
  TORCH_CHECK(dsa::flash_supported((int)D) && S % 64 == 0 && (Hl == 1 || Hl == H) && shift >= 0 && shift <= 6,
              "sparse_flash_bwd: unsupported shape");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * S, "sparse_flash_bwd: lse");
  check_lut(rowptr, cols, masks, Hl, S / 64, "sparse_flash_bwd rowptr/cols/masks");
  check_dev(rows, "rows"); check_dev(masks_t, "masks_t"); check_dev(tasks, "tasks"); check_dev(fin, "fin");
  TORCH_CHECK(rows.scalar_type() == at::kInt && masks_t.scalar_type() == at::kInt &&
                  rows.numel() == 4 * masks_t.numel() && rows.is_contiguous() && masks_t.is_contiguous(),
              "sparse_flash_bwd: transposed LUT");
  check_dev(kgroups, "kgroups");
  TORCH_CHECK(kgroups.scalar_type() == at::kInt && kgroups.is_contiguous() && kgroups.numel() == Hl * (S / 64) * 4,
              "sparse_flash_bwd: kgroups [Hl, S/64, 4]");
  TORCH_CHECK(tasks.scalar_type() == at::kInt && tasks.dim() == 3 && tasks.size(0) == Hl && tasks.size(2) == 4 &&
                  tasks.is_contiguous(), "sparse_flash_bwd: tasks [Hl, ntask, 4]");
  TORCH_CHECK(fin.scalar_type() == at::kInt && fin.dim() == 3 && fin.size(0) == Hl && fin.size(2) == 4 &&
                  fin.is_contiguous(), "sparse_flash_bwd: fin [Hl, nfin, 4]");
  const int64_t ntask = tasks.size(1), nfin = fin.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  Tensor delta = at::empty_like(lse);
  Tensor ws = at::empty({std::max<int64_t>(1, B * H * nslot * 2 * 64 * D)}, q.options().dtype(at::kFloat));
  const SBias sb = sparse_bias(kbias, ebias, q);
  dsa::launch_sparse_flash_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                               lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(),
                               dv.data_ptr(), rowptr.data_ptr<int>(), cols.data_ptr<int>(),
                               reinterpret_cast<const uint32_t*>(masks.data_ptr<int>()), rows.data_ptr<int>(),
                               reinterpret_cast<const uint32_t*>(masks_t.data_ptr<int>()), tasks.data_ptr<int>(),
                               (int)ntask, fin.data_ptr<int>(), (int)nfin, kgroups.data_ptr<int>(), ws.data_ptr<float>(),
                               (int)nslot,
                               (int)(B * H), (int)H, (int)Hl, (int)S, (int)D, causal, (float)scale, (int)shift,
                               dcode(q), cur_stream(), o_bshd ? (int)H : 0, sb.kb, sb.eb, sb.ez, sb.eh, sb.er);
  return {dq, dk, dv};
}

}  // namespace

void register_gemm_lt(pybind11::module& m);  // gemm_lt.cpp

// ----------------------------------------------------------------------------- streams
// A HIP stream whose kernels may only occupy the CUs set in `mask` (bit i = CU i of the
// runtime's CU enumeration).  Side-stream work (an overlapped optimizer step) placed on a
// subset of the CUs leaves the rest of the chip to the compute stream's GEMMs instead of
// interleaving workgroups on every CU.  Returned as the raw handle for torch.cuda.ExternalStream;
// the stream lives for the process.
int64_t cu_masked_stream(std::vector<int64_t> mask_words) {
  std::vector<uint32_t> words(mask_words.begin(), mask_words.end());
  hipStream_t st = nullptr;
  TORCH_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)words.size(), words.data()) == hipSuccess,
              "hipExtStreamCreateWithCUMask failed");
  return reinterpret_cast<int64_t>(st);
}

// A non-blocking stream at a given HIP priority.  HIP keeps one pool of hardware queues per
// priority level, so a stream of another priority never shares the compute stream's queue (a
// shared queue serialises: a side stream's cross-stream wait then stalls the compute stream).
int64_t priority_stream(int64_t priority) {
  hipStream_t st = nullptr;
  TORCH_CHECK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, (int)priority) == hipSuccess,
              "hipStreamCreateWithPriority failed");
  return reinterpret_cast<int64_t>(st);
}

std::vector<int64_t> stream_priority_range() {
  int least = 0, greatest = 0;
  TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess,
              "hipDeviceGetStreamPriorityRange failed");
  return {least, greatest};
}

// Page-locked host memory of exactly `numel` elements (hipHostMalloc), zero-filled, freed with
// the tensor.  torch's caching host allocator rounds every pinned allocation up to a power of two:
// 111 GB of Adam moments then pin 128 GiB, which is what put the 41B peak-parameter run over its
// host-memory budget (profiles/r5c_notes.md).
Tensor pinned_zeros(int64_t numel, int64_t dtype_code) {
  const auto dt = dtype_code == 0 ? at::kFloat : (dtype_code == 1 ? at::kBFloat16 : (dtype_code == 2 ? at::kHalf
                                                                                     : (dtype_code == 3 ? at::kShort : at::kLong)));
  const size_t bytes = (size_t)std::max<int64_t>(numel, 1) * c10::elementSize(dt);
  void* p = nullptr;
  TORCH_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess, "hipHostMalloc of ", bytes, " bytes failed");
  // parallel first touch + zero (one thread would take tens of seconds for 100 GB)
  const int64_t chunk = 1LL << 26;
  const int64_t nchunks = ((int64_t)bytes + chunk - 1) / chunk;
  at::parallel_for(0, nchunks, 1, [&](int64_t b, int64_t e) {
    for (int64_t c = b; c < e; ++c) {
      const int64_t off = c * chunk;
      std::memset((char*)p + off, 0, (size_t)std::min<int64_t>(chunk, (int64_t)bytes - off));
    }
  });
  return at::from_blob(p, {numel}, [](void* q) { (void)hipHostFree(q); }, at::TensorOptions().dtype(dt));
}

int64_t device_cu_count() {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  return n;
}

void profile_marker(int64_t tag) { dsa::launch_profile_marker((int)tag, cur_stream()); }

// dw[V, H] (+)= scatter-sum of dy[n, H] rows by token id, from ids sorted on the device (values and
// the permutation of torch.sort): no device -> host read anywhere (ops/csrc/kernels/embedding.hip)
Tensor embedding_bwd(Tensor sorted_ids, Tensor perm, Tensor dy, Tensor dw, int64_t padding_idx, bool accumulate) {
  check_dev(sorted_ids, "sorted_ids"); check_dev(perm, "perm"); check_dev(dy, "dy"); check_dev(dw, "dw");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kLong && perm.scalar_type() == at::kLong &&
              sorted_ids.is_contiguous() && perm.is_contiguous() && sorted_ids.numel() == perm.numel(),
              "embedding_bwd: int64 sorted ids / permutation of equal length");
  TORCH_CHECK(dy.dim() == 2 && dw.dim() == 2 && dy.size(1) == dw.size(1) && dy.size(0) == sorted_ids.numel(),
              "embedding_bwd: dy [n, H], dw [V, H]");
  TORCH_CHECK(dy.is_contiguous() && dw.is_contiguous() && dy.scalar_type() == dw.scalar_type() &&
              dy.element_size() == 2 && dw.size(1) % 8 == 0, "embedding_bwd: contiguous 16-bit rows, H % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  const int64_t n = dy.size(0), H = dy.size(1);
  const int64_t nc = dsa::embedding_bwd_chunks(n);
  Tensor ws = at::empty({2 * nc * H}, dy.options().dtype(at::kFloat));
  dsa::launch_embedding_bwd_sorted(sorted_ids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dy.data_ptr(),
                                   dw.data_ptr(), ws.data_ptr<float>(), ws.data_ptr<float>() + nc * H, n, (int)H,
                                   padding_idx, accumulate ? 1 : 0, dcode(dy), cur_stream());
  return dw;
}

// dst <- src (same byte count, both contiguous) on the current stream through a DMA engine, never a
// blit kernel: hipMemcpyDeviceToDeviceNoCU.  The pinned-host <-> HBM copies of the host-moments
// optimizer groups otherwise run (D2H) as ROCclr copyBuffer kernels with one workgroup on every CU,
// next to the forward's GEMMs (profiles/r4m_notes.md).  Pinned host memory is device-addressable,
// so the "device to device" DMA copy reaches it directly.
void copy_nocu(at::Tensor dst, at::Tensor src, int64_t kind) {
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "copy_nocu: contiguous tensors");
  const size_t n = (size_t)src.numel() * src.element_size();
  TORCH_CHECK((size_t)dst.numel() * dst.element_size() == n, "copy_nocu: byte counts differ");
  TORCH_CHECK(dst.is_cuda() || dst.is_pinned(), "copy_nocu: dst must be device or pinned host memory");
  TORCH_CHECK(src.is_cuda() || src.is_pinned(), "copy_nocu: src must be device or pinned host memory");
  if (n == 0) return;
  const hipError_t e = hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), n,
                                      kind < 0 ? hipMemcpyDeviceToDeviceNoCU : (hipMemcpyKind)kind, cur_stream());
  TORCH_CHECK(e == hipSuccess, "copy_nocu: hipMemcpyAsync failed: ", hipGetErrorString(e));
}

// dst <- src (byte copy) by copy_narrow_kernel on `wgs` workgroups (HBM -> pinned host memory).
void copy_narrow(at::Tensor dst, at::Tensor src, int64_t wgs) {
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "copy_narrow: contiguous tensors");
  const int64_t n = src.numel() * src.element_size();
  TORCH_CHECK(dst.numel() * dst.element_size() == n, "copy_narrow: byte counts differ");
  TORCH_CHECK(src.is_cuda() && (dst.is_cuda() || dst.is_pinned()), "copy_narrow: device src, device / pinned dst");
  TORCH_CHECK(wgs >= 1 && wgs <= 1024, "copy_narrow: 1..1024 workgroups");
  TORCH_CHECK(((uintptr_t)dst.data_ptr() & 15) == 0 && ((uintptr_t)src.data_ptr() & 15) == 0,
              "copy_narrow: 16-byte aligned pointers");
  dsa::launch_copy_narrow(src.data_ptr(), dst.data_ptr(), n, (int)wgs, cur_stream());
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("profile_marker", &profile_marker);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("cu_masked_stream", &cu_masked_stream);
  m.def("device_cu_count", &device_cu_count);
  m.def("priority_stream", &priority_stream);
  m.def("pinned_zeros", &pinned_zeros);
  m.def("stream_priority_range", &stream_priority_range);
  register_gemm_lt(m);
  m.def("sum_slices", &sum_slices);
  m.def("dropout_bwd_db", &dropout_bwd_db);
  m.def("add3", &add3, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c") = pybind11::none());
  m.def("sparse_flash_fwd", &sparse_flash_fwd);
  m.def("flash_attn_fwd_ex", &flash_attn_fwd_ex);
  m.def("flash_attn_bwd_ex", &flash_attn_bwd_ex);
  m.def("flash_attn_qkv_fwd", &flash_attn_qkv_fwd, py::arg("qkv"), py::arg("kbias"), py::arg("scale"), py::arg("p_drop"),
        py::arg("seed"), py::arg("rng") = py::none(), py::arg("o_out") = py::none());
  m.def("flash_attn_qkv_bwd", &flash_attn_qkv_bwd, py::arg("dout"), py::arg("qkv"), py::arg("o"), py::arg("lse"),
        py::arg("kbias"), py::arg("scale"), py::arg("p_drop"), py::arg("seed"), py::arg("rng") = py::none(),
        py::arg("dqkv_out") = py::none());
  m.def("sparse_flash_bwd", &sparse_flash_bwd);
  m.def("onebit_worker_compress", &onebit_worker_compress);
  m.def("onebit_server_compress", &onebit_server_compress);
  m.def("onebit_unpack", &onebit_unpack);
  m.def("sparse_sdd", &sparse_sdd);
  m.def("sparse_dsd", &sparse_dsd);
  m.def("sparse_softmax_fwd", &sparse_softmax_fwd);
  m.def("sparse_softmax_bwd", &sparse_softmax_bwd);
  m.def("dropout_fwd", &dropout_fwd, py::arg("x"), py::arg("p"), py::arg("seed"), py::arg("offset"),
        py::arg("rng") = py::none());
  m.def("bdr_ln_fwd", &bdr_ln_fwd, py::arg("x"), py::arg("bias"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("p"), py::arg("eps"), py::arg("seed"), py::arg("offset") = 0, py::arg("rng") = py::none(),
        py::arg("y_out") = py::none());
  m.def("bdr_ln_bwd", &bdr_ln_bwd, py::arg("dy"), py::arg("out"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("has_beta"), py::arg("dres"), py::arg("mask"), py::arg("p"), py::arg("dgamma_acc") = py::none(),
        py::arg("dbeta_acc") = py::none(), py::arg("dbias_acc") = py::none(), py::arg("dxb_out") = py::none());
  m.def("bdr_ln_supported", [](int64_t H, int64_t code) { return dsa::bdr_ln_supported((int)H, (int)code); });
  m.def("bias_dropout_residual", &bias_dropout_residual, py::arg("x"), py::arg("bias"), py::arg("res"), py::arg("p"),
        py::arg("seed"), py::arg("offset"), py::arg("rng") = py::none());
  m.def("dropout_bwd", &dropout_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd, py::arg("logits"), py::arg("labels"), py::arg("lse"), py::arg("dloss"),
        py::arg("inplace") = false);
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_attn_bwd", &flash_attn_bwd);
  m.def("rotary_split_fwd", &rotary_split_fwd);
  m.def("rotary_split_bwd", &rotary_split_bwd);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.doc() = "deeperspeed_amd CDNA4 (gfx950) HIP kernels";
  m.def("adam_flat", &adam_flat);
  m.def("adam_compact", &adam_compact);
  m.def("adam_multi", &adam_multi);
  m.def("sumsq_accum", &sumsq_accum);
  m.def("sumsq_multi", &sumsq_multi);
  m.def("copy_narrow", &copy_narrow);
  m.def("copy_nocu", &copy_nocu, py::arg("dst"), py::arg("src"), py::arg("kind") = -1);
  m.def("scale_copy", &scale_copy, pybind11::arg("x"), pybind11::arg("y"), pybind11::arg("scale_t"),
        pybind11::arg("scale"), pybind11::arg("accumulate") = false);
  m.def("lamb", &lamb);
  m.def("lamb_multi", &lamb_multi, py::arg("meta"), py::arg("T"), py::arg("total_chunks"), py::arg("chunk"),
        py::arg("wt"), py::arg("gt"), py::arg("ot"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("wd"), py::arg("bc1"), py::arg("bc2"), py::arg("grad_scale"), py::arg("max_coeff"), py::arg("min_coeff"),
        py::arg("adamw"), py::arg("partial"), py::arg("coeff"), py::arg("scale") = py::none(),
        py::arg("lr_dev") = py::none());
  m.def("ln_fwd", &ln_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("res"),
        py::arg("bias"), py::arg("y_out") = py::none());
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("has_beta"), py::arg("dres") = py::none(), py::arg("dgamma_acc") = py::none(),
        py::arg("dbeta_acc") = py::none());
  m.def("bias_gelu_fwd", &bias_gelu_fwd, py::arg("x"), py::arg("b"), py::arg("approx"), py::arg("out") = py::none());
  m.def("bias_gelu_bwd", &bias_gelu_bwd, py::arg("dy"), py::arg("x"), py::arg("b"), py::arg("approx"),
        py::arg("dx_out") = py::none(), py::arg("db_acc") = py::none());
  m.def("bias_gelu_fwd_t", &bias_gelu_fwd_t);
  m.def("bias_gelu_bwd_t", &bias_gelu_bwd_t);
  m.def("colsum", &colsum, py::arg("x"), py::arg("out") = py::none(), py::arg("accumulate") = false);
  m.def("heads_split", &heads_split);
  m.def("heads_merge", &heads_merge);
  m.def("swap12", &swap12);
  m.def("transpose_batched", &transpose_batched);
  m.def("transpose2d", &transpose2d, py::arg("x"), py::arg("colsum_out") = py::none(), py::arg("accum") = false,
        py::arg("out") = py::none());
}
