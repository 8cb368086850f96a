// PyTorch bindings for the gfx950 kernel library (one extension, `ds_hip_ops`).
// Host-only C++ (compiled with g++ against torch headers); device code lives in the *.hip objects linked in, which
// expose a C ABI taking raw pointers + hipStream_t. Every op launches on torch's current HIP stream, so ops compose
// with torch streams, events and hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <optional>
#include <vector>

extern "C" {
int ds_adam_flat(void*, void*, void*, const void*, void*, int64_t, int, int, int, float, float, float, float, float,
                 float, float, float, int, hipStream_t);
int ds_adam_multi(void**, void**, void**, const void**, void**, const int64_t*, int, int, int, int, float, float,
                  float, float, float, float, float, float, int, hipStream_t);
int ds_adam_multi_split(void**, void**, void**, const void**, void**, const int64_t*, int, int, float, float, float,
                        float, float, float, float, float, int, hipStream_t);
int ds_lion_flat(void*, void*, const void*, void*, int64_t, int, int, int, float, float, float, float, float,
                 hipStream_t);
int ds_adagrad_flat(void*, void*, const void*, void*, int64_t, int, int, int, float, float, float, float, hipStream_t);
int ds_lamb_flat(void*, void*, void*, const void*, void*, float*, float*, float*, int64_t, int, int, int, float,
                 float, float, float, float, float, float, float, float, float, hipStream_t);
int ds_sumsq_multi(const void**, const int64_t*, const int*, int, float*, int, float*, hipStream_t);
int ds_norm_bwd_blocks(int64_t);
int ds_rms_fwd(const void*, const void*, const void*, void*, void*, float*, int64_t, int, float, int, hipStream_t);
int ds_rms_bwd(const void*, const void*, const void*, const float*, const void*, void*, void*, float*, int64_t, int,
               int, hipStream_t);
int ds_ln_fwd(const void*, const void*, const void*, const void*, void*, void*, float*, float*, int64_t, int, float,
              int, hipStream_t);
int ds_ln_bwd(const void*, const void*, const void*, const float*, const float*, const void*, void*, void*, void*,
              float*, int64_t, int, int, hipStream_t);
int ds_gated_act_fwd(const void*, void*, int64_t, int, int, int, hipStream_t);
int ds_gated_act_bwd(const void*, const void*, void*, int64_t, int, int, int, hipStream_t);
int ds_gated_act_fwd_t(const void*, void*, void*, int64_t, int64_t, int, int, int, hipStream_t);
int ds_gated_act_bwd_t(const void*, const void*, void*, void*, int64_t, int64_t, int, int, int, hipStream_t);
int ds_bias_act_fwd(const void*, const void*, void*, int64_t, int, int, int, hipStream_t);
int ds_bias_act_bwd(const void*, const void*, const void*, void*, int64_t, int, int, int, hipStream_t);
int ds_bias_residual(const void*, const void*, const void*, void*, int64_t, int, float, int, hipStream_t);
int ds_dropout_fwd(const void*, const void*, const void*, void*, uint8_t*, int64_t, int, float, uint64_t, uint64_t, int,
                   hipStream_t);
int ds_bias_add2(const void*, const void*, const void*, const void*, void*, int64_t, int, int, hipStream_t);
int ds_dropout_bwd(const void*, void*, int64_t, int, float, uint64_t, uint64_t, int, hipStream_t);
int ds_qkv_rope_fwd(const void*, void*, void*, void*, const float*, const float*, const int*, int, int, int, int, int,
                    int, int, const int64_t*, int, hipStream_t);
int ds_qkv_rope_bwd(const void*, const void*, const void*, void*, const float*, const float*, const int*, int, int,
                    int, int, int, int, int, const int64_t*, int, hipStream_t);
int ds_rope_inplace(void*, int, int, int, int, int64_t, int64_t, int64_t, const float*, const float*, const int*, int,
                    int, int, int, int, hipStream_t);
int ds_flash_fwd(const void*, const void*, const void*, void*, float*, int, int, int, int, int, const int64_t*,
                 const int64_t*, const int64_t*, const int64_t*, float, int, hipStream_t);
int ds_flash_fwd_sparse(const void*, const void*, const void*, void*, float*, int, int, int, int, const int64_t*,
                        const int64_t*, const int64_t*, const int64_t*, float, const int*, const int*, const int*,
                        const uint8_t*, int, int, int, int, const float*, int64_t, const float*, int64_t, const float*,
                        int64_t, int64_t, hipStream_t);
int ds_flash_bwd(const void*, const void*, const void*, const void*, const void*, const float*, float*, float*, void*,
                 void*, void*, int, int, int, int, const int64_t*, const int64_t*, const int64_t*, const int64_t*,
                 const int64_t*, const int64_t*, const int64_t*, const int64_t*, float, int, const int*, const int*,
                 const uint8_t*, int, int, int, int, int, const float*, int64_t, const float*, int64_t, const float*,
                 int64_t, int64_t, hipStream_t);
int ds_transpose16(const void*, void*, int, int, int, int64_t, hipStream_t);
int ds_xent_fwd(const void*, const int64_t*, float*, float*, int64_t, int, int64_t, int, float, int, hipStream_t);
int ds_xent_bwd(const void*, const int64_t*, const float*, const float*, float, void*, int64_t, int, int64_t, int64_t,
                int, float, int, hipStream_t);
}

using torch::Tensor;
using OptT = std::optional<Tensor>;

namespace {

int dcode(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}
hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }
void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed: ", hipGetErrorString((hipError_t)rc));
}
void need(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void* ptr_or_null(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------------------------------ optimizers
void adam_flat(Tensor p, Tensor m, Tensor v, Tensor g, OptT lp, double lr, double b1, double b2, double eps, double wd,
               double bc1, double bc2, double grad_scale, bool adamw) {
  need(p, "p"); need(m, "m"); need(v, "v"); need(g, "g");
  TORCH_CHECK(m.numel() == p.numel() && v.numel() == p.numel() && g.numel() == p.numel(), "adam_flat: size mismatch");
  TORCH_CHECK(m.scalar_type() == p.scalar_type() && v.scalar_type() == p.scalar_type(), "m/v must match p dtype");
  int lpd = -1;
  if (lp.has_value()) { need(*lp, "lp"); TORCH_CHECK(lp->numel() == p.numel(), "lp size"); lpd = dcode(*lp); }
  check(ds_adam_flat(p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(), ptr_or_null(lp), p.numel(), dcode(p),
                     dcode(g), lpd, lr, b1, b2, eps, wd, bc1, bc2, grad_scale, adamw ? 1 : 0, stream()),
        "adam_flat");
}

void adam_multi(std::vector<Tensor> p, std::vector<Tensor> m, std::vector<Tensor> v, std::vector<Tensor> g,
                std::vector<Tensor> lp, double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
                double grad_scale, bool adamw) {
  const size_t n = p.size();
  if (n == 0) return;
  TORCH_CHECK(m.size() == n && v.size() == n && g.size() == n && (lp.empty() || lp.size() == n), "list sizes");
  std::vector<void*> pp(n), mp(n), vp(n), lpp(lp.empty() ? 0 : n);
  std::vector<const void*> gp(n);
  std::vector<int64_t> nn(n);
  const int pd = dcode(p[0]), gd = dcode(g[0]), ld = lp.empty() ? -1 : dcode(lp[0]);
  for (size_t i = 0; i < n; ++i) {
    need(p[i], "p"); need(m[i], "m"); need(v[i], "v"); need(g[i], "g");
    TORCH_CHECK(dcode(p[i]) == pd && dcode(g[i]) == gd, "adam_multi: mixed dtypes within one call");
    TORCH_CHECK(m[i].numel() == p[i].numel() && v[i].numel() == p[i].numel() && g[i].numel() == p[i].numel(),
                "adam_multi: size mismatch");
    pp[i] = p[i].data_ptr(); mp[i] = m[i].data_ptr(); vp[i] = v[i].data_ptr(); gp[i] = g[i].data_ptr();
    nn[i] = p[i].numel();
    if (!lp.empty()) { need(lp[i], "lp"); lpp[i] = lp[i].data_ptr(); }
  }
  check(ds_adam_multi(pp.data(), mp.data(), vp.data(), gp.data(), lp.empty() ? nullptr : lpp.data(), nn.data(), (int)n,
                      pd, gd, ld, lr, b1, b2, eps, wd, bc1, bc2, grad_scale, adamw ? 1 : 0, stream()),
        "adam_multi");
}

// split-master Adam: lo int16 residuals, m/v fp32, g any dtype, hi bf16 weights updated in place
void adam_multi_split(std::vector<Tensor> lo, std::vector<Tensor> m, std::vector<Tensor> v, std::vector<Tensor> g,
                      std::vector<Tensor> hi, double lr, double b1, double b2, double eps, double wd, double bc1,
                      double bc2, double grad_scale, bool adamw) {
  const size_t n = lo.size();
  if (n == 0) return;
  TORCH_CHECK(m.size() == n && v.size() == n && g.size() == n && hi.size() == n, "list sizes");
  std::vector<void*> lp(n), mp(n), vp(n), hp(n);
  std::vector<const void*> gp(n);
  std::vector<int64_t> nn(n);
  const int gd = dcode(g[0]);
  for (size_t i = 0; i < n; ++i) {
    need(lo[i], "lo"); need(m[i], "m"); need(v[i], "v"); need(g[i], "g"); need(hi[i], "hi");
    TORCH_CHECK(lo[i].scalar_type() == at::kShort && hi[i].scalar_type() == at::kBFloat16 &&
                m[i].scalar_type() == at::kFloat && v[i].scalar_type() == at::kFloat && dcode(g[i]) == gd,
                "adam_multi_split: lo int16, hi bf16, m/v fp32, one grad dtype per call");
    const int64_t k = lo[i].numel();
    TORCH_CHECK(m[i].numel() == k && v[i].numel() == k && g[i].numel() == k && hi[i].numel() == k,
                "adam_multi_split: size mismatch");
    lp[i] = lo[i].data_ptr(); mp[i] = m[i].data_ptr(); vp[i] = v[i].data_ptr(); gp[i] = g[i].data_ptr();
    hp[i] = hi[i].data_ptr(); nn[i] = k;
  }
  check(ds_adam_multi_split(lp.data(), mp.data(), vp.data(), gp.data(), hp.data(), nn.data(), (int)n, gd, lr, b1, b2,
                            eps, wd, bc1, bc2, grad_scale, adamw ? 1 : 0, stream()),
        "adam_multi_split");
}

void lion_flat(Tensor p, Tensor m, Tensor g, OptT lp, double lr, double b1, double b2, double wd, double grad_scale) {
  need(p, "p"); need(m, "m"); need(g, "g");
  TORCH_CHECK(m.numel() == p.numel() && g.numel() == p.numel(), "lion_flat: size mismatch");
  check(ds_lion_flat(p.data_ptr(), m.data_ptr(), g.data_ptr(), ptr_or_null(lp), p.numel(), dcode(p), dcode(g),
                     lp.has_value() ? dcode(*lp) : -1, lr, b1, b2, wd, grad_scale, stream()),
        "lion_flat");
}

void adagrad_flat(Tensor p, Tensor s, Tensor g, OptT lp, double lr, double eps, double wd, double grad_scale) {
  need(p, "p"); need(s, "s"); need(g, "g");
  TORCH_CHECK(s.numel() == p.numel() && g.numel() == p.numel(), "adagrad_flat: size mismatch");
  check(ds_adagrad_flat(p.data_ptr(), s.data_ptr(), g.data_ptr(), ptr_or_null(lp), p.numel(), dcode(p), dcode(g),
                        lp.has_value() ? dcode(*lp) : -1, lr, eps, wd, grad_scale, stream()),
        "adagrad_flat");
}

// returns the applied trust ratio (device scalar)
Tensor lamb_flat(Tensor p, Tensor m, Tensor v, Tensor g, OptT lp, double lr, double b1, double b2, double eps,
                 double wd, double bc1, double bc2, double grad_scale, double max_coeff, double min_coeff) {
  need(p, "p"); need(m, "m"); need(v, "v"); need(g, "g");
  TORCH_CHECK(m.numel() == p.numel() && v.numel() == p.numel() && g.numel() == p.numel(), "lamb_flat: size mismatch");
  auto fopt = p.options().dtype(at::kFloat);
  auto u = torch::empty({p.numel()}, fopt);
  auto partials = torch::empty({2 * 512}, fopt);
  auto coeff = torch::empty({1}, fopt);
  check(ds_lamb_flat(p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(), ptr_or_null(lp), u.data_ptr<float>(),
                     partials.data_ptr<float>(), coeff.data_ptr<float>(), p.numel(), dcode(p), dcode(g),
                     lp.has_value() ? dcode(*lp) : -1, lr, b1, b2, eps, wd, bc1, bc2, grad_scale, max_coeff,
                     min_coeff, stream()),
        "lamb_flat");
  return coeff;
}

// sum of squares of all tensors (fp32 device scalar), deterministic
Tensor sumsq_multi(std::vector<Tensor> xs) {
  TORCH_CHECK(!xs.empty(), "sumsq_multi: empty list");
  const int cap = 512 * (int)xs.size();
  auto fopt = xs[0].options().dtype(at::kFloat);
  auto partials = torch::empty({cap}, fopt);
  auto out = torch::zeros({}, fopt);
  std::vector<const void*> ptrs;
  std::vector<int64_t> ns;
  std::vector<int> dts;
  for (auto& x : xs) {
    need(x, "x");
    ptrs.push_back(x.data_ptr());
    ns.push_back(x.numel());
    dts.push_back(dcode(x));
  }
  check(ds_sumsq_multi(ptrs.data(), ns.data(), dts.data(), (int)xs.size(), partials.data_ptr<float>(), cap,
                       out.data_ptr<float>(), stream()),
        "sumsq_multi");
  return out;
}

// ------------------------------------------------------------------------------------------ norms
std::vector<Tensor> rms_fwd(Tensor x, OptT r, Tensor w, double eps) {
  need(x, "x"); need(w, "w");
  const int H = (int)x.size(-1);
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(w.numel() == H && w.scalar_type() == x.scalar_type(), "rms_fwd: weight shape/dtype");
  auto y = torch::empty_like(x);
  auto rstd = torch::empty({rows}, x.options().dtype(at::kFloat));
  Tensor res;
  if (r.has_value()) { need(*r, "r"); TORCH_CHECK(r->sizes() == x.sizes(), "residual shape"); res = torch::empty_like(x); }
  check(ds_rms_fwd(x.data_ptr(), ptr_or_null(r), w.data_ptr(), y.data_ptr(), res.defined() ? res.data_ptr() : nullptr,
                   rstd.data_ptr<float>(), rows, H, eps, dcode(x), stream()),
        "rms_fwd");
  return {y, res.defined() ? res : torch::Tensor(), rstd};
}

std::vector<Tensor> rms_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, OptT dres) {
  need(dy, "dy"); need(x, "x"); need(w, "w"); need(rstd, "rstd");
  const int H = (int)x.size(-1);
  const int64_t rows = x.numel() / H;
  auto dx = torch::empty_like(x);
  auto dw = torch::empty_like(w);
  const int nb = ds_norm_bwd_blocks(rows);
  auto part = torch::empty({((int64_t)nb + 32) * H}, x.options().dtype(at::kFloat));
  if (dres.has_value()) need(*dres, "dres");
  check(ds_rms_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), ptr_or_null(dres),
                   dx.data_ptr(), dw.data_ptr(), part.data_ptr<float>(), rows, H, dcode(x), stream()),
        "rms_bwd");
  return {dx, dw};
}

std::vector<Tensor> ln_fwd(Tensor x, OptT r, Tensor g, Tensor b, double eps) {
  need(x, "x"); need(g, "gamma"); need(b, "beta");
  const int H = (int)x.size(-1);
  const int64_t rows = x.numel() / H;
  auto y = torch::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  auto mean = torch::empty({rows}, fo), rstd = torch::empty({rows}, fo);
  Tensor res;
  if (r.has_value()) { need(*r, "r"); res = torch::empty_like(x); }
  check(ds_ln_fwd(x.data_ptr(), ptr_or_null(r), g.data_ptr(), b.data_ptr(), y.data_ptr(),
                  res.defined() ? res.data_ptr() : nullptr, mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, H,
                  eps, dcode(x), stream()),
        "ln_fwd");
  return {y, res.defined() ? res : torch::Tensor(), mean, rstd};
}

std::vector<Tensor> ln_bwd(Tensor dy, Tensor x, Tensor g, Tensor mean, Tensor rstd, OptT dres) {
  need(dy, "dy"); need(x, "x");
  const int H = (int)x.size(-1);
  const int64_t rows = x.numel() / H;
  auto dx = torch::empty_like(x);
  auto dg = torch::empty_like(g), db = torch::empty_like(g);
  const int nb = ds_norm_bwd_blocks(rows);
  auto part = torch::empty({((int64_t)nb + 32) * 2 * H}, x.options().dtype(at::kFloat));
  check(ds_ln_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                  ptr_or_null(dres), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), part.data_ptr<float>(), rows, H,
                  dcode(x), stream()),
        "ln_bwd");
  return {dx, dg, db};
}

// ------------------------------------------------------------------------------------------ activations
Tensor gated_act_fwd(Tensor gu, int64_t act) {
  need(gu, "gu");
  const int I = (int)(gu.size(-1) / 2);
  const int64_t rows = gu.numel() / (2 * I);
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  auto out = torch::empty(sizes, gu.options());
  check(ds_gated_act_fwd(gu.data_ptr(), out.data_ptr(), rows, I, (int)act, dcode(gu), stream()), "gated_act_fwd");
  return out;
}

Tensor gated_act_bwd(Tensor dout, Tensor gu, int64_t act) {
  need(dout, "dout"); need(gu, "gu");
  const int I = (int)(gu.size(-1) / 2);
  const int64_t rows = gu.numel() / (2 * I);
  auto dgu = torch::empty_like(gu);
  check(ds_gated_act_bwd(dout.data_ptr(), gu.data_ptr(), dgu.data_ptr(), rows, I, (int)act, dcode(gu), stream()),
        "gated_act_bwd");
  return dgu;
}

// gated activation that also writes the token-contiguous copy [I, Tp] (Tp = rows rounded up to `pad`): returns
// {out [.., I], outT [I, Tp]}
std::vector<Tensor> gated_act_fwd_t(Tensor gu, int64_t act, int64_t pad) {
  need(gu, "gu");
  TORCH_CHECK(gu.element_size() == 2, "gated_act_fwd_t: 16-bit dtypes only");
  const int I = (int)(gu.size(-1) / 2);
  const int64_t rows = gu.numel() / (2 * I);
  const int64_t Tp = (rows + pad - 1) / pad * pad;
  TORCH_CHECK(rows % 8 == 0 && I % 8 == 0 && Tp % 8 == 0, "gated_act_fwd_t: rows / features multiples of 8");
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  auto out = torch::empty(sizes, gu.options());
  auto outT = torch::empty({(int64_t)I, Tp}, gu.options());
  check(ds_gated_act_fwd_t(gu.data_ptr(), out.data_ptr(), outT.data_ptr(), rows, Tp, I, (int)act, dcode(gu), stream()),
        "gated_act_fwd_t");
  return {out, outT};
}

// returns {dgu [.., 2I], dguT [2I, Tp]}
std::vector<Tensor> gated_act_bwd_t(Tensor dout, Tensor gu, int64_t act, int64_t pad) {
  need(dout, "dout"); need(gu, "gu");
  TORCH_CHECK(gu.element_size() == 2 && dout.scalar_type() == gu.scalar_type(), "gated_act_bwd_t: 16-bit dtypes");
  const int I = (int)(gu.size(-1) / 2);
  const int64_t rows = gu.numel() / (2 * I);
  const int64_t Tp = (rows + pad - 1) / pad * pad;
  TORCH_CHECK(rows % 8 == 0 && I % 8 == 0 && Tp % 8 == 0 && dout.numel() == rows * I, "gated_act_bwd_t: shapes");
  auto dgu = torch::empty_like(gu);
  auto dguT = torch::empty({(int64_t)2 * I, Tp}, gu.options());
  check(ds_gated_act_bwd_t(dout.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), rows, Tp, I, (int)act,
                           dcode(gu), stream()),
        "gated_act_bwd_t");
  return {dgu, dguT};
}

Tensor bias_act_fwd(Tensor x, OptT bias, int64_t act) {
  need(x, "x");
  const int C = (int)x.size(-1);
  auto y = torch::empty_like(x);
  check(ds_bias_act_fwd(x.data_ptr(), ptr_or_null(bias), y.data_ptr(), x.numel() / C, C, (int)act, dcode(x), stream()),
        "bias_act_fwd");
  return y;
}

Tensor bias_act_bwd(Tensor dy, Tensor x, OptT bias, int64_t act) {
  need(dy, "dy"); need(x, "x");
  const int C = (int)x.size(-1);
  auto dx = torch::empty_like(x);
  check(ds_bias_act_bwd(dy.data_ptr(), x.data_ptr(), ptr_or_null(bias), dx.data_ptr(), x.numel() / C, C, (int)act,
                        dcode(x), stream()),
        "bias_act_bwd");
  return dx;
}

Tensor bias_residual(Tensor x, OptT bias, OptT res, double res_scale) {
  need(x, "x");
  const int C = (int)x.size(-1);
  auto y = torch::empty_like(x);
  check(ds_bias_residual(x.data_ptr(), ptr_or_null(bias), ptr_or_null(res), y.data_ptr(), x.numel() / C, C, res_scale,
                         dcode(x), stream()),
        "bias_residual");
  return y;
}

// x [..., C] channels-last: y = x + bias (+ other) (+ other_bias)
Tensor bias_add2(Tensor x, Tensor bias, OptT other, OptT other_bias) {
  need(x, "x");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0 && bias.numel() == C && bias.scalar_type() == x.scalar_type(), "bias_add2: bias [C], C % 8");
  if (other.has_value()) TORCH_CHECK(other->sizes() == x.sizes() && other->is_contiguous(), "other shape");
  if (other_bias.has_value()) TORCH_CHECK(other_bias->numel() == C, "other_bias [C]");
  auto y = torch::empty_like(x);
  check(ds_bias_add2(x.data_ptr(), bias.data_ptr(), ptr_or_null(other), ptr_or_null(other_bias), y.data_ptr(),
                     x.numel() / C, C, dcode(x), stream()),
        "bias_add2");
  return y;
}

// ------------------------------------------------------------------------------------------ dropout
// y = res + dropout_p(x + bias); the keep mask is a pure function of (seed, offset, element) so the backward
// regenerates it. want_mask returns the packed mask (bit j of byte t = element 8t + j) for tests.
std::vector<Tensor> dropout_fwd(Tensor x, OptT bias, OptT res, double p, int64_t seed, int64_t offset, bool want_mask) {
  need(x, "x");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0, "dropout: last dim must be a multiple of 8");
  if (bias.has_value()) TORCH_CHECK(bias->numel() == C && bias->scalar_type() == x.scalar_type(), "bias [C]");
  if (res.has_value()) TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "residual shape");
  auto y = torch::empty_like(x);
  Tensor mask = want_mask ? torch::empty({x.numel() / 8}, x.options().dtype(at::kByte)) : Tensor();
  check(ds_dropout_fwd(x.data_ptr(), ptr_or_null(bias), ptr_or_null(res), y.data_ptr(),
                       want_mask ? mask.data_ptr<uint8_t>() : nullptr, x.numel() / C, C, (float)p, (uint64_t)seed,
                       (uint64_t)offset, dcode(x), stream()),
        "dropout_fwd");
  if (want_mask) return {y, mask};
  return {y};
}

Tensor dropout_bwd(Tensor dy, double p, int64_t seed, int64_t offset) {
  need(dy, "dy");
  const int C = (int)dy.size(-1);
  auto dx = torch::empty_like(dy);
  check(ds_dropout_bwd(dy.data_ptr(), dx.data_ptr(), dy.numel() / C, C, (float)p, (uint64_t)seed, (uint64_t)offset,
                       dcode(dy), stream()),
        "dropout_bwd");
  return dx;
}

// ------------------------------------------------------------------------------------------ rotary
void hm_strides(const Tensor& q, const Tensor& k, const Tensor& v, int64_t (&st)[9]) {
  const Tensor* ts[3] = {&q, &k, &v};
  for (int i = 0; i < 3; ++i) {
    TORCH_CHECK(ts[i]->dim() == 4 && ts[i]->stride(3) == 1, "q/k/v views need a unit last stride");
    for (int d = 0; d < 3; ++d) st[3 * i + d] = ts[i]->stride(d);
  }
}

// token_major: q/k/v are returned as [B,H,S,D] views of [B,S,H,D] memory (the layout the flash-attention kernel and
// the efficient-attention backward exchange without transposing copies); else contiguous [B,H,S,D].
std::vector<Tensor> qkv_rope_fwd(Tensor qkv, Tensor cos_t, Tensor sin_t, OptT pos, int64_t Hq, int64_t Hk, int64_t rot,
                                 int64_t pos_offset, bool token_major) {
  need(qkv, "qkv"); need(cos_t, "cos"); need(sin_t, "sin");
  TORCH_CHECK(qkv.dim() == 4 && qkv.size(2) == Hq + 2 * Hk, "qkv must be [B,S,Hq+2Hk,D]");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat, "cos/sin tables must be fp32");
  const int B = (int)qkv.size(0), S = (int)qkv.size(1), D = (int)qkv.size(3);
  TORCH_CHECK(cos_t.size(-1) == rot / 2, "cos table width must be rot/2");
  TORCH_CHECK(pos.has_value() || cos_t.size(0) >= S + pos_offset, "rotary table too short");
  auto mk = [&](int64_t H) {
    return token_major ? torch::empty({B, S, H, D}, qkv.options()).transpose(1, 2)
                       : torch::empty({B, H, S, D}, qkv.options());
  };
  auto q = mk(Hq), k = mk(Hk), v = mk(Hk);
  int64_t st[9];
  hm_strides(q, k, v, st);
  const int* pp = nullptr;
  if (pos.has_value()) { need(*pos, "pos"); TORCH_CHECK(pos->scalar_type() == at::kInt, "pos int32"); pp = pos->data_ptr<int>(); }
  check(ds_qkv_rope_fwd(qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cos_t.data_ptr<float>(),
                        sin_t.data_ptr<float>(), pp, B, S, (int)Hq, (int)Hk, D, (int)rot, (int)pos_offset, st,
                        dcode(qkv), stream()),
        "qkv_rope_fwd");
  return {q, k, v};
}

// dq/dk/dv: any [B,H,S,D] views with unit last stride (no contiguous copies)
Tensor qkv_rope_bwd(Tensor dq, Tensor dk, Tensor dv, Tensor cos_t, Tensor sin_t, OptT pos, int64_t rot,
                    int64_t pos_offset) {
  TORCH_CHECK(dq.is_cuda() && dk.is_cuda() && dv.is_cuda(), "qkv_rope_bwd: device tensors");
  Tensor dq_ = dq.stride(3) == 1 ? dq : dq.contiguous(), dk_ = dk.stride(3) == 1 ? dk : dk.contiguous(),
         dv_ = dv.stride(3) == 1 ? dv : dv.contiguous();
  const int B = (int)dq.size(0), Hq = (int)dq.size(1), S = (int)dq.size(2), D = (int)dq.size(3);
  const int Hk = (int)dk.size(1);
  auto dqkv = torch::empty({B, S, Hq + 2 * Hk, D}, dq.options());
  int64_t st[9];
  hm_strides(dq_, dk_, dv_, st);
  const int* pp = pos.has_value() ? pos->data_ptr<int>() : nullptr;
  check(ds_qkv_rope_bwd(dq_.data_ptr(), dk_.data_ptr(), dv_.data_ptr(), dqkv.data_ptr(), cos_t.data_ptr<float>(),
                        sin_t.data_ptr<float>(), pp, B, S, Hq, Hk, D, (int)rot, (int)pos_offset, st, dcode(dq),
                        stream()),
        "qkv_rope_bwd");
  return dqkv;
}

void rope_inplace(Tensor x, Tensor cos_t, Tensor sin_t, OptT pos, int64_t rot, int64_t pos_offset, bool interleaved,
                  bool inverse) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.stride(3) == 1, "x must be a [B,S,H,D] view with unit last stride");
  const int* pp = pos.has_value() ? pos->data_ptr<int>() : nullptr;
  check(ds_rope_inplace(x.data_ptr(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), x.stride(0),
                        x.stride(1), x.stride(2), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp, (int)rot,
                        (int)pos_offset, interleaved ? 1 : 0, inverse ? 1 : 0, dcode(x), stream()),
        "rope_inplace");
}

// ------------------------------------------------------------------------------------------ cross entropy
std::vector<Tensor> xent_fwd(Tensor logits, Tensor labels, int64_t ignore_index, double smoothing) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N,V] row-major");
  need(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  const int64_t N = logits.size(0);
  auto fo = logits.options().dtype(at::kFloat);
  auto loss = torch::empty({N}, fo), lse = torch::empty({N}, fo);
  check(ds_xent_fwd(logits.data_ptr(), labels.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(), N,
                    (int)logits.size(1), logits.stride(0), (int)ignore_index, smoothing, dcode(logits), stream()),
        "xent_fwd");
  return {loss, lse};
}

Tensor xent_bwd(Tensor logits, Tensor labels, Tensor lse, OptT dloss, double dloss_scalar, bool inplace,
                int64_t ignore_index, double smoothing) {
  const int64_t N = logits.size(0);
  Tensor out = inplace ? logits : torch::empty_like(logits);
  const float* dl = nullptr;
  Tensor dlc;
  if (dloss.has_value()) { dlc = dloss->to(at::kFloat).contiguous(); dl = dlc.data_ptr<float>(); }
  check(ds_xent_bwd(logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), dl, (float)dloss_scalar,
                    out.data_ptr(), N, (int)logits.size(1), logits.stride(0), out.stride(0), (int)ignore_index,
                    smoothing, dcode(logits), stream()),
        "xent_bwd");
  return out;
}

// ------------------------------------------------------------------------------------------ flash attention
// q [B,Hq,S,128] / k,v [B,Hk,Skv,128] bf16 views with unit last stride; returns (o [B,Hq,S,128] whose memory is laid
// out [B,S,Hq,128] so the o_proj GEMM reads it without a transpose copy, lse [B,Hq,S] fp32).
// x [R, C] (16-bit, unit last stride) -> x^T contiguous [C, Rp] at HBM speed (K-major wgrad GEMM operands);
// pad_to > R appends zero columns (the contraction dimension rounded up for the GEMM)
Tensor transpose16(Tensor x, int64_t pad_to) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "transpose16: 2-D device tensor, unit last stride");
  TORCH_CHECK(x.element_size() == 2, "transpose16: 16-bit dtypes only");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0 && x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "transpose16: sizes / row stride multiples of 8, 16-B aligned base");
  const int64_t Rp = pad_to > R ? pad_to : R;
  TORCH_CHECK(Rp % 8 == 0 && Rp < (1LL << 31) && C < (1LL << 31), "transpose16: bad padded size / dims too large");
  auto out = torch::empty({C, Rp}, x.options());
  check(ds_transpose16(x.data_ptr(), out.data_ptr(), (int)R, (int)Rp, (int)C, x.stride(0), stream()), "transpose16");
  return out;
}

std::vector<Tensor> flash_fwd(Tensor q, Tensor k, Tensor v, bool causal, double scale, bool want_lse) {
  TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "flash_fwd: device tensors expected");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "flash_fwd: 4-D [B,H,S,D] tensors expected");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 && v.scalar_type() == at::kBFloat16,
              "flash_fwd: bf16 only");
  TORCH_CHECK(q.size(3) == 128 && k.size(3) == 128 && v.size(3) == 128, "flash_fwd: head dim 128 only");
  TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "flash_fwd: unit last stride required");
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), Hk = k.size(1), Skv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Hk && v.size(2) == Skv, "flash_fwd: k/v shape");
  TORCH_CHECK(Hq % Hk == 0, "flash_fwd: Hq must be a multiple of Hk");
  for (const Tensor* t : {&q, &k, &v})
    for (int d = 0; d < 3; ++d) TORCH_CHECK(t->stride(d) % 8 == 0, "flash_fwd: strides must be multiples of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(q.data_ptr()) | reinterpret_cast<uintptr_t>(k.data_ptr()) |
               reinterpret_cast<uintptr_t>(v.data_ptr())) % 16 == 0, "flash_fwd: 16-B aligned data required");
  auto o = torch::empty({B, S, Hq, 128}, q.options()).transpose(1, 2);  // [B,Hq,S,D] view of [B,S,Hq,D] memory
  Tensor lse;
  if (want_lse) lse = torch::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  const int64_t qs[3] = {q.stride(0), q.stride(1), q.stride(2)}, ks[3] = {k.stride(0), k.stride(1), k.stride(2)},
                vs[3] = {v.stride(0), v.stride(1), v.stride(2)}, os[3] = {o.stride(0), o.stride(1), o.stride(2)};
  check(ds_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                     want_lse ? lse.data_ptr<float>() : nullptr, (int)B, (int)Hq, (int)Hk, (int)S, (int)Skv, qs, ks,
                     vs, os, (float)scale, causal ? 1 : 0, stream()),
        "flash_fwd");
  return {o, lse};
}

// Block-sparse flash forward (non-causal; causality belongs to the layout). tiles int32 [LH, nqb, T], ntiles int32
// [LH, nqb], layout uint8 [LH, nb, nb] at granularity blk; LH in {1, Hq}. Same q/k/v/o/lse contract as flash_fwd.
// additive score biases of the block-sparse attention: kbias [B, S], abias [S, S], rpe [H or 1, S, S], fp32 device
// tensors with unit last stride, 16-B aligned rows
struct AttnBias {
  const float *kb = nullptr, *ab = nullptr, *rp = nullptr;
  int64_t kbs = 0, abs_ = 0, rhs = 0, rrs = 0;
};
AttnBias attn_bias(const OptT& kbias, const OptT& abias, const OptT& rpe, int64_t B, int64_t H, int64_t S) {
  AttnBias r;
  auto chk = [](const Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.stride(-1) == 1 &&
                    reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, ": fp32 device tensor, unit last stride, "
                "16-B aligned");
  };
  if (kbias.has_value() && kbias->defined()) {
    chk(*kbias, "kbias");
    TORCH_CHECK(kbias->dim() == 2 && kbias->size(0) == B && kbias->size(1) == S && kbias->stride(0) % 4 == 0, "kbias [B, S]");
    r.kb = kbias->data_ptr<float>(); r.kbs = kbias->stride(0);
  }
  if (abias.has_value() && abias->defined()) {
    chk(*abias, "abias");
    TORCH_CHECK(abias->dim() == 2 && abias->size(0) == S && abias->size(1) == S && abias->stride(0) % 4 == 0, "abias [S, S]");
    r.ab = abias->data_ptr<float>(); r.abs_ = abias->stride(0);
  }
  if (rpe.has_value() && rpe->defined()) {
    chk(*rpe, "rpe");
    TORCH_CHECK(rpe->dim() == 3 && (rpe->size(0) == H || rpe->size(0) == 1) && rpe->size(1) == S && rpe->size(2) == S &&
                    rpe->stride(1) % 4 == 0 && rpe->stride(0) % 4 == 0, "rpe [H or 1, S, S]");
    r.rp = rpe->data_ptr<float>(); r.rhs = rpe->size(0) == 1 ? 0 : rpe->stride(0); r.rrs = rpe->stride(1);
  }
  return r;
}

std::vector<Tensor> flash_fwd_sparse(Tensor q, Tensor k, Tensor v, double scale, Tensor tiles, Tensor ntiles,
                                     Tensor qorder, Tensor layout, int64_t blk, bool want_lse, OptT kbias,
                                     OptT abias, OptT rpe) {
  TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "flash_fwd_sparse: device tensors expected");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "flash_fwd_sparse: 4-D [B,H,S,D] tensors expected");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 && v.scalar_type() == at::kBFloat16,
              "flash_fwd_sparse: bf16 only");
  TORCH_CHECK(q.size(3) == 128 && k.size(3) == 128 && v.size(3) == 128, "flash_fwd_sparse: head dim 128 only");
  TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "flash_fwd_sparse: unit last stride");
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), Hk = k.size(1);
  TORCH_CHECK(k.size(0) == B && k.size(2) == S && v.sizes() == k.sizes(), "flash_fwd_sparse: k/v shape");
  TORCH_CHECK(Hq % Hk == 0, "flash_fwd_sparse: Hq must be a multiple of Hk");
  for (const Tensor* t : {&q, &k, &v})
    for (int d = 0; d < 3; ++d) TORCH_CHECK(t->stride(d) % 8 == 0, "flash_fwd_sparse: strides must be multiples of 8");
  need(tiles, "tiles"); need(ntiles, "ntiles"); need(layout, "layout"); need(qorder, "qorder");
  TORCH_CHECK(tiles.scalar_type() == at::kInt && ntiles.scalar_type() == at::kInt && layout.scalar_type() == at::kByte,
              "flash_fwd_sparse: int32 tiles/ntiles, uint8 layout");
  const int64_t LH = layout.size(0), nb = layout.size(1), nqb = (S + 127) / 128;
  TORCH_CHECK(layout.dim() == 3 && layout.size(2) == nb && nb * blk >= S, "flash_fwd_sparse: layout [LH, nb, nb]");
  TORCH_CHECK((LH == 1 || LH == Hq) && tiles.dim() == 3 && tiles.size(0) == LH && tiles.size(1) == nqb &&
                  ntiles.numel() == LH * nqb && qorder.numel() == LH * nqb && qorder.scalar_type() == at::kInt,
              "flash_fwd_sparse: LUT shape");
  TORCH_CHECK(qorder.min().item<int>() >= 0 && qorder.max().item<int>() < nqb, "flash_fwd_sparse: qorder range");
  // every listed tile must lie inside the key range (the kernel trusts the LUT for its K/V addresses)
  if (tiles.numel() > 0)
    TORCH_CHECK(tiles.min().item<int>() >= 0 && tiles.max().item<int>() < (S + 63) / 64 &&
                    ntiles.max().item<int>() <= tiles.size(2) && ntiles.min().item<int>() >= 0,
                "flash_fwd_sparse: LUT entries out of range");
  auto o = torch::empty({B, S, Hq, 128}, q.options()).transpose(1, 2);
  Tensor lse;
  if (want_lse) lse = torch::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  const AttnBias ab = attn_bias(kbias, abias, rpe, B, Hq, S);
  const int64_t qs[3] = {q.stride(0), q.stride(1), q.stride(2)}, ks[3] = {k.stride(0), k.stride(1), k.stride(2)},
                vs[3] = {v.stride(0), v.stride(1), v.stride(2)}, os[3] = {o.stride(0), o.stride(1), o.stride(2)};
  check(ds_flash_fwd_sparse(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                            want_lse ? lse.data_ptr<float>() : nullptr, (int)B, (int)Hq, (int)Hk, (int)S, qs, ks, vs,
                            os, (float)scale, tiles.data_ptr<int>(), ntiles.data_ptr<int>(), qorder.data_ptr<int>(),
                            layout.data_ptr<uint8_t>(), (int)tiles.size(2), (int)LH, (int)nb, (int)blk, ab.kb, ab.kbs,
                            ab.ab, ab.abs_, ab.rp, ab.rhs, ab.rrs, stream()),
        "flash_fwd_sparse");
  return {o, lse};
}

// Flash backward (csrc/attn/flash_bwd.hip): q/o/dout [B,Hq,S,128], k/v [B,Hk,S,128] bf16 views with unit last stride,
// lse [B,Hq,S] fp32 from flash_fwd. mode 0 full, 1 causal, 2 block-sparse with the column LUT (qtiles int32
// [Hk, nkb, T] of (head-in-group << 16 | 32-row tile), nqt int32 [Hk, nkb], layout uint8 [LH, nb, nb], granularity
// blk). Returns dq, dk, dv laid out [B,S,H,128] in memory (viewed [B,H,S,128]) like flash_fwd's output.
std::vector<Tensor> flash_bwd(Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor dout, double scale,
                              int64_t mode, OptT qtiles, OptT nqt, OptT layout, int64_t blk, OptT kbias, OptT abias,
                              OptT rpe) {
  for (const Tensor* t : {&q, &k, &v, &o, &dout}) {
    TORCH_CHECK(t->is_cuda() && t->dim() == 4 && t->scalar_type() == at::kBFloat16, "flash_bwd: 4-D bf16 device tensors");
    TORCH_CHECK(t->size(3) == 128 && t->stride(3) == 1, "flash_bwd: head dim 128 with unit last stride");
    for (int d = 0; d < 3; ++d) TORCH_CHECK(t->stride(d) % 8 == 0, "flash_bwd: strides must be multiples of 8");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "flash_bwd: 16-B aligned data required");
  }
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), Hk = k.size(1);
  TORCH_CHECK(k.size(0) == B && k.size(2) == S && v.sizes() == k.sizes(), "flash_bwd: k/v shape (S == Skv required)");
  TORCH_CHECK(o.sizes() == q.sizes() && dout.sizes() == q.sizes(), "flash_bwd: o/dout shape");
  TORCH_CHECK(Hq % Hk == 0, "flash_bwd: Hq must be a multiple of Hk");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * Hq * S,
              "flash_bwd: lse [B,Hq,S] fp32 contiguous");
  TORCH_CHECK(mode >= 0 && mode <= 2, "flash_bwd: mode");
  const int* qt = nullptr; const int* nq = nullptr; const uint8_t* lay = nullptr;
  int maxt = 0, LH = 1, nb = 0;
  if (mode == 2) {
    TORCH_CHECK(qtiles.has_value() && nqt.has_value() && layout.has_value(), "flash_bwd: sparse LUT required");
    need(*qtiles, "qtiles"); need(*nqt, "nqt"); need(*layout, "layout");
    TORCH_CHECK(qtiles->scalar_type() == at::kInt && nqt->scalar_type() == at::kInt &&
                    layout->scalar_type() == at::kByte, "flash_bwd: int32 qtiles/nqt, uint8 layout");
    const int64_t nkb = (S + 255) / 256;
    LH = (int)layout->size(0); nb = (int)layout->size(1);
    TORCH_CHECK(layout->dim() == 3 && layout->size(2) == nb && nb * blk >= S && (LH == 1 || LH == Hq),
                "flash_bwd: layout [LH, nb, nb]");
    TORCH_CHECK(qtiles->dim() == 3 && qtiles->size(0) == Hk && qtiles->size(1) == nkb && nqt->numel() == Hk * nkb,
                "flash_bwd: LUT shape");
    maxt = (int)qtiles->size(2);
    if (nqt->numel() > 0) TORCH_CHECK(nqt->max().item<int>() <= maxt && nqt->min().item<int>() >= 0, "flash_bwd: nqt");
    if (qtiles->numel() > 0) {  // the kernel trusts the LUT for its Q / dO addresses
      const int ntq = (int)((S + 31) / 32), rep = (int)(Hq / Hk);
      auto codes = qtiles->masked_fill(qtiles->lt(0), 0);
      TORCH_CHECK((codes.bitwise_and(0xffff)).max().item<int>() < ntq && torch::bitwise_right_shift(codes, 16).max().item<int>() < rep,
                  "flash_bwd: LUT entries out of range");
    }
    qt = qtiles->data_ptr<int>(); nq = nqt->data_ptr<int>(); lay = layout->data_ptr<uint8_t>();
  }
  const AttnBias ab = attn_bias(kbias, abias, rpe, B, Hq, S);
  TORCH_CHECK(mode == 2 || (!ab.kb && !ab.ab && !ab.rp), "flash_bwd: score biases need the block-sparse mode");
  // the kernel loads all three bias terms unconditionally: absent ones read one zero float
  const int flags = (ab.kb ? 1 : 0) | (ab.ab ? 2 : 0) | (ab.rp ? 4 : 0);
  Tensor zero1;
  if (flags) zero1 = torch::zeros({4}, q.options().dtype(at::kFloat));
  auto zp = [&](const float* p) { return (p || !flags) ? p : zero1.data_ptr<float>(); };
  auto mk = [&](int64_t H) { return torch::empty({B, S, H, 128}, q.options()).transpose(1, 2); };
  auto dq = mk(Hq), dk = mk(Hk), dv = mk(Hk);
  auto delta = torch::empty({2 * B * Hq * S}, q.options().dtype(at::kFloat));  // -delta and -LSE/scale rows
  auto dqacc = torch::empty({B * Hq * S * 128}, q.options().dtype(at::kFloat));
  auto st3 = [](const Tensor& t, int64_t* s) { for (int d = 0; d < 3; ++d) s[d] = t.stride(d); };
  int64_t qs[3], ks[3], vs[3], os[3], gs[3], dqs[3], dks[3], dvs[3];
  st3(q, qs); st3(k, ks); st3(v, vs); st3(o, os); st3(dout, gs); st3(dq, dqs); st3(dk, dks); st3(dv, dvs);
  check(ds_flash_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                     delta.data_ptr<float>(), dqacc.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                     (int)B, (int)Hq, (int)Hk, (int)S, qs, ks, vs, os, gs, dqs, dks, dvs, (float)scale, (int)mode, qt,
                     nq, lay, maxt, LH, nb, (int)blk, flags, zp(ab.kb), ab.kbs, zp(ab.ab), ab.abs_, zp(ab.rp), ab.rhs,
                     ab.rrs, stream()),
        "flash_bwd");
  return {dq, dk, dv};
}

}  // namespace

// other binding translation units of this extension
void register_inference_ops(pybind11::module& m);  // bind/infer_bind.cpp
void register_host_mem_ops(pybind11::module& m);   // bind/host_mem.cpp
void register_comm_ops(pybind11::module& m);       // bind/comm_bind.cpp
void register_moe_ops(pybind11::module& m);        // bind/moe_bind.cpp
void register_attn_small_ops(pybind11::module& m); // bind/attn_small_bind.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_inference_ops(m);
  register_host_mem_ops(m);
  register_comm_ops(m);
  register_moe_ops(m);
  register_attn_small_ops(m);
  m.doc() = "deepspeedsyclsupport_amd gfx950 kernels";
  m.def("adam_flat", &adam_flat);
  m.def("adam_multi", &adam_multi);
  m.def("adam_multi_split", &adam_multi_split);
  m.def("lion_flat", &lion_flat);
  m.def("adagrad_flat", &adagrad_flat);
  m.def("lamb_flat", &lamb_flat);
  m.def("sumsq_multi", &sumsq_multi);
  m.def("rms_fwd", &rms_fwd);
  m.def("rms_bwd", &rms_bwd);
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("gated_act_fwd", &gated_act_fwd);
  m.def("gated_act_bwd", &gated_act_bwd);
  m.def("gated_act_fwd_t", &gated_act_fwd_t);
  m.def("gated_act_bwd_t", &gated_act_bwd_t);
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("bias_act_bwd", &bias_act_bwd);
  m.def("bias_residual", &bias_residual);
  m.def("bias_add2", &bias_add2);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("qkv_rope_fwd", &qkv_rope_fwd, py::arg("qkv"), py::arg("cos"), py::arg("sin"), py::arg("pos"), py::arg("hq"),
        py::arg("hk"), py::arg("rot"), py::arg("pos_offset"), py::arg("token_major") = false);
  m.def("qkv_rope_bwd", &qkv_rope_bwd);
  m.def("rope_inplace", &rope_inplace);
  m.def("transpose16", &transpose16, py::arg("x"), py::arg("pad_to") = 0);
  m.def("flash_fwd", &flash_fwd);
  m.def("flash_fwd_sparse", &flash_fwd_sparse, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("scale"),
        py::arg("tiles"), py::arg("ntiles"), py::arg("qorder"), py::arg("layout"), py::arg("blk"), py::arg("want_lse"),
        py::arg("kbias") = py::none(), py::arg("abias") = py::none(), py::arg("rpe") = py::none());
  m.def("flash_bwd", &flash_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("lse"),
        py::arg("dout"), py::arg("scale"), py::arg("mode"), py::arg("qtiles") = py::none(), py::arg("nqt") = py::none(),
        py::arg("layout") = py::none(), py::arg("blk") = 0, py::arg("kbias") = py::none(),
        py::arg("abias") = py::none(), py::arg("rpe") = py::none());
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
}
