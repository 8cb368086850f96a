// Host-side optimizers for ZeRO-Offload / Offload++ Twin-Flow: Adam/AdamW, Adagrad, Lion over fp32 master
// partitions in host DRAM.
//
// Parity: reference `csrc/adam/cpu_adam_impl.cpp` (+ `includes/cpu_adam.h`, `simd.h`), `csrc/adagrad/cpu_adagrad.cpp`,
// `csrc/lion/cpu_lion_impl.cpp`. The reference hand-writes AVX512/AVX2 intrinsics with TILE-sized loops and launches
// an fp16 H2D copy kernel on alternating streams. Here:
//  * the math is a plain fused loop compiled three times via `target_clones` (avx512f / avx2 / baseline) and picked
//    at load time by the dynamic loader, so one .so runs on any x86 host (the GPU box CPU differs from the build host);
//  * OpenMP splits the partition into cache-sized tiles;
//  * the low-precision model copy (bf16/fp16) is written into a caller-provided (pinned) host buffer in the same pass;
//    the Python side issues the H2D copy with `non_blocking=True` on a side HIP stream (Twin-Flow overlap).
#include <torch/extension.h>

#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

constexpr int64_t TILE = 1 << 16;

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float load_any(const void* p, int dt, int64_t i) {
  if (dt == 0) return static_cast<const float*>(p)[i];
  if (dt == 1) return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  return (float)static_cast<const at::Half*>(p)[i];
}
inline void store_lp(void* p, int dt, int64_t i, float v) {
  if (dt == 1) static_cast<uint16_t*>(p)[i] = f32_to_bf16(v);
  else if (dt == 2) static_cast<at::Half*>(p)[i] = at::Half(v);
  else static_cast<float*>(p)[i] = v;
}

int dcode(const torch::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  if (t.scalar_type() == at::kHalf) return 2;
  TORCH_CHECK(false, "unsupported dtype");
  return -1;
}

// ---------------------------------------------------------------- kernels (vectorised per target clone)
__attribute__((target_clones("avx512f", "avx2", "default"))) void adam_tile_f32g(
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, const float* __restrict__ g, int64_t n,
    float lr, float b1, float b2, float eps, float wd, float step_size, float denom_scale, float gs, int adamw) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    float gg = g[i] * gs;
    if (!adamw) gg += wd * p[i];
    const float mm = b1 * m[i] + (1.f - b1) * gg;
    const float vv = b2 * v[i] + (1.f - b2) * gg * gg;
    float upd = mm * step_size / (std::sqrt(vv) * denom_scale + eps);
    if (adamw) upd += wd * p[i];
    p[i] -= lr * upd;
    m[i] = mm;
    v[i] = vv;
  }
}

__attribute__((target_clones("avx512f", "avx2", "default"))) void adam_tile_bf16g(
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, const uint16_t* __restrict__ g, int64_t n,
    float lr, float b1, float b2, float eps, float wd, float step_size, float denom_scale, float gs, int adamw) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u = (uint32_t)g[i] << 16;
    float gg;
    std::memcpy(&gg, &u, 4);
    gg *= gs;
    if (!adamw) gg += wd * p[i];
    const float mm = b1 * m[i] + (1.f - b1) * gg;
    const float vv = b2 * v[i] + (1.f - b2) * gg * gg;
    float upd = mm * step_size / (std::sqrt(vv) * denom_scale + eps);
    if (adamw) upd += wd * p[i];
    p[i] -= lr * upd;
    m[i] = mm;
    v[i] = vv;
  }
}

__attribute__((target_clones("avx512f", "avx2", "default"))) void cvt_bf16_tile(const float* __restrict__ p,
                                                                                uint16_t* __restrict__ o, int64_t n) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u;
    std::memcpy(&u, &p[i], 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    o[i] = (uint16_t)(u >> 16);
  }
}

// Split-master tile: the fp32 master is (hi << 16) + sext(lo) with hi = the bf16 weight (round half away from zero)
// and lo a signed 16-bit residual; `hi_out` may alias `g` (the pinned staging buffer receives the gradient and
// returns the updated weight), which is safe because iteration i reads g[i] before it writes hi_out[i].
template <typename TG>
inline float grad_f32(const TG* g, int64_t i);
template <>
inline float grad_f32<float>(const float* g, int64_t i) { return g[i]; }
template <>
inline float grad_f32<uint16_t>(const uint16_t* g, int64_t i) {
  uint32_t u = (uint32_t)g[i] << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

#define DS_SPLIT_TILE(NAME, TG)                                                                                      \
  __attribute__((target_clones("avx512f", "avx2", "default"))) void NAME(                                           \
      int16_t* __restrict__ lo, float* __restrict__ m, float* __restrict__ v, const TG* g,                           \
      const uint16_t* __restrict__ hi_in, uint16_t* hi_out, int64_t n, float lr, float b1, float b2, float eps,      \
      float wd, float step_size, float denom_scale, float gs, int adamw) {                                           \
    _Pragma("omp simd") for (int64_t i = 0; i < n; ++i) {                                                            \
      uint32_t u = ((uint32_t)hi_in[i] << 16) + (uint32_t)(int32_t)lo[i];                                            \
      float p;                                                                                                       \
      std::memcpy(&p, &u, 4);                                                                                        \
      float gg = grad_f32<TG>(g, i) * gs;                                                                            \
      if (!adamw) gg += wd * p;                                                                                      \
      const float mm = b1 * m[i] + (1.f - b1) * gg;                                                                  \
      const float vv = b2 * v[i] + (1.f - b2) * gg * gg;                                                             \
      float upd = mm * step_size / (std::sqrt(vv) * denom_scale + eps);                                              \
      if (adamw) upd += wd * p;                                                                                      \
      p -= lr * upd;                                                                                                 \
      m[i] = mm;                                                                                                     \
      v[i] = vv;                                                                                                     \
      std::memcpy(&u, &p, 4);                                                                                        \
      hi_out[i] = (uint16_t)((u + 0x8000u) >> 16);                                                                   \
      lo[i] = (int16_t)(u & 0xffffu);                                                                                \
    }                                                                                                                \
  }
DS_SPLIT_TILE(adam_split_tile_bf16g, uint16_t)
DS_SPLIT_TILE(adam_split_tile_f32g, float)

__attribute__((target_clones("avx512f", "avx2", "default"))) void acc_tile_bf16(float* __restrict__ d,
                                                                                const uint16_t* __restrict__ s,
                                                                                int64_t n, float alpha, int first) {
#pragma omp simd
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u = (uint32_t)s[i] << 16;
    float f;
    std::memcpy(&f, &u, 4);
    d[i] = first ? f * alpha : d[i] + f * alpha;
  }
}
__attribute__((target_clones("avx512f", "avx2", "default"))) double sumsq_tile(const float* __restrict__ s,
                                                                               int64_t n) {
  double acc = 0.0;
#pragma omp simd reduction(+ : acc)
  for (int64_t i = 0; i < n; ++i) acc += (double)s[i] * (double)s[i];
  return acc;
}

void check_host(const torch::Tensor& t, const char* n) {
  TORCH_CHECK(t.device().is_cpu() && t.is_contiguous(), n, " must be a contiguous host tensor");
}

}  // namespace

// p (fp32 master), m, v (fp32), g (fp32/bf16/fp16), optional lp output (bf16/fp16/fp32, host, may be pinned)
void cpu_adam_update(torch::Tensor p, torch::Tensor m, torch::Tensor v, torch::Tensor g, c10::optional<torch::Tensor> lp,
                     int64_t step, double lr, double b1, double b2, double eps, double wd, bool bias_correction,
                     bool adamw, double grad_scale) {
  check_host(p, "p"); check_host(m, "m"); check_host(v, "v"); check_host(g, "g");
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "cpu_adam: p/m/v must be fp32");
  const int64_t n = p.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "cpu_adam: size mismatch");
  const float bc1 = bias_correction ? 1.f - std::pow((float)b1, (float)step) : 1.f;
  const float bc2 = bias_correction ? 1.f - std::pow((float)b2, (float)step) : 1.f;
  const float step_size = 1.f / bc1, denom_scale = 1.f / std::sqrt(bc2);  // step_size scales m only
  float* pp = p.data_ptr<float>();
  float* mp = m.data_ptr<float>();
  float* vp = v.data_ptr<float>();
  const int gd = dcode(g);
  void* lpp = nullptr;
  int lpd = -1;
  if (lp.has_value() && lp->defined()) {
    check_host(*lp, "lp");
    TORCH_CHECK(lp->numel() == n, "lp size");
    lpp = lp->data_ptr();
    lpd = dcode(*lp);
  }
  const void* gp = g.data_ptr();
#pragma omp parallel for schedule(static)
  for (int64_t t0 = 0; t0 < n; t0 += TILE) {
    const int64_t len = std::min(TILE, n - t0);
    if (gd == 0)
      adam_tile_f32g(pp + t0, mp + t0, vp + t0, static_cast<const float*>(gp) + t0, len, lr, b1, b2, eps, wd,
                     step_size, denom_scale, grad_scale, adamw);
    else if (gd == 1)
      adam_tile_bf16g(pp + t0, mp + t0, vp + t0, static_cast<const uint16_t*>(gp) + t0, len, lr, b1, b2, eps, wd,
                      step_size, denom_scale, grad_scale, adamw);
    else {
      for (int64_t i = t0; i < t0 + len; ++i) {
        float gg = load_any(gp, gd, i) * (float)grad_scale;
        if (!adamw) gg += (float)wd * pp[i];
        mp[i] = (float)b1 * mp[i] + (1.f - (float)b1) * gg;
        vp[i] = (float)b2 * vp[i] + (1.f - (float)b2) * gg * gg;
        float upd = mp[i] * step_size / (std::sqrt(vp[i]) * denom_scale + (float)eps);
        if (adamw) upd += (float)wd * pp[i];
        pp[i] -= (float)lr * upd;
      }
    }
    if (lpp) {
      if (lpd == 1) cvt_bf16_tile(pp + t0, static_cast<uint16_t*>(lpp) + t0, len);
      else
        for (int64_t i = t0; i < t0 + len; ++i) store_lp(lpp, lpd, i, pp[i]);
    }
  }
}

// Split-master Adam on the host: lo (int16 residuals), m, v (fp32), g (bf16/fp32), hi_in (bf16 weights staged from the
// device), hi_out (bf16, may be the same buffer as g or hi_in).
void cpu_adam_update_split(torch::Tensor lo, torch::Tensor m, torch::Tensor v, torch::Tensor g, torch::Tensor hi_in,
                           torch::Tensor hi_out, int64_t step, double lr, double b1, double b2, double eps, double wd,
                           bool bias_correction, bool adamw, double grad_scale) {
  check_host(lo, "lo"); check_host(m, "m"); check_host(v, "v"); check_host(g, "g");
  check_host(hi_in, "hi_in"); check_host(hi_out, "hi_out");
  const int64_t n = lo.numel();
  TORCH_CHECK(lo.scalar_type() == at::kShort && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat &&
              hi_in.scalar_type() == at::kBFloat16 && hi_out.scalar_type() == at::kBFloat16,
              "cpu_adam_split: lo int16, m/v fp32, hi bf16");
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n && hi_in.numel() == n && hi_out.numel() == n,
              "cpu_adam_split: size mismatch");
  const int gd = dcode(g);
  TORCH_CHECK(gd == 0 || gd == 1, "cpu_adam_split: grads must be fp32 or bf16");
  const float bc1 = bias_correction ? 1.f - std::pow((float)b1, (float)step) : 1.f;
  const float bc2 = bias_correction ? 1.f - std::pow((float)b2, (float)step) : 1.f;
  const float step_size = 1.f / bc1, denom_scale = 1.f / std::sqrt(bc2);
  int16_t* lp = lo.data_ptr<int16_t>();
  float* mp = m.data_ptr<float>();
  float* vp = v.data_ptr<float>();
  const void* gp = g.data_ptr();
  const uint16_t* hin = reinterpret_cast<const uint16_t*>(hi_in.data_ptr());
  uint16_t* hout = reinterpret_cast<uint16_t*>(hi_out.data_ptr());
#pragma omp parallel for schedule(static)
  for (int64_t t0 = 0; t0 < n; t0 += TILE) {
    const int64_t len = std::min(TILE, n - t0);
    if (gd == 1)
      adam_split_tile_bf16g(lp + t0, mp + t0, vp + t0, static_cast<const uint16_t*>(gp) + t0, hin + t0, hout + t0,
                            len, lr, b1, b2, eps, wd, step_size, denom_scale, grad_scale, adamw);
    else
      adam_split_tile_f32g(lp + t0, mp + t0, vp + t0, static_cast<const float*>(gp) + t0, hin + t0, hout + t0, len,
                           lr, b1, b2, eps, wd, step_size, denom_scale, grad_scale, adamw);
  }
}

// dst (fp32) = src * alpha (first) or dst + src * alpha, src bf16 or fp32: host-side gradient accumulation
void cpu_accumulate(torch::Tensor dst, torch::Tensor src, double alpha, bool first) {
  check_host(dst, "dst"); check_host(src, "src");
  const int64_t n = dst.numel();
  TORCH_CHECK(dst.scalar_type() == at::kFloat && src.numel() == n, "cpu_accumulate: fp32 dst, same numel");
  float* d = dst.data_ptr<float>();
  const int sd = dcode(src);
  const void* sp = src.data_ptr();
#pragma omp parallel for schedule(static)
  for (int64_t t0 = 0; t0 < n; t0 += TILE) {
    const int64_t len = std::min(TILE, n - t0);
    if (sd == 1) acc_tile_bf16(d + t0, static_cast<const uint16_t*>(sp) + t0, len, alpha, first);
    else
      for (int64_t i = t0; i < t0 + len; ++i) {
        const float f = load_any(sp, sd, i) * (float)alpha;
        d[i] = first ? f : d[i] + f;
      }
  }
}

double cpu_sumsq(torch::Tensor src) {
  check_host(src, "src");
  TORCH_CHECK(src.scalar_type() == at::kFloat, "cpu_sumsq: fp32 only");
  const int64_t n = src.numel();
  const float* s = src.data_ptr<float>();
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc)
  for (int64_t t0 = 0; t0 < n; t0 += TILE) acc += sumsq_tile(s + t0, std::min(TILE, n - t0));
  return acc;
}

void cpu_adagrad_update(torch::Tensor p, torch::Tensor s, torch::Tensor g, c10::optional<torch::Tensor> lp, double lr,
                        double eps, double wd, double grad_scale) {
  check_host(p, "p"); check_host(s, "s"); check_host(g, "g");
  const int64_t n = p.numel();
  float* pp = p.data_ptr<float>();
  float* sp = s.data_ptr<float>();
  const void* gp = g.data_ptr();
  const int gd = dcode(g);
  void* lpp = (lp.has_value() && lp->defined()) ? lp->data_ptr() : nullptr;
  const int lpd = lpp ? dcode(*lp) : -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    float gg = load_any(gp, gd, i) * (float)grad_scale;
    if (wd != 0) gg += (float)wd * pp[i];
    sp[i] += gg * gg;
    pp[i] -= (float)lr * gg / (std::sqrt(sp[i]) + (float)eps);
    if (lpp) store_lp(lpp, lpd, i, pp[i]);
  }
}

void cpu_lion_update(torch::Tensor p, torch::Tensor m, torch::Tensor g, c10::optional<torch::Tensor> lp, double lr,
                     double b1, double b2, double wd, double grad_scale) {
  check_host(p, "p"); check_host(m, "m"); check_host(g, "g");
  const int64_t n = p.numel();
  float* pp = p.data_ptr<float>();
  float* mp = m.data_ptr<float>();
  const void* gp = g.data_ptr();
  const int gd = dcode(g);
  void* lpp = (lp.has_value() && lp->defined()) ? lp->data_ptr() : nullptr;
  const int lpd = lpp ? dcode(*lp) : -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const float gg = load_any(gp, gd, i) * (float)grad_scale;
    const float c = (float)b1 * mp[i] + (1.f - (float)b1) * gg;
    const float upd = (c > 0.f) ? 1.f : ((c < 0.f) ? -1.f : 0.f);
    pp[i] = pp[i] * (1.f - (float)lr * (float)wd) - (float)lr * upd;
    mp[i] = (float)b2 * mp[i] + (1.f - (float)b2) * gg;
    if (lpp) store_lp(lpp, lpd, i, pp[i]);
  }
}

// fp32 -> bf16 host conversion (used to stage params for H2D)
void cpu_to_bf16(torch::Tensor src, torch::Tensor dst) {
  check_host(src, "src"); check_host(dst, "dst");
  TORCH_CHECK(src.scalar_type() == at::kFloat && dst.scalar_type() == at::kBFloat16 && src.numel() == dst.numel(),
              "cpu_to_bf16: fp32 -> bf16 same numel");
  const int64_t n = src.numel();
  const float* s = src.data_ptr<float>();
  uint16_t* d = reinterpret_cast<uint16_t*>(dst.data_ptr());
#pragma omp parallel for schedule(static)
  for (int64_t t0 = 0; t0 < n; t0 += TILE) cvt_bf16_tile(s + t0, d + t0, std::min(TILE, n - t0));
}

// CPU SIMD width report (parity with reference simd_width / ds_report)
std::string simd_level() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f")) return "AVX512";
  if (__builtin_cpu_supports("avx2")) return "AVX2";
  return "scalar";
}

// OpenMP team size for the calling thread's later update calls (the Twin-Flow worker leaves a core to the thread
// that launches GPU work when the host step overlaps the next forward)
void cpu_set_omp_threads(int64_t n) { omp_set_num_threads((int)std::max<int64_t>(1, n)); }
int64_t cpu_get_omp_threads() { return omp_get_max_threads(); }

void register_cpu_optim(pybind11::module& m) {
  m.def("cpu_set_omp_threads", &cpu_set_omp_threads);
  m.def("cpu_get_omp_threads", &cpu_get_omp_threads);
  // the update loops run without the interpreter lock: the Twin-Flow worker thread steps the host partition while
  // the main thread launches the device optimizer and the next forward
  using nogil = pybind11::call_guard<pybind11::gil_scoped_release>;
  m.def("cpu_adam_update", &cpu_adam_update, nogil());
  m.def("cpu_adam_update_split", &cpu_adam_update_split, nogil());
  m.def("cpu_accumulate", &cpu_accumulate, nogil());
  m.def("cpu_sumsq", &cpu_sumsq, nogil());
  m.def("cpu_adagrad_update", &cpu_adagrad_update, nogil());
  m.def("cpu_lion_update", &cpu_lion_update, nogil());
  m.def("cpu_to_bf16", &cpu_to_bf16, nogil());
  m.def("simd_level", &simd_level);
}
