// Fused optimizer kernels for CDNA4 (gfx950): Adam/AdamW, Lion, Adagrad, LAMB, plus L2-norm / overflow helpers.
//
// Parity targets: reference `csrc/adam/multi_tensor_adam.cu:34-126` (Adam functor), `csrc/lion/multi_tensor_lion.cu`,
// `csrc/lamb/fused_lamb_cuda_kernel.cu:195-300` (3-phase LAMB), `csrc/adagrad/cpu_adagrad.cpp` (update rule).
//
// MI355X design: these are HBM-bound streaming kernels (Adam moves ~32 B/element), so the whole game is
//  * one pass over memory: fp32 master + m + v + grad (any dtype) in, fp32 master + m + v + low-precision param copy
//    out — the bf16 model weights are written by the same kernel, no separate cast pass;
//  * 16 B per lane per access (8 elements/thread/iteration: 2x float4 for fp32 streams, one 16 B load for bf16);
//  * grid = min(work, 256 CUs x 8 blocks) with a grid-stride loop, 256-thread blocks (4 waves);
//  * multi-tensor launches carry their pointer table in the kernel-argument segment (no H2D copy, so the launch is
//    hipGraph-capturable and never synchronises).
#include "../include/ds_hip.h"

namespace {

struct AdamArgs {
  float lr, beta1, beta2, eps, weight_decay;
  float bias_correction1, bias_correction2;  // 1 - beta^t (1.0 when bias correction is disabled)
  float grad_scale;                          // multiplier applied to grads (1/loss_scale * clip coefficient)
  int adamw_mode;                            // 1: decoupled weight decay, 0: L2 added to the gradient
};

// step_size = 1/bias_correction1 (applied to m), denom_scale = 1/sqrt(bias_correction2); the decoupled weight decay
// is scaled by lr only (not lr/bc1), as in the reference functor (`multi_tensor_adam.cu:34-126`) and torch AdamW.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamArgs& a, float rbc1,
                                          float denom_scale) {
  g *= a.grad_scale;
  if (!a.adamw_mode && a.weight_decay != 0.f) g = fmaf(a.weight_decay, p, g);
  m = fmaf(a.beta1, m, (1.f - a.beta1) * g);
  v = fmaf(a.beta2, v, (1.f - a.beta2) * g * g);
  const float denom = sqrtf(v) * denom_scale + a.eps;
  float upd = (m * rbc1) / denom;
  if (a.adamw_mode && a.weight_decay != 0.f) upd = fmaf(a.weight_decay, p, upd);
  p = fmaf(-a.lr, upd, p);
}

// Flat Adam: P (master, fp32 or bf16), M/V same dtype as P, G grad dtype, LP optional low-precision copy.
template <typename TP, typename TG, typename TL, bool HAS_LP, bool VEC>
__global__ void __launch_bounds__(256) adam_flat_kernel(TP* __restrict__ p, TP* __restrict__ m, TP* __restrict__ v,
                                                        const TG* __restrict__ g, TL* __restrict__ lp, int64_t n,
                                                        AdamArgs a) {
  const float step_size = 1.f / a.bias_correction1;
  const float denom_scale = rsqrtf(a.bias_correction2);
  const int64_t nvec = VEC ? n / 8 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int64_t o = i * 8;
    float pp[8], mm[8], vv[8], gg[8];
    Vec8<TP>::load(p + o, pp);
    Vec8<TP>::load(m + o, mm);
    Vec8<TP>::load(v + o, vv);
    Vec8<TG>::load(g + o, gg);
#pragma unroll
    for (int j = 0; j < 8; ++j) adam_elem(pp[j], mm[j], vv[j], gg[j], a, step_size, denom_scale);
    Vec8<TP>::store(p + o, pp);
    Vec8<TP>::store(m + o, mm);
    Vec8<TP>::store(v + o, vv);
    if (HAS_LP) Vec8<TL>::store(lp + o, pp);
  }
  // scalar tail (n % 8)
  for (int64_t i = nvec * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = to_f32(p[i]), mm = to_f32(m[i]), vv = to_f32(v[i]);
    adam_elem(pp, mm, vv, to_f32(g[i]), a, step_size, denom_scale);
    p[i] = from_f32<TP>(pp);
    m[i] = from_f32<TP>(mm);
    v[i] = from_f32<TP>(vv);
    if (HAS_LP) lp[i] = from_f32<TL>(pp);
  }
}

// ---------------------------------------------------------------- multi-tensor (pointer table in kernargs)
constexpr int MT_MAX = 32;
struct MTTable {
  void* p[MT_MAX];
  void* m[MT_MAX];
  void* v[MT_MAX];
  const void* g[MT_MAX];
  void* lp[MT_MAX];
  int64_t n[MT_MAX];
  int block_start[MT_MAX + 1];  // prefix sum of blocks per tensor
  int vec_ok[MT_MAX];           // 16-B aligned & numel%8==0 -> vector path
  int count;
};
constexpr int MT_CHUNK = 256 * 8 * 16;  // elements per block (16 vector iterations of a 256-thread block)

__device__ __forceinline__ int mt_find(const MTTable& t, int b) {
  int lo = 0, hi = t.count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t.block_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <typename TP, typename TG, typename TL, bool HAS_LP>
__global__ void __launch_bounds__(256) adam_mt_kernel(MTTable t, AdamArgs a) {
  const int ti = mt_find(t, blockIdx.x);
  const int64_t chunk = blockIdx.x - t.block_start[ti];
  TP* p = (TP*)t.p[ti];
  TP* m = (TP*)t.m[ti];
  TP* v = (TP*)t.v[ti];
  const TG* g = (const TG*)t.g[ti];
  TL* lp = (TL*)t.lp[ti];
  const int64_t n = t.n[ti];
  const int64_t beg = chunk * MT_CHUNK, end = min(n, beg + (int64_t)MT_CHUNK);
  const float step_size = 1.f / a.bias_correction1;
  const float denom_scale = rsqrtf(a.bias_correction2);
  if (t.vec_ok[ti]) {
    for (int64_t o = beg + threadIdx.x * 8; o < end; o += 256 * 8) {
      float pp[8], mm[8], vv[8], gg[8];
      Vec8<TP>::load(p + o, pp);
      Vec8<TP>::load(m + o, mm);
      Vec8<TP>::load(v + o, vv);
      Vec8<TG>::load(g + o, gg);
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem(pp[j], mm[j], vv[j], gg[j], a, step_size, denom_scale);
      Vec8<TP>::store(p + o, pp);
      Vec8<TP>::store(m + o, mm);
      Vec8<TP>::store(v + o, vv);
      if (HAS_LP) Vec8<TL>::store(lp + o, pp);
    }
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
      float pp = to_f32(p[i]), mm = to_f32(m[i]), vv = to_f32(v[i]);
      adam_elem(pp, mm, vv, to_f32(g[i]), a, step_size, denom_scale);
      p[i] = from_f32<TP>(pp);
      m[i] = from_f32<TP>(mm);
      v[i] = from_f32<TP>(vv);
      if (HAS_LP) lp[i] = from_f32<TL>(pp);
    }
  }
}


// ---------------------------------------------------------------- split-master Adam (bf16 weight + 16 low bits)
// The fp32 master value is not stored separately: its bit pattern is (hi << 16) + sext(lo), where `hi` is the bf16
// model weight itself (the master rounded to nearest, ties away from zero) and `lo` a signed 16-bit residual in
// fp32 ulps. The update reconstructs the exact fp32 master, applies Adam and writes both halves back, so training
// is bit-identical to an fp32 master whose bf16 copy is rounded half-up — at 2 B/param less memory and traffic.
__device__ __forceinline__ float split_join(uint16_t hi, int16_t lo) {
  return __uint_as_float(((uint32_t)hi << 16) + (uint32_t)(int32_t)lo);
}
__device__ __forceinline__ void split_cut(float f, uint16_t& hi, int16_t& lo) {
  const uint32_t u = __float_as_uint(f);
  hi = (uint16_t)((u + 0x8000u) >> 16);
  lo = (int16_t)(u & 0xffffu);
}

template <typename TG>
__global__ void __launch_bounds__(256) adam_mt_split_kernel(MTTable t, AdamArgs a) {
  const int ti = mt_find(t, blockIdx.x);
  const int64_t chunk = blockIdx.x - t.block_start[ti];
  int16_t* lo = (int16_t*)t.p[ti];
  float* m = (float*)t.m[ti];
  float* v = (float*)t.v[ti];
  const TG* g = (const TG*)t.g[ti];
  uint16_t* hi = (uint16_t*)t.lp[ti];
  const int64_t n = t.n[ti];
  const int64_t beg = chunk * MT_CHUNK, end = min(n, beg + (int64_t)MT_CHUNK);
  const float step_size = 1.f / a.bias_correction1;
  const float denom_scale = rsqrtf(a.bias_correction2);
  if (t.vec_ok[ti]) {
    for (int64_t o = beg + threadIdx.x * 8; o < end; o += 256 * 8) {
      float pp[8], mm[8], vv[8], gg[8];
      s16x8 h = *reinterpret_cast<const s16x8*>(hi + o);
      s16x8 l = *reinterpret_cast<const s16x8*>(lo + o);
      Vec8<float>::load(m + o, mm);
      Vec8<float>::load(v + o, vv);
      Vec8<TG>::load(g + o, gg);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pp[j] = split_join((uint16_t)h[j], (int16_t)l[j]);
        adam_elem(pp[j], mm[j], vv[j], gg[j], a, step_size, denom_scale);
        uint16_t hh; int16_t ll;
        split_cut(pp[j], hh, ll);
        h[j] = (short)hh;
        l[j] = ll;
      }
      *reinterpret_cast<s16x8*>(hi + o) = h;
      *reinterpret_cast<s16x8*>(lo + o) = l;
      Vec8<float>::store(m + o, mm);
      Vec8<float>::store(v + o, vv);
    }
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
      float pp = split_join(hi[i], lo[i]), mm = m[i], vv = v[i];
      adam_elem(pp, mm, vv, to_f32(g[i]), a, step_size, denom_scale);
      uint16_t hh; int16_t ll;
      split_cut(pp, hh, ll);
      hi[i] = hh; lo[i] = ll; m[i] = mm; v[i] = vv;
    }
  }
}

// ---------------------------------------------------------------- Lion
struct LionArgs {
  float lr, beta1, beta2, weight_decay, grad_scale;
};
template <typename TP, typename TG, typename TL, bool HAS_LP>
__global__ void __launch_bounds__(256) lion_flat_kernel(TP* __restrict__ p, TP* __restrict__ m,
                                                        const TG* __restrict__ g, TL* __restrict__ lp, int64_t n,
                                                        LionArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = to_f32(p[i]), mm = to_f32(m[i]), gg = to_f32(g[i]) * a.grad_scale;
    const float c = fmaf(a.beta1, mm, (1.f - a.beta1) * gg);
    const float upd = (c > 0.f) ? 1.f : ((c < 0.f) ? -1.f : 0.f);
    pp = pp * (1.f - a.lr * a.weight_decay) - a.lr * upd;
    mm = fmaf(a.beta2, mm, (1.f - a.beta2) * gg);
    p[i] = from_f32<TP>(pp);
    m[i] = from_f32<TP>(mm);
    if (HAS_LP) lp[i] = from_f32<TL>(pp);
  }
}

// ---------------------------------------------------------------- Adagrad
struct AdagradArgs {
  float lr, eps, weight_decay, grad_scale;
};
template <typename TP, typename TG, typename TL, bool HAS_LP>
__global__ void __launch_bounds__(256) adagrad_flat_kernel(TP* __restrict__ p, TP* __restrict__ s,
                                                           const TG* __restrict__ g, TL* __restrict__ lp, int64_t n,
                                                           AdagradArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = to_f32(p[i]), ss = to_f32(s[i]), gg = to_f32(g[i]) * a.grad_scale;
    if (a.weight_decay != 0.f) gg = fmaf(a.weight_decay, pp, gg);
    ss = fmaf(gg, gg, ss);
    pp -= a.lr * gg / (sqrtf(ss) + a.eps);
    p[i] = from_f32<TP>(pp);
    s[i] = from_f32<TP>(ss);
    if (HAS_LP) lp[i] = from_f32<TL>(pp);
  }
}

// ---------------------------------------------------------------- LAMB (2 passes + tiny reduction)
// pass 1: m,v update; u = m_hat/(sqrt(v_hat)+eps) + wd*p stored to `u`; per-block partial ||p||^2 and ||u||^2.
template <typename TP, typename TG>
__global__ void __launch_bounds__(256) lamb_phase1_kernel(const TP* __restrict__ p, TP* __restrict__ m,
                                                          TP* __restrict__ v, const TG* __restrict__ g,
                                                          float* __restrict__ u, float* __restrict__ partials,
                                                          int64_t n, AdamArgs a) {
  __shared__ float red[8];
  float wsq = 0.f, usq = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float rb1 = 1.f / a.bias_correction1, rb2 = 1.f / a.bias_correction2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float pp = to_f32(p[i]);
    const float gg = to_f32(g[i]) * a.grad_scale;
    float mm = fmaf(a.beta1, to_f32(m[i]), (1.f - a.beta1) * gg);
    float vv = fmaf(a.beta2, to_f32(v[i]), (1.f - a.beta2) * gg * gg);
    m[i] = from_f32<TP>(mm);
    v[i] = from_f32<TP>(vv);
    const float uu = (mm * rb1) / (sqrtf(vv * rb2) + a.eps) + a.weight_decay * pp;
    u[i] = uu;
    wsq = fmaf(pp, pp, wsq);
    usq = fmaf(uu, uu, usq);
  }
  wsq = block_sum(wsq, red);
  usq = block_sum(usq, red + 4);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = wsq;
    partials[2 * blockIdx.x + 1] = usq;
  }
}
// pass 2: each block re-reduces the (few hundred) partials, computes the trust ratio and applies the update.
template <typename TP, typename TL, bool HAS_LP>
__global__ void __launch_bounds__(256) lamb_phase2_kernel(TP* __restrict__ p, const float* __restrict__ u,
                                                          const float* __restrict__ partials, int nparts,
                                                          TL* __restrict__ lp, int64_t n, float lr, float max_coeff,
                                                          float min_coeff, float* __restrict__ coeff_out) {
  __shared__ float red[8];
  float w = 0.f, uu = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    w += partials[2 * i];
    uu += partials[2 * i + 1];
  }
  w = sqrtf(block_sum(w, red));
  uu = sqrtf(block_sum(uu, red + 4));
  float trust = (w > 0.f && uu > 0.f) ? w / uu : 1.f;
  trust = fminf(fmaxf(trust, min_coeff), max_coeff);
  if (blockIdx.x == 0 && threadIdx.x == 0 && coeff_out) *coeff_out = trust;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float pp = to_f32(p[i]) - lr * trust * u[i];
    p[i] = from_f32<TP>(pp);
    if (HAS_LP) lp[i] = from_f32<TL>(pp);
  }
}

// ---------------------------------------------------------------- norms / overflow
// Sum of squares of a flat tensor into per-block partials (deterministic 2-pass; pass 2 in `finalize`).
template <typename T>
__global__ void __launch_bounds__(256) sumsq_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ partials,
                                                    int slot_offset) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t nvec = (((uintptr_t)x) % 16 == 0) ? n / 8 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float vv[8];
    Vec8<T>::load(x + i * 8, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(vv[j], vv[j], acc);
  }
  for (int64_t i = nvec * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float f = to_f32(x[i]);
    acc = fmaf(f, f, acc);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partials[slot_offset + blockIdx.x] = acc;
}
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ partials, int n,
                                                           float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) *out = acc;
}

template <typename T> struct DT;
template <> struct DT<float> { static constexpr int v = DS_F32; };
template <> struct DT<bf16> { static constexpr int v = DS_BF16; };
template <> struct DT<fp16> { static constexpr int v = DS_F16; };

}  // namespace

// ============================================================================ C ABI launchers
// All launchers return 0 on success or a hipError_t code. dtype codes: 0 fp32, 1 bf16, 2 fp16; lp_dtype -1 = none.

#define DISPATCH_G(gdt, ...)                                        \
  do {                                                              \
    if ((gdt) == DS_F32) { using TG = float; __VA_ARGS__; }         \
    else if ((gdt) == DS_BF16) { using TG = bf16; __VA_ARGS__; }    \
    else { using TG = fp16; __VA_ARGS__; }                          \
  } while (0)
#define DISPATCH_P(pdt, ...)                                        \
  do {                                                              \
    if ((pdt) == DS_F32) { using TP = float; __VA_ARGS__; }         \
    else if ((pdt) == DS_BF16) { using TP = bf16; __VA_ARGS__; }    \
    else { using TP = fp16; __VA_ARGS__; }                          \
  } while (0)
#define DISPATCH_LP(ldt, ...)                                                         \
  do {                                                                                \
    if ((ldt) < 0) { using TL = float; constexpr bool HL = false; __VA_ARGS__; }      \
    else if ((ldt) == DS_F32) { using TL = float; constexpr bool HL = true; __VA_ARGS__; } \
    else if ((ldt) == DS_BF16) { using TL = bf16; constexpr bool HL = true; __VA_ARGS__; } \
    else { using TL = fp16; constexpr bool HL = true; __VA_ARGS__; }                  \
  } while (0)

extern "C" int ds_adam_flat(void* p, void* m, void* v, const void* g, void* lp, int64_t n, int p_dtype, int g_dtype,
                            int lp_dtype, float lr, float beta1, float beta2, float eps, float wd, float bc1,
                            float bc2, float grad_scale, int adamw_mode, hipStream_t stream) {
  if (n <= 0) return 0;
  AdamArgs a{lr, beta1, beta2, eps, wd, bc1, bc2, grad_scale, adamw_mode};
  const int grid = ds_grid_for((n + 7) / 8, 256);
  auto al = [](const void* q) { return q == nullptr || ((uintptr_t)q % 16) == 0; };
  const bool vec = al(p) && al(m) && al(v) && al(g) && al(lp);
  if (vec) {
    DISPATCH_P(p_dtype, DISPATCH_G(g_dtype, DISPATCH_LP(lp_dtype,
        hipLaunchKernelGGL((adam_flat_kernel<TP, TG, TL, HL, true>), dim3(grid), dim3(256), 0, stream, (TP*)p,
                           (TP*)m, (TP*)v, (const TG*)g, (TL*)lp, n, a))));
  } else {
    DISPATCH_P(p_dtype, DISPATCH_G(g_dtype, DISPATCH_LP(lp_dtype,
        hipLaunchKernelGGL((adam_flat_kernel<TP, TG, TL, HL, false>), dim3(ds_grid_for(n, 256)), dim3(256), 0,
                           stream, (TP*)p, (TP*)m, (TP*)v, (const TG*)g, (TL*)lp, n, a))));
  }
  DS_CHECK_LAUNCH();
  return 0;
}

// Multi-tensor Adam: arrays of `count` pointers; processed in launches of up to MT_MAX tensors.
extern "C" int ds_adam_multi(void** p, void** m, void** v, const void** g, void** lp, const int64_t* n, int count,
                             int p_dtype, int g_dtype, int lp_dtype, float lr, float beta1, float beta2, float eps,
                             float wd, float bc1, float bc2, float grad_scale, int adamw_mode, hipStream_t stream) {
  AdamArgs a{lr, beta1, beta2, eps, wd, bc1, bc2, grad_scale, adamw_mode};
  for (int base = 0; base < count; base += MT_MAX) {
    MTTable t;
    t.count = count - base < MT_MAX ? count - base : MT_MAX;
    int blocks = 0;
    for (int i = 0; i < t.count; ++i) {
      const int k = base + i;
      t.p[i] = p[k]; t.m[i] = m[k]; t.v[i] = v[k]; t.g[i] = g[k]; t.lp[i] = lp ? lp[k] : nullptr; t.n[i] = n[k];
      t.block_start[i] = blocks;
      blocks += (int)((n[k] + MT_CHUNK - 1) / MT_CHUNK);
      auto al = [](const void* q) { return ((uintptr_t)q % 16) == 0; };
      bool ok = (n[k] % 8 == 0) && al(p[k]) && al(m[k]) && al(v[k]) && al(g[k]) && (!lp || al(lp[k]));
      t.vec_ok[i] = ok ? 1 : 0;
    }
    t.block_start[t.count] = blocks;
    if (blocks == 0) continue;
    DISPATCH_P(p_dtype, DISPATCH_G(g_dtype, DISPATCH_LP(lp ? lp_dtype : -1,
        hipLaunchKernelGGL((adam_mt_kernel<TP, TG, TL, HL>), dim3(blocks), dim3(256), 0, stream, t, a))));
    DS_CHECK_LAUNCH();
  }
  return 0;
}

// Split-master multi-tensor Adam: lo (int16 residuals), m/v (fp32), g (any dtype), hi (bf16 weights, in/out).
extern "C" int ds_adam_multi_split(void** lo, void** m, void** v, const void** g, void** hi, const int64_t* n,
                                   int count, int g_dtype, float lr, float beta1, float beta2, float eps, float wd,
                                   float bc1, float bc2, float grad_scale, int adamw_mode, hipStream_t stream) {
  AdamArgs a{lr, beta1, beta2, eps, wd, bc1, bc2, grad_scale, adamw_mode};
  for (int base = 0; base < count; base += MT_MAX) {
    MTTable t;
    t.count = count - base < MT_MAX ? count - base : MT_MAX;
    int blocks = 0;
    for (int i = 0; i < t.count; ++i) {
      const int k = base + i;
      t.p[i] = lo[k]; t.m[i] = m[k]; t.v[i] = v[k]; t.g[i] = g[k]; t.lp[i] = hi[k]; t.n[i] = n[k];
      t.block_start[i] = blocks;
      blocks += (int)((n[k] + MT_CHUNK - 1) / MT_CHUNK);
      auto al = [](const void* q) { return ((uintptr_t)q % 16) == 0; };
      t.vec_ok[i] = ((n[k] % 8 == 0) && al(lo[k]) && al(m[k]) && al(v[k]) && al(g[k]) && al(hi[k])) ? 1 : 0;
    }
    t.block_start[t.count] = blocks;
    if (blocks == 0) continue;
    DISPATCH_G(g_dtype, hipLaunchKernelGGL((adam_mt_split_kernel<TG>), dim3(blocks), dim3(256), 0, stream, t, a));
    DS_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int ds_lion_flat(void* p, void* m, const void* g, void* lp, int64_t n, int p_dtype, int g_dtype,
                            int lp_dtype, float lr, float beta1, float beta2, float wd, float grad_scale,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  LionArgs a{lr, beta1, beta2, wd, grad_scale};
  const int grid = ds_grid_for(n, 256);
  DISPATCH_P(p_dtype, DISPATCH_G(g_dtype, DISPATCH_LP(lp_dtype,
      hipLaunchKernelGGL((lion_flat_kernel<TP, TG, TL, HL>), dim3(grid), dim3(256), 0, stream, (TP*)p, (TP*)m,
                         (const TG*)g, (TL*)lp, n, a))));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_adagrad_flat(void* p, void* s, const void* g, void* lp, int64_t n, int p_dtype, int g_dtype,
                               int lp_dtype, float lr, float eps, float wd, float grad_scale, hipStream_t stream) {
  if (n <= 0) return 0;
  AdagradArgs a{lr, eps, wd, grad_scale};
  const int grid = ds_grid_for(n, 256);
  DISPATCH_P(p_dtype, DISPATCH_G(g_dtype, DISPATCH_LP(lp_dtype,
      hipLaunchKernelGGL((adagrad_flat_kernel<TP, TG, TL, HL>), dim3(grid), dim3(256), 0, stream, (TP*)p, (TP*)s,
                         (const TG*)g, (TL*)lp, n, a))));
  DS_CHECK_LAUNCH();
  return 0;
}

// LAMB: `u` is an fp32 scratch of n elements; `partials` has room for 2*512 floats.
extern "C" int ds_lamb_flat(void* p, void* m, void* v, const void* g, void* lp, float* u, float* partials,
                            float* coeff_out, int64_t n, int p_dtype, int g_dtype, int lp_dtype, float lr,
                            float beta1, float beta2, float eps, float wd, float bc1, float bc2, float grad_scale,
                            float max_coeff, float min_coeff, hipStream_t stream) {
  if (n <= 0) return 0;
  AdamArgs a{lr, beta1, beta2, eps, wd, bc1, bc2, grad_scale, 1};
  const int grid = ds_grid_for(n, 256, 512);
  DISPATCH_P(p_dtype, DISPATCH_G(g_dtype,
      hipLaunchKernelGGL((lamb_phase1_kernel<TP, TG>), dim3(grid), dim3(256), 0, stream, (const TP*)p, (TP*)m,
                         (TP*)v, (const TG*)g, u, partials, n, a)));
  DS_CHECK_LAUNCH();
  DISPATCH_P(p_dtype, DISPATCH_LP(lp_dtype,
      hipLaunchKernelGGL((lamb_phase2_kernel<TP, TL, HL>), dim3(grid), dim3(256), 0, stream, (TP*)p, u, partials,
                         grid, (TL*)lp, n, lr, max_coeff, min_coeff, coeff_out)));
  DS_CHECK_LAUNCH();
  return 0;
}

// Sum of squares over a list of flat tensors -> *out (fp32). `partials` needs sum(blocks) floats; returns via out.
extern "C" int ds_sumsq_multi(const void** x, const int64_t* n, const int* dtypes, int count, float* partials,
                              int partials_cap, float* out, hipStream_t stream) {
  int slot = 0;
  for (int i = 0; i < count; ++i) {
    if (n[i] <= 0) continue;
    int grid = ds_grid_for((n[i] + 7) / 8, 256, 512);
    if (slot + grid > partials_cap) grid = partials_cap - slot;
    if (grid <= 0) return (int)hipErrorInvalidValue;
    if (dtypes[i] == DS_F32)
      hipLaunchKernelGGL((sumsq_kernel<float>), dim3(grid), dim3(256), 0, stream, (const float*)x[i], n[i], partials, slot);
    else if (dtypes[i] == DS_BF16)
      hipLaunchKernelGGL((sumsq_kernel<bf16>), dim3(grid), dim3(256), 0, stream, (const bf16*)x[i], n[i], partials, slot);
    else
      hipLaunchKernelGGL((sumsq_kernel<fp16>), dim3(grid), dim3(256), 0, stream, (const fp16*)x[i], n[i], partials, slot);
    DS_CHECK_LAUNCH();
    slot += grid;
  }
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream, partials, slot, out);
  DS_CHECK_LAUNCH();
  return 0;
}
