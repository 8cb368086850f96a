// Gated / biased activations, fwd+bwd, CDNA4.
//
// Parity: reference `csrc/transformer/gelu_kernels.cu` (gelu_kernel, fused_bias_gelu, d_gelu_func),
// `csrc/transformer/inference/csrc/gelu.cu` (fused_bias_gelu, fused_gate_activation = GEGLU/SwiGLU),
// `relu.cu`, v2 `core_ops/bias_activations`, `core_ops/gated_activations`.
//
// Memory-bound: 8 elements per lane per iteration (16 B for bf16), grid-stride over 256 CUs x 8 blocks.
// Gated layout is the fused gate_up projection output [rows, 2*I] = [gate | up] per row (one GEMM for both).
#include "../include/ds_hip.h"

namespace {

enum Act : int { ACT_SILU = 0, ACT_GELU_TANH = 1, ACT_GELU_ERF = 2, ACT_RELU = 3, ACT_IDENTITY = 4 };

template <int A>
__device__ __forceinline__ float act_f(float x) {
  if (A == ACT_SILU) return x / (1.f + __expf(-x));
  if (A == ACT_GELU_TANH) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
  }
  if (A == ACT_GELU_ERF) return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
  if (A == ACT_RELU) return fmaxf(x, 0.f);
  return x;
}
template <int A>
__device__ __forceinline__ float act_df(float x) {
  if (A == ACT_SILU) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
  if (A == ACT_GELU_TANH) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (x + k1 * x * x * x);
    const float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  }
  if (A == ACT_GELU_ERF) {
    return 0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
  }
  if (A == ACT_RELU) return x > 0.f ? 1.f : 0.f;
  return 1.f;
}

// out[r, i] = act(gu[r, i]) * gu[r, I + i]
template <typename T, int A>
__global__ void __launch_bounds__(256) gated_fwd_kernel(const T* __restrict__ gu, T* __restrict__ out, int64_t rows,
                                                        int I) {
  const int64_t nvec_row = I / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float g[8], u[8], o[8];
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g[j]) * u[j];
    Vec8<T>::store(out + r * I + c, o);
  }
}
// dgu[r, i] = dout * u * act'(g) ; dgu[r, I+i] = dout * act(g)
template <typename T, int A>
__global__ void __launch_bounds__(256) gated_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ gu,
                                                        T* __restrict__ dgu, int64_t rows, int I) {
  const int64_t nvec_row = I / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
    Vec8<T>::load(dout + r * I + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dg[j] = d[j] * u[j] * act_df<A>(g[j]);
      du[j] = d[j] * act_f<A>(g[j]);
    }
    Vec8<T>::store(dgu + r * 2 * I + c, dg);
    Vec8<T>::store(dgu + r * 2 * I + I + c, du);
  }
}

// y = act(x + bias) (bias optional, broadcast over rows of length C)
template <typename T, int A, bool BIAS>
__global__ void __launch_bounds__(256) bias_act_fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                           T* __restrict__ y, int64_t rows, int C) {
  const int64_t nvec_row = C / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float v[8], b[8];
    Vec8<T>::load(x + r * C + c, v);
    if (BIAS) Vec8<T>::load(bias + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_f<A>(BIAS ? v[j] + b[j] : v[j]);
    Vec8<T>::store(y + r * C + c, v);
  }
}
// dx = dy * act'(x + bias)  (bias grad = column sum of dx, done by the caller's colsum or torch.sum)
template <typename T, int A, bool BIAS>
__global__ void __launch_bounds__(256) bias_act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const T* __restrict__ bias, T* __restrict__ dx,
                                                           int64_t rows, int C) {
  const int64_t nvec_row = C / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float v[8], b[8], d[8];
    Vec8<T>::load(x + r * C + c, v);
    Vec8<T>::load(dy + r * C + c, d);
    if (BIAS) Vec8<T>::load(bias + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= act_df<A>(BIAS ? v[j] + b[j] : v[j]);
    Vec8<T>::store(dx + r * C + c, d);
  }
}

// y = x + bias + residual (inference `fused_bias_residual` / v2 bias_add)
template <typename T>
__global__ void __launch_bounds__(256) bias_residual_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                            const T* __restrict__ res, T* __restrict__ y,
                                                            int64_t rows, int C, float res_scale) {
  const int64_t nvec_row = C / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float v[8], b[8], rr[8];
    Vec8<T>::load(x + r * C + c, v);
    if (bias) Vec8<T>::load(bias + c, b);
    if (res) Vec8<T>::load(res + r * C + c, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] + (bias ? b[j] : 0.f) + (res ? rr[j] * res_scale : 0.f);
    Vec8<T>::store(y + r * C + c, v);
  }
}

// y = x + bias + other + other_bias over channels-last rows (spatial `nhwc_bias_add_bias_add`; diffusers UNet/VAE
// residual joins). Either of (other, other_bias) may be null.
template <typename T>
__global__ void __launch_bounds__(256) bias_add2_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                        const T* __restrict__ other, const T* __restrict__ obias,
                                                        T* __restrict__ y, int64_t rows, int C) {
  const int64_t nvec_row = C / 8;
  const int64_t total = rows * nvec_row;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvec_row, c = (t - r * nvec_row) * 8;
    float v[8], b[8], o[8], ob[8];
    Vec8<T>::load(x + r * C + c, v);
    Vec8<T>::load(bias + c, b);
    if (other) Vec8<T>::load(other + r * C + c, o);
    if (obias) Vec8<T>::load(obias + c, ob);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += b[j] + (other ? o[j] : 0.f) + (obias ? ob[j] : 0.f);
    Vec8<T>::store(y + r * C + c, v);
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                    \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)
#define DISPATCH_ACT(a, ...)                                                  \
  do {                                                                        \
    if ((a) == ACT_SILU) { constexpr int A = ACT_SILU; __VA_ARGS__; }         \
    else if ((a) == ACT_GELU_TANH) { constexpr int A = ACT_GELU_TANH; __VA_ARGS__; } \
    else if ((a) == ACT_GELU_ERF) { constexpr int A = ACT_GELU_ERF; __VA_ARGS__; }   \
    else if ((a) == ACT_RELU) { constexpr int A = ACT_RELU; __VA_ARGS__; }    \
    else { constexpr int A = ACT_IDENTITY; __VA_ARGS__; }                     \
  } while (0)

extern "C" int ds_gated_act_fwd(const void* gu, void* out, int64_t rows, int I, int act, int dtype, hipStream_t s) {
  if (I % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(rows * (I / 8), 256);
  DISPATCH_T(dtype, DISPATCH_ACT(act, hipLaunchKernelGGL((gated_fwd_kernel<T, A>), dim3(grid), dim3(256), 0, s,
                                                         (const T*)gu, (T*)out, rows, I)));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_gated_act_bwd(const void* dout, const void* gu, void* dgu, int64_t rows, int I, int act, int dtype,
                                hipStream_t s) {
  if (I % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(rows * (I / 8), 256);
  DISPATCH_T(dtype, DISPATCH_ACT(act, hipLaunchKernelGGL((gated_bwd_kernel<T, A>), dim3(grid), dim3(256), 0, s,
                                                         (const T*)dout, (const T*)gu, (T*)dgu, rows, I)));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_bias_act_fwd(const void* x, const void* bias, void* y, int64_t rows, int C, int act, int dtype,
                               hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  DISPATCH_T(dtype, DISPATCH_ACT(act, {
    if (bias)
      hipLaunchKernelGGL((bias_act_fwd_kernel<T, A, true>), dim3(grid), dim3(256), 0, s, (const T*)x,
                         (const T*)bias, (T*)y, rows, C);
    else
      hipLaunchKernelGGL((bias_act_fwd_kernel<T, A, false>), dim3(grid), dim3(256), 0, s, (const T*)x, nullptr,
                         (T*)y, rows, C);
  }));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_bias_act_bwd(const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int C, int act,
                               int dtype, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  DISPATCH_T(dtype, DISPATCH_ACT(act, {
    if (bias)
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, A, true>), dim3(grid), dim3(256), 0, s, (const T*)dy, (const T*)x,
                         (const T*)bias, (T*)dx, rows, C);
    else
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, A, false>), dim3(grid), dim3(256), 0, s, (const T*)dy,
                         (const T*)x, nullptr, (T*)dx, rows, C);
  }));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_bias_residual(const void* x, const void* bias, const void* res, void* y, int64_t rows, int C,
                                float res_scale, int dtype, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((bias_residual_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)x,
                                       (const T*)bias, (const T*)res, (T*)y, rows, C, res_scale));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_bias_add2(const void* x, const void* bias, const void* other, const void* obias, void* y,
                            int64_t rows, int C, int dtype, hipStream_t s) {
  if (C % 8 || bias == nullptr) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((bias_add2_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)x,
                                       (const T*)bias, (const T*)other, (const T*)obias, (T*)y, rows, C));
  DS_CHECK_LAUNCH();
  return 0;
}
