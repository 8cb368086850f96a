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

// ---------------------------------------------------------------- gated activation with K-major side outputs
// The training step needs the SwiGLU output X twice: row-major [T, I] for the forward down-projection GEMM and
// token-contiguous ("K-major") X^T [I, Tp] for the weight-gradient GEMM dW = dY^T X, which contracts over tokens (the
// library GEMM runs ~40 % faster on K-major operands). Likewise the backward's d(gate|up) is needed row-major for the
// data-gradient GEMM and K-major for the weight gradient. These kernels write both layouts in the pass that computes
// the values, so no separate transpose kernel re-reads them: one workgroup owns a 64-token x 64-feature tile, computes
// it from 16-B row loads, stores it row-major, parks it in LDS (rows padded to 33 dwords) and stores its transpose
// with 16-B stores along the token axis. Tp >= T pads the token axis with zeros (a multiple of 256 for the GEMM).
constexpr int GT_TS = 64;
constexpr int GT_LROW = 33;

template <typename T>
__device__ __forceinline__ void tile_store_transposed(const uint32_t* tile, T* __restrict__ outT, int c0, int r0,
                                                      int C, int64_t Tp, int lr, int lc) {
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int j = lr + 32 * p, oc = c0 + j;
    const int64_t orow0 = r0 + 8 * lc;
    if (oc >= C || orow0 >= Tp) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = t16[(8 * lc + 2 * e) * GT_LROW * 2 + j];
      const uint32_t hi = t16[(8 * lc + 2 * e + 1) * GT_LROW * 2 + j];
      w[e] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(outT) + (int64_t)oc * Tp + orow0) =
        make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <typename T>
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  uint4 r;
  T* h = reinterpret_cast<T*>(&r);
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (T)v[j];
  return r;
}

// out[r, i] = act(g) * u, outT[i, r] the same values token-contiguous
template <typename T, int A>
__global__ void __launch_bounds__(256) gated_fwd_t_kernel(const T* __restrict__ gu, T* __restrict__ out,
                                                          T* __restrict__ outT, int64_t rows, int64_t Tp, int I,
                                                          int tiles_r, int tiles_c) {
  __shared__ uint32_t tile[GT_TS * GT_LROW];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tr = bid % tiles_r, tc = bid / tiles_r;
  const int r0 = tr * GT_TS, c0 = tc * GT_TS;
  const int t = threadIdx.x, lr = t >> 3, lc = t & 7;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = lr + 32 * p;
    const int64_t gr = (int64_t)r0 + r;
    const int gc = c0 + 8 * lc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gr < rows && gc < I) {
      float g[8], u[8], o[8];
      Vec8<T>::load(gu + gr * 2 * I + gc, g);
      Vec8<T>::load(gu + gr * 2 * I + I + gc, u);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g[j]) * u[j];
      v = pack8<T>(o);
      *reinterpret_cast<uint4*>(out + gr * I + gc) = v;
    }
    uint32_t* dst = tile + r * GT_LROW + 4 * lc;
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();
  tile_store_transposed<T>(tile, outT, c0, r0, I, Tp, lr, lc);
}

// dgu[r, i] = dout * u * act'(g), dgu[r, I + i] = dout * act(g); dguT[2I, Tp] the same values token-contiguous
template <typename T, int A>
__global__ void __launch_bounds__(256) gated_bwd_t_kernel(const T* __restrict__ dout, const T* __restrict__ gu,
                                                          T* __restrict__ dgu, T* __restrict__ dguT, int64_t rows,
                                                          int64_t Tp, int I, int tiles_r, int tiles_c) {
  __shared__ uint32_t tile_g[GT_TS * GT_LROW];
  __shared__ uint32_t tile_u[GT_TS * GT_LROW];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tr = bid % tiles_r, tc = bid / tiles_r;
  const int r0 = tr * GT_TS, c0 = tc * GT_TS;
  const int t = threadIdx.x, lr = t >> 3, lc = t & 7;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = lr + 32 * p;
    const int64_t gr = (int64_t)r0 + r;
    const int gc = c0 + 8 * lc;
    uint4 vg = make_uint4(0u, 0u, 0u, 0u), vu = vg;
    if (gr < rows && gc < I) {
      float g[8], u[8], d[8], dg[8], du[8];
      Vec8<T>::load(gu + gr * 2 * I + gc, g);
      Vec8<T>::load(gu + gr * 2 * I + I + gc, u);
      Vec8<T>::load(dout + gr * I + gc, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dg[j] = d[j] * u[j] * act_df<A>(g[j]);
        du[j] = d[j] * act_f<A>(g[j]);
      }
      vg = pack8<T>(dg);
      vu = pack8<T>(du);
      *reinterpret_cast<uint4*>(dgu + gr * 2 * I + gc) = vg;
      *reinterpret_cast<uint4*>(dgu + gr * 2 * I + I + gc) = vu;
    }
    uint32_t* dg_ = tile_g + r * GT_LROW + 4 * lc;
    uint32_t* du_ = tile_u + r * GT_LROW + 4 * lc;
    dg_[0] = vg.x; dg_[1] = vg.y; dg_[2] = vg.z; dg_[3] = vg.w;
    du_[0] = vu.x; du_[1] = vu.y; du_[2] = vu.z; du_[3] = vu.w;
  }
  __syncthreads();
  tile_store_transposed<T>(tile_g, dguT, c0, r0, I, Tp, lr, lc);
  tile_store_transposed<T>(tile_u, dguT + (int64_t)I * Tp, c0, r0, I, Tp, lr, lc);
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

// 16-bit dtypes only; rows, Tp, I multiples of 8, Tp >= rows; outT [I, Tp] / dguT [2I, Tp] contiguous.
extern "C" int ds_gated_act_fwd_t(const void* gu, void* out, void* outT, int64_t rows, int64_t Tp, int I, int act,
                                  int dtype, hipStream_t s) {
  if (I % 8 || rows % 8 || Tp % 8 || Tp < rows || dtype == DS_F32) return (int)hipErrorInvalidValue;
  const int64_t tiles_r = (Tp + GT_TS - 1) / GT_TS, tiles_c = (I + GT_TS - 1) / GT_TS;
  if (tiles_r * tiles_c > 0x7fffffff) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)(tiles_r * tiles_c);
  if (dtype == DS_BF16) {
    using T = bf16;
    DISPATCH_ACT(act, hipLaunchKernelGGL((gated_fwd_t_kernel<T, A>), dim3(grid), dim3(256), 0, s, (const T*)gu,
                                         (T*)out, (T*)outT, rows, Tp, I, (int)tiles_r, (int)tiles_c));
  } else {
    using T = fp16;
    DISPATCH_ACT(act, hipLaunchKernelGGL((gated_fwd_t_kernel<T, A>), dim3(grid), dim3(256), 0, s, (const T*)gu,
                                         (T*)out, (T*)outT, rows, Tp, I, (int)tiles_r, (int)tiles_c));
  }
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_gated_act_bwd_t(const void* dout, const void* gu, void* dgu, void* dguT, int64_t rows, int64_t Tp,
                                  int I, int act, int dtype, hipStream_t s) {
  if (I % 8 || rows % 8 || Tp % 8 || Tp < rows || dtype == DS_F32) return (int)hipErrorInvalidValue;
  const int64_t tiles_r = (Tp + GT_TS - 1) / GT_TS, tiles_c = (I + GT_TS - 1) / GT_TS;
  if (tiles_r * tiles_c > 0x7fffffff) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)(tiles_r * tiles_c);
  if (dtype == DS_BF16) {
    using T = bf16;
    DISPATCH_ACT(act, hipLaunchKernelGGL((gated_bwd_t_kernel<T, A>), dim3(grid), dim3(256), 0, s, (const T*)dout,
                                         (const T*)gu, (T*)dgu, (T*)dguT, rows, Tp, I, (int)tiles_r, (int)tiles_c));
  } else {
    using T = fp16;
    DISPATCH_ACT(act, hipLaunchKernelGGL((gated_bwd_t_kernel<T, A>), dim3(grid), dim3(256), 0, s, (const T*)dout,
                                         (const T*)gu, (T*)dgu, (T*)dguT, rows, Tp, I, (int)tiles_r, (int)tiles_c));
  }
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
