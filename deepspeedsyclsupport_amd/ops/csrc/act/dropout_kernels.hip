// Fused (bias +) dropout (+ residual) forward / backward for CDNA4, mask regenerated from (seed, offset) in the
// backward instead of stored.
//
// Reference counterparts (behaviour, not code): `csrc/transformer/dropout_kernels.cu:10-726` — `dropout_kernel`,
// `dropout_kernel_bwd`, the bias / bias+residual fused variants used by `ds_transformer_cuda.cpp` — which keep a
// uint8 mask per element in HBM between forward and backward.
//
// MI355X design:
//  * counter-based RNG: one Philox-4x32 (10 rounds) evaluation per 8-element vector, keyed by the 64-bit seed,
//    counter = (vector index, offset). Each 32-bit output yields two 16-bit uniforms, so 8 elements cost one Philox
//    call; keep <=> u16 >= round(p * 65536). The backward re-derives the identical mask from the same counter, so
//    no mask tensor is written or read: the bwd moves 2 tensors (dy in, dx out) instead of 3;
//  * 16-byte vector loads / stores (8 x bf16), grid-stride loop over rows * C / 8 vectors, wave64-sized blocks;
//  * optional per-column bias (added before dropout) and residual (added after), fp32 math, output in the input
//    dtype. Bias gradient = column sum of dx (taken by the caller with one reduction).
#include "ds_hip.h"

namespace {

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  return {c0, c1, c2, c3};
}

// 8 keep bits for vector v
__device__ __forceinline__ uint32_t keep_bits(uint64_t seed, uint64_t offset, uint64_t v, uint32_t thresh) {
  const U4 r = philox((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)seed,
                      (uint32_t)(seed >> 32));
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bits |= ((w[j] & 0xffffu) >= thresh ? 1u : 0u) << (2 * j);
    bits |= ((w[j] >> 16) >= thresh ? 1u : 0u) << (2 * j + 1);
  }
  return bits;
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                          const T* __restrict__ res, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask_out, int64_t rows, int C,
                                                          uint64_t seed, uint64_t offset, uint32_t thresh,
                                                          float scale) {
  const int64_t nvr = C / 8, total = rows * nvr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t r = t / nvr, c = (t - r * nvr) * 8;
    float v[8], b[8], rr[8];
    Vec8<T>::load(x + r * C + c, v);
    if (bias) Vec8<T>::load(bias + c, b);
    if (res) Vec8<T>::load(res + r * C + c, rr);
    const uint32_t keep = keep_bits(seed, offset, (uint64_t)t, thresh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float h = v[j] + (bias ? b[j] : 0.f);
      v[j] = ((keep >> j) & 1u ? h * scale : 0.f) + (res ? rr[j] : 0.f);
    }
    Vec8<T>::store(y + r * C + c, v);
    if (mask_out) mask_out[t] = (uint8_t)keep;  // optional packed mask (8 elements / byte) for inspection
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int64_t rows,
                                                          int C, uint64_t seed, uint64_t offset, uint32_t thresh,
                                                          float scale) {
  const int64_t nvr = C / 8, total = rows * nvr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    float g[8];
    Vec8<T>::load(dy + t * 8, g);
    const uint32_t keep = keep_bits(seed, offset, (uint64_t)t, thresh);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (keep >> j) & 1u ? g[j] * scale : 0.f;
    Vec8<T>::store(dx + t * 8, g);
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                    \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)

static uint32_t dropout_threshold(float p) {
  const float t = p * 65536.f + 0.5f;
  return t <= 0.f ? 0u : (t >= 65536.f ? 65536u : (uint32_t)t);
}

extern "C" int ds_dropout_fwd(const void* x, const void* bias, const void* res, void* y, uint8_t* mask, int64_t rows,
                              int C, float p, uint64_t seed, uint64_t offset, int dtype, hipStream_t s) {
  if (C % 8 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  const float scale = 1.f / (1.f - p);
  const uint32_t th = dropout_threshold(p);
  DISPATCH_T(dtype, hipLaunchKernelGGL((dropout_fwd_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)x,
                                       (const T*)bias, (const T*)res, (T*)y, mask, rows, C, seed, offset, th, scale));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_dropout_bwd(const void* dy, void* dx, int64_t rows, int C, float p, uint64_t seed, uint64_t offset,
                              int dtype, hipStream_t s) {
  if (C % 8 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int grid = ds_grid_for(rows * (C / 8), 256);
  const float scale = 1.f / (1.f - p);
  const uint32_t th = dropout_threshold(p);
  DISPATCH_T(dtype, hipLaunchKernelGGL((dropout_bwd_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)dy, (T*)dx,
                                       rows, C, seed, offset, th, scale));
  DS_CHECK_LAUNCH();
  return 0;
}
