// Group-wise int8 / int4 quantisation for ZeRO++ (qwZ weights, qgZ gradients), MoQ / QAT fake-quant and
// weight-only inference, CDNA4.
//
// Parity: reference `csrc/quantization/{quantize.cu (cached_quantization), dequantize.cu, fake_quantizer.cu
// (fake_quantize_kernel, sr_fake_quantize_kernel, *_asym), quant_reduce.cu (dequant_reduce),
// quantize_intX.cu (dequantize_int4/8_to_half)}` and the inference `dequantize.cu`.
//
// Layout: groups of `gs` consecutive elements, ONE WAVE PER GROUP (gs <= 4096 -> <= 64 elements per lane, 16-B
// loads); the group's absmax (or min/max for asymmetric) is a 64-lane butterfly, no LDS. int4 packs two values per
// byte (low nibble = even element). Scales are fp32 per group: q = round(x / scale), x ~= q * scale (+ zero for
// asymmetric, where q is unsigned).
#include "../include/ds_hip.h"

namespace {

__device__ __forceinline__ float rnd(float x, bool sr, uint32_t& state) {
  if (!sr) return rintf(x);
  // xorshift32 stochastic rounding (deterministic per element seed)
  state ^= state << 13;
  state ^= state >> 17;
  state ^= state << 5;
  const float u = (state & 0xFFFFFF) * (1.0f / 16777216.0f);
  return floorf(x + u);
}

template <typename T, int BITS, bool ASYM>
__global__ void __launch_bounds__(256) quantize_kernel(const T* __restrict__ x, int8_t* __restrict__ q,
                                                       float* __restrict__ scales, float* __restrict__ zeros,
                                                       int64_t groups, int gs, int sr, uint32_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= groups) return;
  const T* xg = x + g * gs;
  float mx = -INFINITY, mn = INFINITY, amax = 0.f;
  for (int i = lane * 8; i < gs; i += 512) {
    float v[8];
    Vec8<T>::load(xg + i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mx = fmaxf(mx, v[j]);
      mn = fminf(mn, v[j]);
      amax = fmaxf(amax, fabsf(v[j]));
    }
  }
  constexpr int QMAX = (1 << (BITS - 1)) - 1;   // 127 / 7
  constexpr int QLEVELS = (1 << BITS) - 1;       // 255 / 15
  float scale, zero = 0.f;
  if (ASYM) {
    mx = wave_max(mx);
    mn = -wave_max(-mn);
    scale = (mx - mn) / QLEVELS;
    if (scale == 0.f) scale = 1.f;
    zero = mn;
  } else {
    amax = wave_max(amax);
    scale = amax / QMAX;
    if (scale == 0.f) scale = 1.f;
  }
  if (lane == 0) {
    scales[g] = scale;
    if (ASYM) zeros[g] = zero;
  }
  const float inv = 1.f / scale;
  uint32_t st = seed ^ (uint32_t)(g * 2654435761u) ^ (uint32_t)(lane * 40503u);
  for (int i = lane * 8; i < gs; i += 512) {
    float v[8];
    Vec8<T>::load(xg + i, v);
    int qi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = ASYM ? (v[j] - zero) * inv : v[j] * inv;
      t = rnd(t, sr, st);
      qi[j] = ASYM ? (int)fminf(fmaxf(t, 0.f), (float)QLEVELS) : (int)fminf(fmaxf(t, (float)-QMAX), (float)QMAX);
    }
    if (BITS == 8) {
      int8_t* dst = q + g * gs + i;
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo |= (uint32_t)(uint8_t)qi[j] << (8 * j);
        hi |= (uint32_t)(uint8_t)qi[j + 4] << (8 * j);
      }
      *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
    } else {
      uint8_t* dst = reinterpret_cast<uint8_t*>(q) + (g * gs + i) / 2;
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w |= (uint32_t)(((qi[2 * j] & 0xF) | ((qi[2 * j + 1] & 0xF) << 4)) & 0xFF) << (8 * j);
      *reinterpret_cast<uint32_t*>(dst) = w;
    }
  }
}

template <typename T, int BITS, bool ASYM>
__global__ void __launch_bounds__(256) dequantize_kernel(const int8_t* __restrict__ q, const float* __restrict__ scales,
                                                         const float* __restrict__ zeros, T* __restrict__ out,
                                                         int64_t n, int gs) {
  const int64_t nvec = n / 8;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = v * 8;
    const int64_t g = i / gs;
    const float s = scales[g];
    const float z = ASYM ? zeros[g] : 0.f;
    float o[8];
    if (BITS == 8) {
      const uint2 w = *reinterpret_cast<const uint2*>(q + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int a = ASYM ? (int)((w.x >> (8 * j)) & 0xFF) : (int)(int8_t)((w.x >> (8 * j)) & 0xFF);
        const int b = ASYM ? (int)((w.y >> (8 * j)) & 0xFF) : (int)(int8_t)((w.y >> (8 * j)) & 0xFF);
        o[j] = a * s + z;
        o[j + 4] = b * s + z;
      }
    } else {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(q) + i / 2);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int nib = (w >> (4 * j)) & 0xF;
        if (!ASYM && nib > 7) nib -= 16;
        o[j] = nib * s + z;
      }
    }
    Vec8<T>::store(out + i, o);
  }
}

// qgZ dequant-reduce: `in` holds `nsrc` quantised copies of the same [n] vector (int8 sym, group gs), back to back;
// out = sum_k dequant(in_k) (fp32 or bf16). Reference `quant_reduce.cu` dequant_reduce.
template <typename T>
__global__ void __launch_bounds__(256) dequant_reduce_kernel(const int8_t* __restrict__ q,
                                                             const float* __restrict__ scales, T* __restrict__ out,
                                                             int64_t n, int gs, int nsrc, float out_scale) {
  const int64_t nvec = n / 8;
  const int64_t ngroups = n / gs;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = v * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < nsrc; ++k) {
      const float s = scales[k * ngroups + i / gs];
      const uint2 w = *reinterpret_cast<const uint2*>(q + (int64_t)k * n + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] += (int)(int8_t)((w.x >> (8 * j)) & 0xFF) * s;
        acc[j + 4] += (int)(int8_t)((w.y >> (8 * j)) & 0xFF) * s;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= out_scale;
    Vec8<T>::store(out + i, acc);
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                    \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)

extern "C" int ds_quantize(const void* x, int8_t* q, float* scales, float* zeros, int64_t n, int gs, int bits,
                           int asym, int sr, unsigned seed, int dtype, hipStream_t s) {
  if (gs % 8 || n % gs || gs > 4096 || (bits != 8 && bits != 4)) return (int)hipErrorInvalidValue;
  const int64_t groups = n / gs;
  const int grid = (int)((groups + 3) / 4);
  DISPATCH_T(dtype, {
    if (bits == 8 && !asym)
      hipLaunchKernelGGL((quantize_kernel<T, 8, false>), dim3(grid), dim3(256), 0, s, (const T*)x, q, scales, zeros,
                         groups, gs, sr, seed);
    else if (bits == 8)
      hipLaunchKernelGGL((quantize_kernel<T, 8, true>), dim3(grid), dim3(256), 0, s, (const T*)x, q, scales, zeros,
                         groups, gs, sr, seed);
    else if (!asym)
      hipLaunchKernelGGL((quantize_kernel<T, 4, false>), dim3(grid), dim3(256), 0, s, (const T*)x, q, scales, zeros,
                         groups, gs, sr, seed);
    else
      hipLaunchKernelGGL((quantize_kernel<T, 4, true>), dim3(grid), dim3(256), 0, s, (const T*)x, q, scales, zeros,
                         groups, gs, sr, seed);
  });
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_dequantize(const int8_t* q, const float* scales, const float* zeros, void* out, int64_t n, int gs,
                             int bits, int asym, int dtype, hipStream_t s) {
  if (gs % 8 || n % gs || (bits != 8 && bits != 4)) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(n / 8, 256);
  DISPATCH_T(dtype, {
    if (bits == 8 && !asym)
      hipLaunchKernelGGL((dequantize_kernel<T, 8, false>), dim3(grid), dim3(256), 0, s, q, scales, zeros, (T*)out, n,
                         gs);
    else if (bits == 8)
      hipLaunchKernelGGL((dequantize_kernel<T, 8, true>), dim3(grid), dim3(256), 0, s, q, scales, zeros, (T*)out, n,
                         gs);
    else if (!asym)
      hipLaunchKernelGGL((dequantize_kernel<T, 4, false>), dim3(grid), dim3(256), 0, s, q, scales, zeros, (T*)out, n,
                         gs);
    else
      hipLaunchKernelGGL((dequantize_kernel<T, 4, true>), dim3(grid), dim3(256), 0, s, q, scales, zeros, (T*)out, n,
                         gs);
  });
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_dequant_reduce(const int8_t* q, const float* scales, void* out, int64_t n, int gs, int nsrc,
                                 float out_scale, int dtype, hipStream_t s) {
  if (gs % 8 || n % gs) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for(n / 8, 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((dequant_reduce_kernel<T>), dim3(grid), dim3(256), 0, s, q, scales, (T*)out,
                                       n, gs, nsrc, out_scale));
  DS_CHECK_LAUNCH();
  return 0;
}
