// Common CDNA4 (gfx950) device helpers for deepspeedsyclsupport_amd kernels.
// Wave64 everywhere: reductions use 64-lane shuffles / DPP-friendly xor patterns, block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DS_WAVE 64

typedef __bf16 bf16;
typedef _Float16 fp16;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 fp16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 fp16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// dtype tags shared with the Python side (ops/native.py DTYPE_CODE)
enum DsDtype : int { DS_F32 = 0, DS_BF16 = 1, DS_F16 = 2 };

// ---------------------------------------------------------------- 8-wide vector load/store in any dtype
// Loads 8 consecutive elements (16 B for bf16/fp16, 32 B for fp32) and widens to fp32.
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[i + 4] = b[i]; }
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = v[i]; b[i] = v[i + 4]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};
template <> struct Vec8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    f32x4 lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) { lo[i] = v[i]; hi[i] = v[i + 4]; }
    bf16x4 a = __builtin_convertvector(lo, bf16x4);
    bf16x4 b = __builtin_convertvector(hi, bf16x4);
    bf16x8 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) { r[i] = a[i]; r[i + 4] = b[i]; }
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};
template <> struct Vec8<fp16> {
  __device__ __forceinline__ static void load(const fp16* p, float (&v)[8]) {
    fp16x8 a = *reinterpret_cast<const fp16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  __device__ __forceinline__ static void store(fp16* p, const float (&v)[8]) {
    fp16x8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (fp16)v[i];
    *reinterpret_cast<fp16x8*>(p) = r;
  }
};

template <typename T> __device__ __forceinline__ float to_f32(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// ---------------------------------------------------------------- wave64 / block reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Block sum for up to 1024 threads. `red` must hold >= blockDim/64 floats. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}

// ---------------------------------------------------------------- launch helpers
#define DS_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

static inline int ds_grid_for(int64_t work_items, int block, int max_blocks = 256 * 8) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

// XCD-aware bijective remap of a linear workgroup id (guide §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD under round-robin dispatch, so give each XCD a contiguous chunk of tiles.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
