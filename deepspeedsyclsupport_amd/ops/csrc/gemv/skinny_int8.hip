// Weight-only int8 skinny GEMM for decode: y[M, N] = X[M, K] . (Q[N, K] * s[N, K / gs])^T (+ bias), M <= 8.
//
// Reference counterparts (behaviour, not code): the weight-only int8 inference path of `transformer_inference`
// (`ds_vector_matmul_int8` / `dequantize_kernel`, `csrc/transformer/inference/csrc/pt_binding.cpp:13xx`,
// `dequantize.cu:15-86`) and v2's `mixed_gemm` (CUTLASS, prebuilt) — both materialise or stream-dequantise the
// weight and run a library GEMM.
//
// MI355X design: decode GEMMs are pure weight streams, so int8 weights halve the HBM bytes of a bf16 decode step.
// The dequantisation is fused into the stream: no bf16 copy of the weight is ever written.
//  * each wave owns 4 consecutive output rows at a time (grid-stride over row quads), each lane a 16-element K chunk
//    per row per step: one 16-byte non-temporal load per row; the group scale of that chunk (groups of >= 16
//    elements along K, the quantiser's layout) is one fp32 load;
//  * UNR chunks are issued before any is consumed (4 rows x UNR x 16 B in flight per lane) to cover HBM latency;
//  * X (M <= 8 rows) is staged once per workgroup into LDS as bf16 when it fits (<= 64 KB), else read through L2;
//  * int8 -> f32 by byte extract + convert, fp32 FMA, one wave reduction per (row, token) at the end.
#include "ds_hip.h"

namespace {

constexpr int ROWS = 4;        // output rows per wave
constexpr int UNR = 4;         // K chunks in flight per lane
constexpr int XLDS_LIMIT = 64 * 1024;

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void x16(const bf16* p, float (&x)[16]) {
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
  const bf16x8 b = *reinterpret_cast<const bf16x8*>(p + 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = (float)a[j]; x[j + 8] = (float)b[j]; }
}

template <int MM>
__global__ void __launch_bounds__(256) skinny_i8_kernel(const bf16* __restrict__ X, const int8_t* __restrict__ Q,
                                                        const float* __restrict__ S, const bf16* __restrict__ bias,
                                                        bf16* __restrict__ Y, int N, int K, int gs, int xlds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (xlds) {
    const int nvec = MM * K / 8;
    for (int i = tid; i < nvec; i += 256)
      reinterpret_cast<bf16x8*>(xs)[i] = reinterpret_cast<const bf16x8*>(X)[i];
    __syncthreads();
  }
  const bf16* Xp = xlds ? xs : X;
  const int ngroups = K / gs;
  const int nwaves = gridDim.x * 4;
  for (int n0 = (blockIdx.x * 4 + wid) * ROWS; n0 < N; n0 += nwaves * ROWS) {
    float acc[MM][ROWS];
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int r = 0; r < ROWS; ++r) acc[m][r] = 0.f;
    for (int kb = lane * 16; kb < K; kb += 64 * 16 * UNR) {
      i32x4 w[UNR][ROWS];
      float sc[UNR][ROWS];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int k = kb + u * 64 * 16;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          const int n = n0 + r;
          if (k < K && n < N) {
            w[u][r] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(Q + (int64_t)n * K + k));
            sc[u][r] = S[(int64_t)n * ngroups + k / gs];
          } else {
            w[u][r] = i32x4{0, 0, 0, 0};
            sc[u][r] = 0.f;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int k = kb + u * 64 * 16;
        if (k >= K) break;
        float x[MM][16];
#pragma unroll
        for (int m = 0; m < MM; ++m) x16(Xp + (int64_t)m * K + k, x[m]);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          float part[MM];
#pragma unroll
          for (int m = 0; m < MM; ++m) part[m] = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int word = w[u][r][c];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const float wv = (float)(int8_t)((word >> (8 * b)) & 0xff);
#pragma unroll
              for (int m = 0; m < MM; ++m) part[m] = fmaf(wv, x[m][4 * c + b], part[m]);
            }
          }
#pragma unroll
          for (int m = 0; m < MM; ++m) acc[m][r] = fmaf(part[m], sc[u][r], acc[m][r]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        const float v = wave_sum(acc[m][r]);
        const int n = n0 + r;
        if (lane == 0 && n < N) Y[(int64_t)m * N + n] = (bf16)(v + (bias ? (float)bias[n] : 0.f));
      }
  }
}

}  // namespace

extern "C" int ds_skinny_i8_ok(int M, int K, int gs) {
  return M >= 1 && M <= 8 && K % 16 == 0 && gs >= 16 && gs % 16 == 0 && K % gs == 0;
}

// X [M, K] bf16, Q int8 [N, K] row-major, S fp32 [N * K / gs], bias bf16 [N] or null -> Y [M, N] bf16
extern "C" int ds_skinny_i8(const void* X, const int8_t* Q, const float* S, const void* bias, void* Y, int M, int N,
                            int K, int gs, hipStream_t st) {
  if (!ds_skinny_i8_ok(M, K, gs) || N <= 0) return (int)hipErrorInvalidValue;
  const int xbytes = M * K * 2;
  const int xlds = xbytes <= XLDS_LIMIT ? 1 : 0;
  const int shm = xlds ? xbytes : 0;
  const int quads = (N + ROWS - 1) / ROWS;
  const int grid = min((quads + 3) / 4, 256 * 8);
  static bool attr = false;
  if (!attr) {
    const void* ks[8] = {reinterpret_cast<const void*>(&skinny_i8_kernel<1>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<2>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<3>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<4>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<5>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<6>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<7>),
                         reinterpret_cast<const void*>(&skinny_i8_kernel<8>)};
    for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, XLDS_LIMIT);
    attr = true;
  }
  auto xb = (const bf16*)X;
  auto bb = (const bf16*)bias;
  auto yb = (bf16*)Y;
#define DS_I8_CASE(MMV)                                                                                      \
  case MMV:                                                                                                  \
    hipLaunchKernelGGL(skinny_i8_kernel<MMV>, dim3(grid), dim3(256), shm, st, xb, Q, S, bb, yb, N, K, gs, xlds); \
    break;
  switch (M) {
    DS_I8_CASE(1) DS_I8_CASE(2) DS_I8_CASE(3) DS_I8_CASE(4) DS_I8_CASE(5) DS_I8_CASE(6) DS_I8_CASE(7)
    default: hipLaunchKernelGGL(skinny_i8_kernel<8>, dim3(grid), dim3(256), shm, st, xb, Q, S, bb, yb, N, K, gs, xlds);
  }
#undef DS_I8_CASE
  DS_CHECK_LAUNCH();
  return 0;
}
