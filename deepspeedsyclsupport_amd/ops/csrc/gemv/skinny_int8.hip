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
// That VALU path costs M FMAs per weight byte, so from 4 token rows on the MFMA variant below takes over:
//  * one workgroup = one 16-row slab of W; its 4 waves split K into quarters; per 64-element K chunk each lane
//    loads 16 int8 of one row (16 B), turns them into u = q + 128 (sign-bit flip, one v_cvt_f32_ubyte per element,
//    exact in bf16) and feeds two v_mfma_f32_16x16x32_bf16 with A = u (rows = output features) and B = X^T (cols =
//    tokens, zero beyond M); two more MFMAs against ones give sum_k x_k, so W.x = s * (u.x - 128 sum x) is applied
//    per chunk to the accumulator with the row's group scale (no per-element multiply). Both operands use the same
//    k permutation (lane group g holds k = 16g + j, then 16g + 8 + j), which a sum over k does not see. MFMA
//    throughput is far above the weight stream, so the cost per byte no longer depends on M (<= 16); the four
//    quarter sums meet in LDS. Measured ~3 TB/s flat in M (VALU path: 6.1-6.4 TB/s at one row): the lane->row
//    mapping the MFMA operand dictates gives 64-B row segments per load instruction, which the HBM stream
//    pays for; staging whole 1-KB row pieces through LDS is the next step.
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

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int MF_UNR = 8;  // 64-element chunks in flight per lane

__global__ void __launch_bounds__(256) skinny_i8_mfma_kernel(const bf16* __restrict__ X, const int8_t* __restrict__ Q,
                                                             const float* __restrict__ S,
                                                             const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                             int M, int N, int K, int gs) {
  __shared__ float red[4][16][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int n0 = blockIdx.x * 16;
  const int n = min(n0 + l16, N - 1);       // A row of this lane (clamped; rows >= N are never stored)
  const int m = l16;                         // B column (token) of this lane
  const bool xvalid = m < M;
  const int nchunks = K / 64;
  const int ngroups = K / gs;
  const int per = (nchunks + 3) / 4;
  const int c0 = wid * per, c1 = min(c0 + per, nchunks);
  const int8_t* qrow = Q + (int64_t)n * K + 16 * g;
  const bf16* xrow = X + (int64_t)(xvalid ? m : 0) * K + 16 * g;
  // accumulator rows of this lane are output features 4g + i; their group scales
  const float* srows[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) srows[i] = S + (int64_t)min(n0 + 4 * g + i, N - 1) * ngroups;
  bf16x8_t ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  for (int c = c0; c < c1; c += MF_UNR) {
    // issue every load of the batch (weights, scales AND the X operand) before any math, so HBM and L2 latency
    // overlap instead of serialising behind each chunk's MFMAs
    i32x4 w[MF_UNR];
    float sc[MF_UNR][4];
    bf16x8_t b[MF_UNR][2];
#pragma unroll
    for (int u = 0; u < MF_UNR; ++u) {
      const int cc = c + u;
      const bool live = cc < c1;
      w[u] = live ? __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(qrow + (int64_t)cc * 64))
                  : i32x4{0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[u][i] = live ? srows[i][(cc * 64) / gs] : 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (xvalid && live) {
          b[u][h] = *reinterpret_cast<const bf16x8_t*>(xrow + (int64_t)cc * 64 + 8 * h);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) b[u][h][j] = (__bf16)0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < MF_UNR; ++u) {
      if (c + u >= c1) break;
      // q (int8) -> u = q + 128 (unsigned byte, exact in bf16) by flipping the sign bits; the -128 offset is
      // applied to the product afterwards via sum_k x_k (an extra MFMA against ones)
      bf16x8_t a[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned lo = (unsigned)w[u][2 * h] ^ 0x80808080u, hi = (unsigned)w[u][2 * h + 1] ^ 0x80808080u;
        f32x4 flo, fhi;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          flo[j] = (float)((lo >> (8 * j)) & 0xffu);
          fhi[j] = (float)((hi >> (8 * j)) & 0xffu);
        }
        const bf16x4 blo = __builtin_convertvector(flo, bf16x4), bhi = __builtin_convertvector(fhi, bf16x4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[h][j] = blo[j]; a[h][4 + j] = bhi[j]; }
      }
      f32x4 pu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[u][0], zero4, 0, 0, 0);
      pu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[u][1], pu, 0, 0, 0);
      f32x4 px = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, b[u][0], zero4, 0, 0, 0);
      px = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, b[u][1], px, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(sc[u][i], fmaf(-128.f, px[i], pu[i]), acc[i]);
    }
  }
  // C: col = token (lane & 15), rows = output features 4g + i
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wid][4 * g + i][l16] = acc[i];
  __syncthreads();
  const int row = tid >> 4, tok = tid & 15;
  if (tok < M && n0 + row < N) {
    const float v = red[0][row][tok] + red[1][row][tok] + red[2][row][tok] + red[3][row][tok];
    Y[(int64_t)tok * N + n0 + row] = (bf16)(v + (bias ? (float)bias[n0 + row] : 0.f));
  }
}

}  // namespace

extern "C" int ds_skinny_i8_mfma_ok(int M, int K, int gs) {
  return M >= 1 && M <= 16 && K % 64 == 0 && gs % 64 == 0 && K % gs == 0;
}

// same contract as ds_skinny_i8 for M <= 16 token rows (K % 64 == 0, group size a multiple of 64)
extern "C" int ds_skinny_i8_mfma(const void* X, const int8_t* Q, const float* S, const void* bias, void* Y, int M,
                                 int N, int K, int gs, hipStream_t st) {
  if (!ds_skinny_i8_mfma_ok(M, K, gs) || N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(skinny_i8_mfma_kernel, dim3((N + 15) / 16), dim3(256), 0, st, (const bf16*)X, Q, S,
                     (const bf16*)bias, (bf16*)Y, M, N, K, gs);
  DS_CHECK_LAUNCH();
  return 0;
}

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
