// MFMA skinny GEMM for decode batches of 1..16 token rows: y[M, N] = X[M, K] . W[N, K]^T.
//
// Same weight-streaming job as the VALU kernel in skinny_gemm.hip, but the dot products run on the matrix cores
// (v_mfma_f32_16x16x32_bf16) so the kernel stays HBM-bound up to M = 16 (the VALU version becomes FMA-bound around
// M = 8). Layout (gfx950 16x16x32 operands): lane l holds A[row l&15][8 k-slots of group l>>4] and
// B[same k-slots][col l&15]; C lane l holds rows 4*(l>>4)+r, column l&15.
//   A = 16 weight rows  -> loaded straight from HBM in the operand layout (no LDS), 16-byte non-temporal loads;
//                          k-slots are permuted so each lane reads 32 contiguous bytes per MFMA pair and every row
//                          is fetched in whole 128-byte lines;
//   B = X^T (token rows)-> from LDS when the input is RMS-normalised in-kernel (IN 1), else straight from L2;
//   split-K across the 8 waves of a workgroup, partial 16x16 tiles reduced through LDS.
// One workgroup owns 16 output rows (GATED: 16 gate rows + the matching 16 up rows, writes act(gate) * up).
#include "ds_hip.h"

namespace {

constexpr int NW = 8;            // waves per workgroup (split-K)
constexpr int GRP = 8;           // MFMA steps per load group (all loads of a group in flight together)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_f(float g, int act) {
  switch (act) {
    case 0: return g / (1.f + __expf(-g));
    case 1: return 0.5f * g * (1.f + tanhf(0.7978845608f * (g + 0.044715f * g * g * g)));
    case 2: return 0.5f * g * (1.f + erff(g * 0.70710678f));
    case 3: return fmaxf(g, 0.f);
    default: return g;
  }
}

// k offset (within a K-slice) of MFMA step s for lane-group q = lane >> 4: steps come in pairs sharing one 32-byte
// contiguous run per lane (pair i covers k in [64 i, 64 i + 64), group q owns [64 i + 16 q, 64 i + 16 q + 16)).
// A trailing unpaired step (odd step count, e.g. K-slice 1376 = 43 x 32) uses the plain [32 s + 8 q, +8) slots so
// it never leaves the slice.
__device__ __forceinline__ int kofs(int s, int q, int paired) {
  return s < paired ? (s >> 1) * 64 + q * 16 + (s & 1) * 8 : s * 32 + q * 8;
}

template <int T, int IN, bool GATED>
__global__ void __launch_bounds__(NW * 64) skinny_mfma_kernel(
    const bf16* __restrict__ W, const bf16* __restrict__ x, const bf16* __restrict__ r, const bf16* __restrict__ nw,
    const bf16* __restrict__ bias, const bf16* __restrict__ add, bf16* __restrict__ y, bf16* __restrict__ res_out,
    int M, int N, int K, float eps, int act) {
  extern __shared__ __attribute__((aligned(16))) bf16 xs[];   // IN 1: [M][K + 8] normalised activations
  __shared__ float part[NW][T][64][4];                       // split-K partial tiles
  __shared__ float red[NW][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4, col = lane & 15;
  const int KP = K + 8;
  const int Nout = GATED ? N / 2 : N;
  const int n0 = blockIdx.x * 16;
  const int Ks = K / NW, kw = wid * Ks, steps = Ks / 32, paired = steps & ~1;

  // weight rows of this lane for each tile (clamped: rows past the end are loaded but never written)
  const bf16* wrow[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    int n = n0 + col;
    if (n >= Nout) n = Nout - 1;
    if (GATED && t == 1) n += Nout;
    wrow[t] = W + (int64_t)n * K + kw;
  }

  // ------------------------------------------------------------ stage normalised X in LDS (IN 1)
  if (IN == 1) {
    for (int m = 0; m < M; ++m) {
      float ss = 0.f;
      for (int c = tid * 8; c < K; c += NW * 512) {
        float v[8], o[8];
        Vec8<bf16>::load(x + (int64_t)m * K + c, v);
        if (r) {
          Vec8<bf16>::load(r + (int64_t)m * K + c, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (float)(bf16)(v[j] + o[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss = fmaf(v[j], v[j], ss);
      }
      ss = wave_sum(ss);
      if (lane == 0) red[wid][m] = ss;
    }
    __syncthreads();
    for (int m = 0; m < M; ++m) {
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) tot += red[w][m];
      const float rs = rsqrtf(tot / K + eps);
      for (int c = tid * 8; c < K; c += NW * 512) {
        float v[8], o[8], g[8];
        Vec8<bf16>::load(x + (int64_t)m * K + c, v);
        if (r) {
          Vec8<bf16>::load(r + (int64_t)m * K + c, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (float)(bf16)(v[j] + o[j]);
        }
        if (res_out && blockIdx.x == 0) Vec8<bf16>::store(res_out + (int64_t)m * K + c, v);
        Vec8<bf16>::load(nw + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (float)(bf16)(v[j] * rs) * g[j];
        Vec8<bf16>::store(xs + (int64_t)m * KP + c, v);
      }
    }
    __syncthreads();
  }

  // ------------------------------------------------------------ split-K MFMA stream
  f4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const bool live = col < M;  // B column = token row
  const bf16* xb = IN == 1 ? xs + (int64_t)col * KP + kw : x + (int64_t)col * K + kw;
  for (int s0 = 0; s0 < steps; s0 += GRP) {
    bf16x8_t a[T][GRP], b[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      if (s0 + i < steps) {
        const int ko = kofs(s0 + i, q, paired);
#pragma unroll
        for (int t = 0; t < T; ++t)
          a[t][i] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(wrow[t] + ko));
        if (live) {
          b[i] = *reinterpret_cast<const bf16x8_t*>(xb + ko);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) b[i][j] = (bf16)0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      if (s0 + i < steps) {
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][i], b[i], acc[t], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[wid][t][lane][j] = acc[t][j];
  __syncthreads();

  // ------------------------------------------------------------ reduce the NW partial tiles + epilogue
  for (int e = tid; e < 64 * 4; e += NW * 64) {
    const int l = e >> 2, j = e & 3;
    const int n = n0 + (l >> 4) * 4 + j, m = l & 15;
    if (m >= M || n >= Nout) continue;
    float v[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float sacc = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sacc += part[w][t][l][j];
      v[t] = sacc;
    }
    float o;
    if (GATED) {
      const float g = (float)(bf16)(v[0] + (bias ? (float)bias[n] : 0.f));
      const float u = (float)(bf16)(v[1] + (bias ? (float)bias[Nout + n] : 0.f));
      o = act_f(g, act) * u;
    } else {
      o = v[0] + (bias ? (float)bias[n] : 0.f);
    }
    if (add) o += (float)add[(int64_t)m * Nout + n];
    y[(int64_t)m * Nout + n] = (bf16)o;
  }
}

template <int T, int IN, bool G>
int launch(const bf16* W, const bf16* x, const bf16* r, const bf16* nw, const bf16* bias, const bf16* add, bf16* y,
           bf16* res_out, int M, int N, int K, float eps, int act, hipStream_t s) {
  const int Nout = G ? N / 2 : N;
  const int grid = (Nout + 15) / 16;
  const size_t lds = IN == 1 ? (size_t)M * (K + 8) * sizeof(bf16) : 0;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_mfma_kernel<T, IN, G>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL((skinny_mfma_kernel<T, IN, G>), dim3(grid), dim3(NW * 64), lds, s, W, x, r, nw, bias, add, y,
                     res_out, M, N, K, eps, act);
  DS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// LDS the IN 1 staging needs (bytes); the caller falls back to a separate RMSNorm above the budget.
extern "C" int ds_skinny_mfma_ok(int M, int K, int in_mode) {
  if (M < 1 || M > 16 || K % (NW * 32) != 0) return 0;
  if (in_mode == 1 && (int64_t)M * (K + 8) * 2 > 140 * 1024) return 0;  // + 16 KB split-K tiles <= 160 KB
  return 1;
}

extern "C" int ds_skinny_mfma(const void* W, const void* x, const void* r, const void* nw, const void* bias,
                              const void* add, void* y, void* res_out, int M, int N, int K, int in_mode, int gated,
                              int act, float eps, hipStream_t s) {
  if (!ds_skinny_mfma_ok(M, K, in_mode) || (gated && N % 2)) return (int)hipErrorInvalidValue;
  auto W_ = (const bf16*)W;
  auto x_ = (const bf16*)x;
  auto r_ = (const bf16*)r;
  auto nw_ = (const bf16*)nw;
  auto b_ = (const bf16*)bias;
  auto a_ = (const bf16*)add;
  auto y_ = (bf16*)y;
  auto ro_ = (bf16*)res_out;
  if (in_mode == 1) {
    if (gated) return launch<2, 1, true>(W_, x_, r_, nw_, b_, a_, y_, ro_, M, N, K, eps, act, s);
    return launch<1, 1, false>(W_, x_, r_, nw_, b_, a_, y_, ro_, M, N, K, eps, act, s);
  }
  if (gated) return launch<2, 0, true>(W_, x_, r_, nw_, b_, a_, y_, ro_, M, N, K, eps, act, s);
  return launch<1, 0, false>(W_, x_, r_, nw_, b_, a_, y_, ro_, M, N, K, eps, act, s);
}
