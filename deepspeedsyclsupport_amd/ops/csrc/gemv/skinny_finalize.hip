// Consumers of the weight-only decode streams' fp32 split-K workspace (skinny_int8.hip / skinny_int4.hip).
//
// The int8 / int4 MFMA streams add their partial sums into a [16, NP] fp32 workspace and leave "convert to bf16 (+ bias)
// and re-zero" to a second small kernel. At decode sizes every kernel costs 4-5 us of launch / drain latency whatever
// it does, and a Llama layer has four such GEMVs, so the plain finalize pass is ~18 us of a ~90 us layer. The kernels
// here ARE that pass, fused with the element-wise op that consumes the GEMV anyway (reference counterparts of the
// fused ops: `csrc/transformer/inference/csrc/rms_norm.cu` pre_rms_norm, `gelu.cu` fused_gate_activation):
//  * finalize + bias + residual add + RMSNorm  (attention-output and MLP-down projections feed the next norm);
//  * finalize + bias + gated activation        (the fused gate/up projection feeds act(gate) * up).
// Each re-zeroes the workspace rows it read (all NP padded columns), keeping the streams' contract: the workspace is
// zero between calls, without a memset (capturable in a HIP graph).
#include "ds_hip.h"

namespace {

enum Act : int { ACT_SILU = 0, ACT_GELU_TANH = 1, ACT_GELU_ERF = 2, ACT_RELU = 3, ACT_IDENTITY = 4 };

__device__ __forceinline__ float act_any(int a, float x) {
  switch (a) {
    case ACT_SILU: return x / (1.f + __expf(-x));
    case ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
    }
    case ACT_GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
    case ACT_RELU: return fmaxf(x, 0.f);
    default: return x;
  }
}

// One block per token row. v = acc + bias + residual -> res_out; y = v * rsqrt(mean(v^2) + eps) * w.
// Elements are kept in registers between the two phases (EPT per thread, N <= 1024 * EPT).
template <int EPT>
__global__ void __launch_bounds__(1024) finalize_rms_kernel(float* __restrict__ acc, const bf16* __restrict__ bias,
                                                            const bf16* __restrict__ residual,
                                                            const bf16* __restrict__ w, bf16* __restrict__ y,
                                                            bf16* __restrict__ res_out, int N, int NP, float eps) {
  __shared__ float red[16];
  const int t = blockIdx.x, tid = threadIdx.x, nthr = blockDim.x;
  float* arow = acc + (int64_t)t * NP;
  float v[EPT];
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int n = tid + e * nthr;
    float x = 0.f;
    if (n < NP) {
      x = arow[n];
      arow[n] = 0.f;
    }
    if (n < N) {
      x += (bias ? (float)bias[n] : 0.f) + (residual ? (float)residual[(int64_t)t * N + n] : 0.f);
      // the norm sees the residual stream as it is stored (bf16), like the unfused rms kernel reading res_out back
      const bf16 xb = (bf16)x;
      if (res_out) res_out[(int64_t)t * N + n] = xb;
      x = (float)xb;
      ss = fmaf(x, x, ss);
    } else {
      x = 0.f;
    }
    v[e] = x;
  }
  ss = block_sum(ss, red);
  const float rs = rsqrtf(ss / N + eps);
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int n = tid + e * nthr;
    if (n < N) y[(int64_t)t * N + n] = (bf16)(v[e] * rs * (float)w[n]);
  }
}

// out[t, i] = act(acc[t, i] + b[i]) * (acc[t, I + i] + b[I + i]),  N = 2 I
__global__ void __launch_bounds__(256) finalize_gated_kernel(float* __restrict__ acc, const bf16* __restrict__ bias,
                                                             bf16* __restrict__ out, int M, int I, int NP, int act) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int half = NP - I;  // columns [I, NP) hold the up half and the padding
  if (e >= (int64_t)M * half) return;
  const int t = (int)(e / half), j = (int)(e % half);
  float* arow = acc + (int64_t)t * NP;
  const float u = arow[I + j];
  arow[I + j] = 0.f;
  if (j < I) {
    const float g = arow[j];
    arow[j] = 0.f;
    const float gb = bias ? (float)bias[j] : 0.f, ub = bias ? (float)bias[I + j] : 0.f;
    out[(int64_t)t * I + j] = (bf16)(act_any(act, g + gb) * (u + ub));
  }
}

// y = bf16(acc + bias), workspace re-zeroed (the streams' own finalize, for callers that ran them unfinalized)
__global__ void __launch_bounds__(256) finalize_plain_kernel(float* __restrict__ acc, const bf16* __restrict__ bias,
                                                             bf16* __restrict__ y, int M, int N, int NP) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * NP) return;
  const int t = (int)(e / NP), n = (int)(e % NP);
  const float v = acc[e];
  acc[e] = 0.f;
  if (n < N) y[(int64_t)t * N + n] = (bf16)(v + (bias ? (float)bias[n] : 0.f));
}

}  // namespace

extern "C" int ds_skinny_finalize_rms(float* ws, const void* bias, const void* residual, const void* w, void* y,
                                      void* res_out, int M, int N, int NP, float eps, hipStream_t st) {
  if (M < 1 || M > 16 || N < 1 || NP < N || NP > 16 * 1024 || w == nullptr) return (int)hipErrorInvalidValue;
  const int nthr = NP <= 2048 ? 256 : (NP <= 8192 ? 512 : 1024);
  const int ept = (NP + nthr - 1) / nthr;
#define DS_FR(E)                                                                                                   \
  hipLaunchKernelGGL((finalize_rms_kernel<E>), dim3(M), dim3(nthr), 0, st, ws, (const bf16*)bias,                  \
                     (const bf16*)residual, (const bf16*)w, (bf16*)y, (bf16*)res_out, N, NP, eps)
  if (ept <= 4) DS_FR(4);
  else if (ept <= 8) DS_FR(8);
  else DS_FR(16);
#undef DS_FR
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_skinny_finalize_gated(float* ws, const void* bias, void* out, int M, int N, int NP, int act,
                                        hipStream_t st) {
  if (M < 1 || M > 16 || N < 2 || N % 2 || NP < N) return (int)hipErrorInvalidValue;
  const int I = N / 2;
  const int64_t total = (int64_t)M * (NP - I);
  hipLaunchKernelGGL(finalize_gated_kernel, dim3((int)((total + 255) / 256)), dim3(256), 0, st, ws, (const bf16*)bias,
                     (bf16*)out, M, I, NP, act);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_skinny_finalize_plain(float* ws, const void* bias, void* y, int M, int N, int NP, hipStream_t st) {
  if (M < 1 || M > 16 || N < 1 || NP < N) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(finalize_plain_kernel, dim3((int)(((int64_t)M * NP + 255) / 256)), dim3(256), 0, st, ws,
                     (const bf16*)bias, (bf16*)y, M, N, NP);
  DS_CHECK_LAUNCH();
  return 0;
}
