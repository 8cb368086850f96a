// Fused softmax cross-entropy over the vocabulary (LM loss), CDNA4.
//
// The reference has no fused LM loss (users call torch CE on materialised fp32 logits). On MI355X the logits
// tensor of a 7B model step is [tokens, 32000] — ~1 GB in bf16 — so the loss must stay one read for forward and
// one read + one write for backward:
//   fwd: one block per row, online max/sum-exp in one pass (16 B loads), loss = lse - x[label], lse saved.
//   bwd: dlogits = (exp(x - lse) - onehot(label)) * dloss[row], written IN PLACE over the logits when requested
//        (the logits are dead after the loss), so no second vocab-sized buffer is allocated.
#include "../include/ds_hip.h"

namespace {

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse_out,
                                                       int64_t rows, int V, int64_t ld, int ignore_index,
                                                       float smoothing) {
  __shared__ float sm_m[4], sm_s[4], sm_x[4];
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const T* x = logits + row * ld;
  float m = -INFINITY, s = 0.f, sumx = 0.f;
  const bool vec = (V % 8 == 0) && ((((uintptr_t)x) & 15) == 0);
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      Vec8<T>::load(x + c, v);
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { ls += __expf(v[j] - lm); sumx += v[j]; }
      online_merge(m, s, lm, ls);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float v = (float)x[c];
      online_merge(m, s, v, 1.f);
      sumx += v;
    }
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
    sumx += __shfl_xor(sumx, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm_m[wid] = m; sm_s[wid] = s; sm_x[wid] = sumx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm_m[0], Ssum = sm_s[0], X = sm_x[0];
    for (int i = 1; i < 4; ++i) { online_merge(M, Ssum, sm_m[i], sm_s[i]); X += sm_x[i]; }
    const float lse = M + __logf(Ssum);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    if (lab == ignore_index || lab < 0 || lab >= V) {
      loss[row] = 0.f;
    } else {
      const float nll = lse - (float)x[lab];
      loss[row] = smoothing > 0.f ? (1.f - smoothing) * nll + smoothing * (lse - X / V) : nll;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss,
                                                       float dloss_scalar, T* __restrict__ dlogits, int64_t rows,
                                                       int V, int64_t ld, int64_t ldo, int ignore_index,
                                                       float smoothing) {
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const T* x = logits + row * ld;
  T* dx = dlogits + row * ldo;
  const int64_t lab = labels[row];
  const bool ignored = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ignored ? 0.f : (dloss ? dloss[row] : dloss_scalar);
  const float L = lse[row];
  const float sm_off = smoothing / V;
  const bool vec = (V % 8 == 0) && ((((uintptr_t)x) & 15) == 0) && ((((uintptr_t)dx) & 15) == 0);
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      Vec8<T>::load(x + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __expf(v[j] - L);
        const float tgt = (c + j == lab ? (1.f - smoothing) : 0.f) + sm_off;
        v[j] = (p - tgt) * g;
      }
      Vec8<T>::store(dx + c, v);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float p = __expf((float)x[c] - L);
      const float tgt = (c == lab ? (1.f - smoothing) : 0.f) + sm_off;
      dx[c] = (T)((p - tgt) * g);
    }
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                    \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)

extern "C" int ds_xent_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int64_t rows, int V,
                           int64_t ld, int ignore_index, float smoothing, int dtype, hipStream_t s) {
  if (rows <= 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL((xent_fwd_kernel<T>), dim3((unsigned)rows), dim3(256), 0, s, (const T*)logits,
                                       labels, loss, lse, rows, V, ld, ignore_index, smoothing));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_xent_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                           float dloss_scalar, void* dlogits, int64_t rows, int V, int64_t ld, int64_t ldo,
                           int ignore_index, float smoothing, int dtype, hipStream_t s) {
  if (rows <= 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL((xent_bwd_kernel<T>), dim3((unsigned)rows), dim3(256), 0, s, (const T*)logits,
                                       labels, lse, dloss, dloss_scalar, (T*)dlogits, rows, V, ld, ldo, ignore_index,
                                       smoothing));
  DS_CHECK_LAUNCH();
  return 0;
}
