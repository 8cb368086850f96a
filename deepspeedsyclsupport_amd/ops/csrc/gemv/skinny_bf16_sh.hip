// bf16 skinny GEMM for decode over a PRE-SHUFFLED weight: y[M, N] = X[M, K] . W[N, K]^T (+ bias), M <= 16.
//
// Reference counterpart (behaviour): the bf16 / fp16 decode GEMMs of `transformer_inference` (`qkv_gemm`,
// `vector_matmul`, `mlp_gemm`; `csrc/transformer/inference/csrc/pt_binding.cpp`), which call the vendor GEMM on the
// row-major weight.
//
// MI355X design: a decode GEMM is a weight stream and the HBM stream only runs at full rate when every load
// instruction covers long contiguous segments. Read from a row-major matrix, the MFMA operand layout is 16 rows x
// 64 B per instruction, which measured 4.4 - 5.0 TB/s loads-only (`profiles/int8_load_patterns_r2.jsonl`), and the
// row-major bf16 kernels of this directory run at 3 - 4.2 TB/s end to end. Inference weights are constants, so —
// exactly like the int8 / int4 streams — the matrix is re-laid ONCE into operand order:
//   Wsh[nb][kq][h][lane][8] = W[16 nb + (lane & 15)][64 kq + 16 (lane >> 4) + 8 h + 0..7]    (2 KB per 16 x 64 tile)
// so each 16-byte-per-lane load reads 1 KB contiguous and IS the B operand of one v_mfma_f32_16x16x32_bf16 (X is
// loaded with the same k permutation). The kernel is the int8 stream (skinny_int8.hip) minus the dequantisation:
// a wave owns FB row blocks and walks a contiguous range of the (block group, k quarter) sequence with P quarters
// in flight in registers; ranges may start / end inside a block group (split-K without a fixed factor); partial
// sums go to the fp32 workspace shared with the int8 / int4 streams by f32 atomics, and the same finalize kernels
// (skinny_finalize.hip: plain, + residual + RMSNorm, gated activation) convert and re-zero it.
// Prefill (more than 16 token rows) un-shuffles into a row-major temporary for the library GEMM (`ds_unshuffle_sh16`),
// or uses the row-major copy the caller kept.
#include "ds_hip.h"

#include <algorithm>

extern "C" int ds_skinny_finalize_plain(float* ws, const void* bias, void* y, int M, int N, int NP, hipStream_t st);

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

struct B16Args {
  const bf16* x;
  const bf16* w;  // shuffled
  float* acc;     // [16, NP] fp32 workspace, zero between calls
  int M, N, K, NB, KQ, NBG;
  int NP;         // workspace row length: NBG * FB * 16
  int64_t total;  // NBG * KQ
};

template <int FB>
struct B16Stage {
  bf16x8_t w0[FB], w1[FB];
  bf16x8_t x0, x1;
};

template <int FB, int P>
__global__ void __launch_bounds__(256) skinny_b16_mfma_kernel(B16Args a) {
  const int lane = threadIdx.x & 63;
  // wave-uniform bookkeeping lives in SGPRs (readfirstlane): scalar branches keep the vmcnt counts static
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  const int lo = (int)(a.total * gw / nw), hi = (int)(a.total * (gw + 1) / nw);
  if (lo >= hi) return;
  const int r = lane & 15, g = lane >> 4;

  // issue cursor: wave-uniform offsets advanced per quarter; block offsets recomputed only when entering a group
  int ibg = 0, ikq = 0;
  bool hold = false;
  int64_t iw = 0, ix = 0, fw[FB];
  const int64_t xlane = (int64_t)min(r, a.M - 1) * a.K + 16 * g;  // token rows >= M re-read row M - 1
  auto enter = [&](int bgv, int kqv) {
    if (bgv >= a.NBG) {  // past the end of the range: keep re-loading the last quarter (static vmcnt)
      bgv = a.NBG - 1;
      kqv = a.KQ - 1;
      hold = true;
    }
    ibg = bgv;
    ikq = kqv;
#pragma unroll
    for (int f = 0; f < FB; ++f) fw[f] = (int64_t)min(bgv * FB + f, a.NB - 1) * a.KQ * 1024;  // (elements)
    iw = (int64_t)kqv * 1024;
    ix = (int64_t)kqv * 64;
  };
  auto advance = [&]() {
    if (hold) return;
    if (++ikq == a.KQ) {
      enter(ibg + 1, 0);
      return;
    }
    iw += 1024;
    ix += 64;
  };
  auto load = [&](B16Stage<FB>& st) {
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const bf16* p = a.w + fw[f] + iw + lane * 8;
      st.w0[f] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(p));
      st.w1[f] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(p + 512));
    }
    const bf16* xp = a.x + xlane + ix;
    st.x0 = *reinterpret_cast<const bf16x8_t*>(xp);
    st.x1 = *reinterpret_cast<const bf16x8_t*>(xp + 8);
  };

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[FB];
#pragma unroll
  for (int f = 0; f < FB; ++f) acc[f] = zero4;

  int bg = lo / a.KQ, kq = lo - bg * a.KQ;
  enter(bg, kq);
  B16Stage<FB> st[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {  // same issue order as the steady state
    load(st[p]);
    advance();
    __builtin_amdgcn_sched_barrier(0);
  }
  // partial sums of block group `grp` -> fp32 workspace (padded to whole groups; features >= N are never read)
  auto spill = [&](int grp) {
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const int n = (grp * FB + f) * 16 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < a.M) unsafeAtomicAdd(a.acc + (int64_t)(4 * g + i) * a.NP + n, acc[f][i]);
      acc[f] = zero4;
    }
  };
  // Straight-line steady state: every reload follows the compute that frees its registers; steps past the range end
  // re-load the last quarter and skip the (wave-uniform) MFMA block.
  for (int base = lo; base < hi; base += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool live = base + p < hi;
      if (live) {
#pragma unroll
        for (int f = 0; f < FB; ++f) {
          acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x0, st[p].w0[f], acc[f], 0, 0, 0);
          acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x1, st[p].w1[f], acc[f], 0, 0, 0);
        }
        if (kq == a.KQ - 1) spill(bg);
      }
      if (++kq == a.KQ) { kq = 0; ++bg; }
      __builtin_amdgcn_sched_barrier(0);
      load(st[p]);
      advance();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if ((hi % a.KQ) != 0) spill((hi - 1) / a.KQ);  // the range ends inside a group
}

// Pre-shuffled bf16 -> row-major bf16 [N, K]. One thread per 16-byte lane chunk (8 weights of one row).
__global__ void __launch_bounds__(256) unshuffle_sh16_kernel(const bf16* __restrict__ Wsh, bf16* __restrict__ W, int N,
                                                             int KQ) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk = ((nb * KQ + kq) * 2 + h) * 64 + lane
  const int lane = (int)(c & 63);
  const int h = (int)((c >> 6) & 1);
  const int64_t t = c >> 7;
  const int kq = (int)(t % KQ);
  const int64_t nb = t / KQ;
  const int64_t row = nb * 16 + (lane & 15);
  if (row >= N) return;
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(Wsh + c * 8);
  *reinterpret_cast<bf16x8*>(W + row * KQ * 64 + kq * 64 + 16 * (lane >> 4) + 8 * h) = v;
}

int g_b16_cfg = 0, g_b16_wpc = 0;

}  // namespace

extern "C" void ds_skinny_b16_tune(int cfg, int wpc) {
  g_b16_cfg = cfg;
  g_b16_wpc = wpc;
}

extern "C" int ds_skinny_b16_mfma_ok(int M, int K) { return M >= 1 && M <= 16 && K % 64 == 0; }

extern "C" int ds_unshuffle_sh16(const void* Wsh, void* W, int N, int K, hipStream_t st) {
  if (N <= 0 || K % 64) return (int)hipErrorInvalidValue;
  const int KQ = K / 64, NB = (N + 15) / 16;
  const int64_t chunks = (int64_t)NB * KQ * 128;
  hipLaunchKernelGGL(unshuffle_sh16_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st,
                     (const bf16*)Wsh, (bf16*)W, N, KQ);
  DS_CHECK_LAUNCH();
  return 0;
}

// X [M, K] bf16 (M <= 16), Wsh in the shuffled layout above (N padded to a multiple of 16), bias bf16 [N] or null
// -> Y [M, N] bf16 (Y == null: leave the sums in the workspace, row length ws_floats / 16, un-finalized). The
// workspace is the int8 stream's: fp32 [16 x N padded to whole groups of 4 row blocks], zero between calls.
extern "C" int ds_skinny_b16_mfma(const void* X, const void* Wsh, const void* bias, void* Y, float* ws, int M, int N,
                                  int K, hipStream_t st) {
  if (!ds_skinny_b16_mfma_ok(M, K) || N <= 0) return (int)hipErrorInvalidValue;
  B16Args a;
  a.x = (const bf16*)X;
  a.w = (const bf16*)Wsh;
  a.acc = ws;
  a.M = M;
  a.N = N;
  a.K = K;
  a.NB = (N + 15) / 16;
  a.KQ = K / 64;
  auto go = [&](auto kern, int P, int FB, int wpc) {
    // one resident round of waves (wpc per CU, from the VGPR budget), each with the same number of quarters
    const int nbg = (a.NB + FB - 1) / FB;
    a.NBG = nbg;
    a.NP = ((a.NB + 3) / 4) * 64;  // the shared workspace row length (whole groups of 4 row blocks)
    a.total = (int64_t)nbg * a.KQ;
    const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(a.total / (2 * P), 256 * wpc));
    hipLaunchKernelGGL(kern, dim3((int)((waves + 3) / 4)), dim3(256), 0, st, a);
  };
  int cfg = g_b16_cfg ? g_b16_cfg : 1;
  const int wpc = g_b16_wpc;
  switch (cfg) {
    case 2: go(skinny_b16_mfma_kernel<4, 2>, 2, 4, wpc ? wpc : 8); break;
    case 3: go(skinny_b16_mfma_kernel<2, 3>, 3, 2, wpc ? wpc : 12); break;
    case 4: go(skinny_b16_mfma_kernel<4, 1>, 1, 4, wpc ? wpc : 12); break;
    default: go(skinny_b16_mfma_kernel<2, 2>, 2, 2, wpc ? wpc : 8);
  }
  DS_CHECK_LAUNCH();
  if (Y == nullptr) return 0;  // sums stay in the workspace for a fused consumer (skinny_finalize.hip)
  return ds_skinny_finalize_plain(ws, bias, Y, M, N, a.NP, st);
}
