// Weight-only int8 skinny GEMM for decode: y[M, N] = X[M, K] . (Q[N, K] * s[N, K / gs])^T (+ bias), M <= 16.
//
// Reference counterparts (behaviour, not code): the weight-only int8 inference path of `transformer_inference`
// (`ds_vector_matmul_int8` / `dequantize_kernel`, `csrc/transformer/inference/csrc/pt_binding.cpp:13xx`,
// `dequantize.cu:15-86`) and v2's `mixed_gemm` (CUTLASS, prebuilt) — both materialise or stream-dequantise the
// weight and run a library GEMM.
//
// MI355X design: decode GEMMs are pure weight streams, so int8 weights halve the HBM bytes of a bf16 decode step.
// The dequantisation is fused into the stream: no bf16 copy of the weight is ever written. Two kernels:
//  * VALU stream over a ROW-MAJOR weight (<= 8 rows; kept for callers holding the quantiser's layout): each wave owns
//    4 consecutive output rows at a time, each lane a 16-element K chunk per row per step (one 16-byte non-temporal
//    load + one fp32 group scale), UNR chunks in flight, X staged in LDS when it fits, int8 -> f32 by byte extract +
//    convert, fp32 FMA, one wave reduction per (row, token). Costs M FMAs per weight byte: 6.2 TB/s at one row,
//    1.5 at eight.
//  * MFMA stream over the PRE-SHUFFLED weight (ops/int8_gemv.py), the decode path of the inference engine: below.
#include "ds_hip.h"

#include <algorithm>

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

// ---------------------------------------------------------------------------------------------- MFMA stream
// Pre-shuffled weights. The HBM stream wants every load instruction to cover long contiguous segments: measured
// loads-only (tools/probe_load_patterns.hip, profiles/int8_load_patterns_r2.jsonl) 16 rows x 64 B per instruction
// (the MFMA operand layout read from a row-major weight: lane & 15 = row) caps at 4.4-5.0 TB/s, 4 rows x 256 B or
// 1 row x 1 KB reach 6-6.9. Staging a row-major tile through LDS (LDS-DMA, 3-slot ring) fixes the pattern but LDS
// then bounds the bytes in flight to ~64 KB per CU, which at the loaded HBM latency (~4 us) is 1.5 TB/s (measured).
// Weights of an inference model are constants, so the quantiser output is re-laid ONCE into operand order instead:
//   Qsh[nb][kq][lane][16 B] = Q[16 nb + (lane & 15)][64 kq + 16 (lane >> 4) + 0..15]   (1 KB per 16 rows x 64 k)
//   Ssh[nb][group][16]      = S[16 nb + r][group]
// so one 16-byte-per-lane load IS the v_mfma_f32_16x16x32_bf16 B operand of two MFMAs (k permuted 16g + j for the
// first, 16g + 8 + j for the second, X loaded with the same permutation) and each instruction reads 1 KB contiguous.
//  * a wave owns FB = 4 row blocks (64 output features) and walks a contiguous range of the (block group, k quarter)
//    sequence; P = 2-3 quarters of weights, X and scales are in flight in registers (compiler-counted vmcnt; the
//    prologue and every reload are fenced with sched_barrier so hipcc keeps the issue order that makes the counts
//    static), 12 waves per CU. MORE in flight is slower (measured: 8 waves x 8 KB beat 8 x 32 KB by 1.5x): the
//    memory pipeline reorders deep per-CU queues into a DRAM-unfriendly stream;
//  * B = u = q + 128 (byte extract + packed bf16 convert), A = X (token = lane & 15; rows >= M re-read row M-1); two
//    MFMAs per block for u.x and two per quarter against ones for sum(x), W.x = s * (u.x - 128 sum x) with the
//    lane's single scale (its accumulator rows are 4 tokens of ONE feature);
//  * ranges may start / end inside a block group (split-K without a fixed factor, every wave gets the same number
//    of quarters); partial sums go to a fp32 workspace with f32 atomics and a second small kernel converts it (+ bias)
//    to bf16 and re-zeroes it: no memset, capturable in a HIP graph. (A last-arriver finalize inside the main kernel
//    needs device-scope fences, which on the multi-XCD part write back / invalidate the XCD's L2 — measured 3.2 vs
//    5.4 TB/s for the same loop.)
// Measured (profiles/int8_skinny_gemv_r2.jsonl, BLOOM-176B shapes 57344x14336 / 14336x57344): 6.3 TB/s at 1 token
// row, 6.0-6.1 at 8, 5.5-5.9 at 16 (round 1's MFMA kernel: 2.2-3.0; the VALU stream: 6.3 at 1 row, 1.5 at 8).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

struct I8Args {
  const bf16* x;
  const int8_t* q;   // shuffled
  const float* s;    // shuffled
  const bf16* bias;
  bf16* y;
  float* acc;  // [16, NP] fp32 workspace, zero between calls
  int M, N, K, gs, ngroups, NB, KQ, NBG;
  int qpg;        // k quarters per scale group (gs / 64)
  int NP;         // workspace row length: NBG * FB * 16
  int64_t total;  // NBG * KQ
};

// 16 int8 -> two bf16x8 of u = q + 128 (exact)
__device__ __forceinline__ void u8x16_to_bf16(const i32x4 wq, bf16x8_t& lo, bf16x8_t& hi) {
  bf16x8_t o[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned a = (unsigned)wq[2 * h] ^ 0x80808080u, b = (unsigned)wq[2 * h + 1] ^ 0x80808080u;
    f32x4 fa, fb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fa[j] = (float)((a >> (8 * j)) & 0xffu);
      fb[j] = (float)((b >> (8 * j)) & 0xffu);
    }
    const bf16x4 ba = __builtin_convertvector(fa, bf16x4), bb = __builtin_convertvector(fb, bf16x4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[h][j] = ba[j]; o[h][4 + j] = bb[j]; }
  }
  lo = o[0];
  hi = o[1];
}

template <int FB>
struct I8Stage {
  i32x4 w[FB];
  bf16x8_t x0, x1;
  float sc[FB];
};

template <int FB, int P>
__global__ void __launch_bounds__(256) skinny_i8_mfma_kernel(I8Args a) {
  const int lane = threadIdx.x & 63;
  // wave-uniform bookkeeping lives in SGPRs (readfirstlane): scalar branches keep the vmcnt counts static
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  const int lo = (int)(a.total * gw / nw), hi = (int)(a.total * (gw + 1) / nw);
  if (lo >= hi) return;
  const int r = lane & 15, g = lane >> 4;

  // issue cursor: wave-uniform (SGPR) pointers advanced per quarter; divisions only when entering a block group
  int ibg = 0, ikq = 0, iql = 0;
  bool hold = false;
  int64_t iw = 0, is = 0, ix = 0, fw[FB], fs[FB];
  const int64_t xlane = (int64_t)min(r, a.M - 1) * a.K + 16 * g + 0;  // token rows >= M re-read row M - 1
  auto enter = [&](int bgv, int kqv) {
    if (bgv >= a.NBG) {  // past the end of the range: keep re-loading the last quarter (static vmcnt)
      bgv = a.NBG - 1;
      kqv = a.KQ - 1;
      hold = true;
    }
    ibg = bgv;
    ikq = kqv;
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      const int64_t nb = min(bgv * FB + f, a.NB - 1);
      fw[f] = nb * a.KQ * 1024;
      fs[f] = nb * a.ngroups * 16;
    }
    iw = (int64_t)kqv * 1024;
    is = (int64_t)(kqv / a.qpg) * 16;
    iql = a.qpg - kqv % a.qpg;
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
    if (--iql == 0) {
      is += 16;
      iql = a.qpg;
    }
  };
  auto load = [&](I8Stage<FB>& st) {
#pragma unroll
    for (int f = 0; f < FB; ++f)
      st.w[f] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(a.q + fw[f] + iw + lane * 16));
#pragma unroll
    for (int f = 0; f < FB; ++f) st.sc[f] = a.s[fs[f] + is + r];
    const bf16* xp = a.x + xlane + ix;
    st.x0 = *reinterpret_cast<const bf16x8_t*>(xp);
    st.x1 = *reinterpret_cast<const bf16x8_t*>(xp + 8);
  };

  bf16x8_t ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[FB];
#pragma unroll
  for (int f = 0; f < FB; ++f) acc[f] = zero4;

  int bg = lo / a.KQ, kq = lo - bg * a.KQ;
  enter(bg, kq);
  I8Stage<FB> st[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {  // same issue order as the steady state (else vmcnt at the loop head drains all)
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
  // Straight-line steady state (no early exit, no fence): hipcc keeps each reload right after the compute that frees
  // its registers and counts vmcnt statically; steps past the range end compute on re-loaded data with scale 0.
  for (int base = lo; base < hi; base += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool live = base + p < hi;
      f32x4 px = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x0, ones, zero4, 0, 0, 0);
      px = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x1, ones, px, 0, 0, 0);
#pragma unroll
      for (int f = 0; f < FB; ++f) {
        bf16x8_t b0, b1;
        u8x16_to_bf16(st[p].w[f], b0, b1);
        f32x4 pu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x0, b0, zero4, 0, 0, 0);
        pu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x1, b1, pu, 0, 0, 0);
        const float sc = live ? st[p].sc[f] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[f][i] = fmaf(sc, fmaf(-128.f, px[i], pu[i]), acc[f][i]);
      }
      if (live && kq == a.KQ - 1) spill(bg);
      if (++kq == a.KQ) { kq = 0; ++bg; }
      __builtin_amdgcn_sched_barrier(0);
      load(st[p]);
      advance();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if ((hi % a.KQ) != 0) spill((hi - 1) / a.KQ);  // the range ends inside a group
}

// y = bf16(workspace + bias) for the M token rows; the workspace is re-zeroed over everything the spills touched
// (rows < M, all NP padded columns), so the next call — whatever its N — starts from 0.
__global__ void __launch_bounds__(256) skinny_i8_finalize(float* __restrict__ acc, const bf16* __restrict__ bias,
                                                          bf16* __restrict__ y, int M, int N, int NP) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * NP) return;
  const int t = (int)(e / NP), n = (int)(e % NP);
  const float v = acc[e];
  acc[e] = 0.f;
  if (n < N) y[(int64_t)t * N + n] = (bf16)(v + (bias ? (float)bias[n] : 0.f));
}

// Pre-shuffled int8 -> row-major bf16 [N, K] (prefill: the library GEMM wants the plain matrix). One thread per
// 16-byte lane chunk: 16 weights of one row, one scale, 32 contiguous output bytes.
__global__ void __launch_bounds__(256) dequant_sh_kernel(const int8_t* __restrict__ Qsh, const float* __restrict__ Ssh,
                                                         bf16* __restrict__ W, int N, int KQ, int ngroups, int qpg) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk index = (nb * KQ + kq) * 64 + lane
  const int lane = (int)(c & 63);
  const int64_t t = c >> 6;
  const int kq = (int)(t % KQ), nb = (int)(t / KQ);
  const int row = nb * 16 + (lane & 15);
  if (row >= N) return;
  const float sc = Ssh[((int64_t)nb * ngroups + kq / qpg) * 16 + (lane & 15)];
  const i32x4 q = *reinterpret_cast<const i32x4*>(Qsh + c * 16);
  bf16x8 o[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[h][j] = (bf16)(sc * (float)(int8_t)((q[2 * h + j / 4] >> (8 * (j & 3))) & 0xff));
  bf16* dst = W + (int64_t)row * KQ * 64 + kq * 64 + 16 * (lane >> 4);
  *reinterpret_cast<bf16x8*>(dst) = o[0];
  *reinterpret_cast<bf16x8*>(dst + 8) = o[1];
}

}  // namespace

extern "C" int ds_dequant_sh(const int8_t* Qsh, const float* Ssh, void* W, int N, int K, int gs, hipStream_t st) {
  if (N <= 0 || K % 64 || gs % 64 || K % gs) return (int)hipErrorInvalidValue;
  const int KQ = K / 64, NB = (N + 15) / 16;
  const int64_t chunks = (int64_t)NB * KQ * 64;
  hipLaunchKernelGGL(dequant_sh_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st, Qsh, Ssh, (bf16*)W,
                     N, KQ, K / gs, gs / 64);
  DS_CHECK_LAUNCH();
  return 0;
}

// Variant override for tools/sweep_int8_gemv.py (0 = measured default below): (FB, P) kernel and resident waves / CU.
static int g_i8_cfg = 0, g_i8_wpc = 0;
extern "C" void ds_skinny_i8_tune(int cfg, int wpc, int) {
  g_i8_cfg = cfg;
  g_i8_wpc = wpc;
}

extern "C" int ds_skinny_i8_mfma_ok(int M, int K, int gs) {
  return M >= 1 && M <= 16 && K % 64 == 0 && gs % 64 == 0 && K % gs == 0;
}

// workspace the caller keeps per stream: fp32 [16 rows x N padded to whole block groups], zero-filled once
extern "C" int64_t ds_skinny_i8_mfma_ws_floats(int N) { return 16LL * (((N + 15) / 16 + 3) / 4) * 64; }

// X [M, K] bf16 (M <= 16), Qsh / Ssh in the shuffled layout above (N padded to a multiple of 16), bias bf16 [N] or
// null -> Y [M, N] bf16 (Y == null: leave the sums in the workspace, row length ws_floats / 16, un-finalized)
extern "C" int ds_skinny_i8_mfma(const void* X, const int8_t* Qsh, const float* Ssh, const void* bias, void* Y,
                                 float* ws, int M, int N, int K, int gs, hipStream_t st) {
  if (!ds_skinny_i8_mfma_ok(M, K, gs) || N <= 0) return (int)hipErrorInvalidValue;
  I8Args a;
  a.x = (const bf16*)X;
  a.q = Qsh;
  a.s = Ssh;
  a.bias = (const bf16*)bias;
  a.y = (bf16*)Y;
  a.acc = ws;
  a.M = M;
  a.N = N;
  a.K = K;
  a.gs = gs;
  a.ngroups = K / gs;
  a.qpg = gs / 64;
  a.NB = (N + 15) / 16;
  a.KQ = K / 64;
  auto go = [&](auto kern, int P, int FB, int wpc) {
    // one resident round of waves (wpc per CU, from the VGPR budget), each with the same number of quarters
    const int nbg = (a.NB + FB - 1) / FB;
    a.NBG = nbg;
    a.NP = nbg * FB * 16;
    a.total = (int64_t)nbg * a.KQ;
    const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(a.total / (2 * P), 256 * wpc));
    hipLaunchKernelGGL(kern, dim3((int)((waves + 3) / 4)), dim3(256), 0, st, a);
    if (Y == nullptr) return;  // sums stay in the workspace for a fused consumer (skinny_finalize.hip)
    hipLaunchKernelGGL(skinny_i8_finalize, dim3((int)(((int64_t)M * a.NP + 255) / 256)), dim3(256), 0, st, ws,
                       (const bf16*)bias, (bf16*)Y, M, N, a.NP);
  };
  // measured (tools/sweep_int8_gemv.py, profiles/int8_skinny_gemv_r2.jsonl): FB 4 / P 2 at 12 waves per CU (128
  // registers) up to 8 token rows, FB 4 / P 3 at 8 waves per CU above (more MFMA work per byte wants fewer waves)
  int cfg = g_i8_cfg ? g_i8_cfg : (M > 8 ? 2 : 1);
  const int wpc = g_i8_wpc;
  switch (cfg) {
    case 2: go(skinny_i8_mfma_kernel<4, 3>, 3, 4, wpc ? wpc : 8); break;
    case 3: go(skinny_i8_mfma_kernel<4, 4>, 4, 4, wpc ? wpc : 8); break;
    case 4: go(skinny_i8_mfma_kernel<2, 2>, 2, 2, wpc ? wpc : 16); break;
    default: go(skinny_i8_mfma_kernel<4, 2>, 2, 4, wpc ? wpc : 12);
  }
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
