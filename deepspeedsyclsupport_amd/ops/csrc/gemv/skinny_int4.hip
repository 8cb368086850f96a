// Weight-only int4 (group-quantised) skinny GEMM for decode: y[M, N] = X[M, K] . (Q[N, K] * s[N, K / gs])^T (+ bias),
// M <= 16, plus the dequantiser that turns the same packed layout into a row-major bf16 weight for prefill GEMMs.
//
// Reference counterparts (behaviour, not code): inference v2's CUTLASS `mixed_gemm` with `num_bits = 4`
// (`inference/v2/kernels/cutlass_ops/mixed_gemm/mixed_gemm.py`, built by `op_builder/inference_cutlass_builder.py:59-92`)
// and the v1 weight-quantiser's int4 path (`runtime/weight_quantizer.py`): a library GEMM over weights dequantised on
// the fly.
//
// MI355X design. Decode GEMMs are pure weight streams, so int4 weights quarter the HBM bytes of a bf16 decode step; the
// dequantisation is fused into the stream and costs no convert instruction at all:
//  * symmetric int4 q in [-8, 7] is stored as the nibble u = q + 8. The bf16 bit pattern 0x4300 | u IS the number
//    128 + u exactly (bf16 has 7 mantissa bits and 128 <= 128 + u < 256, so the mantissa's unit is 1). One
//    v_and_or_b32 per register turns two nibbles of a packed word into a ready pair of bf16 MFMA operand elements:
//        reg_t = ((word >> 4 t) & 0x000F000F) | 0x43004300,  t = 0..3   (low half = nibble t, high half = nibble t + 4)
//    and W.x = s * ((128 + u).x - 136 * sum(x)), with sum(x) from MFMAs against a vector of ones shared by every
//    feature block of the wave.
//  * weights are constants, so they are re-laid ONCE (ops/int4_gemv.py) into operand order, 1 KB contiguous per
//    wave-wide load (the pattern that sustains the HBM stream, see skinny_int8.hip):
//        word i of Q4[nb][kq][lane] = the 8 weights W[16 nb + (lane & 15)][128 kq + 32 i + 8 (lane >> 4) + j], j = 0..7,
//        weight j in nibble (j even ? j / 2 : 4 + j / 2)
//        S4[nb][group][16] = s[16 nb + r][group]
//    so word i is the B operand of the i-th v_mfma_f32_16x16x32_bf16 of a "quarter" (128 k), whose K range is the 32
//    consecutive k 128 kq + 32 i .. + 31: scale groups of 32, 64 or any multiple of 128 all line up with whole MFMAs.
//    X is loaded with the same k mapping (four 16-byte loads per lane and quarter, L2-resident);
//  * the schedule is skinny_int8.hip's: a wave owns FB = 4 row blocks (64 features) and a contiguous range of the
//    (block group, quarter) sequence, P quarters in flight in registers with compiler-counted vmcnt, equal work per
//    wave (split-K without a fixed factor), fp32 atomics into a workspace that a finalize kernel converts (+ bias) and
//    re-zeroes (no memset: capturable in a HIP graph).
#include "ds_hip.h"

#include <algorithm>

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

struct I4Args {
  const bf16* x;
  const int8_t* q;   // shuffled, 16 bytes per lane and quarter
  const float* s;    // shuffled
  const bf16* bias;
  bf16* y;
  float* acc;        // [16, NP] fp32 workspace, zero between calls
  int M, N, K, gs, ngroups, NB, KQ, NBG;
  int qpg;           // quarters per scale group (gs / 128, 1 when gs < 128)
  int NP;            // workspace row length: NBG * FB * 16
  int64_t total;     // NBG * KQ
};

// one packed word -> the 8 bf16 values 128 + u of one MFMA operand
__device__ __forceinline__ bf16x8_t unpack_u4(unsigned w) {
  u32x4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = ((w >> (4 * t)) & 0x000F000Fu) | 0x43004300u;
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int FB, int SPQ>
struct I4Stage {
  i32x4 w[FB];
  bf16x8_t x[4];
  float sc[FB][SPQ];
};

// SPQ = scale groups per quarter: 1 (gs a multiple of 128), 2 (gs 64) or 4 (gs 32)
template <int FB, int P, int SPQ>
__global__ void __launch_bounds__(256) skinny_i4_mfma_kernel(I4Args a) {
  constexpr int MPS = 4 / SPQ;  // MFMAs per scale group
  const int lane = threadIdx.x & 63;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  const int lo = (int)(a.total * gw / nw), hi = (int)(a.total * (gw + 1) / nw);
  if (lo >= hi) return;
  const int r = lane & 15, g = lane >> 4;

  // issue cursor: wave-uniform pointers advanced per quarter; divisions only when entering a block group
  int ibg = 0, ikq = 0, iql = 0;
  bool hold = false;
  int64_t iw = 0, is = 0, ix = 0, fw[FB], fs[FB];
  const int64_t xlane = (int64_t)min(r, a.M - 1) * a.K + 8 * g;  // token rows >= M re-read row M - 1
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
    is = SPQ > 1 ? (int64_t)kqv * SPQ * 16 : (int64_t)(kqv / a.qpg) * 16;
    iql = a.qpg - kqv % a.qpg;
    ix = (int64_t)kqv * 128;
  };
  auto advance = [&]() {
    if (hold) return;
    if (++ikq == a.KQ) {
      enter(ibg + 1, 0);
      return;
    }
    iw += 1024;
    ix += 128;
    if (SPQ > 1) {
      is += SPQ * 16;
    } else if (--iql == 0) {
      is += 16;
      iql = a.qpg;
    }
  };
  auto load = [&](I4Stage<FB, SPQ>& st) {
#pragma unroll
    for (int f = 0; f < FB; ++f)
      st.w[f] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(a.q + fw[f] + iw + lane * 16));
#pragma unroll
    for (int f = 0; f < FB; ++f)
#pragma unroll
      for (int sg = 0; sg < SPQ; ++sg) st.sc[f][sg] = a.s[fs[f] + is + sg * 16 + r];
    const bf16* xp = a.x + xlane + ix;
#pragma unroll
    for (int i = 0; i < 4; ++i) st.x[i] = *reinterpret_cast<const bf16x8_t*>(xp + 32 * i);
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
  I4Stage<FB, SPQ> st[P];
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
  // Straight-line steady state (no early exit): steps past the range end compute on re-loaded data with scale 0.
  for (int base = lo; base < hi; base += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool live = base + p < hi;
      f32x4 px[SPQ];
#pragma unroll
      for (int sg = 0; sg < SPQ; ++sg) {
        px[sg] = zero4;
#pragma unroll
        for (int i = 0; i < MPS; ++i)
          px[sg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x[sg * MPS + i], ones, px[sg], 0, 0, 0);
      }
#pragma unroll
      for (int f = 0; f < FB; ++f) {
#pragma unroll
        for (int sg = 0; sg < SPQ; ++sg) {
          f32x4 pu = zero4;
#pragma unroll
          for (int i = 0; i < MPS; ++i)
            pu = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st[p].x[sg * MPS + i],
                                                         unpack_u4((unsigned)st[p].w[f][sg * MPS + i]), pu, 0, 0, 0);
          const float sc = live ? st[p].sc[f][sg] : 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[f][i] = fmaf(sc, fmaf(-136.f, px[sg][i], pu[i]), acc[f][i]);
        }
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

// y = bf16(workspace + bias) for the M token rows; the workspace is re-zeroed over everything the spills touched.
__global__ void __launch_bounds__(256) skinny_i4_finalize(float* __restrict__ acc, const bf16* __restrict__ bias,
                                                          bf16* __restrict__ y, int M, int N, int NP) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * NP) return;
  const int t = (int)(e / NP), n = (int)(e % NP);
  const float v = acc[e];
  acc[e] = 0.f;
  if (n < N) y[(int64_t)t * N + n] = (bf16)(v + (bias ? (float)bias[n] : 0.f));
}

// Packed int4 -> row-major bf16 [N, K] (prefill: the library GEMM wants the plain matrix). One thread per 16-byte lane
// chunk: 4 words x 8 weights of one row, four 16-byte stores.
__global__ void __launch_bounds__(256) dequant_sh4_kernel(const int8_t* __restrict__ Q4, const float* __restrict__ S4,
                                                          bf16* __restrict__ W, int N, int KQ, int ngroups, int gs) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk index = (nb * KQ + kq) * 64 + lane
  const int lane = (int)(c & 63);
  const int64_t t = c >> 6;
  const int kq = (int)(t % KQ), nb = (int)(t / KQ);
  const int row = nb * 16 + (lane & 15);
  if (row >= N) return;
  const i32x4 q = *reinterpret_cast<const i32x4*>(Q4 + c * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k0 = kq * 128 + 32 * i;
    const float sc = S4[((int64_t)nb * ngroups + k0 / gs) * 16 + (lane & 15)];
    const unsigned w = (unsigned)q[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int nib = (j & 1) ? 4 + (j >> 1) : (j >> 1);
      o[j] = (bf16)(sc * (float)((int)((w >> (4 * nib)) & 0xFu) - 8));
    }
    *reinterpret_cast<bf16x8*>(W + (int64_t)row * KQ * 128 + k0 + 8 * (lane >> 4)) = o;
  }
}

}  // namespace

extern "C" int ds_skinny_i4_mfma_ok(int M, int K, int gs) {
  return M >= 1 && M <= 16 && K % 128 == 0 && gs > 0 && K % gs == 0 && (gs == 32 || gs == 64 || gs % 128 == 0);
}

extern "C" int ds_dequant_sh4(const int8_t* Q4, const float* S4, void* W, int N, int K, int gs, hipStream_t st) {
  if (N <= 0 || !ds_skinny_i4_mfma_ok(1, K, gs)) return (int)hipErrorInvalidValue;
  const int KQ = K / 128, NB = (N + 15) / 16;
  const int64_t chunks = (int64_t)NB * KQ * 64;
  hipLaunchKernelGGL(dequant_sh4_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st, Q4, S4, (bf16*)W, N,
                     KQ, K / gs, gs);
  DS_CHECK_LAUNCH();
  return 0;
}

// workspace the caller keeps per stream: fp32 [16 rows x N padded to whole block groups], zero-filled once
extern "C" int64_t ds_skinny_i4_mfma_ws_floats(int N) { return 16LL * (((N + 15) / 16 + 3) / 4) * 64; }

// Variant override for tools/bench_int4_gemv.py (0 = default): in-flight quarters P and resident waves per CU.
static int g_i4_p = 0, g_i4_wpc = 0, g_i4_rounds = 0;
extern "C" void ds_skinny_i4_tune(int p, int wpc, int rounds) {
  g_i4_p = p;
  g_i4_wpc = wpc;
  g_i4_rounds = rounds;
}

// X [M, K] bf16 (M <= 16), Q4 / S4 in the packed layout above (N padded to a multiple of 16), bias bf16 [N] or null
// -> Y [M, N] bf16. Y == null leaves the sums in the workspace (rows < M, row length ds_skinny_i4_mfma_ws_floats / 16)
// for a fused consumer (skinny_finalize.hip), which then owes the re-zeroing.
extern "C" int ds_skinny_i4_mfma(const void* X, const int8_t* Q4, const float* S4, const void* bias, void* Y, float* ws,
                                 int M, int N, int K, int gs, hipStream_t st) {
  if (!ds_skinny_i4_mfma_ok(M, K, gs) || N <= 0) return (int)hipErrorInvalidValue;
  constexpr int FB = 4;
  I4Args a;
  a.x = (const bf16*)X;
  a.q = Q4;
  a.s = S4;
  a.bias = (const bf16*)bias;
  a.y = (bf16*)Y;
  a.acc = ws;
  a.M = M;
  a.N = N;
  a.K = K;
  a.gs = gs;
  a.ngroups = K / gs;
  a.qpg = gs >= 128 ? gs / 128 : 1;
  a.NB = (N + 15) / 16;
  a.KQ = K / 128;
  a.NBG = (a.NB + FB - 1) / FB;
  a.NP = a.NBG * FB * 16;
  a.total = (int64_t)a.NBG * a.KQ;
  const int P = g_i4_p ? g_i4_p : 2;
  const int wpc = g_i4_wpc ? g_i4_wpc : 12;
  // one resident round of waves, each with the same number of quarters (at least two rounds of the pipeline each)
  const int rounds = g_i4_rounds ? g_i4_rounds : 2;
  const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(a.total / (rounds * P), 256 * wpc));
  const dim3 grid((int)((waves + 3) / 4));
  const int spq = gs >= 128 ? 1 : 128 / gs;
#define DS_I4_GO(PP, SS) hipLaunchKernelGGL((skinny_i4_mfma_kernel<FB, PP, SS>), grid, dim3(256), 0, st, a)
  if (P == 3) {
    if (spq == 1) DS_I4_GO(3, 1); else if (spq == 2) DS_I4_GO(3, 2); else DS_I4_GO(3, 4);
  } else {
    if (spq == 1) DS_I4_GO(2, 1); else if (spq == 2) DS_I4_GO(2, 2); else DS_I4_GO(2, 4);
  }
#undef DS_I4_GO
  DS_CHECK_LAUNCH();
  if (Y == nullptr) return 0;
  hipLaunchKernelGGL(skinny_i4_finalize, dim3((int)(((int64_t)M * a.NP + 255) / 256)), dim3(256), 0, st, ws,
                     (const bf16*)bias, (bf16*)Y, M, N, a.NP);
  DS_CHECK_LAUNCH();
  return 0;
}
