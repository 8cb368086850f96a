// Ragged paged flash attention for inference prefill / prompt chunks (SplitFuse), bf16, head dims 64 / 80 / 96 / 128 /
// 256 (GPT-2 / Phi / GPT-NeoX-20B / Llama / GPT-J).
//
// Reference counterpart (behaviour): inference v2's `blocked_flash` (`inference/v2/kernels/ragged_ops/blocked_flash/
// blocked_flash.cpp:21-100`, a prebuilt flash-attention over the blocked KV cache driven by the ragged batch's
// `atoms`) and v1's `softmax_context` with ALiBi / local windows (`csrc/transformer/inference/csrc/softmax.cu:35,256`).
//
// One launch covers every prompt / chunk sequence of a ragged batch:
//  * queries are the batch's concatenated new tokens q [T, Hq, D] (cu_q gives each sequence's slice); keys and
//    values are read straight from the paged cache [blocks, Hk, BS, D] through the block table — the new tokens'
//    K/V were appended by the fused QKV epilogue first, so a chunk sees its whole cached prefix plus itself;
//  * a host-built work list names (sequence, 128-row query block) pairs, so ragged lengths cost no padding beyond one
//    block; every q head of a work item sits on one XCD (xcd_remap) so the GQA group's K/V tiles are shared in L2;
//  * per query row the position is start + i: causal masking against absolute positions, ALiBi bias
//    slope_h * (key - pos) folded into the score before the online softmax, sliding window key > pos - window; tiles
//    entirely outside [pos - window, pos] are never loaded;
//  * the compute core is flash_fwd.hip's: 4 waves x 32 rows, S^T = K.Q^T on v_mfma_f32_32x32x16_bf16 so each lane
//    owns one query row's scores, P reused as the A operand of O += P.V, V by ds_read_b64_tr_b16 from the same
//    XOR-swizzled LDS image, next tile's loads issued before the current tile's MFMAs;
//  * the head dim is a template parameter: D / 16 MFMA steps for the scores, ceil(D / 32) output column tiles (D = 80
//    computes a third, half-used tile over zero-filled LDS columns), LDS rows pitched to 16 (D <= 128) or 32 (D = 256)
//    16-byte chunks so one swizzle serves every size.
#include "ds_hip.h"

namespace {

constexpr int BM = 128;
constexpr int BN = 64;
constexpr int NTHR = 256;

template <int D>
struct Cfg {
  static_assert(D % 16 == 0 && D >= 64 && D <= 256, "head dim");
  static constexpr int KC = D / 16;               // MFMA steps of the score product
  static constexpr int DT = (D + 31) / 32;        // 32-column output tiles
  static constexpr int CH = D / 8;                // 16-byte chunks holding data in one K / V row
  static constexpr int PCH = D <= 128 ? 16 : 32;  // chunks per LDS row (pitch)
  static constexpr int ROWB = PCH * 16;
  static constexpr int TILE_BYTES = BN * ROWB;
  static constexpr int NLD = BN * PCH / NTHR;     // chunks staged per thread per tile
  static constexpr int LDS_BYTES = 4 * TILE_BYTES + 4 * 32 * 4;
  static constexpr int OCC = D <= 128 ? 2 : 1;
};

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int ROWB>
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * ROWB + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

struct PagedArgs {
  const bf16* q;          // [T, Hq, D]
  const bf16* kc;         // [blocks, Hk, BS, D]
  const bf16* vc;
  bf16* o;                // [T, Hq, D]
  const int* block_table; // [nseq, max_blocks]
  const int* start;       // [nseq] cached tokens before this step
  const int* cu_q;        // [nseq + 1] token offsets of each sequence's new tokens
  const int* work;        // [nwork, 2] (sequence, query block)
  const float* alibi;     // [Hq] slopes or null
  int Hq, Hk, BS, max_blocks, window;
  float c;                // softmax scale * log2(e)
  float inv_scale;        // 1 / softmax scale (ALiBi bias in score units)
};

template <int D>
__global__ void __launch_bounds__(NTHR, Cfg<D>::OCC) paged_prefill_kernel(PagedArgs a) {
  using C = Cfg<D>;
  constexpr int KC = C::KC, DT = C::DT, CH = C::CH, PCH = C::PCH, ROWB = C::ROWB, TILE_BYTES = C::TILE_BYTES,
                NLD = C::NLD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int w = logical / a.Hq, hq = logical % a.Hq, hk = hq / (a.Hq / a.Hk);
  const int seq = a.work[2 * w], qb = a.work[2 * w + 1];
  const int t0 = a.cu_q[seq], n = a.cu_q[seq + 1] - t0, start = a.start[seq], Skv = start + n;
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int* bt = a.block_table + (int64_t)seq * a.max_blocks;
  const float slope = a.alibi ? a.alibi[hq] * a.inv_scale : 0.f;

  bf16x8_t qf[KC];
  {
    const int qr = min(q0w + l32, n - 1);
    const bf16* qrow = a.q + ((int64_t)(t0 + qr) * a.Hq + hq) * D + 8 * h;
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) qf[kk] = *reinterpret_cast<const bf16x8_t*>(qrow + 16 * kk);
  }
  const int pos_lane = start + q0w + l32;                // this lane's query position
  const int pos_hi = start + min(q0 + BM, n) - 1;        // last query position of the block
  const int wpos_lo = start + q0w, wpos_hi = start + q0w + 31;
  int kt1 = min((Skv + BN - 1) / BN, pos_hi / BN + 1);
  int kt0 = a.window > 0 ? max(0, (start + q0 - a.window + 1) / BN) : 0;
  if (kt0 > kt1) kt0 = kt1;

  float* scratch = reinterpret_cast<float*>(smem + 4 * TILE_BYTES) + wid * 32;
  u32x4_t kreg[NLD], vreg[NLD];
  auto stage_load = [&](int tile) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int cidx = tid + i * NTHR, row = cidx / PCH, ch = cidx % PCH;
      if (ch < CH) {
        const int key = min(tile * BN + row, Skv - 1);
        const int64_t off = (((int64_t)bt[key / a.BS] * a.Hk + hk) * a.BS + key % a.BS) * D + ch * 8;
        kreg[i] = *reinterpret_cast<const u32x4_t*>(a.kc + off);
        vreg[i] = *reinterpret_cast<const u32x4_t*>(a.vc + off);
      } else {  // pitch padding: zero columns (read by the last, partly used output tile of D = 80)
        kreg[i] = u32x4_t{0u, 0u, 0u, 0u};
        vreg[i] = u32x4_t{0u, 0u, 0u, 0u};
      }
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int cidx = tid + i * NTHR, row = cidx / PCH, ch = cidx % PCH;
      if (ch < 4 * DT) {
        *reinterpret_cast<u32x4_t*>(smem + buf * TILE_BYTES + lds_off<ROWB>(row, ch)) = kreg[i];
        *reinterpret_cast<u32x4_t*>(smem + (2 + buf) * TILE_BYTES + lds_off<ROWB>(row, ch)) = vreg[i];
      }
    }
  };

  f32x16_t o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  if (kt1 > kt0) {
    stage_load(kt0);
    stage_store(0);
  }
  __syncthreads();
  for (int j = kt0; j < kt1; ++j) {
    const int cur = (j - kt0) & 1;
    if (j + 1 < kt1) stage_load(j + 1);
    const int k0 = j * BN;
    const bool active = q0w < n && k0 <= wpos_hi && (a.window <= 0 || k0 + BN - 1 > wpos_lo - a.window);
    if (active) {
      const char* Kt = smem + cur * TILE_BYTES;
      const char* Vt = smem + (2 + cur) * TILE_BYTES;
      f32x16_t s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t][r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
          const bf16x8_t av = *reinterpret_cast<const bf16x8_t*>(Kt + lds_off<ROWB>(t * 32 + l32, 2 * kk + h));
          s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, qf[kk], s[t], 0, 0, 0);
        }
      }
      // ALiBi bias, causal diagonal, window, key tail (lane = one query row, r = 32 keys of the 64)
      const bool need_mask = k0 + BN - 1 > wpos_lo || k0 + BN > Skv ||
                             (a.window > 0 && k0 <= wpos_hi - a.window);
      if (a.alibi || need_mask) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = fmaf(slope, (float)(key - pos_lane), s[t][r]);
            if (key >= Skv || key > pos_lane || (a.window > 0 && key <= pos_lane - a.window)) v = -INFINITY;
            s[t][r] = v;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f((m_run - m_use) * a.c);
      const float mc = m_use * a.c;
      float psum = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[t][r], a.c, -mc));
          s[t][r] = p;
          psum += p;
        }
      l_run = l_run * alpha + psum;
      m_run = m_new;
      if (!__all(alpha == 1.f)) {
        if (lane < 32) scratch[lane] = alpha;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        float a4[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(scratch + 8 * g + 4 * h);
#pragma unroll
          for (int i = 0; i < 4; ++i) a4[4 * g + i] = v[i];
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= a4[r];
        __builtin_amdgcn_wave_barrier();
      }
      bf16x8_t pa[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int e = 0; e < 8; ++e) pa[t][ss][e] = (bf16)s[t][8 * ss + e];
      const int gq = (lane >> 2) & 3, gch = (lane >> 1) & 1, gb = 8 * (lane & 1), colhalf = (lane >> 4) & 1;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int rb = t * 32 + 16 * ss + 4 * h;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(Vt + lds_off<ROWB>(rb + gq, ch0) + gb));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(Vt + lds_off<ROWB>(rb + 8 + gq, ch0) + gb));
            s16x8 vv;
#pragma unroll
            for (int e = 0; e < 4; ++e) { vv[e] = lo[e]; vv[4 + e] = hi[e]; }
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[t][ss], __builtin_bit_cast(bf16x8_t, vv), o[dt], 0,
                                                           0, 0);
          }
      }
    }
    if (j + 1 < kt1) stage_store(cur ^ 1);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (lane < 32) scratch[lane] = inv;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  float iv[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(scratch + 8 * g + 4 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) iv[4 * g + i] = v[i];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qi = q0w + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (qi < n) {
      bf16* orow = a.o + ((int64_t)(t0 + qi) * a.Hq + hq) * D + l32;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        if (D % 32 == 0 || dt * 32 + l32 < D) orow[dt * 32] = (bf16)(o[dt][r] * iv[r]);
    }
  }
}

template <int D>
int launch(const PagedArgs& a, int nwork, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&paged_prefill_kernel<D>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, Cfg<D>::LDS_BYTES);
    attr = true;
  }
  hipLaunchKernelGGL((paged_prefill_kernel<D>), dim3(nwork * a.Hq), dim3(NTHR), Cfg<D>::LDS_BYTES, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// q / o [T, Hq, D] bf16 (contiguous), caches [blocks, Hk, BS, D] bf16, D in {64, 80, 96, 128, 256}, block_table
// [nseq, max_blocks] int32, start [nseq], cu_q [nseq + 1], work [nwork, 2] (sequence, 128-row query block) int32,
// alibi [Hq] fp32 or null, window <= 0 for none.
extern "C" int ds_paged_prefill(const void* q, const void* kc, const void* vc, void* o, const int* block_table,
                                const int* start, const int* cu_q, const int* work, int nwork, const float* alibi,
                                int Hq, int Hk, int D, int BS, int max_blocks, int window, float scale,
                                hipStream_t st) {
  if (nwork <= 0) return 0;
  if (Hk <= 0 || Hq % Hk || BS <= 0 || max_blocks <= 0 || scale <= 0.f) return (int)hipErrorInvalidValue;
  PagedArgs a{(const bf16*)q, (const bf16*)kc, (const bf16*)vc, (bf16*)o, block_table, start, cu_q, work, alibi,
              Hq, Hk, BS, max_blocks, window, scale * 1.4426950408889634f, 1.f / scale};
  switch (D) {
    case 64: return launch<64>(a, nwork, st);
    case 80: return launch<80>(a, nwork, st);
    case 96: return launch<96>(a, nwork, st);
    case 128: return launch<128>(a, nwork, st);
    case 256: return launch<256>(a, nwork, st);
    default: return (int)hipErrorInvalidValue;
  }
}
