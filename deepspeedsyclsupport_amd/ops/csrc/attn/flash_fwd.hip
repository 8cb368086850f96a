// CDNA4 flash-attention forward (training / prefill), bf16, head dim 128.
//
// Reference counterparts: the fused softmax-context path of `csrc/transformer/inference/csrc/pt_binding.cpp:434-557`,
// the Triton `_flash_packed_kernel` (`ops/transformer/inference/triton/attention.py:253`) and the prebuilt
// `flash_attn_by_atoms` of inference v2 (`inference/v2/kernels/ragged_ops/blocked_flash/blocked_flash.cpp:21-100`).
// This is a gfx950 design, not a translation of any of them:
//
//  * one workgroup = 4 waves = 128 query rows (32 per wave); K/V tiles of 64 keys are staged once per workgroup into
//    LDS (double buffered, 2 x 32 KB) and shared by the 4 waves; 2 workgroups per CU (launch bounds 256 x 2);
//  * S^T = K . Q^T on `v_mfma_f32_32x32x16_bf16` ("swapped" product): each lane ends up holding 32 of the 64 scores
//    of ONE query row, so the online-softmax row max / row sum are lane-local plus a single xor-32 exchange;
//  * the score accumulator is re-used directly as the A operand of O += P . V (accumulator-as-operand, no LDS round
//    trip for P); V is consumed column-wise with the hardware transposed read `ds_read_b64_tr_b16`;
//  * K and V share one LDS image (256-B rows, 16-B chunks XOR-swizzled by the row) that is conflict-free both for the
//    row reads of K (`ds_read_b128`) and the transposed reads of V;
//  * global->LDS staging is split (issue the next tile's loads before the current tile's MFMAs, write LDS after them),
//    so HBM latency hides under the MFMA work; one barrier per tile;
//  * causal: fully-masked tiles are skipped per wave, heavy query blocks are launched first, and the block->tile map
//    keeps every (batch, head) on one XCD so its K/V stay in that XCD's L2.
//  * block-sparse variant (SPARSE=true, reference `ops/sparse_attention` SDD/softmax/DSD Triton kernels): each
//    workgroup walks only the 64-key tiles listed for its (layout head, 128-row query block) in a host-built LUT, and
//    masks inside a tile at the layout's block granularity (16/32/64/128) with a per-lane 64-bit allow mask built
//    from the block layout — compute and K/V traffic scale with the layout's density, not with S^2.
// Outputs O (any [B,H,S,D] strides, e.g. written straight into the [B,S,H,D] layout the o_proj GEMM wants) and the
// natural-log LSE [B,H,S] in fp32 that the backward pass consumes.
#include "ds_hip.h"

namespace {

constexpr int D = 128;
constexpr int BM = 128;            // query rows per workgroup
constexpr int BN = 64;             // keys per tile
constexpr int NTHR = 256;
constexpr int TILE_BYTES = BN * D * 2;     // 16 KB
constexpr int LDS_BYTES = 4 * TILE_BYTES + 4 * 32 * 4;  // K0 K1 V0 V1 + per-wave row scratch

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// byte offset of 16-B chunk `ch` (0..15) of row `row` in a [64][128 x bf16] tile: 256-B rows, chunk index XORed with
// a bijection of row mod 16 so both the row reads (32 consecutive rows, one chunk) and the 4-row transposed reads
// touch distinct banks.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// block-sparse LUT: tiles [lay_heads, nqb, max_tiles] (ascending 64-key tile ids), ntiles [lay_heads, nqb],
// layout [lay_heads, nb, nb] (uint8, block granularity blk)
struct SparseLut {
  const int* tiles;
  const int* ntiles;
  const int* qorder;  // [lay_heads, nqb] query blocks by descending tile count
  const uint8_t* layout;
  int max_tiles, lay_heads, nb, blk;
};

template <bool CAUSAL, bool SPARSE>
__global__ void __launch_bounds__(NTHR, 2) flash_fwd_kernel(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, bf16* __restrict__ O,
    float* __restrict__ LSE, int B, int Hq, int Hk, int S, int Skv, int64_t qsb, int64_t qsh, int64_t qss,
    int64_t ksb, int64_t ksh, int64_t kss, int64_t vsb, int64_t vsh, int64_t vss, int64_t osb, int64_t osh,
    int64_t oss, float c /* softmax scale * log2(e) */, float scale, SparseLut lut) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;

  // ------------------------------------------------------------------ block -> (batch, head, query block)
  const int nqb = (S + BM - 1) / BM;
  const int nwg = gridDim.x;
  const int logical = xcd_remap(blockIdx.x, nwg);
  // (batch, head)-major so one head's query blocks share an XCD's L2 (K/V tiles reused across its query blocks);
  // within a head the heaviest query blocks go first (causal: the longest rows; sparse: the LUT's order by tile
  // count, so global-attention rows do not start last). Measured: query-block-major heavy-first order loses more
  // to L2 misses than it gains in tail length (tools/bench_sparse_attn.py).
  const int bh = logical / nqb;
  const int qbi = logical % nqb;
  const int b = bh / Hq, hq = bh % Hq, hk = hq / (Hq / Hk);
  const int lh = SPARSE ? (lut.lay_heads == 1 ? 0 : hq) : 0;
  const int qb = SPARSE ? lut.qorder[lh * nqb + qbi] : (CAUSAL ? nqb - 1 - qbi : qbi);  // heaviest first
  const int q0 = qb * BM, q0w = q0 + wid * 32;

  const bf16* Qp = Q + b * qsb + hq * qsh;
  const bf16* Kp = K + b * ksb + hk * ksh;
  const bf16* Vp = V + b * vsb + hk * vsh;

  // ------------------------------------------------------------------ Q fragments (B operand of S^T = K.Q^T)
  bf16x8_t qf[8];
  {
    const int qr = min(q0w + l32, S - 1);
    const bf16* qrow = Qp + (int64_t)qr * qss + 8 * h;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) qf[kk] = *reinterpret_cast<const bf16x8_t*>(qrow + 16 * kk);
  }

  int nt = (Skv + BN - 1) / BN;
  if (CAUSAL) nt = min(nt, (q0 + BM + BN - 1) / BN);
  const int* tlist = nullptr;
  if constexpr (SPARSE) {
    nt = lut.ntiles[lh * nqb + qb];
    tlist = lut.tiles + ((int64_t)lh * nqb + qb) * lut.max_tiles;
  }
  auto tile_of = [&](int j) { return SPARSE ? tlist[j] : j; };

  // LDS: [K0][K1][V0][V1][scratch]
  float* scratch = reinterpret_cast<float*>(smem + 4 * TILE_BYTES) + wid * 32;

  // staging: thread t moves chunks t, t+256, t+512, t+768 (row = c>>4, 16-B chunk = c&15) of both K and V
  u32x4_t kreg[4], vreg[4];
  auto stage_load = [&](int tile) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cidx = tid + i * NTHR, row = cidx >> 4, ch = cidx & 15;
      const int key = min(tile * BN + row, Skv - 1);
      kreg[i] = *reinterpret_cast<const u32x4_t*>(Kp + (int64_t)key * kss + ch * 8);
      vreg[i] = *reinterpret_cast<const u32x4_t*>(Vp + (int64_t)key * vss + ch * 8);
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cidx = tid + i * NTHR, row = cidx >> 4, ch = cidx & 15;
      *reinterpret_cast<u32x4_t*>(smem + buf * TILE_BYTES + lds_off(row, ch)) = kreg[i];
      *reinterpret_cast<u32x4_t*>(smem + (2 + buf) * TILE_BYTES + lds_off(row, ch)) = vreg[i];
    }
  };

  f32x16_t o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const int qrow_lane = q0w + l32;  // the query row this lane's scores belong to

  if (nt > 0) {  // uniform per workgroup (a sparse row block may have no tiles)
    stage_load(tile_of(0));
    stage_store(0);
  }
  __syncthreads();

  for (int j = 0; j < nt; ++j) {
    const int cur = j & 1;
    if (j + 1 < nt) stage_load(tile_of(j + 1));
    const int k0 = tile_of(j) * BN;
    const bool active = !CAUSAL || k0 <= q0w + 31;
    if (active) {
      const char* Kt = smem + cur * TILE_BYTES;
      const char* Vt = smem + (2 + cur) * TILE_BYTES;
      // ---------------- S^T = K . Q^T  (two 32-key halves)
      f32x16_t s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t][r] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Kt + lds_off(t * 32 + l32, 2 * kk + h));
          s[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[kk], s[t], 0, 0, 0);
        }
      }
      // ---------------- block-sparse mask at the layout's granularity (this lane's query row vs the 64 keys)
      if constexpr (SPARSE) {
        const int qr = min(qrow_lane, S - 1);
        const uint8_t* lrow = lut.layout + ((int64_t)lh * lut.nb + qr / lut.blk) * lut.nb;
        uint64_t allow = 0;
        for (int kb = k0 / lut.blk; kb < lut.nb && kb * lut.blk < k0 + BN; ++kb) {
          if (!lrow[kb]) continue;
          const int lo = max(kb * lut.blk - k0, 0), hi = min((kb + 1) * lut.blk - k0, BN);
          allow |= (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1)) << lo;
        }
        if (allow != ~0ull) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rel = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              if (!((allow >> rel) & 1ull)) s[t][r] = -INFINITY;
            }
        }
      }
      // ---------------- masking (causal diagonal / ragged key tail)
      const bool need_mask = (CAUSAL && k0 + BN - 1 > q0w) || (k0 + BN > Skv);
      if (need_mask) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= Skv || (CAUSAL && key > qrow_lane)) s[t][r] = -INFINITY;
          }
      }
      // ---------------- online softmax (row = this lane's query; partner lane^32 holds the other 32 keys)
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = fast_exp2((m_run - m_use) * c);
      const float mc = m_use * c;
      float psum = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(s[t][r], c, -mc));
          s[t][r] = p;
          psum += p;
        }
      l_run = l_run * alpha + psum;
      m_run = m_new;
      // ---------------- rescale O rows (alpha lives on the lane of its row; O rows live in registers)
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
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= a4[r];
        __builtin_amdgcn_wave_barrier();
      }
      // ---------------- O += P . V  (P straight from the score registers; V via transposed LDS reads)
      bf16x8_t pa[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int e = 0; e < 8; ++e) pa[t][ss][e] = (bf16)s[t][8 * ss + e];
      const int gq = (lane >> 2) & 3;        // row within the 4-row block this lane addresses
      const int gch = (lane >> 1) & 1;       // chunk within the 16-column group
      const int gb = 8 * (lane & 1);         // byte within the chunk
      const int colhalf = (lane >> 4) & 1;   // which 16 columns of the 32-column tile
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int rb = t * 32 + 16 * ss + 4 * h;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(Vt + lds_off(rb + gq, ch0) + gb));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(Vt + lds_off(rb + 8 + gq, ch0) + gb));
            s16x8 vv;
#pragma unroll
            for (int e = 0; e < 4; ++e) { vv[e] = lo[e]; vv[4 + e] = hi[e]; }
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[t][ss], __builtin_bit_cast(bf16x8_t, vv), o[dt], 0,
                                                           0, 0);
          }
      }
    }
    if (j + 1 < nt) stage_store(cur ^ 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue: O / l, LSE
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
  bf16* Op = O + b * osb + hq * osh;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = q0w + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (q < S) {
      bf16* orow = Op + (int64_t)q * oss + l32;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) orow[dt * 32] = (bf16)(o[dt][r] * iv[r]);
    }
  }
  if (LSE != nullptr && lane < 32 && qrow_lane < S) {
    LSE[((int64_t)b * Hq + hq) * S + qrow_lane] =
        l_tot > 0.f ? (m_run * c + __log2f(l_tot)) * 0.69314718055994531f : INFINITY;
  }
  (void)scale;
}

template <bool C, bool SP>
int launch(const bf16* q, const bf16* k, const bf16* v, bf16* o, float* lse, int B, int Hq, int Hk, int S, int Skv,
           const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os, float scale, hipStream_t st,
           SparseLut lut = SparseLut{nullptr, nullptr, nullptr, nullptr, 0, 1, 0, 1}) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&flash_fwd_kernel<C, SP>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr = true;
  }
  const int nqb = (S + BM - 1) / BM;
  const int grid = nqb * B * Hq;
  const float c = scale * 1.4426950408889634f;
  hipLaunchKernelGGL((flash_fwd_kernel<C, SP>), dim3(grid), dim3(NTHR), LDS_BYTES, st, q, k, v, o, lse, B, Hq, Hk, S,
                     Skv, qs[0], qs[1], qs[2], ks[0], ks[1], ks[2], vs[0], vs[1], vs[2], os[0], os[1], os[2], c, scale,
                     lut);
  DS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// q [B,Hq,S,128], k/v [B,Hk,Skv,128] (bf16, unit last stride, any outer strides), o [B,Hq,S,128] (any outer strides),
// lse [B,Hq,S] fp32 (optional). strides are (batch, head, seq) in elements. Top-left causal alignment (SDPA's).
extern "C" int ds_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Hq, int Hk,
                            int S, int Skv, const int64_t* qs, const int64_t* ks, const int64_t* vs,
                            const int64_t* os, float scale, int causal, hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || S <= 0 || Skv <= 0) return (int)hipErrorInvalidValue;
  auto q_ = (const bf16*)q;
  auto k_ = (const bf16*)k;
  auto v_ = (const bf16*)v;
  auto o_ = (bf16*)o;
  return causal ? launch<true, false>(q_, k_, v_, o_, lse, B, Hq, Hk, S, Skv, qs, ks, vs, os, scale, st)
                : launch<false, false>(q_, k_, v_, o_, lse, B, Hq, Hk, S, Skv, qs, ks, vs, os, scale, st);
}

// Block-sparse forward: same tensors as ds_flash_fwd (non-causal; causality, if wanted, is part of the layout) plus
// the LUT described at SparseLut. lay_heads is 1 (shared layout) or Hq. Requires S == Skv.
extern "C" int ds_flash_fwd_sparse(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Hq,
                                   int Hk, int S, const int64_t* qs, const int64_t* ks, const int64_t* vs,
                                   const int64_t* os, float scale, const int* tiles, const int* ntiles,
                                   const int* qorder, const uint8_t* layout, int max_tiles, int lay_heads, int nb,
                                   int blk, hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || S <= 0 || blk <= 0 || nb * blk < S || max_tiles < 0 ||
      (lay_heads != 1 && lay_heads != Hq) || tiles == nullptr || ntiles == nullptr || qorder == nullptr ||
      layout == nullptr)
    return (int)hipErrorInvalidValue;
  return launch<false, true>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, B, Hq, Hk, S, S, qs, ks,
                             vs, os, scale, st,
                             SparseLut{tiles, ntiles, qorder, layout, max_tiles, lay_heads, nb, blk});
}
