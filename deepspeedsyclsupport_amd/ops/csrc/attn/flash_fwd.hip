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

#include <type_traits>

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

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
typedef __attribute__((address_space(3))) bf16x8_t lds_bf16x8;

// LDS-DMA: every lane fetches 16 bytes from its own global address; they land at lds_base + 16 * lane. Issued from
// inline asm on purpose: hipcc tracks its own global_load_lds builtins and then waits vmcnt(0) before every LDS read it
// cannot prove disjoint from the DMA target, draining the prefetch. Out of its sight the DMA is ordered only by the
// `s_waitcnt vmcnt(0)` + barrier at the end of each tile (see flash_bwd.hip for the same idiom).
__device__ __forceinline__ void glds16(const void* g, const char* lds_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_char*)lds_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}
// same with a wave-uniform 64-bit base (scalar registers) and a 32-bit per-lane byte offset
__device__ __forceinline__ void glds16_s(const char* base, uint32_t voff, const char* lds_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_char*)lds_base);
  const uint64_t sb = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  const uint64_t ub = ((uint64_t)hi << 32) | lo;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(ub), "s"(dst)
               : "memory");
}

// byte offset of 16-B chunk `ch` (0..15) of row `row` in a [64][128 x bf16] tile: 256-B rows, chunk index XORed with
// a bijection of row mod 16 so both the row reads (32 consecutive rows, one chunk) and the 4-row transposed reads
// touch distinct banks.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
constexpr float RESCALE_LOG2 = 8.f;

// two fp32 -> one dword of two bf16 (round to nearest even), lo in bits 0..15
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// block-sparse LUT: tiles [lay_heads, nqb, max_tiles] (ascending 64-key tile ids), ntiles [lay_heads, nqb],
// layout [lay_heads, nb, nb] (uint8, block granularity blk)
struct SparseLut {
  const int* tiles;
  const int* ntiles;
  const int* qorder;  // [lay_heads, nqb] query blocks by descending tile count
  const uint8_t* layout;
  int max_tiles, lay_heads, nb, blk;
  // additive biases on the scaled scores (reference `ops/sparse_attention/softmax.py:37-70`: key-padding mask,
  // attention mask and relative position embedding are applied inside the sparse softmax); any may be null
  const float* kbias;      // [B, Skv] per-key (key_padding_mask in additive form), row stride kb_stride
  const float* abias;      // [S, Skv] shared by batch and heads (attn_mask in additive form), row stride ab_stride
  const float* rpe;        // [H or 1, S, Skv] per head, head stride rpe_hs (0 = shared), row stride rpe_rs
  int64_t kb_stride, ab_stride, rpe_hs, rpe_rs;
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
  const lds_char* s3 = (const lds_char*)smem;  // 32-bit LDS addressing: per-lane base + compile-time displacement

  // ------------------------------------------------------------------ K/V staging by LDS-DMA
  // A 64-key tile of K (or V) is sixteen 1-KB pieces (4 rows each); wave w moves pieces w, w+4, w+8, w+12 of both
  // with `global_load_lds_dwordx4`: no staging registers, no ds_write, and the transfer of tile j+1 runs under the
  // MFMAs of tile j. Lane L of piece p lands at physical chunk L%16 of row 4p + L/16, so it fetches the logical
  // chunk (L%16) ^ swizzle(row) — the image's XOR swizzle goes on the SOURCE address. The row's low four bits
  // (4w + L/16) do not depend on the piece, so one 32-bit byte offset per lane serves all pieces of all tiles; the
  // tile / piece part of the address is wave-uniform (scalar base). Only a ragged last tile builds clamped
  // per-lane addresses.
  const int drow = 4 * wid + (lane >> 4);
  const int dch = (lane & 15) ^ (((drow & 3) << 2) | ((drow >> 2) & 3));
  const uint32_t kdma = (uint32_t)((drow * kss + dch * 8) * 2);
  const uint32_t vdma = (uint32_t)((drow * vss + dch * 8) * 2);
  auto dma_tile = [&](int tile, int buf) {
    if (tile * BN + BN <= Skv) {
      const char* kb = reinterpret_cast<const char*>(Kp + (int64_t)tile * BN * kss);
      const char* vb = reinterpret_cast<const char*>(Vp + (int64_t)tile * BN * vss);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        glds16_s(kb + (int64_t)32 * i * kss, kdma, smem + buf * TILE_BYTES + 1024 * (wid + 4 * i));
        glds16_s(vb + (int64_t)32 * i * vss, vdma, smem + (2 + buf) * TILE_BYTES + 1024 * (wid + 4 * i));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = min(tile * BN + 16 * i + drow, Skv - 1);
        glds16(Kp + (int64_t)key * kss + dch * 8, smem + buf * TILE_BYTES + 1024 * (wid + 4 * i));
        glds16(Vp + (int64_t)key * vss + dch * 8, smem + (2 + buf) * TILE_BYTES + 1024 * (wid + 4 * i));
      }
    }
  };
  // every wave: its own DMA pieces have landed (vmcnt) and its LDS reads are done (lgkmcnt), then the barrier
  auto tile_barrier = [&]() { asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  // ------------------------------------------------------------------ per-lane LDS read addresses
  // K row reads: lds_off(32t + l32, 2kk + h) = kaddr[kk] + 8192 t; V transposed reads (lane geometry of
  // ds_read_b64_tr_b16: lane reads row rb + gq, 16-B chunk 4dt + 2 colhalf + gch, byte gb):
  // lds_off(32t + 16ss + 4h + 8hi + gq, ...) + gb = vaddr[hi][dt] + 256 (32t + 16ss). The XOR swizzle only involves
  // the row's low four bits, so tile half, k-step and buffer are compile-time displacements (the ds offset field).
  const int gq = (lane >> 2) & 3, gch = (lane >> 1) & 1, gb = 8 * (lane & 1), colhalf = (lane >> 4) & 1;
  uint32_t kaddr[8], vaddr[2][4];
  {
    const int f = ((l32 & 3) << 2) | ((l32 >> 2) & 3);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) kaddr[kk] = (uint32_t)(l32 * 256 + 16 * ((2 * kk + h) ^ f));
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int row = 4 * h + 8 * hi + gq, g = ((row & 3) << 2) | ((row >> 2) & 3);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        vaddr[hi][dt] = (uint32_t)(2 * TILE_BYTES + row * 256 + 16 * ((dt * 4 + colhalf * 2 + gch) ^ g) + gb);
    }
  }

  f32x16_t o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float rescale_thr = RESCALE_LOG2 / c;  // in raw score units
  const int qrow_lane = q0w + l32;  // the query row this lane's scores belong to

  // the Q fragments are the only loads hipcc tracks: retire them before the first DMA so its own counted waits
  // never have to look past transfers it does not know about
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) asm volatile("" : : "v"(qf[kk]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nt > 0) dma_tile(tile_of(0), 0);  // uniform per workgroup (a sparse row block may have no tiles)
  tile_barrier();

  // one tile; `cur` (the LDS buffer) is a compile-time constant so it folds into the displacements
  auto tile_step = [&](int j, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (j + 1 < nt) dma_tile(tile_of(j + 1), cur ^ 1);
    const int k0 = tile_of(j) * BN;
    const bool active = !CAUSAL || k0 <= q0w + 31;
    if (active) {
      // ---------------- S^T = K . Q^T  (two 32-key halves), K fragments read three MFMAs ahead: left to itself
      // hipcc issued each ds_read right before its MFMA and waited lgkmcnt(0) in between, so every MFMA paid a
      // full LDS round trip. The order is pinned with sched_barrier (VALU and SALU may cross, MFMA / LDS may not).
      auto ldk = [&](int i) {
        return *reinterpret_cast<const lds_bf16x8*>(s3 + kaddr[i & 7] + (cur * TILE_BYTES + (i >> 3) * 8192));
      };
      f32x16_t s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t][r] = 0.f;
      {
        bf16x8_t k0f = ldk(0), k1f = ldk(1), k2f = ldk(2);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          bf16x8_t k3f;
          if (i + 3 < 16) k3f = ldk(i + 3);
          __builtin_amdgcn_sched_barrier(0x6);
          s[i >> 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0f, qf[i & 7], s[i >> 3], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0x6);
          k0f = k1f;
          k1f = k2f;
          k2f = k3f;
        }
      }
      // V operand i = (dt, t, ss): both transposed reads of the 16-key x 32-column slab; the first two are issued
      // here so they fly under the softmax arithmetic
      auto ldv = [&](int i) {
        const int dt = i >> 2, t = (i >> 1) & 1, ss = i & 1;
        const int disp = cur * TILE_BYTES + (t * 32 + 16 * ss) * 256;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s3 + vaddr[0][dt] + disp));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s3 + vaddr[1][dt] + disp));
        s16x8 vv;
#pragma unroll
        for (int e = 0; e < 4; ++e) { vv[e] = lo[e]; vv[4 + e] = hi[e]; }
        return __builtin_bit_cast(bf16x8_t, vv);
      };
      bf16x8_t v0f = ldv(0), v1f = ldv(1);
      // ---------------- additive biases (key padding / attention mask / relative position), in raw score units
      // (bias / scale), then the block-sparse mask at the layout's granularity (this lane's query row vs the 64 keys)
      if constexpr (SPARSE) {
        if (lut.kbias != nullptr || lut.abias != nullptr || lut.rpe != nullptr) {
          const float inv_scale = 1.f / scale;
          const int qr = min(qrow_lane, S - 1);
          const float* kbp = lut.kbias ? lut.kbias + (int64_t)b * lut.kb_stride : nullptr;
          const float* abp = lut.abias ? lut.abias + (int64_t)qr * lut.ab_stride : nullptr;
          const float* rpp = lut.rpe ? lut.rpe + (int64_t)hq * lut.rpe_hs + (int64_t)qr * lut.rpe_rs : nullptr;
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int key = k0 + t * 32 + 8 * g + 4 * h;  // four consecutive keys: registers 4g .. 4g+3
              if (key + 3 < Skv) {
                f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
                if (kbp) bsum += *reinterpret_cast<const f32x4*>(kbp + key);
                if (abp) bsum += *reinterpret_cast<const f32x4*>(abp + key);
                if (rpp) bsum += *reinterpret_cast<const f32x4*>(rpp + key);
#pragma unroll
                for (int i = 0; i < 4; ++i) s[t][4 * g + i] = fmaf(bsum[i], inv_scale, s[t][4 * g + i]);
              } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  if (key + i >= Skv) continue;
                  float bv = 0.f;
                  if (kbp) bv += kbp[key + i];
                  if (abp) bv += abp[key + i];
                  if (rpp) bv += rpp[key + i];
                  s[t][4 * g + i] = fmaf(bv, inv_scale, s[t][4 * g + i]);
                }
              }
            }
        }
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
      // row max: one v_max3 per register pair (fmaxf on MFMA outputs makes hipcc canonicalise every input first)
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = max3f(mx, s[0][r], s[1][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // deferred rescale: the running reference maximum only moves when the new maximum exceeds it by more than
      // RESCALE_LOG2 in the exponent's units, so most tiles skip the rescale of O entirely; until then the
      // probabilities are at most 2^RESCALE_LOG2 (exact in fp32, in range for bf16), and l / LSE use the same
      // reference, so the result is unchanged.
      const float m_new = mx > m_run + rescale_thr ? mx : m_run;
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
      // two probabilities per v_cvt_pk_bf16_f32 (hipcc lowers an element-wise fptrunc to one convert plus a
      // v_perm per element, and the VALU issue slots are what this loop runs out of)
      bf16x8_t pa[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          u32x4_t pu;
#pragma unroll
          for (int i = 0; i < 4; ++i) pu[i] = pack_bf16(s[t][8 * ss + 2 * i], s[t][8 * ss + 2 * i + 1]);
          pa[t][ss] = __builtin_bit_cast(bf16x8_t, pu);
        }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        bf16x8_t v2f;
        if (i + 2 < 16) v2f = ldv(i + 2);
        __builtin_amdgcn_sched_barrier(0x6);
        o[i >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[(i >> 1) & 1][i & 1], v0f, o[i >> 2], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0x6);
        v0f = v1f;
        v1f = v2f;
      }
    }
    tile_barrier();
  };
  for (int j = 0; j < nt; j += 2) {
    tile_step(j, std::integral_constant<int, 0>{});
    if (j + 1 < nt) tile_step(j + 1, std::integral_constant<int, 1>{});
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
}

template <bool C, bool SP>
int launch(const bf16* q, const bf16* k, const bf16* v, bf16* o, float* lse, int B, int Hq, int Hk, int S, int Skv,
           const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os, float scale, hipStream_t st,
           SparseLut lut = SparseLut{nullptr, nullptr, nullptr, nullptr, 0, 1, 0, 1, nullptr, nullptr, nullptr, 0, 0,
                                     0, 0}) {
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
                                   int blk, const float* kbias, int64_t kb_stride, const float* abias,
                                   int64_t ab_stride, const float* rpe, int64_t rpe_hs, int64_t rpe_rs,
                                   hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || S <= 0 || blk <= 0 || nb * blk < S || max_tiles < 0 ||
      (lay_heads != 1 && lay_heads != Hq) || tiles == nullptr || ntiles == nullptr || qorder == nullptr ||
      layout == nullptr)
    return (int)hipErrorInvalidValue;
  // bias rows are read four keys at a time
  auto al = [](const float* p, int64_t st) { return p == nullptr || (((uintptr_t)p % 16) == 0 && st % 4 == 0); };
  if (!al(kbias, kb_stride) || !al(abias, ab_stride) || !al(rpe, rpe_rs) || rpe_hs % 4) return (int)hipErrorInvalidValue;
  return launch<false, true>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, B, Hq, Hk, S, S, qs, ks,
                             vs, os, scale, st,
                             SparseLut{tiles, ntiles, qorder, layout, max_tiles, lay_heads, nb, blk, kbias, abias,
                                       rpe, kb_stride, ab_stride, rpe_hs, rpe_rs});
}
