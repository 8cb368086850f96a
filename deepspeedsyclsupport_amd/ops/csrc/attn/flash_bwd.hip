// CDNA4 flash-attention backward (training), bf16, head dim 128, GQA-native, causal / full / block-sparse.
//
// Reference counterparts: the training attention backward of the BERT kernel (`csrc/transformer/softmax_kernels.cu:
// 443-592` softmax backward + the strided-batched dQ/dK/dV GEMMs of `csrc/transformer/ds_transformer_cuda.cpp:302+`)
// and the block-sparse Triton backward (`deepspeed/ops/sparse_attention/matmul.py:605` DSD/SDD transposes,
// `softmax.py:213`). Both materialise the [B,H,S,S] probabilities; this kernel recomputes them from the forward's
// natural-log LSE instead (FlashAttention-2 style), laid out for gfx950:
//
//  * one workgroup = 8 waves = 256 keys of one (batch, kv head); wave w owns keys 32w..32w+31 and keeps dK^T and dV^T
//    of its keys (2 x 4 x 32x32 fp32 tiles = 128 accumulator registers) while the workgroup sweeps every query head of
//    the kv group (GQA: no repeat_interleave, no dK/dV reduction afterwards) x every 32-row query tile;
//  * "key on the lane": S = Q.K^T and dP = dO.V^T put the key on the MFMA column, so their accumulators are already
//    the B operands of dV^T += dO^T.P and dK^T += Q^T.dS (accumulator-as-operand, no LDS round trip); the query-side
//    A operands of those two products come from the same LDS image of the Q / dO tile through the hardware transposed
//    read `ds_read_b64_tr_b16`; the image is XOR-swizzled so row reads (S, dP) and transposed reads are conflict-free;
//  * dP's accumulator starts at -delta (delta = rowsum(dO*O), one preprocessing pass), so dS = P*(dP-delta) is one
//    multiply; P = exp2(S*c - LSE*log2e) needs no row max;
//  * dS crosses LDS once (dS^T image, 64-B rows, 8-B units swizzled by key so the packed stores of 8 rows and the
//    transposed reads are both conflict-free); waves 0..3 then compute the 32x128 dQ tile over all 256 keys
//    (A = dS by transposed read, B = K by transposed read of the resident K image) and add it with packed-row f32
//    atomics (one 32x32 accumulator register = two 128-B row segments = the full-rate atomic shape); waves 4..7 run
//    ahead into the next tile, so the two waves on a SIMD keep its matrix core busy across the dQ phase;
//  * one barrier per tile: the next Q / dO tile is fetched into registers before the current tile's MFMAs and written
//    to the other LDS buffer after them (double-buffered Q/dO and dS images);
//  * causal: waves whose 32 keys lie entirely above a tile skip it, the dQ product stops at the diagonal, workgroups
//    with the most tiles (low key blocks) start first, and each (batch, kv head)'s key blocks share an XCD (Q / dO
//    reuse in L2);
//  * block-sparse: each workgroup walks only the 32-row query tiles its key block meets in the layout (a host-built
//    column LUT) and masks at the layout's block granularity (16/32/64/128) — cost scales with the layout density.
#include "ds_hip.h"

namespace {

constexpr int D = 128;
constexpr int NW = 8;                  // waves per workgroup
constexpr int NTHR = NW * 64;
constexpr int KB = 32 * NW;            // keys per workgroup
constexpr int QT = 32;                 // query rows per tile
constexpr int TILE = QT * D * 2;       // 8 KB: one Q or dO tile
constexpr int K_BYTES = KB * 256;      // resident K image
constexpr int DS_BYTES = KB * 64;      // dS^T image [KB keys][32 q] bf16
constexpr int LDS_BYTES = K_BYTES + 4 * TILE + 2 * DS_BYTES + 2 * 64 * 4 + 2 * NW;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

// 256-B rows of 16 x 16-B chunks, chunk XOR-swizzled by row mod 16 (same image as flash_fwd.hip): conflict-free for
// 32-row b128 reads of one chunk and for 4-row transposed reads.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
// dS^T image: 64-B rows (32 queries), 8-B unit u (4 queries) XOR-swizzled by (key >> 1) & 7 so that 16 lanes storing
// one unit of 16 consecutive keys hit 32 distinct banks.
__device__ __forceinline__ int ds_off(int key, int u) { return key * 64 + 8 * (u ^ ((key >> 1) & 7)); }

// row of a 32x32 accumulator register r for lane half h
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ s16x4_t tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t join(s16x4_t lo, s16x4_t hi) {
  s16x8 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[4 + e] = hi[e]; }
  return __builtin_bit_cast(bf16x8_t, v);
}

struct BwdArgs {
  const bf16 *q, *k, *v, *dout;
  const float *lse, *delta;
  float* dqacc;  // [B, Hq, S, 128] fp32, pre-zeroed
  bf16 *dk, *dv;
  int B, Hq, Hk, S;
  int64_t qsb, qsh, qss, ksb, ksh, kss, vsb, vsh, vss, osb, osh, oss, dksb, dksh, dkss, dvsb, dvsh, dvss;
  float c;      // softmax scale * log2(e)
  float scale;
  // block-sparse column LUT: qtiles [Hk, nkb, maxt] = (query head within the kv group << 16 | 32-row query tile)
  // for every tile key block kb meets, nqt [Hk, nkb] = list lengths; layout [LH, nb, nb] uint8 at granularity blk
  const int* qtiles;
  const int* nqt;
  const uint8_t* layout;
  int maxt, lay_heads, nb, blk;
};

template <bool CAUSAL, bool SPARSE>
__global__ void __launch_bounds__(NTHR, 1) flash_bwd_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int S = a.S;
  const int nkb = (S + KB - 1) / KB;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kb = logical % nkb;  // causal: low key blocks (most tiles) first within a head
  const int b = bh / a.Hk, hk = bh % a.Hk, rep = a.Hq / a.Hk;
  const int k0 = kb * KB;
  const int ntq = (S + QT - 1) / QT;

  char* Kimg = smem;
  char* QD = smem + K_BYTES;               // [buf][Q tile | dO tile]
  char* DSimg = QD + 4 * TILE;             // [buf][KB][32] bf16
  float* LD = reinterpret_cast<float*>(DSimg + 2 * DS_BYTES);  // [buf][lse/scale (32) | delta (32)]
  uint8_t* FL = reinterpret_cast<uint8_t*>(LD + 2 * 64);            // [buf][wave]: slab met the tile

  const bf16* Kp = a.k + b * a.ksb + hk * a.ksh;
  const bf16* Vp = a.v + b * a.vsb + hk * a.vsh;

  // ------------------------------------------------------------------ iteration space: (query head, query tile)
  const int t0 = CAUSAL ? k0 / QT : 0;
  const int per_head_dense = ntq - t0;
  int n_it = rep * per_head_dense;
  const int* lut = nullptr;
  if constexpr (SPARSE) {
    lut = a.qtiles + ((int64_t)hk * nkb + kb) * a.maxt;
    n_it = a.nqt[hk * nkb + kb];
  }
  // it -> (query head, query tile); the sparse LUT lists (head-in-group << 16 | tile) per (kv head, key block)
  auto tile_at = [&](int it, int& hq, int& qt) {
    if constexpr (SPARSE) {
      const int code = lut[it];
      hq = hk * rep + (code >> 16);
      qt = code & 0xffff;
    } else {
      hq = hk * rep + it / per_head_dense;
      qt = t0 + it % per_head_dense;
    }
  };

  // ------------------------------------------------------------------ staging of one (Q, dO, lse, delta) tile
  // thread t moves 16-B chunk t of the Q tile and of the dO tile (32 rows x 16 chunks = 512 each)
  u32x4_t qreg, oreg;
  float lreg = 0.f;
  const float inv_scale = 1.f / a.scale;
  const int srow = tid >> 4, sch = tid & 15;
  auto stage_load = [&](int it) {
    int hq, qt;
    tile_at(it, hq, qt);
    const int qrow = qt * QT + srow;
    const int qr = min(qrow, S - 1);
    qreg = *reinterpret_cast<const u32x4_t*>(a.q + b * a.qsb + hq * a.qsh + (int64_t)qr * a.qss + sch * 8);
    oreg = *reinterpret_cast<const u32x4_t*>(a.dout + b * a.osb + hq * a.osh + (int64_t)qr * a.oss + sch * 8);
    if (tid < 64) {
      const int r = qt * QT + (tid & 31);
      const int64_t idx = ((int64_t)b * a.Hq + hq) * S + min(r, S - 1);
      if (tid < 32)
        lreg = r < S ? a.lse[idx] * inv_scale : INFINITY;  // S starts at -LSE/scale; p = 0 on padded rows
      else
        lreg = r < S ? a.delta[idx] : 0.f;
    }
  };
  auto stage_store = [&](int buf) {
    *reinterpret_cast<u32x4_t*>(QD + buf * 2 * TILE + lds_off(srow, sch)) = qreg;
    *reinterpret_cast<u32x4_t*>(QD + buf * 2 * TILE + TILE + lds_off(srow, sch)) = oreg;
    if (tid < 64) LD[buf * 64 + tid] = lreg;
  };

  // ------------------------------------------------------------------ resident K image + per-wave K / V fragments
  for (int i = tid; i < KB * 16; i += NTHR) {
    const int row = i >> 4, ch = i & 15;
    const int key = min(k0 + row, S - 1);
    *reinterpret_cast<u32x4_t*>(Kimg + lds_off(row, ch)) =
        *reinterpret_cast<const u32x4_t*>(Kp + (int64_t)key * a.kss + ch * 8);
  }
  const int kw0 = k0 + 32 * w;        // first key of this wave
  const int mykey = kw0 + l32;        // this lane's key (column of S / dP)
  // V rows stay in registers (B operand of dP); K rows are read from the resident image (it also feeds dQ)
  bf16x8_t vf[8];
  {
    const int kr = min(mykey, S - 1);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
      vf[kk] = *reinterpret_cast<const bf16x8_t*>(Vp + (int64_t)kr * a.vss + 16 * kk + 8 * h);
  }

  f32x16_t dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[dt][r] = dv[dt][r] = 0.f;

  if (n_it > 0) {
    stage_load(0);
    stage_store(0);
  }
  __syncthreads();

  for (int it = 0; it < n_it; ++it) {
    const int cur = it & 1;
    // Lane-derived LDS offsets are recomputed every tile from a laundered lane id: hoisted out of the loop they cost
    // ~40 registers, which at 2 waves per SIMD is the difference between spilling and not.
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int h = ln >> 5, l32 = ln & 31;
    // transposed-read lane geometry (see flash_fwd.hip): lane reads row rb + gq, 16-B chunk c0 + 2*colhalf + gch,
    // byte gb; it receives rows rb..rb+3 of column (lane & 31) of the addressed 32-column slab
    const int gq = (ln >> 2) & 3, gch = (ln >> 1) & 1, gb = 8 * (ln & 1), colhalf = (ln >> 4) & 1;
    const int ds_unit = 4 * colhalf + 2 * gch + (ln & 1);
    int hq, qt;
    tile_at(it, hq, qt);
    const int q0 = qt * QT;
    if (it + 1 < n_it) stage_load(it + 1);

    const char* Qt = QD + cur * 2 * TILE;
    const char* Ot = Qt + TILE;
    const float* lse2 = LD + cur * 64;
    const float* dlt = lse2 + 32;
    char* DSc = DSimg + cur * DS_BYTES;

    // ---------------- does this wave's 32-key slab meet the tile? keep = bit r set if accumulator row r is unmasked
    bool active = kw0 < S;
    if (CAUSAL) active = active && kw0 <= q0 + QT - 1;
    unsigned keep = mykey < S ? 0xffffu : 0u;
    if constexpr (SPARSE) {
      const int lh = a.lay_heads == 1 ? 0 : hq;
      const int kbl = min(mykey, S - 1) / a.blk;
      const uint8_t* lay = a.layout + (int64_t)lh * a.nb * a.nb;
      const int r0 = q0 / a.blk;
      const unsigned a0 = lay[(int64_t)r0 * a.nb + kbl] ? 0xffffu : 0u;
      if (a.blk < QT) {  // 16-row blocks: registers 0..7 are rows 0..15 of the tile, 8..15 rows 16..31
        const unsigned a1 = lay[(int64_t)min(r0 + 1, a.nb - 1) * a.nb + kbl] ? 0xffffu : 0u;
        keep &= (a0 & 0x00ffu) | (a1 & 0xff00u);
      } else {
        keep &= a0;
      }
      active = active && __any(keep != 0);
    }
    if (active) {
      // ---------------- S' = Q.K^T - LSE/scale and dP' = dO.V^T - delta (query rows in registers, key on the
      // lane); the row constants are the accumulators' initial values
      f32x16_t s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(lse2 + 8 * g + 4 * h);
        const f32x4 y = *reinterpret_cast<const f32x4*>(dlt + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s[4 * g + i] = -x[i]; dp[4 * g + i] = -y[i]; }
      }
      const char* Kw = Kimg + 32 * w * 256;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const bf16x8_t qa = *reinterpret_cast<const bf16x8_t*>(Qt + lds_off(l32, 2 * kk + h));
        const bf16x8_t kb_ = *reinterpret_cast<const bf16x8_t*>(Kw + lds_off(l32, 2 * kk + h));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kb_, s, 0, 0, 0);
      }
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const bf16x8_t oa = *reinterpret_cast<const bf16x8_t*>(Ot + lds_off(l32, 2 * kk + h));
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa, vf[kk], dp, 0, 0, 0);
      }
      // ---------------- P and dS
      const bool need_mask = keep != 0xffffu || (CAUSAL && kw0 + 31 > q0);
      if (CAUSAL && need_mask) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (mykey > q0 + crow(r, h)) keep &= ~(1u << r);
      }
      bf16x8_t pb[2], dsb[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __builtin_amdgcn_exp2f(s[r] * a.c);
        if (need_mask && !((keep >> r) & 1u)) p = 0.f;
        pb[r >> 3][r & 7] = (bf16)p;
        dsb[r >> 3][r & 7] = (bf16)(p * dp[r]);
      }
      // ---------------- dS^T -> LDS (row = key, 8-B unit g*2+h holds queries 8g+4h .. +3)
      {
        const int kr = 32 * w + l32;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          // whole-vector bit cast: per-element __builtin_bit_cast(short, bf16 element) is miscompiled by hipcc
          // (ROCm 7.2) into a splat of one element (tools/probe_flash_bwd2.py)
          const s16x8 d8 = __builtin_bit_cast(s16x8, dsb[g >> 1]);
          s16x4 v4;
#pragma unroll
          for (int i = 0; i < 4; ++i) v4[i] = d8[4 * (g & 1) + i];
          *reinterpret_cast<s16x4*>(DSc + ds_off(kr, 2 * g + h)) = v4;
        }
      }
      // ---------------- dV^T += dO^T.P, dK^T += Q^T.dS   (A operands by transposed reads of the tile images)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int rb = 16 * s2 + 4 * h;
          const bf16x8_t oT = join(tr_read(Ot + lds_off(rb + gq, ch0) + gb), tr_read(Ot + lds_off(rb + 8 + gq, ch0) + gb));
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oT, pb[s2], dv[dt], 0, 0, 0);
          const bf16x8_t qT = join(tr_read(Qt + lds_off(rb + gq, ch0) + gb), tr_read(Qt + lds_off(rb + 8 + gq, ch0) + gb));
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qT, dsb[s2], dk[dt], 0, 0, 0);
        }
        // bound the operand prefetch window (register budget: 2 waves per SIMD)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the dQ product walks only the slabs that met this tile
    if (lane == 0) FL[cur * NW + w] = active ? 1 : 0;

    if (it + 1 < n_it) stage_store(cur ^ 1);
    __syncthreads();

    // ---------------- dQ[q0:q0+32, 32w:32w+32] += dS . K   (waves 0..3; keys up to the diagonal)
    if (w < 4) {
      const uint64_t fl = *reinterpret_cast<const uint64_t*>(FL + cur * NW);
      const uint32_t flo = __builtin_amdgcn_readfirstlane((uint32_t)fl), fhi = __builtin_amdgcn_readfirstlane((uint32_t)(fl >> 32));
      f32x16_t dq;
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[r] = 0.f;
      int nks = 0;
      const int ch0 = w * 4 + colhalf * 2 + gch;
      for (int slab = 0; slab < NW; ++slab) {
        if (!(((slab < 4 ? flo : fhi) >> (8 * (slab & 3))) & 0xff)) continue;
#pragma unroll
        for (int s2 = 2 * slab; s2 < 2 * slab + 2; ++s2) {
          const int rb = 16 * s2 + 8 * h;
          const bf16x8_t dsa = join(tr_read(DSc + ds_off(rb + gq, ds_unit)), tr_read(DSc + ds_off(rb + 4 + gq, ds_unit)));
          const bf16x8_t kb_ = join(tr_read(Kimg + lds_off(rb + gq, ch0) + gb), tr_read(Kimg + lds_off(rb + 4 + gq, ch0) + gb));
          dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dsa, kb_, dq, 0, 0, 0);
        }
        ++nks;
      }
      if (nks > 0) {
        float* dqp = a.dqacc + (((int64_t)b * a.Hq + hq) * S + q0) * D + 32 * w + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = crow(r, h);
          if (q0 + qr < S) unsafeAtomicAdd(dqp + (int64_t)qr * D, dq[r]);
        }
      }
    }
  }

  // ------------------------------------------------------------------ epilogue: dK = scale * dK^T^T, dV
  if (mykey < S) {
    bf16* dkp = a.dk + b * a.dksb + hk * a.dksh + (int64_t)mykey * a.dkss;
    bf16* dvp = a.dv + b * a.dvsb + hk * a.dvsh + (int64_t)mykey * a.dvss;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 k4, v4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          k4[i] = (bf16)(dk[dt][4 * g + i] * a.scale);
          v4[i] = (bf16)dv[dt][4 * g + i];
        }
        const int d0 = 32 * dt + 8 * g + 4 * h;
        *reinterpret_cast<bf16x4*>(dkp + d0) = k4;
        *reinterpret_cast<bf16x4*>(dvp + d0) = v4;
      }
  }
}

// delta[b,h,q] = sum_d O*dO (fp32), and zero the dQ accumulator row. 16 threads per row, 8 elements each.
__global__ void __launch_bounds__(256) flash_bwd_pre_kernel(const bf16* __restrict__ O, const bf16* __restrict__ dO,
                                                            float* __restrict__ delta, float* __restrict__ dqacc,
                                                            int Hq, int S, int64_t rows, int64_t osb, int64_t osh,
                                                            int64_t oss, int64_t gsb, int64_t gsh, int64_t gss) {
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  if (row >= rows) return;
  const int q = (int)(row % S);
  const int64_t bh = row / S;
  const int hh = (int)(bh % Hq);
  const int64_t bb = bh / Hq;
  const bf16x8 o = *reinterpret_cast<const bf16x8*>(O + bb * osb + hh * osh + (int64_t)q * oss + sub * 8);
  const bf16x8 g = *reinterpret_cast<const bf16x8*>(dO + bb * gsb + hh * gsh + (int64_t)q * gss + sub * 8);
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc = fmaf((float)o[i], (float)g[i], acc);
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (sub == 0) delta[row] = acc;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  *reinterpret_cast<f32x4*>(dqacc + row * D + sub * 8) = z;
  *reinterpret_cast<f32x4*>(dqacc + row * D + sub * 8 + 4) = z;
}

// dq = bf16(scale * dqacc), any [B,H,S,D] output strides
__global__ void __launch_bounds__(256) flash_bwd_post_kernel(const float* __restrict__ dqacc, bf16* __restrict__ dq,
                                                             int Hq, int S, int64_t rows, int64_t sb, int64_t sh,
                                                             int64_t ss, float scale) {
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  if (row >= rows) return;
  const int q = (int)(row % S);
  const int64_t bh = row / S;
  const int hh = (int)(bh % Hq);
  const int64_t bb = bh / Hq;
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(dqacc + row * D + sub * 8);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(dqacc + row * D + sub * 8 + 4);
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = (bf16)(x0[i] * scale);
    r[4 + i] = (bf16)(x1[i] * scale);
  }
  *reinterpret_cast<bf16x8*>(dq + bb * sb + hh * sh + (int64_t)q * ss + sub * 8) = r;
}

template <bool C, bool SP>
int launch_main(const BwdArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&flash_bwd_kernel<C, SP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr = true;
  }
  const int nkb = (a.S + KB - 1) / KB;
  const int grid = a.B * a.Hk * nkb;
  hipLaunchKernelGGL((flash_bwd_kernel<C, SP>), dim3(grid), dim3(NTHR), LDS_BYTES, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// Strides are (batch, head, seq) in elements, unit last stride everywhere, all bf16 rows 16-B aligned.
// q/o/dout/dq [B,Hq,S,128], k/v/dk/dv [B,Hk,S,128], lse [B,Hq,S] natural-log (flash_fwd's), workspace:
// delta [B*Hq*S] fp32 and dqacc [B*Hq*S*128] fp32. mode: 0 full, 1 causal (top-left), 2 block-sparse (LUT below).
extern "C" int ds_flash_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, float* delta, float* dqacc, void* dq, void* dk, void* dv, int B, int Hq,
                            int Hk, int S, const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os,
                            const int64_t* dos, const int64_t* dqs, const int64_t* dks, const int64_t* dvs,
                            float scale, int mode, const int* qtiles, const int* nqt, const uint8_t* layout, int maxt,
                            int lay_heads, int nb, int blk, hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || S <= 0 || B <= 0) return (int)hipErrorInvalidValue;
  if (mode == 2 && (qtiles == nullptr || nqt == nullptr || layout == nullptr || (lay_heads != 1 && lay_heads != Hq) ||
                    (blk != 16 && blk != 32 && blk != 64 && blk != 128) || nb * blk < S))
    return (int)hipErrorInvalidValue;
  const int64_t rows = (int64_t)B * Hq * S;
  const int pgrid = (int)((rows + 15) / 16);
  hipLaunchKernelGGL(flash_bwd_pre_kernel, dim3(pgrid), dim3(256), 0, st, (const bf16*)o, (const bf16*)dout, delta,
                     dqacc, Hq, S, rows, os[0], os[1], os[2], dos[0], dos[1], dos[2]);
  DS_CHECK_LAUNCH();
  BwdArgs a;
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.dout = (const bf16*)dout;
  a.lse = lse; a.delta = delta; a.dqacc = dqacc; a.dk = (bf16*)dk; a.dv = (bf16*)dv;
  a.B = B; a.Hq = Hq; a.Hk = Hk; a.S = S;
  a.qsb = qs[0]; a.qsh = qs[1]; a.qss = qs[2];
  a.ksb = ks[0]; a.ksh = ks[1]; a.kss = ks[2];
  a.vsb = vs[0]; a.vsh = vs[1]; a.vss = vs[2];
  a.osb = dos[0]; a.osh = dos[1]; a.oss = dos[2];
  a.dksb = dks[0]; a.dksh = dks[1]; a.dkss = dks[2];
  a.dvsb = dvs[0]; a.dvsh = dvs[1]; a.dvss = dvs[2];
  a.c = scale * 1.4426950408889634f;
  a.scale = scale;
  a.qtiles = qtiles; a.nqt = nqt; a.layout = layout; a.maxt = maxt; a.lay_heads = lay_heads; a.nb = nb; a.blk = blk;
  int rc = mode == 1 ? launch_main<true, false>(a, st)
                     : (mode == 2 ? launch_main<false, true>(a, st) : launch_main<false, false>(a, st));
  if (rc) return rc;
  hipLaunchKernelGGL(flash_bwd_post_kernel, dim3(pgrid), dim3(256), 0, st, dqacc, (bf16*)dq, Hq, S, rows, dqs[0],
                     dqs[1], dqs[2], scale);
  DS_CHECK_LAUNCH();
  return 0;
}
