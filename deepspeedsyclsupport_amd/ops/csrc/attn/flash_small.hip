// CDNA4 flash attention for small head dims (32 / 64) with additive biases and attention dropout: forward and
// backward. Serves the DS4Science Evoformer attention and the BERT training layer.
//
// Reference counterparts (behaviour): `csrc/deepspeed4science/evoformer_attn/attention_cu.cu:12-160` +
// `attention_back.cu` (CUTLASS fMHA with a [B,N,1,1,S] per-key bias and a [B,1,H,S,S] pair bias, gradients for both)
// and the BERT layer's masked softmax + attention dropout (`csrc/transformer/softmax_kernels.cu:28-158`,
// `dropout_kernels.cu`). Neither bias nor the probability matrix is ever materialised at [batch, H, S, S].
//
// Tensors are [Z, S, H, D] with arbitrary (z, s, h) strides (Z = B*N for Evoformer, B for BERT); bias1 is indexed
// [z, key] (per-key mask bias), bias2 is [Z / b2_div, H, S, S] (pair bias shared by b2_div consecutive z).
//  * forward: one workgroup = 4 waves x 32 query rows of one (z, h); 64-key K/V tiles double-buffered in LDS (rows
//    padded to 2D + 16 bytes: conflict-free b128 row reads without a swizzle); S^T = K.Q^T on
//    v_mfma_f32_32x32x16 so each lane owns one query row's scores, biases added in natural units, online softmax,
//    P reused as the A operand of O += P.V (V by the hardware transposed read); dropout multiplies P by
//    keep / (1 - p) after the normaliser (Philox-4x32 keyed by (z, h, query, key), regenerated in the backward);
//  * backward: three atomic-free passes (dQ query-outer; dK/dV key-outer; the shared pair-bias gradient summed over
//    the z that share it in registers), P recomputed from the saved LSE in each — see the backward section.
#include "ds_hip.h"

#include <algorithm>

namespace {

constexpr int BM = 128;    // query rows per workgroup
constexpr int BN = 64;     // keys per tile
constexpr int NTHR = 256;

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

template <typename T> struct MF;
template <> struct MF<bf16> {
  typedef bf16x8_t V8;
  __device__ __forceinline__ static f32x16_t mma(V8 a, V8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MF<fp16> {
  typedef f16x8_t V8;
  __device__ __forceinline__ static f32x16_t mma(V8 a, V8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

template <int D> constexpr int RS() { return 2 * D + 16; }   // LDS row stride (bytes)
template <int D> constexpr int TILE() { return BN * RS<D>(); }

// row of accumulator register r (32x32 C layout) for lane half h
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---------------------------------------------------------------- dropout: Philox-4x32-7, 4 keep bits per call
__device__ __forceinline__ uint32_t keep4(uint64_t seed, uint64_t row, uint32_t key4, uint32_t thresh) {
  uint32_t c0 = key4, c1 = (uint32_t)row, c2 = (uint32_t)(row >> 32), c3 = 0x5bd1e995u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return (c0 >= thresh ? 1u : 0u) | (c1 >= thresh ? 2u : 0u) | (c2 >= thresh ? 4u : 0u) | (c3 >= thresh ? 8u : 0u);
}

template <typename T>
struct SmallArgs {
  const T* q; const T* k; const T* v; const T* o; const T* dout;
  T* out;          // forward O / backward dQ
  float* lse;      // [Z, H, S]
  const T* b1;     // [z, key] (stride b1_zs) or null
  const T* b2;     // [Z / b2_div, H, S, S] or null
  T* dk; T* dv;    // backward [Z, S, H, D] (dense)
  float* delta;    // backward rowsum(dO * O) [Z, H, S], written by the dQ pass
  float* db1;      // [Z, S] fp32 (zeroed; summed over heads by atomics) or null
  float* db2;      // [Z / b2_div, H, S, S] fp32 or null
  int64_t qz, qs, qh, kz, ks, kh, vz, vs, vh, oz, os_, oh, gz, gs, gh, dz, ds, dh;  // (z, s, h) strides: q k v o dO dQ
  int64_t b1_zs;
  int Z, H, S, b2_div;
  float scale;
  float pdrop;     // 0 = no dropout
  uint32_t thresh; // keep if philox >= thresh
  uint64_t seed;
  int vec_bias;    // bias rows in whole 16-B chunks (Sk % 8 == 0, 16-B aligned rows): one load per 8 keys
  int nsplit;      // dB2 pass: the b2_div sharing z are split over this many workgroups (atomics when > 1)
  int Sk;          // keys (the forward may attend to a context of another length; the backward needs Sk == S)
};

// 4 consecutive 16-bit values (8-B aligned) added to f as fp32 / stored from fp32
__device__ __forceinline__ void add4(const bf16* p, float (&f)[4]) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] += (float)v[i];
}
__device__ __forceinline__ void add4(const fp16* p, float (&f)[4]) {
  const fp16x4 v = *reinterpret_cast<const fp16x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] += (float)v[i];
}
__device__ __forceinline__ void store4(bf16* p, const float (&f)[4]) {
  bf16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (bf16)f[i];
  *reinterpret_cast<bf16x4*>(p) = v;
}
__device__ __forceinline__ void store4(fp16* p, const float (&f)[4]) {
  fp16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (fp16)f[i];
  *reinterpret_cast<fp16x4*>(p) = v;
}

// 16 B (8 keys) of a bias row starting at key kb; never reads past key S-1 (vec: S % 8 == 0 and 16-B rows)
template <typename T>
__device__ __forceinline__ u32x4_t bias_chunk(const T* row, int kb, int S, int vec) {
  if (vec) {
    if (kb < S) return *reinterpret_cast<const u32x4_t*>(row + kb);
    return u32x4_t{0u, 0u, 0u, 0u};
  }
  typename MF<T>::V8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = kb + i < S ? row[kb + i] : (T)0.f;
  return __builtin_bit_cast(u32x4_t, v);
}

__device__ __forceinline__ void st16_as_2x8(char* p, u32x4_t v) {  // 8-B aligned LDS destination
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  *reinterpret_cast<u32x2_t*>(p) = u32x2_t{v[0], v[1]};
  *reinterpret_cast<u32x2_t*>(p + 8) = u32x2_t{v[2], v[3]};
}

template <typename T, int D>
struct Tiles {
  // staging: chunk c (row = c / (D/8), 16-B chunk = c % (D/8)); D/8 * 64 chunks, D/32 per thread
  static constexpr int CPR = D / 8, PER = CPR * BN / NTHR;
};

// One 64-key tile for the query-row kernels (forward, dQ, dB2): K and V rows, bias1 of the 64 keys and the
// workgroup's [128 q][64 key] bias2 block, staged global -> registers -> LDS (two-phase so the loads of tile j+1
// are in flight while tile j computes). bias2 rows are 136 B apart: the 8-B reads of 32 different rows by one wave
// land on 64 distinct banks.
template <typename T, int D>
struct KeyTile {
  static constexpr int PER = Tiles<T, D>::PER, CPR = Tiles<T, D>::CPR;
  static constexpr int B2RS = 2 * BN + 8;
  static constexpr int OFF_V = TILE<D>(), OFF_B2 = 2 * TILE<D>(), OFF_B1 = OFF_B2 + BM * B2RS;
  static constexpr int BYTES = OFF_B1 + 2 * BN;
  u32x4_t rk[PER], rv[PER], rb2[4], rb1;
  // b2blk: the [S, S] bias2 matrix of this (z-group, head) or null; qrow0: first query row of the workgroup
  __device__ __forceinline__ void load(const SmallArgs<T>& a, const T* Kp, const T* Vp, const T* b1p,
                                       const T* b2blk, int qrow0, int k0, int tid, bool kv = true) {
    if (kv) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = tid + i * NTHR, row = c / CPR, ch = c % CPR;
        const int key = min(k0 + row, a.Sk - 1);
        rk[i] = *reinterpret_cast<const u32x4_t*>(Kp + (int64_t)key * a.ks + ch * 8);
        rv[i] = *reinterpret_cast<const u32x4_t*>(Vp + (int64_t)key * a.vs + ch * 8);
      }
    }
    if (b2blk) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * NTHR, row = c >> 3, ch = c & 7;
        const int q = min(qrow0 + row, a.S - 1);
        rb2[i] = bias_chunk(b2blk + (int64_t)q * a.Sk, k0 + ch * 8, a.Sk, a.vec_bias);
      }
    }
    if (b1p && tid < BN / 8) rb1 = bias_chunk(b1p, k0 + tid * 8, a.Sk, a.vec_bias);
  }
  __device__ __forceinline__ void store(char* buf, int tid, bool hb1, bool hb2, bool kv = true) {
    if (kv) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = tid + i * NTHR, row = c / CPR, ch = c % CPR;
        *reinterpret_cast<u32x4_t*>(buf + row * RS<D>() + ch * 16) = rk[i];
        *reinterpret_cast<u32x4_t*>(buf + OFF_V + row * RS<D>() + ch * 16) = rv[i];
      }
    }
    if (hb2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * NTHR, row = c >> 3, ch = c & 7;
        st16_as_2x8(buf + OFF_B2 + row * B2RS + ch * 16, rb2[i]);
      }
    }
    if (hb1 && tid < BN / 8) *reinterpret_cast<u32x4_t*>(buf + OFF_B1 + tid * 16) = rb1;
  }
};

// bias1 + bias2 of the 4 keys kr..kr+3 of the tile (kr % 4 == 0) for LDS bias2 row `brow`; keys >= S give -inf
template <typename T, int D>
__device__ __forceinline__ void tile_bias4(const char* buf, const char* b2buf, bool hb1, bool hb2, int brow, int kr,
                                           int key0, int S, float (&bb)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) bb[i] = key0 + i < S ? 0.f : -INFINITY;
  if (hb1) add4(reinterpret_cast<const T*>(buf + KeyTile<T, D>::OFF_B1 + kr * 2), bb);
  if (hb2) add4(reinterpret_cast<const T*>(b2buf + KeyTile<T, D>::OFF_B2 + brow * KeyTile<T, D>::B2RS + kr * 2), bb);
}

// transposed 4+4-row read of a row-major 16-bit image into an MFMA operand (k slots = rows rb+{0..3}, rb+8+{0..3})
template <typename V8>
__device__ __forceinline__ V8 tr_read(const char* img, int rs, int rb, int ch0, int lane) {
  const int gq = (lane >> 2) & 3, gb = 8 * (lane & 1);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(img + (rb + gq) * rs + ch0 * 16 + gb));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(img + (rb + 8 + gq) * rs + ch0 * 16 + gb));
  s16x8 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = lo[e]; v[4 + e] = hi[e]; }
  return __builtin_bit_cast(V8, v);
}

// ================================================================================================== forward
template <typename T, int D>
__global__ void __launch_bounds__(NTHR, 2) small_fwd_kernel(SmallArgs<T> a) {
  typedef typename MF<T>::V8 V8;
  typedef KeyTile<T, D> KT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (a.S + BM - 1) / BM;
  const int qb = blockIdx.x % nqb, hd = (blockIdx.x / nqb) % a.H, z = blockIdx.x / (nqb * a.H);
  const int q0w = qb * BM + wid * 32, qrow = q0w + l32;
  const T* Qp = a.q + z * a.qz + hd * a.qh;
  const T* Kp = a.k + z * a.kz + hd * a.kh;
  const T* Vp = a.v + z * a.vz + hd * a.vh;
  const T* b1p = a.b1 ? a.b1 + z * a.b1_zs : nullptr;
  const T* b2blk = a.b2 ? a.b2 + ((int64_t)(z / a.b2_div) * a.H + hd) * a.S * a.Sk : nullptr;
  const bool hb1 = b1p != nullptr, hb2 = b2blk != nullptr;
  const uint64_t drow = ((uint64_t)z * a.H + hd) * (uint64_t)a.S + (uint64_t)qrow;

  V8 qf[D / 16];
  {
    const T* qr = Qp + (int64_t)min(qrow, a.S - 1) * a.qs + 8 * h;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const V8*>(qr + 16 * kk);
  }
  float* scratch = reinterpret_cast<float*>(smem + 2 * KT::BYTES) + wid * 32;
  KT stg;

  f32x16_t o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const int nt = (a.Sk + BN - 1) / BN;
  const float LOG2E = 1.4426950408889634f;
  const float inv_keep = a.pdrop > 0.f ? 1.f / (1.f - a.pdrop) : 1.f;
  const int gch = (lane >> 1) & 1, colhalf = (lane >> 4) & 1;

  stg.load(a, Kp, Vp, b1p, b2blk, qb * BM, 0, tid);
  stg.store(smem, tid, hb1, hb2);
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const int cur = j & 1, k0 = j * BN;
    if (j + 1 < nt) stg.load(a, Kp, Vp, b1p, b2blk, qb * BM, k0 + BN, tid);
    const char* buf = smem + cur * KT::BYTES;
    const char* Vt = buf + KT::OFF_V;
    f32x16_t s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[t][r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const V8 av = *reinterpret_cast<const V8*>(buf + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        s[t] = MF<T>::mma(av, qf[kk], s[t]);
      }
    }
    // natural-unit logits: scale * q.k + bias1[key] + bias2[q, key]; keys past S masked
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int kr = t * 32 + 8 * g + 4 * h;
        float bb[4];
        tile_bias4<T, D>(buf, buf, hb1, hb2, wid * 32 + l32, kr, k0 + kr, a.Sk, bb);
#pragma unroll
        for (int i = 0; i < 4; ++i) s[t][4 * g + i] = s[t][4 * g + i] * a.scale + bb[i];
      }
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_use) * LOG2E);
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f((s[t][r] - m_use) * LOG2E);
        s[t][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (a.pdrop > 0.f) {  // dropout after the normaliser: O accumulates P * keep / (1 - p)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t kb = keep4(a.seed, drow, (uint32_t)((k0 + t * 32 + 8 * g + 4 * h) >> 2), a.thresh);
#pragma unroll
          for (int i = 0; i < 4; ++i) s[t][4 * g + i] *= ((kb >> i) & 1u) ? inv_keep : 0.f;
        }
    }
    if (!__all(alpha == 1.f)) {
      if (lane < 32) scratch[lane] = alpha;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      float a4[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 vv = *reinterpret_cast<const f32x4*>(scratch + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[4 * g + i] = vv[i];
      }
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= a4[r];
      __builtin_amdgcn_wave_barrier();
    }
    V8 pa[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int e = 0; e < 8; ++e) pa[t][ss][e] = (T)s[t][8 * ss + e];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
          o[dt] = MF<T>::mma(pa[t][ss], tr_read<V8>(Vt, RS<D>(), t * 32 + 16 * ss + 4 * h, ch0, lane), o[dt]);
    }
    if (j + 1 < nt) stg.store(smem + (cur ^ 1) * KT::BYTES, tid, hb1, hb2);
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
    const f32x4 vv = *reinterpret_cast<const f32x4*>(scratch + 8 * g + 4 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) iv[4 * g + i] = vv[i];
  }
  T* Op = a.out + z * a.oz + hd * a.oh;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qi = q0w + crow(r, h);
    if (qi < a.S) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) Op[(int64_t)qi * a.os_ + dt * 32 + l32] = (T)(o[dt][r] * iv[r]);
    }
  }
  if (lane < 32 && qrow < a.S)
    a.lse[((int64_t)z * a.H + hd) * a.S + qrow] = l_tot > 0.f ? m_run + __logf(l_tot) : INFINITY;
}

// ================================================================================================== backward
// Three passes, no fp32 atomics on the big tensors:
//  1. dQ pass (query-outer, same tiling as the forward): delta = rowsum(dO * O) written for the other passes,
//     dQ += dS.K in registers; dB2 stored directly when every z has its own pair bias (b2_div == 1);
//  2. dK/dV pass (key-outer): a wave owns 32 keys (K, V rows in registers as B operands), Q / dO / lse / delta and
//     the [64 q x 128 key] bias2 block stream through LDS; S = Q.K^T lands with the key on the lane so P^T / dS^T
//     feed dV += P^T.dO and dK += dS^T.Q as the A operand straight from registers (dO, Q by transposed read);
//     dB1 column sums per lane, one atomic per (z, head, key);
//  3. dB2 pass (b2_div > 1): a workgroup owns one [128 q x 64 key] tile of the shared pair bias and loops over the
//     z that share it (split over a few workgroups when the tile grid alone cannot fill the chip), summing dS in
//     registers.

// ---------------------------------------------------------------- pass 1: dQ, delta (and unshared dB2)
template <typename T, int D>
__global__ void __launch_bounds__(NTHR, D == 32 ? 2 : 1) small_bwd_dq_kernel(SmallArgs<T> a) {
  typedef typename MF<T>::V8 V8;
  typedef KeyTile<T, D> KT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (a.S + BM - 1) / BM;
  const int qb = blockIdx.x % nqb, hd = (blockIdx.x / nqb) % a.H, z = blockIdx.x / (nqb * a.H);
  const int q0w = qb * BM + wid * 32, qrow = q0w + l32;
  const int qc = min(qrow, a.S - 1);
  const bool qlive = qrow < a.S;
  const T* Kp = a.k + z * a.kz + hd * a.kh;
  const T* Vp = a.v + z * a.vz + hd * a.vh;
  const T* b1p = a.b1 ? a.b1 + z * a.b1_zs : nullptr;
  const int64_t b2mat = ((int64_t)(z / a.b2_div) * a.H + hd) * a.S * a.S;
  const T* b2blk = a.b2 ? a.b2 + b2mat : nullptr;
  const bool hb1 = b1p != nullptr, hb2 = b2blk != nullptr;
  float* db2p = (a.db2 && a.b2_div == 1) ? a.db2 + b2mat + (int64_t)qc * a.S : nullptr;
  const uint64_t drow = ((uint64_t)z * a.H + hd) * (uint64_t)a.S + (uint64_t)qrow;

  V8 qf[D / 16], gf[D / 16];
  float delta = 0.f;
  {
    const T* qr = a.q + z * a.qz + hd * a.qh + (int64_t)qc * a.qs;
    const T* gr = a.dout + z * a.gz + hd * a.gh + (int64_t)qc * a.gs;
    const T* orr = a.o + z * a.oz + hd * a.oh + (int64_t)qc * a.os_;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) {
      qf[kk] = *reinterpret_cast<const V8*>(qr + 16 * kk + 8 * h);
      gf[kk] = *reinterpret_cast<const V8*>(gr + 16 * kk + 8 * h);
      const V8 ov = *reinterpret_cast<const V8*>(orr + 16 * kk + 8 * h);
#pragma unroll
      for (int e = 0; e < 8; ++e) delta += (float)gf[kk][e] * (float)ov[e];
    }
    delta += __shfl_xor(delta, 32, 64);
  }
  const int64_t lrow = ((int64_t)z * a.H + hd) * a.S;
  if (lane < 32 && qlive) a.delta[lrow + qrow] = delta;
  const float lse = a.lse[lrow + qc];
  const float LOG2E = 1.4426950408889634f;
  const float inv_keep = a.pdrop > 0.f ? 1.f / (1.f - a.pdrop) : 1.f;
  f32x16_t dq[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;
  const int nt = (a.S + BN - 1) / BN;
  const int gch = (lane >> 1) & 1, colhalf = (lane >> 4) & 1;
  const bool st4 = (a.S & 3) == 0;

  KT stg;
  stg.load(a, Kp, Vp, b1p, b2blk, qb * BM, 0, tid);
  stg.store(smem, tid, hb1, hb2);
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const int cur = j & 1, k0 = j * BN;
    if (j + 1 < nt) stg.load(a, Kp, Vp, b1p, b2blk, qb * BM, k0 + BN, tid);
    const char* buf = smem + cur * KT::BYTES;
    const char* Vt = buf + KT::OFF_V;
    f32x16_t s[2], dp[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[t][r] = 0.f; dp[t][r] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const V8 kv = *reinterpret_cast<const V8*>(buf + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        s[t] = MF<T>::mma(kv, qf[kk], s[t]);
        const V8 vv = *reinterpret_cast<const V8*>(Vt + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        dp[t] = MF<T>::mma(vv, gf[kk], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int kr = t * 32 + 8 * g + 4 * h, kb4 = k0 + kr;
        uint32_t kb = 0xfu;
        if (a.pdrop > 0.f) kb = keep4(a.seed, drow, (uint32_t)(kb4 >> 2), a.thresh);
        float bb[4];
        tile_bias4<T, D>(buf, buf, hb1, hb2, wid * 32 + l32, kr, kb4, a.S, bb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float x = s[t][r] * a.scale + bb[i];
          const float p = (kb4 + i < a.S && qlive) ? __builtin_amdgcn_exp2f((x - lse) * LOG2E) : 0.f;
          const float kf = ((kb >> i) & 1u) ? inv_keep : 0.f;
          s[t][r] = p * (dp[t][r] * kf - delta);  // dS (natural units)
        }
        if (db2p && qlive) {
          if (st4) {
            if (kb4 < a.S) {
              f32x4 w;
#pragma unroll
              for (int i = 0; i < 4; ++i) w[i] = s[t][4 * g + i];
              *reinterpret_cast<f32x4*>(db2p + kb4) = w;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (kb4 + i < a.S) db2p[kb4 + i] = s[t][4 * g + i];
          }
        }
      }
    V8 da[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int e = 0; e < 8; ++e) da[t][ss][e] = (T)s[t][8 * ss + e];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
          dq[dt] = MF<T>::mma(da[t][ss], tr_read<V8>(buf, RS<D>(), t * 32 + 16 * ss + 4 * h, ch0, lane), dq[dt]);
    }
    if (j + 1 < nt) stg.store(smem + (cur ^ 1) * KT::BYTES, tid, hb1, hb2);
    __syncthreads();
  }
  T* Gq = a.out + z * a.dz + hd * a.dh;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qi = q0w + crow(r, h);
    if (qi < a.S) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) Gq[(int64_t)qi * a.ds + dt * 32 + l32] = (T)(dq[dt][r] * a.scale);
    }
  }
}

// ---------------------------------------------------------------- pass 2: dK, dV (key-outer), dB1
// One 64-query tile: Q and dO rows, lse / delta of the 64 queries, and the [64 q][128 key] bias2 block of the
// workgroup's keys (272-B rows; the wave reads 32 consecutive 2-B keys of one row).
template <typename T, int D>
struct QueryTile {
  static constexpr int PER = Tiles<T, D>::PER, CPR = Tiles<T, D>::CPR;
  static constexpr int B2RS = 2 * BM + 16;
  static constexpr int OFF_G = TILE<D>(), OFF_L = 2 * TILE<D>(), OFF_B2 = OFF_L + 2 * BN * 4;
  static constexpr int BYTES = OFF_B2 + BN * B2RS;
  u32x4_t rq[PER], rg[PER], rb2[4];
  float rl;
  __device__ __forceinline__ void load(const SmallArgs<T>& a, const T* Qp, const T* Gp, int64_t lrow,
                                       const T* b2blk, int key0, int q0, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTHR, row = c / CPR, ch = c % CPR;
      const int q = min(q0 + row, a.S - 1);
      rq[i] = *reinterpret_cast<const u32x4_t*>(Qp + (int64_t)q * a.qs + ch * 8);
      rg[i] = *reinterpret_cast<const u32x4_t*>(Gp + (int64_t)q * a.gs + ch * 8);
    }
    if (tid < 2 * BN) {
      const int q = min(q0 + (tid & (BN - 1)), a.S - 1);
      rl = tid < BN ? a.lse[lrow + q] : a.delta[lrow + q];
    }
    if (b2blk) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * NTHR, row = c >> 4, ch = c & 15;
        const int q = min(q0 + row, a.S - 1);
        rb2[i] = bias_chunk(b2blk + (int64_t)q * a.S, key0 + ch * 8, a.S, a.vec_bias);
      }
    }
  }
  __device__ __forceinline__ void store(char* buf, int tid, bool hb2) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTHR, row = c / CPR, ch = c % CPR;
      *reinterpret_cast<u32x4_t*>(buf + row * RS<D>() + ch * 16) = rq[i];
      *reinterpret_cast<u32x4_t*>(buf + OFF_G + row * RS<D>() + ch * 16) = rg[i];
    }
    if (tid < 2 * BN) reinterpret_cast<float*>(buf + OFF_L)[tid] = rl;
    if (hb2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * NTHR, row = c >> 4, ch = c & 15;
        *reinterpret_cast<u32x4_t*>(buf + OFF_B2 + row * B2RS + ch * 16) = rb2[i];
      }
    }
  }
};

template <typename T, int D>
__global__ void __launch_bounds__(NTHR, D == 32 ? 2 : 1) small_bwd_dkv_kernel(SmallArgs<T> a) {
  typedef typename MF<T>::V8 V8;
  typedef QueryTile<T, D> QT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int nkb = (a.S + BM - 1) / BM;
  const int kbk = blockIdx.x % nkb, hd = (blockIdx.x / nkb) % a.H, z = blockIdx.x / (nkb * a.H);
  const int key0w = kbk * BM + wid * 32, key = key0w + l32;
  const int kc = min(key, a.S - 1);
  const bool klive = key < a.S;
  const T* Qp = a.q + z * a.qz + hd * a.qh;
  const T* Gp = a.dout + z * a.gz + hd * a.gh;
  const T* b2blk = a.b2 ? a.b2 + ((int64_t)(z / a.b2_div) * a.H + hd) * a.S * a.S : nullptr;
  const bool hb2 = b2blk != nullptr;

  // B operands (column = this lane's key): K and V rows
  V8 kB[D / 16], vB[D / 16];
  {
    const T* kr = a.k + z * a.kz + hd * a.kh + (int64_t)kc * a.ks;
    const T* vr = a.v + z * a.vz + hd * a.vh + (int64_t)kc * a.vs;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) {
      kB[kk] = *reinterpret_cast<const V8*>(kr + 16 * kk + 8 * h);
      vB[kk] = *reinterpret_cast<const V8*>(vr + 16 * kk + 8 * h);
    }
  }
  const float b1v = (a.b1 && klive) ? (float)a.b1[z * a.b1_zs + key] : 0.f;
  const int64_t lrow = ((int64_t)z * a.H + hd) * a.S;
  const float LOG2E = 1.4426950408889634f;
  const float inv_keep = a.pdrop > 0.f ? 1.f / (1.f - a.pdrop) : 1.f;
  f32x16_t dk[D / 32], dv[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  float colsum = 0.f;
  const int nt = (a.S + BN - 1) / BN;
  const int gch = (lane >> 1) & 1, colhalf = (lane >> 4) & 1;

  QT stg;
  stg.load(a, Qp, Gp, lrow, b2blk, kbk * BM, 0, tid);
  stg.store(smem, tid, hb2);
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const int cur = j & 1, q0 = j * BN;
    if (j + 1 < nt) stg.load(a, Qp, Gp, lrow, b2blk, kbk * BM, q0 + BN, tid);
    const char* Qt = smem + cur * QT::BYTES;
    const char* Gt = Qt + QT::OFF_G;
    const float* lseT = reinterpret_cast<const float*>(Qt + QT::OFF_L);
    const float* delT = lseT + BN;
    const char* b2t = Qt + QT::OFF_B2 + (wid * 32 + l32) * 2;
    // one 32-query half at a time (keeps the transient score / dP registers at 2 x 16)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const V8 qa = *reinterpret_cast<const V8*>(Qt + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        s = MF<T>::mma(qa, kB[kk], s);
        const V8 ga = *reinterpret_cast<const V8*>(Gt + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        dp = MF<T>::mma(ga, vB[kk], dp);
      }
      // rows = queries q0 + t*32 + crow(r, h), column = this lane's key
      V8 pa[2], da[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(lseT + t * 32 + 8 * g + 4 * h);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(delT + t * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i, qr = t * 32 + 8 * g + 4 * h + i, q = q0 + qr;
          const bool live = klive && q < a.S;
          float x = s[r] * a.scale + b1v;
          if (hb2) x += (float)*reinterpret_cast<const T*>(b2t + qr * QT::B2RS);
          const float p = live ? __builtin_amdgcn_exp2f((x - l4[i]) * LOG2E) : 0.f;
          float kf = 1.f;
          if (a.pdrop > 0.f) {
            const uint32_t kb = keep4(a.seed, (uint64_t)lrow + (uint64_t)q, (uint32_t)(key >> 2), a.thresh);
            kf = ((kb >> (key & 3)) & 1u) ? inv_keep : 0.f;
          }
          const float ds = p * (dp[r] * kf - d4[i]);
          colsum += ds;
          pa[r >> 3][r & 7] = (T)(p * kf);
          da[r >> 3][r & 7] = (T)ds;
        }
      }
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int ch0 = dt * 4 + colhalf * 2 + gch;
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int rb = t * 32 + 16 * ss + 4 * h;
          dv[dt] = MF<T>::mma(pa[ss], tr_read<V8>(Gt, RS<D>(), rb, ch0, lane), dv[dt]);
          dk[dt] = MF<T>::mma(da[ss], tr_read<V8>(Qt, RS<D>(), rb, ch0, lane), dk[dt]);
        }
      }
    }
    if (j + 1 < nt) stg.store(smem + (cur ^ 1) * QT::BYTES, tid, hb2);
    __syncthreads();
  }
  if (a.db1) {
    colsum += __shfl_xor(colsum, 32, 64);
    if (lane < 32 && klive) unsafeAtomicAdd(a.db1 + (int64_t)z * a.S + key, colsum);
  }
  const int64_t obase = ((int64_t)z * a.S) * a.H * D + (int64_t)hd * D;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int kr = key0w + crow(r, h);
    if (kr < a.S) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int64_t idx = obase + (int64_t)kr * a.H * D + dt * 32 + l32;
        a.dk[idx] = (T)(dk[dt][r] * a.scale);
        a.dv[idx] = (T)dv[dt][r];
      }
    }
  }
}

// ---------------------------------------------------------------- pass 3: dB2 summed over the z sharing it
template <typename T, int D, bool DROP>
__global__ void __launch_bounds__(NTHR, (D == 32 && !DROP) ? 2 : 1) small_bwd_db2_kernel(SmallArgs<T> a) {
  typedef typename MF<T>::V8 V8;
  typedef KeyTile<T, D> KT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (a.S + BM - 1) / BM, nkt = (a.S + BN - 1) / BN;
  int bid = blockIdx.x;
  const int kt = bid % nkt; bid /= nkt;
  const int qb = bid % nqb; bid /= nqb;
  const int hd = bid % a.H; bid /= a.H;
  const int zb = bid % (a.Z / a.b2_div), split = bid / (a.Z / a.b2_div);
  const int chunk = (a.b2_div + a.nsplit - 1) / a.nsplit;
  const int n_lo = split * chunk, n_hi = min(a.b2_div, n_lo + chunk);
  const int q0w = qb * BM + wid * 32, qrow = q0w + l32;
  const int qc = min(qrow, a.S - 1);
  const bool qlive = qrow < a.S;
  const int k0 = kt * BN;
  const int64_t b2mat = ((int64_t)zb * a.H + hd) * a.S * a.S;
  const bool hb1 = a.b1 != nullptr;
  const float LOG2E = 1.4426950408889634f;
  const float inv_keep = a.pdrop > 0.f ? 1.f / (1.f - a.pdrop) : 1.f;
  f32x16_t acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  if (n_lo >= n_hi) return;  // uniform per workgroup (before any barrier)

  // per-z operands of the lane's query row, prefetched one z ahead
  V8 qf[D / 16], gf[D / 16];
  float lse = 0.f, delta = 0.f;
  auto load_rows = [&](int z) {
    const T* qr = a.q + z * a.qz + hd * a.qh + (int64_t)qc * a.qs;
    const T* gr = a.dout + z * a.gz + hd * a.gh + (int64_t)qc * a.gs;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) {
      qf[kk] = *reinterpret_cast<const V8*>(qr + 16 * kk + 8 * h);
      gf[kk] = *reinterpret_cast<const V8*>(gr + 16 * kk + 8 * h);
    }
    const int64_t lrow = ((int64_t)z * a.H + hd) * a.S;
    lse = a.lse[lrow + qc];
    delta = a.delta[lrow + qc];
  };
  KT stg;
  {
    const int z = zb * a.b2_div + n_lo;
    stg.load(a, a.k + z * a.kz + hd * a.kh, a.v + z * a.vz + hd * a.vh, hb1 ? a.b1 + z * a.b1_zs : nullptr,
             a.b2 + b2mat, qb * BM, k0, tid);
    stg.store(smem, tid, hb1, true);  // the bias2 block lives in buffer 0 for the whole loop
  }
  load_rows(zb * a.b2_div + n_lo);
  __syncthreads();
  for (int n = n_lo; n < n_hi; ++n) {
    const int z = zb * a.b2_div + n, cur = (n - n_lo) & 1;
    const bool more = n + 1 < n_hi;
    if (more) {
      const int zn = z + 1;
      stg.load(a, a.k + zn * a.kz + hd * a.kh, a.v + zn * a.vz + hd * a.vh, hb1 ? a.b1 + zn * a.b1_zs : nullptr,
               nullptr, qb * BM, k0, tid);
    }
    const char* buf = smem + cur * KT::BYTES;
    const uint64_t drow = ((uint64_t)z * a.H + hd) * (uint64_t)a.S + (uint64_t)qrow;
    const float lse_n = lse, delta_n = delta;
    V8 qc_[D / 16], gc_[D / 16];
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) { qc_[kk] = qf[kk]; gc_[kk] = gf[kk]; }
    if (more) load_rows(z + 1);
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // one 32-key half at a time
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const V8 kv = *reinterpret_cast<const V8*>(buf + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        s = MF<T>::mma(kv, qc_[kk], s);
        const V8 vv = *reinterpret_cast<const V8*>(buf + KT::OFF_V + (t * 32 + l32) * RS<D>() + (2 * kk + h) * 16);
        dp = MF<T>::mma(vv, gc_[kk], dp);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int kr = t * 32 + 8 * g + 4 * h, kb4 = k0 + kr;
        uint32_t kb = 0xfu;
        if (DROP) kb = keep4(a.seed, drow, (uint32_t)(kb4 >> 2), a.thresh);
        float bb[4];
        tile_bias4<T, D>(buf, smem, hb1, true, wid * 32 + l32, kr, kb4, a.S, bb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float x = s[r] * a.scale + bb[i];
          const float p = (kb4 + i < a.S && qlive) ? __builtin_amdgcn_exp2f((x - lse_n) * LOG2E) : 0.f;
          const float kf = ((kb >> i) & 1u) ? inv_keep : 0.f;
          acc[t][r] += p * (dp[r] * kf - delta_n);
        }
      }
    }
    if (more) stg.store(smem + (cur ^ 1) * KT::BYTES, tid, hb1, false);
    __syncthreads();
  }
  if (!qlive) return;
  float* out = a.db2 + b2mat + (int64_t)qrow * a.S;
  const bool st4 = (a.S & 3) == 0;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int kb4 = k0 + t * 32 + 8 * g + 4 * h;
      if (a.nsplit > 1) {  // partial sums of several workgroups (dB2 zeroed by the caller)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (kb4 + i < a.S) unsafeAtomicAdd(out + kb4 + i, acc[t][4 * g + i]);
      } else if (st4) {
        if (kb4 < a.S) {
          f32x4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = acc[t][4 * g + i];
          *reinterpret_cast<f32x4*>(out + kb4) = w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (kb4 + i < a.S) out[kb4 + i] = acc[t][4 * g + i];
      }
    }
}

template <typename K>
void set_lds(K* fn, int bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <typename T, int D>
int launch_small(SmallArgs<T> a, bool bwd, hipStream_t st) {
  const int nqb = (a.S + BM - 1) / BM;
  const dim3 grid(nqb * a.H * a.Z);
  constexpr int lds_f = 2 * KeyTile<T, D>::BYTES + 4 * 32 * 4;
  constexpr int lds_kv = 2 * QueryTile<T, D>::BYTES;
  static bool attr = false;
  if (!attr) {
    set_lds(&small_fwd_kernel<T, D>, lds_f);
    set_lds(&small_bwd_dq_kernel<T, D>, lds_f);
    set_lds(&small_bwd_dkv_kernel<T, D>, lds_kv);
    set_lds(&small_bwd_db2_kernel<T, D, false>, lds_f);
    set_lds(&small_bwd_db2_kernel<T, D, true>, lds_f);
    attr = true;
  }
  if (!bwd) {
    hipLaunchKernelGGL((small_fwd_kernel<T, D>), grid, dim3(NTHR), lds_f, st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL((small_bwd_dq_kernel<T, D>), grid, dim3(NTHR), lds_f, st, a);
  DS_CHECK_LAUNCH();
  hipLaunchKernelGGL((small_bwd_dkv_kernel<T, D>), grid, dim3(NTHR), lds_kv, st, a);
  DS_CHECK_LAUNCH();
  if (a.db2 && a.b2_div > 1) {
    // enough workgroups to fill 256 CUs a few times over: split the sharing z when the tile grid is small
    const int base = (a.Z / a.b2_div) * a.H * nqb * ((a.S + BN - 1) / BN);
    a.nsplit = std::max(1, std::min(a.b2_div / 4, 1024 / base));
    const dim3 g3(base * a.nsplit);
    if (a.pdrop > 0.f)
      hipLaunchKernelGGL((small_bwd_db2_kernel<T, D, true>), g3, dim3(NTHR), lds_f, st, a);
    else
      hipLaunchKernelGGL((small_bwd_db2_kernel<T, D, false>), g3, dim3(NTHR), lds_f, st, a);
    DS_CHECK_LAUNCH();
  }
  return 0;
}

template <typename T>
int dispatch_small(SmallArgs<T> a, int D, bool bwd, hipStream_t st) {
  if (D == 32) return launch_small<T, 32>(a, bwd, st);
  if (D == 64) return launch_small<T, 64>(a, bwd, st);
  return (int)hipErrorInvalidValue;
}

}  // namespace

// Forward. strides[12] = (q z,s,h)(k)(v)(o); dtype DS_BF16 / DS_F16; b1 / b2 may be null.
extern "C" int ds_flash_small_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const void* b1,
                                  const void* b2, const int64_t* st, int64_t b1_zs, int Z, int H, int S, int Sk, int D,
                                  int b2_div, float scale, float pdrop, uint64_t seed, int vec_bias, int dtype,
                                  hipStream_t stream) {
  if (Z <= 0 || H <= 0 || S <= 0 || Sk <= 0 || b2_div <= 0 || (D != 32 && D != 64) || pdrop < 0.f || pdrop >= 1.f)
    return (int)hipErrorInvalidValue;
  const uint32_t thresh = (uint32_t)fminf(4294967295.f, pdrop * 4294967296.f);
#define DS_SMALL_ARGS(T)                                                                                        \
  SmallArgs<T> a{(const T*)q, (const T*)k, (const T*)v, nullptr, nullptr, (T*)o, lse, (const T*)b1, (const T*)b2, \
                 nullptr, nullptr, nullptr, nullptr, nullptr, st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7],     \
                 st[8], st[9], st[10], st[11], 0, 0, 0, 0, 0, 0, b1_zs, Z, H, S, b2_div, scale, pdrop, thresh, seed, vec_bias, 1, Sk};
  if (dtype == DS_BF16) {
    DS_SMALL_ARGS(bf16)
    return dispatch_small<bf16>(a, D, false, stream);
  }
  if (dtype == DS_F16) {
    DS_SMALL_ARGS(fp16)
    return dispatch_small<fp16>(a, D, false, stream);
  }
  return (int)hipErrorInvalidValue;
#undef DS_SMALL_ARGS
}

// Backward. strides[18] = (q)(k)(v)(o)(dO)(dQ); dk / dv dense [Z, S, H, D] in the input dtype; delta fp32 [Z, H, S]
// scratch; db1 [Z, S] fp32 (zeroed by the caller) or null; db2 [Z / b2_div, H, S, S] fp32 (fully written) or null.
extern "C" int ds_flash_small_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                  const float* lse, const void* b1, const void* b2, void* dq, void* dk, void* dv,
                                  float* delta, float* db1, float* db2, const int64_t* st, int64_t b1_zs, int Z, int H, int S, int D,
                                  int b2_div, float scale, float pdrop, uint64_t seed, int vec_bias, int dtype,
                                  hipStream_t stream) {
  if (Z <= 0 || H <= 0 || S <= 0 || b2_div <= 0 || (D != 32 && D != 64) || pdrop < 0.f || pdrop >= 1.f)
    return (int)hipErrorInvalidValue;
  const uint32_t thresh = (uint32_t)fminf(4294967295.f, pdrop * 4294967296.f);
#define DS_SMALL_ARGS(T)                                                                                           \
  SmallArgs<T> a{(const T*)q, (const T*)k, (const T*)v, (const T*)o, (const T*)dout, (T*)dq, (float*)lse,           \
                 (const T*)b1, (const T*)b2, (T*)dk, (T*)dv, delta, db1, db2, st[0], st[1], st[2], st[3], st[4], st[5], st[6],      \
                 st[7], st[8], st[9], st[10], st[11], st[12], st[13], st[14], st[15], st[16], st[17], b1_zs, Z, H, S, b2_div, scale, pdrop, \
                 thresh, seed, vec_bias, 1, S};
  if (dtype == DS_BF16) {
    DS_SMALL_ARGS(bf16)
    return dispatch_small<bf16>(a, D, true, stream);
  }
  if (dtype == DS_F16) {
    DS_SMALL_ARGS(fp16)
    return dispatch_small<fp16>(a, D, true, stream);
  }
  return (int)hipErrorInvalidValue;
#undef DS_SMALL_ARGS
}
