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
//    read `ds_read_b64_tr_b16`; the image is XOR-swizzled so row reads (S, dP) and transposed reads are conflict-free
//    (SQ_LDS_BANK_CONFLICT = 0 measured);
//  * S's accumulator starts at -LSE/scale and dP's at -delta (delta = rowsum(dO*O), one preprocessing pass), so
//    P = exp2(c*S') needs no row max and dS = P*dP' is one multiply;
//  * dS crosses LDS once (dS^T image, 64-B rows, 8-B units swizzled by key so the packed stores of 8 rows and the
//    transposed reads are both conflict-free); waves 0..3 then compute the 32x128 dQ tile over all 256 keys
//    (A = dS by transposed read, B = K by transposed read of the resident K image) and add it with packed-row f32
//    atomics (one 32x32 accumulator register = two 128-B row segments = the full-rate atomic shape); waves 4..7 run
//    ahead into the next tile, so the two waves on a SIMD keep its matrix core busy across the dQ phase;
//  * Q / dO / lse / delta tiles arrive by LDS-DMA (global_load_lds, issued from inline asm so hipcc does not drain it)
//    two tiles ahead into a 3-deep ring, with the swizzle applied on the source address; one raw barrier per tile
//    behind a counted `s_waitcnt vmcnt(N)`;
//  * every LDS address is a per-lane base + an XOR toggle + a compile-time displacement; the bases are laundered per
//    tile so hipcc does not hoist ~40 derived addresses into registers (2 waves per SIMD leave 256 per lane);
//  * causal: waves whose 32 keys lie entirely above a tile skip it, the dQ product stops at the diagonal, workgroups
//    with the most tiles (low key blocks) start first, and each (batch, kv head)'s key blocks share an XCD (Q / dO
//    reuse in L2);
//  * block-sparse: each workgroup walks only the 32-row query tiles its key block meets in the layout (a host-built
//    column LUT) and masks at the layout's block granularity (16/32/64/128) — cost scales with the layout density.
// Measured (tools/bench_flash_bwd.py, profiles/flash_bwd_bench_r2_final.jsonl): B8 H32 S4096 D128 causal 4.2-4.3 ms
// (round-2 start: 4.58). SQ PMC of the round-2 start: ~29 % MFMA busy, ~9 VALU per MFMA -- the VALU issue slots, not
// the matrix pipe, are what the trims above (packed converts, pre-scaled row constants, uniform mask skip) buy back.
// Where the time goes now: the dQ sum. Every 32-row query tile receives one 16-KB fp32 tile-add per 256-key block it
// meets: B8 H32 S4096 causal = 278.5k tile-adds = 4.56 GB of float atomics, and the memory-side atomic units retire
// ~1.3 TB/s chip-wide (one 256-B wave-instruction per ~50 ns per CU), i.e. a 3.5 ms floor for the main kernel at
// this key-block size whatever the MFMA loop does (measured 3.8 ms + 0.3 ms pre/post; 4 heads x 32k: floor 3.3 ms,
// measured 3.9 + 0.3). Pipelining the S / dP operand reads two MFMAs ahead (round 3) therefore bought only 2 %.
// Going below the floor needs fewer adds per dQ element (512 keys per workgroup: the dK/dV accumulators no longer
// fit two waves per SIMD) or bf16 atomics (2-3x the rounding error on dQ) -- neither taken.
// Tried and measured slower: dQ partial stores + a summing pass instead of atomics (5.5 ms), pairing heavy and light
// key blocks across XCDs for few-head long sequences (32k: 5.0 vs 4.75 ms; the dispatcher balances heavy-first),
// splitting long key blocks' query ranges over several workgroups with fp32 dK/dV atomics (4 heads x 32k: 6.7 vs
// 4.3 ms; +10 SGPR spills and the split bookkeeping slowed every shape).
#include "ds_hip.h"

#include <cstdlib>

namespace {

constexpr int D = 128;
constexpr int KB = 256;                // keys per workgroup
constexpr int QT = 32;                 // query rows per tile
constexpr int TILE = QT * D * 2;       // 8 KB: one Q or dO tile
constexpr int K_BYTES = KB * 256;      // resident K image
constexpr int DS_BYTES = KB * 64;      // dS^T image [KB keys][32 q] bf16
constexpr int NBUF = 3;                // Q / dO / lse / delta tiles in flight: two ahead of the one in use
template <int NW>
constexpr int lds_bytes() { return K_BYTES + NBUF * 2 * TILE + 2 * DS_BYTES + NBUF * 64 * 4 + 2 * 8; }

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) bf16x8_t lds_bf16x8;
typedef __attribute__((address_space(1))) void glob_void;

// LDS-DMA: every lane fetches `size` bytes from its own global address; they land at lds_base + lane * size.
// Issued from inline asm on purpose: hipcc tracks its own global_load_lds builtins and then waits vmcnt(0) before
// every LDS read it cannot prove disjoint from the DMA target (i.e. all of them, one LDS array) and before every use
// of an older ordinary load, draining the prefetch. Out of its sight the DMA is ordered only by the counted
// `s_waitcnt vmcnt(N)` + barrier below (in-order vmcnt: the compiler's own counts stay conservative).
__device__ __forceinline__ void glds16(const void* g, const char* lds_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}
__device__ __forceinline__ void glds4(const void* g, const char* lds_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

// 256-B rows of 16 x 16-B chunks, chunk XOR-swizzled by row mod 16 (same image as flash_fwd.hip): conflict-free for
// 32-row b128 reads of one chunk and for 4-row transposed reads.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
// dS^T image: 64-B rows (32 queries), 8-B unit u (4 queries) XOR-swizzled by (key >> 1) & 7 so that 16 lanes storing
// one unit of 16 consecutive keys hit 32 distinct banks.
__device__ __forceinline__ int ds_off(int key, int u) { return key * 64 + 8 * (u ^ ((key >> 1) & 7)); }

// two fp32 -> one dword of two bf16 (round to nearest even), lo in bits 0..15
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

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
  // additive score biases of the block-sparse path (see flash_fwd.hip SparseLut), any may be null
  const float *kbias, *abias, *rpe;
  int64_t kb_stride, ab_stride, rpe_hs, rpe_rs;
  // 1 = kbias, 2 = abias, 4 = rpe are real; with any of them set the others point at one zero float and their
  // strides and key multipliers (ab_km / rpe_km) are 0, so the kernel loads unconditionally (a uniform branch around
  // these loads runs into a hipcc ROCm 7.2 code generation error)
  int bias_flags, kb_km, ab_km, rpe_km;
  int dbg;  // experiment switches (DS_FLASH_BWD_DBG): 1 no atomics, 2 no dQ phase, 4 no dK/dV products, 8 no S/dP
};

// NW waves per workgroup, each owning KPW = 256 / NW keys (NC = KPW / 32 column tiles of the S / dP accumulators).
// NW = 4: one wave per SIMD with the whole 512-register file (dK^T/dV^T of 64 keys = 256 accumulator registers),
// every wave also computes one 32-column slice of the tile's dQ; NW = 8: two waves per SIMD, 32 keys each, waves
// 0..3 compute dQ.
template <int NW, bool CAUSAL, bool SPARSE, int BIASED = 0>
__global__ void __launch_bounds__(NW * 64, 1) flash_bwd_kernel(BwdArgs a) {
  constexpr int NTHR = NW * 64, KPW = KB / NW, NC = KPW / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the wave index lives in a scalar register (wave-uniform), everything lane-dependent in vector registers
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            l32 = lane & 31;
  const int S = a.S;
  const int nkb = (S + KB - 1) / KB;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = logical / nkb, kb = logical % nkb;  // causal: low key blocks (most tiles) first within a head
  const int b = bh / a.Hk, hk = bh % a.Hk, rep = a.Hq / a.Hk;
  const int k0 = kb * KB;
  const int ntq = (S + QT - 1) / QT;

  char* Kimg = smem;
  char* QD = smem + K_BYTES;                      // [NBUF][Q tile | dO tile]
  char* DSimg = QD + NBUF * 2 * TILE;             // [2][KB][32] bf16
  float* LD = reinterpret_cast<float*>(DSimg + 2 * DS_BYTES);  // [NBUF][lse (32) | delta (32)]
  uint8_t* FL = reinterpret_cast<uint8_t*>(LD + NBUF * 64);       // [2][8 slabs]: slab met the tile

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
  // by LDS-DMA, two tiles ahead of the one being computed (no staging registers, no wait until the barrier that
  // precedes its use). Only the waves that issue no dQ atomics stage: `s_waitcnt vmcnt` counts loads, LDS-DMA and
  // atomics together in issue order, so a wave that had its tile's 16 dQ atomics in flight ahead of its next DMA
  // would have to wait for those memory-side atomics to retire (thousands of cycles with every CU adding) before
  // the barrier that publishes the DMA — and every wave of the workgroup waits at that barrier. With the staging on
  // the loader waves the atomics of waves 0..3 are never waited on inside the loop (they drain in the background,
  // the hardware's outstanding-request limit is the only back-pressure).
  // Loader wave lw fills the 1-KB pieces lw + 4i of the swizzled Q and dO images: lane L of piece j lands at physical
  // chunk 64j + L, i.e. row 4j + L/16, physical chunk L%16, so it fetches the logical chunk (L%16) ^ swizzle(row) —
  // the swizzle goes on the SOURCE address. Loader 0 also moves the 32 lse and 32 delta values (4 B per lane).
  static_assert(NW == 8, "the loader / dQ wave split assumes 8 waves");
  constexpr int NLOAD = 4, LPIECES = 8 / NLOAD;  // loader waves 4..7, 1-KB pieces of one 8-KB tile per loader
  const bool loader = w >= NW - NLOAD;
  const int lw = w - (NW - NLOAD);
  auto stage = [&](int it, int buf) {
    if (!loader) return;
    int hq, qt;
    tile_at(it, hq, qt);
    int lane = threadIdx.x & 63;  // re-derived (and laundered) here: hoisted lane values were spilled
    asm volatile("" : "+v"(lane));
    const bf16* qb = a.q + b * a.qsb + hq * a.qsh;
    const bf16* ob = a.dout + b * a.osb + hq * a.osh;
#pragma unroll
    for (int i = 0; i < LPIECES; ++i) {
      const int j = lw + i * NLOAD, row = 4 * j + (lane >> 4), pch = lane & 15;
      const int ch = pch ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const int64_t qr = min(qt * QT + row, S - 1);
      glds16(qb + qr * a.qss + ch * 8, QD + buf * 2 * TILE + 1024 * j);
      glds16(ob + qr * a.oss + ch * 8, QD + buf * 2 * TILE + TILE + 1024 * j);
    }
    if (lw == 0) {
      const int r = min(qt * QT + (lane & 31), S - 1);
      const int64_t idx = ((int64_t)b * a.Hq + hq) * S + r;
      glds4(lane < 32 ? (const void*)(a.lse + idx) : (const void*)(a.delta + idx), (const char*)(LD + buf * 64));
    }
  };
  // loaders: s_waitcnt vmcnt(N) with N = the DMA instructions they issued for the newest tile (so the older tile has
  // landed); everyone: lgkmcnt(0) (this wave's LDS writes done) and the raw barrier (no vmcnt(0) drain)
  auto barrier_keep_newest = [&](bool newest_in_flight) {
    if (!loader) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (newest_in_flight) {
      if (lw == 0) asm volatile("s_waitcnt vmcnt(5)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };

  // ------------------------------------------------------------------ resident K image + per-wave V fragments
  for (int i = tid; i < KB * 16; i += NTHR) {
    const int row = i >> 4, ch = i & 15;
    const int key = min(k0 + row, S - 1);
    *reinterpret_cast<u32x4_t*>(Kimg + lds_off(row, ch)) =
        *reinterpret_cast<const u32x4_t*>(Kp + (int64_t)key * a.kss + ch * 8);
  }
  const int kw0 = k0 + KPW * w;       // first key of this wave
  // V rows stay in registers (B operand of dP); K rows are read from the resident image (it also feeds dQ)
  bf16x8_t vf[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int kr = min(kw0 + 32 * c + l32, S - 1);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
      vf[c][kk] = *reinterpret_cast<const bf16x8_t*>(Vp + (int64_t)kr * a.vss + 16 * kk + 8 * h);
  }

  // ------------------------------------------------------------------ per-lane LDS address bases
  // transposed-read lane geometry (see flash_fwd.hip): lane reads row rb + gq, 16-B chunk c0 + 2*colhalf + gch,
  // byte gb; it receives rows rb..rb+3 of column (lane & 31) of the addressed 32-column slab. Displacements of 16
  // rows keep the swizzle phase, so every address is  base + (small XOR term) + compile-time displacement: the
  // XOR of the chunk index with the row's swizzle splits into a per-lane base and a 2-3-bit per-lane toggle.
  // The bases are laundered at the top of each tile (asm) so hipcc recomputes the few derived addresses (2 VALU
  // each) instead of hoisting ~40 of them into registers — at 2 waves per SIMD that is the difference between
  // spilling and not.
  const int gq = (lane >> 2) & 3, gch = (lane >> 1) & 1, gb = 8 * (lane & 1), colhalf = (lane >> 4) & 1;
  const int ds_unit = 4 * colhalf + 2 * gch + (lane & 1);
  auto swz = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
  // row reads (operands of S and dP): lds_off(l32, 2kk+h) for the eight k-steps, as 32-bit LDS addresses of this
  // wave's K rows; the Q / dO tile rows of the ring buffer in use sit at a wave-uniform distance from them, so a
  // tile's sixteen Q / dO reads cost eight adds in all and everything else is a compile-time displacement
  const lds_char* s3 = (const lds_char*)smem;
  uint32_t kaddr[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) kaddr[kk] = (uint32_t)((KPW * w + l32) * 256 + 16 * ((2 * kk + h) ^ swz(l32)));
  // transposed tile reads: lds_off(4h+8hi+gq, 4dt + 2colhalf + gch) + gb = tbase[hi] + 64 * (dt ^ ttog[hi])
  int tbase[2], ttog[2];
  // dQ: transposed reads of the K image and of the dS^T image (no toggle: 16-row steps)
  const int wq = w & 3;  // the 32-column d slice of dQ this wave computes (waves 0..3)
  int kqoff[2], dsqoff[2];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi) {
    const int row = 4 * h + 8 * hi + gq, f = swz(row);
    tbase[hi] = row * 256 + 16 * ((colhalf * 2 + gch) ^ (f & 3)) + gb;
    ttog[hi] = f >> 2;
    kqoff[hi] = lds_off(8 * h + 4 * hi + gq, wq * 4 + colhalf * 2 + gch) + gb;
    dsqoff[hi] = ds_off(8 * h + 4 * hi + gq, ds_unit);
  }
  // dS^T stores: ds_off(l32, 2g+h) = dwbase + 16 * (g ^ dwtog)
  const int dsx = (l32 >> 1) & 7;
  int dwbase = l32 * 64 + 8 * (h ^ (dsx & 1)), dwtog = dsx >> 1;

  f32x16_t dk[NC][4], dv[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) dk[c][dt][r] = dv[c][dt][r] = 0.f;

  // K image / V rows landed before the DMA starts: consuming the V fragments here makes hipcc's own waitcnt pass
  // retire them now instead of waiting vmcnt(0) (= draining the DMA) at their first use inside the tile loop
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) asm volatile("" : : "v"(vf[c][kk]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (n_it > 0) stage(0, 0);
  if (n_it > 1) stage(1, 1);
  barrier_keep_newest(n_it > 1);

  for (int it = 0; it < n_it; ++it) {
    const int cur = it & 1, tb = it % NBUF;
    asm volatile("" : "+v"(tbase[0]), "+v"(tbase[1]), "+v"(ttog[0]), "+v"(ttog[1]),
                 "+v"(dwbase), "+v"(dwtog), "+v"(kqoff[0]), "+v"(kqoff[1]), "+v"(dsqoff[0]), "+v"(dsqoff[1]));
    int hq, qt;
    tile_at(it, hq, qt);
    const int q0 = qt * QT;
    if (it + 2 < n_it) stage(it + 2, (it + 2) % NBUF);

    const char* Qt = QD + tb * 2 * TILE;
    const char* Ot = Qt + TILE;
    const float* lse2 = LD + tb * 64;
    const float* dlt = lse2 + 32;
    char* DSc = DSimg + cur * DS_BYTES;

    // ---------------- which of this wave's 32-key slabs meet the tile? keep[c] bit r: accumulator row r unmasked
    bool act[NC];
    unsigned keep[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ks = kw0 + 32 * c, mykey = ks + l32;
      act[c] = ks < S && (!CAUSAL || ks <= q0 + QT - 1);
      keep[c] = mykey < S ? 0xffffu : 0u;
      if constexpr (SPARSE) {
        const int lh = a.lay_heads == 1 ? 0 : hq;
        const int kbl = min(mykey, S - 1) / a.blk;
        const uint8_t* lay = a.layout + (int64_t)lh * a.nb * a.nb;
        const int r0 = q0 / a.blk;
        const unsigned a0 = lay[(int64_t)r0 * a.nb + kbl] ? 0xffffu : 0u;
        if (a.blk < QT) {  // 16-row blocks: registers 0..7 are rows 0..15 of the tile, 8..15 rows 16..31
          const unsigned a1 = lay[(int64_t)min(r0 + 1, a.nb - 1) * a.nb + kbl] ? 0xffffu : 0u;
          keep[c] &= (a0 & 0x00ffu) | (a1 & 0xff00u);
        } else {
          keep[c] &= a0;
        }
        act[c] = act[c] && __any(keep[c] != 0);
      }
      if (q0 + QT > S) {  // padded query rows of the last tile
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (q0 + crow(r, h) >= S) keep[c] &= ~(1u << r);
      }
      if (CAUSAL && act[c] && ks + 31 > q0) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (mykey > q0 + crow(r, h)) keep[c] &= ~(1u << r);
      }
    }
    // one 32-key slab at a time (bounds the live S / dP accumulators to 32 registers)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!act[c] || (a.dbg & 8)) continue;
      // ---------------- S' = Q.K^T - LSE/scale and dP' = dO.V^T - delta (query rows in registers, key on the
      // lane); the row constants are the accumulators' initial values
      f32x16_t s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(lse2 + 8 * g + 4 * h);
        const f32x4 y = *reinterpret_cast<const f32x4*>(dlt + 8 * g + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s[4 * g + i] = x[i]; dp[4 * g + i] = y[i]; }
      }
      // Operand reads run two MFMAs ahead of their use (S: Q and K rows, dP: dO rows; V is in registers): left to
      // itself hipcc issued each ds_read right before its MFMA with lgkmcnt(0) in between, so all sixteen MFMAs paid
      // a full LDS round trip. sched_barrier pins the order (VALU / SALU may cross, MFMA / LDS may not).
      {
        const uint32_t qdelta = (uint32_t)(K_BYTES + tb * 2 * TILE - KPW * w * 256);  // wave-uniform
        uint32_t qaddr[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) qaddr[kk] = kaddr[kk] + qdelta;
        auto ld_q = [&](int kk) { return *reinterpret_cast<const lds_bf16x8*>(s3 + qaddr[kk]); };
        auto ld_o = [&](int kk) { return *reinterpret_cast<const lds_bf16x8*>(s3 + qaddr[kk] + TILE); };
        auto ld_k = [&](int kk) { return *reinterpret_cast<const lds_bf16x8*>(s3 + kaddr[kk] + 32 * c * 256); };
        bf16x8_t a0 = ld_q(0), b0 = ld_k(0), a1 = ld_q(1), b1 = ld_k(1);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          bf16x8_t a2, b2;
          if (i + 2 < 8) {
            a2 = ld_q(i + 2);
            b2 = ld_k(i + 2);
          } else if (i + 2 < 16) {
            a2 = ld_o(i + 2 - 8);
          }
          __builtin_amdgcn_sched_barrier(0x6);
          if (i < 8) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, s, 0, 0, 0);
          else dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, vf[c][i - 8], dp, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0x6);
          a0 = a1;
          b0 = b1;
          a1 = a2;
          b1 = b2;
        }
      }
      // ---------------- P and dS, dS^T -> LDS (row = key, 8-B unit g*2+h holds queries 8g+4h .. +3)
      // P and dS in fp32, then packed two per instruction (v_cvt_pk_bf16_f32; hipcc lowers a vector fptrunc to one
      // convert + v_perm per element). Masking only when some lane of the wave needs it (diagonal / padded tiles):
      // the per-element select costs 4 VALU and the VALU issue slots are the co-bottleneck beside the MFMAs.
      float pf[16], df[16];
      const bool need_mask = keep[c] != 0xffffu;
      if constexpr (BIASED != 0) {
        // P = exp2(c * S' + log2(e) * bias): the per-key bias is one constant per lane, attention-mask / relative
        // position values are read per (query row, key) — consecutive lanes read consecutive keys of one row.
        // BIASED == 1: per-key bias only (BERT padding masks); 2: all three terms.
        const int mykey = min(kw0 + 32 * c + l32, S - 1);
        const float l2e = 1.4426950408889634f;
        const float kb = a.kbias[(int64_t)b * a.kb_stride + (int64_t)mykey * a.kb_km] * l2e;
        const float* abp = a.abias + (int64_t)mykey * a.ab_km;
        const float* rpp = a.rpe + (int64_t)hq * a.rpe_hs + (int64_t)mykey * a.rpe_km;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float bv = kb;
          if constexpr (BIASED == 2) {
            const int qr = min(q0 + crow(r, h), S - 1);
            bv = fmaf(abp[(int64_t)qr * a.ab_stride] + rpp[(int64_t)qr * a.rpe_rs], l2e, bv);
          }
          float p = __builtin_amdgcn_exp2f(fmaf(s[r], a.c, bv));
          if (!((keep[c] >> r) & 1u)) p = 0.f;
          pf[r] = p;
          df[r] = p * dp[r];
        }
      } else if (__any(need_mask)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = __builtin_amdgcn_exp2f(s[r] * a.c);
          if (!((keep[c] >> r) & 1u)) p = 0.f;
          pf[r] = p;
          df[r] = p * dp[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          pf[r] = __builtin_amdgcn_exp2f(s[r] * a.c);
          df[r] = pf[r] * dp[r];
        }
      }
      bf16x8_t pb[2], dsb[2];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        u32x4_t pu, du;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pu[i] = pack_bf16(pf[8 * g + 2 * i], pf[8 * g + 2 * i + 1]);
          du[i] = pack_bf16(df[8 * g + 2 * i], df[8 * g + 2 * i + 1]);
        }
        pb[g] = __builtin_bit_cast(bf16x8_t, pu);
        dsb[g] = __builtin_bit_cast(bf16x8_t, du);
      }
      char* dsw = DSc + (KPW * w + 32 * c) * 64;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // whole-vector bit cast: per-element __builtin_bit_cast(short, bf16 element) is miscompiled by hipcc
        // (ROCm 7.2) into a splat of one element (tools/probe_flash_bwd2.py)
        const s16x8 d8 = __builtin_bit_cast(s16x8, dsb[g >> 1]);
        s16x4 v4;
#pragma unroll
        for (int i = 0; i < 4; ++i) v4[i] = d8[4 * (g & 1) + i];
        *reinterpret_cast<s16x4*>(dsw + dwbase + 16 * (g ^ dwtog)) = v4;
      }
      // ---------------- dV^T += dO^T.P, dK^T += Q^T.dS   (A operands by transposed reads of the tile images)
      // 16 MFMAs, i = (dt, s2, O|Q). The transposed reads of operand i+2 are issued before MFMA i and the order is
      // pinned with sched_barrier (ALU may cross, MFMA / LDS may not; a full barrier hits a hipcc ROCm 7.2 codegen
      // error): left to itself the scheduler reused one operand quad and waited lgkmcnt(0) in front of every MFMA
      // (LDS latency fully exposed; SQ_VALU_MFMA_BUSY_CYCLES put the kernel at ~29 % MFMA utilisation).
      if (!(a.dbg & 4)) {
        auto opnd = [&](int i) {
          const int dt = i >> 2, s2 = (i >> 1) & 1;
          const char* base = Qt + ((i & 1) ? 0 : TILE) + 4096 * s2;  // Ot = Qt + TILE (integer select)
          const int t0a = tbase[0] + 64 * (dt ^ ttog[0]), t1a = tbase[1] + 64 * (dt ^ ttog[1]);
          return join(tr_read(base + t0a), tr_read(base + t1a));
        };
        bf16x8_t o0 = opnd(0), o1 = opnd(1);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          bf16x8_t o2;
          if (i + 2 < 16) o2 = opnd(i + 2);
          __builtin_amdgcn_sched_barrier(0x7);
          const int dt = i >> 2, s2 = (i >> 1) & 1;
          if (i & 1) dk[c][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o0, dsb[s2], dk[c][dt], 0, 0, 0);
          else dv[c][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o0, pb[s2], dv[c][dt], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0x7);
          o0 = o1;
          o1 = o2;
        }
      }
    }
    // the dQ product walks only the slabs that met this tile
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) FL[cur * 8 + NC * w + c] = act[c] ? 1 : 0;
    }

    barrier_keep_newest(it + 2 < n_it);

    // ---------------- dQ[q0:q0+32, 32wq:32wq+32] += dS . K over the slabs that met the tile (waves 0..3; waves
    // 4..7 run ahead into the next tile, so the SIMDs stay busy). Measured against an even 8-wave split on
    // 16x16x32 MFMAs: this form is 5% faster end to end (fewer transposed reads per MFMA).
    if (w < 4 && !(a.dbg & 2)) {
      const uint64_t fl = *reinterpret_cast<const uint64_t*>(FL + cur * 8);
      const uint32_t flo = __builtin_amdgcn_readfirstlane((uint32_t)fl),
                     fhi = __builtin_amdgcn_readfirstlane((uint32_t)(fl >> 32));
      f32x16_t dq;
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[r] = 0.f;
      int nks = 0;
      auto ld_a = [&](int s2) {
        return join(tr_read(DSc + 1024 * s2 + dsqoff[0]), tr_read(DSc + 1024 * s2 + dsqoff[1]));
      };
      auto ld_b = [&](int s2) {
        return join(tr_read(Kimg + 4096 * s2 + kqoff[0]), tr_read(Kimg + 4096 * s2 + kqoff[1]));
      };
      if constexpr (SPARSE) {
#pragma unroll 1
        for (int slab = 0; slab < 8; ++slab) {
          if (!(((slab < 4 ? flo : fhi) >> (8 * (slab & 3))) & 0xff)) continue;
          const bf16x8_t a0 = ld_a(2 * slab), b0 = ld_b(2 * slab), a1 = ld_a(2 * slab + 1), b1 = ld_b(2 * slab + 1);
          dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, dq, 0, 0, 0);
          dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, dq, 0, 0, 0);
          ++nks;
        }
      } else {
        // keys up to the diagonal (causal) / the sequence end, as 16-key MFMA steps
        int kmax = min(KB, S - k0);
        if (CAUSAL) kmax = min(kmax, q0 + QT - k0);
        nks = (kmax + 15) >> 4;
        (void)flo;
        (void)fhi;
        if (nks == KB / 16) {  // every key block but the diagonal one: straight-line, scheduled by hipcc
#pragma unroll
          for (int s2 = 0; s2 < KB / 16; ++s2)
            dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_a(s2), ld_b(s2), dq, 0, 0, 0);
        } else {
#pragma unroll 1
          for (int s2 = 0; s2 < nks; ++s2)
            dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_a(s2), ld_b(s2), dq, 0, 0, 0);
        }
      }
      if (nks > 0 && !(a.dbg & 1)) {
        // lane part of the 16 destination rows, laundered so that hipcc forms each address next to its atomic
        // instead of keeping 16 64-bit addresses live across the loop (they spilled). One register of a 32x32
        // accumulator = two 128-B row segments, the full-rate atomic shape.
        int ln = threadIdx.x;
        asm volatile("" : "+v"(ln));
        const int lofs = 4 * ((ln >> 5) & 1) * D + 32 * ((ln >> 6) & 3) + (ln & 31);
        // wave-uniform 64-bit base (scalar registers) + 32-bit per-lane element offset: the atomics take the
        // saddr form instead of a 64-bit VGPR address built with an add/addc pair per atomic
        float* dqb = a.dqacc + (((int64_t)b * a.Hq + hq) * S + q0) * D;
        const int lim = S - q0 - 4 * ((ln >> 5) & 1);  // rows (r&3) + 8(r>>2) below lim are inside the sequence
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = (r & 3) + 8 * (r >> 2);
          if (qr < lim) unsafeAtomicAdd(dqb + (lofs + qr * D), dq[r]);
        }
      }
    }
  }

  // ------------------------------------------------------------------ epilogue: dK = scale * dK^T^T, dV
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int mykey = kw0 + 32 * c + l32;
    if (mykey >= S) continue;
    bf16* dkp = a.dk + b * a.dksb + hk * a.dksh + (int64_t)mykey * a.dkss;
    bf16* dvp = a.dv + b * a.dvsb + hk * a.dvsh + (int64_t)mykey * a.dvss;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 k4, v4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          k4[i] = (bf16)(dk[c][dt][4 * g + i] * a.scale);
          v4[i] = (bf16)dv[c][dt][4 * g + i];
        }
        const int d0 = 32 * dt + 8 * g + 4 * h;
        *reinterpret_cast<bf16x4*>(dkp + d0) = k4;
        *reinterpret_cast<bf16x4*>(dvp + d0) = v4;
      }
  }
}

// Row constants of the main kernel's accumulator initialisation, pre-negated / pre-scaled so the main loop spends
// no VALU on them: nrow[row] = -sum_d O*dO (-delta), nrow[rows + row] = -LSE / scale. Also zeroes the dQ accumulator
// row. 16 threads per row, 8 elements each.
__global__ void __launch_bounds__(256) flash_bwd_pre_kernel(const bf16* __restrict__ O, const bf16* __restrict__ dO,
                                                            const float* __restrict__ lse, float* __restrict__ nrow,
                                                            float* __restrict__ dqacc, int Hq, int S, int64_t rows,
                                                            int64_t osb, int64_t osh, int64_t oss, int64_t gsb,
                                                            int64_t gsh, int64_t gss, float inv_scale) {
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
  if (sub == 0) {
    nrow[row] = -acc;
    nrow[rows + row] = -lse[row] * inv_scale;
  }
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

template <int NW, bool C, bool SP, int BI = 0>
int launch_main(const BwdArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&flash_bwd_kernel<NW, C, SP, BI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<NW>());
    attr = true;
  }
  const int nkb = (a.S + KB - 1) / KB;
  const int grid = a.B * a.Hk * nkb;
  hipLaunchKernelGGL((flash_bwd_kernel<NW, C, SP, BI>), dim3(grid), dim3(NW * 64), lds_bytes<NW>(), st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

template <int NW>
int launch_mode(const BwdArgs& a, int mode, hipStream_t st) {
  if (mode == 2 && a.bias_flags == 1) return launch_main<NW, false, true, 1>(a, st);
  if (mode == 2 && a.bias_flags) return launch_main<NW, false, true, 2>(a, st);
  return mode == 1 ? launch_main<NW, true, false>(a, st)
                   : (mode == 2 ? launch_main<NW, false, true>(a, st) : launch_main<NW, false, false>(a, st));
}

}  // namespace

// Strides are (batch, head, seq) in elements, unit last stride everywhere, all bf16 rows 16-B aligned.
// q/o/dout/dq [B,Hq,S,128], k/v/dk/dv [B,Hk,S,128], lse [B,Hq,S] natural-log (flash_fwd's), workspace:
// delta [2*B*Hq*S] fp32 (the pre kernel's -delta and -LSE/scale rows) and dqacc [B*Hq*S*128] fp32.
// mode: 0 full, 1 causal (top-left), 2 block-sparse (LUT below).
extern "C" int ds_flash_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, float* delta, float* dqacc, void* dq, void* dk, void* dv, int B, int Hq,
                            int Hk, int S, const int64_t* qs, const int64_t* ks, const int64_t* vs, const int64_t* os,
                            const int64_t* dos, const int64_t* dqs, const int64_t* dks, const int64_t* dvs,
                            float scale, int mode, const int* qtiles, const int* nqt, const uint8_t* layout, int maxt,
                            int lay_heads, int nb, int blk, int bias_flags, const float* kbias, int64_t kb_stride,
                            const float* abias, int64_t ab_stride, const float* rpe, int64_t rpe_hs, int64_t rpe_rs,
                            hipStream_t st) {
  if (Hk <= 0 || Hq % Hk != 0 || S <= 0 || B <= 0) return (int)hipErrorInvalidValue;
  if (mode == 2 && (qtiles == nullptr || nqt == nullptr || layout == nullptr || (lay_heads != 1 && lay_heads != Hq) ||
                    (blk != 16 && blk != 32 && blk != 64 && blk != 128) || nb * blk < S))
    return (int)hipErrorInvalidValue;
  const int64_t rows = (int64_t)B * Hq * S;
  const int pgrid = (int)((rows + 15) / 16);
  hipLaunchKernelGGL(flash_bwd_pre_kernel, dim3(pgrid), dim3(256), 0, st, (const bf16*)o, (const bf16*)dout, lse,
                     delta, dqacc, Hq, S, rows, os[0], os[1], os[2], dos[0], dos[1], dos[2], 1.f / scale);
  DS_CHECK_LAUNCH();
  BwdArgs a;
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.dout = (const bf16*)dout;
  a.lse = delta + rows; a.delta = delta; a.dqacc = dqacc; a.dk = (bf16*)dk; a.dv = (bf16*)dv;  // pre-kernel rows
  a.B = B; a.Hq = Hq; a.Hk = Hk; a.S = S;
  a.qsb = qs[0]; a.qsh = qs[1]; a.qss = qs[2];
  a.ksb = ks[0]; a.ksh = ks[1]; a.kss = ks[2];
  a.vsb = vs[0]; a.vsh = vs[1]; a.vss = vs[2];
  a.osb = dos[0]; a.osh = dos[1]; a.oss = dos[2];
  a.dksb = dks[0]; a.dksh = dks[1]; a.dkss = dks[2];
  a.dvsb = dvs[0]; a.dvsh = dvs[1]; a.dvss = dvs[2];
  a.c = scale * 1.4426950408889634f;
  a.scale = scale;
  { const char* e = getenv("DS_FLASH_BWD_DBG"); a.dbg = e ? atoi(e) : 0; }
  a.qtiles = qtiles; a.nqt = nqt; a.layout = layout; a.maxt = maxt; a.lay_heads = lay_heads; a.nb = nb; a.blk = blk;
  // biases: block-sparse path only; with any bias present every pointer must be valid (see BwdArgs::bias_flags)
  if (bias_flags && (mode != 2 || !kbias || !abias || !rpe)) return (int)hipErrorInvalidValue;
  a.kbias = kbias; a.abias = abias; a.rpe = rpe;
  a.bias_flags = bias_flags;
  a.kb_km = bias_flags & 1; a.ab_km = (bias_flags >> 1) & 1; a.rpe_km = (bias_flags >> 2) & 1;
  a.kb_stride = a.kb_km ? kb_stride : 0; a.ab_stride = a.ab_km ? ab_stride : 0;
  a.rpe_hs = a.rpe_km ? rpe_hs : 0; a.rpe_rs = a.rpe_km ? rpe_rs : 0;
  int rc = launch_mode<8>(a, mode, st);
  if (rc) return rc;
  hipLaunchKernelGGL(flash_bwd_post_kernel, dim3(pgrid), dim3(256), 0, st, dqacc, (bf16*)dq, Hq, S, rows, dqs[0],
                     dqs[1], dqs[2], scale);
  DS_CHECK_LAUNCH();
  return 0;
}
