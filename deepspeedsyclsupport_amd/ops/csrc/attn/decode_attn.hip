// Paged (blocked-KV) decode attention for inference, CDNA4 (gfx950).
//
// Parity: reference v1 `softmax_context` over the in-workspace KV cache (`csrc/transformer/inference/csrc/
// pt_binding.cpp:434-557`, `softmax.cu` attn_softmax_v2 with alibi / causal) and v2 `flash_attn_by_atoms` over the
// blocked KV cache (`inference/v2/kernels/ragged_ops/blocked_flash`). One kernel serves both engines: a contiguous
// per-sequence cache is the special case "one block of max_len tokens per sequence".
//
// Decode is HBM-bound (every cached K and V byte is read once per token), so the design is flash-decoding:
//  * grid = (batch, kv_head, split): each workgroup reads ONE kv head's K/V for a contiguous slice of the sequence
//    once and serves all G = Hq/Hk query heads of that GQA group from it (no K/V re-read per query head);
//  * the sequence is split so the launch has >= ~2 workgroups per CU even at batch 1 (256 CUs);
//  * scores for the slice live in LDS; softmax runs on LDS; P·V streams V rows with 16-B loads, 16 lanes per row;
//  * partial (max, sum, unnormalised acc) per split are merged by a small combine kernel (log-sum-exp). (An in-kernel
//    last-block merge was measured 2x slower: the device-scope fences it needs write back L2.)
// Optional ALiBi slopes (BLOOM) and a sliding window (Mistral) are applied on the fly.
#include "../include/ds_hip.h"

namespace {

constexpr int THREADS = 256;
constexpr int MAXG = 8;          // query heads per kv head handled per workgroup (GQA group)
constexpr int MAX_CHUNK = 1024;  // keys per split (LDS: MAXG * MAX_CHUNK * 4 B = 32 KiB)

template <int D>
__global__ void __launch_bounds__(THREADS) paged_decode_kernel(
    const bf16* __restrict__ q,          // [B, Hq, D]
    const bf16* __restrict__ kc,         // [NB, Hk, BS, D]
    const bf16* __restrict__ vc,         // [NB, Hk, BS, D]
    const int* __restrict__ block_table, // [B, max_blocks]
    const int* __restrict__ seq_lens,    // [B]
    const float* __restrict__ alibi,     // [Hq] or null
    float* __restrict__ part_acc,        // [B, Hq, S, D]  (only if S > 1)
    float* __restrict__ part_ml,         // [B, Hq, S, 2]
    bf16* __restrict__ out,              // [B, Hq, D]  (written directly when S == 1)
    int Hq, int Hk, int BS, int max_blocks, int chunk, float scale, int window) {
  static_assert(D % 16 == 0 && D >= 64 && D <= 256, "head dim");
  extern __shared__ __attribute__((aligned(16))) float sm[];  // scores [G][chunk] + reduction scratch
  const int b = blockIdx.x, kh = blockIdx.y, split = blockIdx.z, S = gridDim.z;
  const int G = Hq / Hk;
  const int T = seq_lens[b];
  const int t0 = split * chunk;
  const int t1 = min(T, t0 + chunk);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tlo = window > 0 ? max(0, T - window) : 0;
  float* scores = sm;                       // [G][chunk]
  float* red = sm + MAXG * MAX_CHUNK;       // [THREADS/64 * MAXG * 2]

  // ---- q of the G heads of this GQA group; LPR lanes cover one row, 8 elements each. LPR is D/8 rounded up to a
  // power of two (head dims 80 and 96 use 16 lanes per row): the surplus lanes carry a zero query, re-read the row's
  // last chunk (a cache hit) and never write
  constexpr int CPR = D / 8;                                   // 16-byte chunks per row
  constexpr int LPR = CPR <= 8 ? 8 : (CPR <= 16 ? 16 : 32);    // lanes per key row (16 for D=128)
  constexpr int RPW = 64 / LPR;                                // rows per wave instruction
  const int sub = lane / LPR, li_raw = lane % LPR, li = li_raw < CPR ? li_raw : CPR - 1;
  const float lane_on = li_raw < CPR ? 1.f : 0.f;
  float qv[MAXG][8];
  // unconditional loads (clamped head index): a guarded load would make the compiler wait on each one in turn
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    const int gc = g < G ? g : G - 1;
    Vec8<bf16>::load(q + ((int64_t)b * Hq + kh * G + gc) * D + li * 8, qv[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[g][j] *= scale * lane_on;
  }
  // ---- phase 1: scores for keys of this split (UNR key rows per lane-group in flight per iteration)
  constexpr int UNR = 4;
  const int* bt = block_table + (int64_t)b * max_blocks;
  const int kstride = (THREADS / 64) * RPW;
  for (int tb = t0 + wid * RPW + sub; tb < t1; tb += kstride * UNR) {
    float kv[UNR][8];
    int blk[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) blk[u] = bt[min(tb + u * kstride, t1 - 1) / BS];  // clamped: always valid
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int tc = min(tb + u * kstride, t1 - 1);
      Vec8<bf16>::load(kc + (((int64_t)blk[u] * Hk + kh) * BS + tc % BS) * D + li * 8, kv[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int t = tb + u * kstride;
      if (t >= t1) continue;  // uniform across the LPR lanes of one key row (the shuffle partners)
#pragma unroll
      for (int g = 0; g < MAXG; ++g) {
        if (g < G) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) s = fmaf(qv[g][j], kv[u][j], s);
#pragma unroll
          for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
          if (li_raw == 0) {
            if (alibi) s += alibi[kh * G + g] * (float)(t - (T - 1));
            if (t < tlo) s = -INFINITY;
            scores[g * MAX_CHUNK + (t - t0)] = s;
          }
        }
      }
    }
  }
  // V rows do not depend on the scores: start the first P.V pass's loads before the softmax phases
  constexpr int ROWS = THREADS / LPR;
  const int r = tid / LPR, c_raw = tid % LPR, c = c_raw < CPR ? c_raw : CPR - 1;
  float vpre[8];
  if (t0 + r < t1) {
    const int blk = bt[(t0 + r) / BS], off = (t0 + r) % BS;
    Vec8<bf16>::load(vc + (((int64_t)blk * Hk + kh) * BS + off) * D + c * 8, vpre);
  }
  __syncthreads();
  // ---- phase 2: per-head max and sum over the split (one wave per head group, strided)
  const int n = t1 - t0;
  for (int g = wid; g < G; g += THREADS / 64) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, scores[g * MAX_CHUNK + i]);
    m = wave_max(m);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = (m == -INFINITY) ? 0.f : __expf(scores[g * MAX_CHUNK + i] - m);
      scores[g * MAX_CHUNK + i] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) {
      red[g * 2] = m;
      red[g * 2 + 1] = l;
    }
  }
  __syncthreads();
  // ---- phase 3: acc[g][d] = sum_t p[g][t] * v[t][d]; LPR lanes per V row, THREADS/LPR rows in flight
  float acc[MAXG][8];
#pragma unroll
  for (int g = 0; g < MAXG; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int tb = t0 + r; tb < t1; tb += ROWS * UNR) {
    float vv[UNR][8];
    int vblk[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) vblk[u] = bt[min(tb + u * ROWS, t1 - 1) / BS];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int tc = min(tb + u * ROWS, t1 - 1);
      if (u == 0 && tb == t0 + r) {
#pragma unroll
        for (int j = 0; j < 8; ++j) vv[u][j] = vpre[j];
      } else {
        Vec8<bf16>::load(vc + (((int64_t)vblk[u] * Hk + kh) * BS + tc % BS) * D + c * 8, vv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int t = tb + u * ROWS;
      if (t >= t1) continue;
#pragma unroll
      for (int g = 0; g < MAXG; ++g) {
        if (g < G) {
          const float p = scores[g * MAX_CHUNK + (t - t0)];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] = fmaf(p, vv[u][j], acc[g][j]);
        }
      }
    }
  }
  __syncthreads();  // scores are dead: reuse their LDS as a [ROWS][D] buffer, one query head at a time
  float* rb = sm;
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    if (g >= G) break;  // block-uniform
    if (c_raw < CPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) rb[r * D + c * 8 + j] = acc[g][j];
    }
    __syncthreads();
    for (int idx = tid; idx < D; idx += THREADS) {
      float s = 0.f;
      for (int rr = 0; rr < ROWS; ++rr) s += rb[rr * D + idx];
      const int hq = kh * G + g;
      const float m = red[g * 2], l = red[g * 2 + 1];
      if (S == 1) {
        out[((int64_t)b * Hq + hq) * D + idx] = (bf16)(l > 0.f ? s / l : 0.f);
      } else {
        part_acc[(((int64_t)b * Hq + hq) * S + split) * D + idx] = s;
        if (idx == 0) {
          part_ml[(((int64_t)b * Hq + hq) * S + split) * 2] = m;
          part_ml[(((int64_t)b * Hq + hq) * S + split) * 2 + 1] = l;
        }
      }
    }
    __syncthreads();
  }
}

template <int D>
__global__ void __launch_bounds__(D) combine_kernel(const float* __restrict__ part_acc,
                                                    const float* __restrict__ part_ml, bf16* __restrict__ out, int S) {
  const int bh = blockIdx.x, d = threadIdx.x;
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, part_ml[((int64_t)bh * S + s) * 2]);
  float num = 0.f, den = 0.f;
  for (int s = 0; s < S; ++s) {
    const float m = part_ml[((int64_t)bh * S + s) * 2], l = part_ml[((int64_t)bh * S + s) * 2 + 1];
    if (m == -INFINITY) continue;
    const float w = __expf(m - M);
    num = fmaf(w, part_acc[((int64_t)bh * S + s) * D + d], num);
    den = fmaf(w, l, den);
  }
  out[(int64_t)bh * D + d] = (bf16)(den > 0.f ? num / den : 0.f);
}

// Write new K/V rows into the paged cache: k,v [B, n_new, Hk, D] token-major; positions start at seq_lens_before[b].
__global__ void __launch_bounds__(256) kv_append_kernel(const bf16* __restrict__ k, const bf16* __restrict__ v,
                                                        bf16* __restrict__ kc, bf16* __restrict__ vc,
                                                        const int* __restrict__ block_table,
                                                        const int* __restrict__ start_pos, int B, int n_new, int Hk,
                                                        int D, int BS, int max_blocks) {
  const int64_t vec_per_row = D / 8;
  const int64_t total = (int64_t)B * n_new * Hk * vec_per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cvec = (int)(i % vec_per_row);
    int64_t r = i / vec_per_row;
    const int h = (int)(r % Hk);
    r /= Hk;
    const int j = (int)(r % n_new), b = (int)(r / n_new);
    const int t = start_pos[b] + j;
    const int blk = block_table[(int64_t)b * max_blocks + t / BS], off = t % BS;
    const int64_t src = (((int64_t)b * n_new + j) * Hk + h) * D + cvec * 8;
    const int64_t dst = (((int64_t)blk * Hk + h) * BS + off) * D + cvec * 8;
    *reinterpret_cast<bf16x8*>(kc + dst) = *reinterpret_cast<const bf16x8*>(k + src);
    *reinterpret_cast<bf16x8*>(vc + dst) = *reinterpret_cast<const bf16x8*>(v + src);
  }
}

// Fused QKV epilogue for inference: split the fused projection output, apply RoPE (rotate-half or GPT-J interleaved,
// partial rotary dims allowed) to q and k, write q [T, Hq, D] and scatter k/v straight into the paged cache
// (optionally also returning contiguous k/v for the prefill attention). Replaces split + 3 copies + 2 RoPE launches
// + kv_append. One workgroup per token; token t belongs to sequence t / n_new at cache slot start_pos[b] + t % n_new.
__global__ void __launch_bounds__(256) qkv_rope_append_kernel(
    const bf16* __restrict__ qkv, const float* __restrict__ cosT, const float* __restrict__ sinT,
    const int* __restrict__ pos, bf16* __restrict__ q_out, bf16* __restrict__ k_out, bf16* __restrict__ v_out,
    bf16* __restrict__ kc, bf16* __restrict__ vc, const int* __restrict__ block_table,
    const int* __restrict__ start_pos, const int* __restrict__ seq_ids, int n_new, int Hq, int Hk, int D, int rot,
    int interleaved, int BS, int max_blocks, float* __restrict__ acc, const bf16* __restrict__ acc_bias, int NP) {
  // grid = (tokens, head groups): 256 threads cover 256 / (D/2) heads of one token, one thread per element pair
  const int H3 = Hq + 2 * Hk, half = D / 2, rh = rot / 2;
  const int tph = half < (int)blockDim.x ? half : (int)blockDim.x;
  // uniform batch: token t is row t % n_new of sequence t / n_new; ragged batch (seq_ids): sequence seq_ids[t],
  // cache slot = its position
  const int t = blockIdx.x, h = blockIdx.y * (blockDim.x / tph) + threadIdx.x / tph;
  const int b = seq_ids ? seq_ids[t] : t / n_new, j = seq_ids ? 0 : t % n_new;
  // acc != null: the fused projection's sums still sit in the weight-only GEMV's fp32 split-K workspace [rows, NP]
  // (skinny_int8.hip / skinny_int4.hip without their finalize pass): read them (+ bias) from there and re-zero what
  // was read, padding columns included, so this kernel IS that GEMV's finalize pass
  float* arow = acc ? acc + (int64_t)t * NP : nullptr;
  if (arow && blockIdx.y == 0)
    for (int i = H3 * D + threadIdx.x; i < NP; i += blockDim.x) arow[i] = 0.f;
  // (head dims whose half does not divide the block leave a few surplus threads at the end)
  if (h >= H3 || (int)threadIdx.x / tph >= (int)blockDim.x / tph) return;
  const bf16* src = acc ? nullptr : qkv + ((int64_t)t * H3 + h) * D;
  auto ld = [&](int d) -> float {
    if (arow == nullptr) return (float)src[d];
    const float v = arow[h * D + d] + (acc_bias ? (float)acc_bias[h * D + d] : 0.f);
    arow[h * D + d] = 0.f;
    return (float)(bf16)v;  // the unfused path rounds the projection to bf16 before RoPE
  };
  bf16* dst;
  bf16* extra = nullptr;
  if (h < Hq) {
    dst = q_out + ((int64_t)t * Hq + h) * D;
  } else {
    const bool isk = h < Hq + Hk;
    const int kh = isk ? h - Hq : h - Hq - Hk;
    const int slot = seq_ids ? pos[t] : start_pos[b] + j;
    const int blk = block_table[(int64_t)b * max_blocks + slot / BS], off = slot % BS;
    dst = (isk ? kc : vc) + (((int64_t)blk * Hk + kh) * BS + off) * D;
    if (isk ? k_out : v_out) extra = (isk ? k_out : v_out) + ((int64_t)t * Hk + kh) * D;
  }
  const int p = pos[t];
  for (int i = threadIdx.x % tph; i < half; i += tph) {
    int d0, d1;
    if (i < rh) {
      d0 = interleaved ? 2 * i : i;
      d1 = interleaved ? 2 * i + 1 : i + rh;
    } else {
      d0 = rot + 2 * (i - rh);
      d1 = d0 + 1;
    }
    float a = ld(d0), c = ld(d1);
    if (i < rh && h < Hq + Hk) {
      const float cs = cosT[(int64_t)p * rh + i], sn = sinT[(int64_t)p * rh + i];
      const float a2 = a * cs - c * sn;
      c = c * cs + a * sn;
      a = a2;
    }
    dst[d0] = (bf16)a;
    dst[d1] = (bf16)c;
    if (extra) {
      extra[d0] = (bf16)a;
      extra[d1] = (bf16)c;
    }
  }
}

}  // namespace

extern "C" int ds_paged_decode_splits(int B, int Hk, int max_len) {
  // enough workgroups to cover the chip ~2x, splits of >= 64 keys, <= MAX_CHUNK keys per split
  const int want = (512 + B * Hk - 1) / (B * Hk);
  int chunk = (max_len + want - 1) / want;
  chunk = ((chunk + 63) / 64) * 64;
  if (chunk < 64) chunk = 64;
  if (chunk > MAX_CHUNK) chunk = MAX_CHUNK;
  return (max_len + chunk - 1) / chunk;
}

extern "C" int ds_paged_decode(const void* q, const void* kc, const void* vc, const int* block_table,
                               const int* seq_lens, const float* alibi, float* part_acc, float* part_ml, void* out,
                               int B, int Hq, int Hk, int D, int BS, int max_blocks, int max_len, int splits,
                               float scale, int window, hipStream_t s) {
  if (Hq % Hk || Hq / Hk > MAXG) return (int)hipErrorInvalidValue;
  const int chunk = ((max_len + splits - 1) / splits + 63) / 64 * 64;
  if (chunk > MAX_CHUNK) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(MAXG * MAX_CHUNK + 64) * sizeof(float);
  dim3 grid(B, Hk, splits);
#define LAUNCH(DD)                                                                                                  \
  hipLaunchKernelGGL((paged_decode_kernel<DD>), grid, dim3(THREADS), lds, s, (const bf16*)q, (const bf16*)kc,       \
                     (const bf16*)vc, block_table, seq_lens, alibi, part_acc, part_ml, (bf16*)out, Hq, Hk, BS,       \
                     max_blocks, chunk, scale, window);                                                             \
  DS_CHECK_LAUNCH();                                                                                                \
  if (splits > 1) {                                                                                                 \
    hipLaunchKernelGGL((combine_kernel<DD>), dim3(B * Hq), dim3(DD), 0, s, part_acc, part_ml, (bf16*)out, splits);  \
    DS_CHECK_LAUNCH();                                                                                              \
  }
  if (D == 64) { LAUNCH(64) }
  else if (D == 80) { LAUNCH(80) }
  else if (D == 96) { LAUNCH(96) }
  else if (D == 128) { LAUNCH(128) }
  else if (D == 256) { LAUNCH(256) }
  else return (int)hipErrorInvalidValue;
#undef LAUNCH
  return 0;
}

extern "C" int ds_kv_append(const void* k, const void* v, void* kc, void* vc, const int* block_table,
                            const int* start_pos, int B, int n_new, int Hk, int D, int BS, int max_blocks,
                            hipStream_t s) {
  if (D % 8) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for((int64_t)B * n_new * Hk * (D / 8), 256);
  hipLaunchKernelGGL(kv_append_kernel, dim3(grid), dim3(256), 0, s, (const bf16*)k, (const bf16*)v, (bf16*)kc,
                     (bf16*)vc, block_table, start_pos, B, n_new, Hk, D, BS, max_blocks);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_qkv_rope_append(const void* qkv, const float* cosT, const float* sinT, const int* pos, void* q_out,
                                  void* k_out, void* v_out, void* kc, void* vc, const int* block_table,
                                  const int* start_pos, const int* seq_ids, int T, int n_new, int Hq, int Hk, int D,
                                  int rot, int interleaved, int BS, int max_blocks, float* acc, const void* acc_bias,
                                  int NP, hipStream_t s) {
  if (D % 2 || rot % 2 || rot > D || (D - rot) % 2 || T <= 0) return T == 0 ? 0 : (int)hipErrorInvalidValue;
  if (acc != nullptr && (NP < (Hq + 2 * Hk) * D || T > 16)) return (int)hipErrorInvalidValue;
  if (acc == nullptr && qkv == nullptr) return (int)hipErrorInvalidValue;
  const int tph = D / 2 < 256 ? D / 2 : 256, hpb = 256 / tph;
  hipLaunchKernelGGL(qkv_rope_append_kernel, dim3(T, (Hq + 2 * Hk + hpb - 1) / hpb), dim3(256), 0, s, (const bf16*)qkv, cosT, sinT, pos,
                     (bf16*)q_out, (bf16*)k_out, (bf16*)v_out, (bf16*)kc, (bf16*)vc, block_table, start_pos, seq_ids,
                     n_new, Hq, Hk, D, rot, interleaved, BS, max_blocks, acc, (const bf16*)acc_bias, NP);
  DS_CHECK_LAUNCH();
  return 0;
}
