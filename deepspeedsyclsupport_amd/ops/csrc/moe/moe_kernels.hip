// Mixture-of-experts routing + grouped expert GEMM, and the ragged-batch gathers of inference v2, CDNA4.
//
// Reference counterparts (behaviour, not code): `inference/v2/kernels/ragged_ops/top_k_gating/top_k_gating.cu:15`,
// `moe_scatter/moe_scatter.cu:23`, `moe_gather/moe_gather.cu:21`, the CUTLASS grouped `moe_gemm`
// (`inference/v2/kernels/cutlass_ops/moe_gemm`, prebuilt libdeepspeedft), `ragged_embed/embed.cu:19`,
// `logits_gather/logits_gather.cu:19`.
//
// MI355X design:
//  * top-k gating: one wave64 per token, each lane owns up to 4 experts (E <= 256); k rounds of a wave argmax with
//    lower-index tie-break (torch.topk / argmax semantics), softmax over all E in fp32, optional renormalisation of
//    the k weights; expert slot = atomicAdd on the expert's counter, so no host sync and no sort;
//  * scatter: every block rebuilds the exclusive prefix of the E counters in LDS (E <= 256: one wave scan) and
//    copies its token row to each assigned expert slot with 16-B vector moves; block 0 publishes the cumsum;
//  * grouped GEMM Y[rows of e] = X[rows of e] . W_e^T on v_mfma_f32_32x32x16_bf16: 128x128 output tiles, K tiles of
//    128 staged through a 256-B-row LDS image whose 16-B chunks are XOR-swizzled by row (conflict-free row reads for
//    both operands), global loads for the next K tile issued before the current tile's MFMAs; the m-tile -> expert
//    map is derived on device from the counters, so the whole MoE block is capturable in a hipGraph;
//  * gather: out[t] = sum_k w[t,k] * Y[slot[t,k]] in fp32, one block per token, 16-B vectors.
#include "ds_hip.h"

namespace {

constexpr int MAXE = 256;

// ------------------------------------------------------------------------------------------------ top-k gating
template <typename T>
__global__ void __launch_bounds__(256) topk_gating_kernel(const T* __restrict__ logits, float* __restrict__ scores,
                                                          int* __restrict__ experts, int* __restrict__ slots,
                                                          int* __restrict__ counts, int T_, int E, int K,
                                                          int renorm) {
  const int lane = threadIdx.x & 63;
  const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= T_) return;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = lane + 64 * i;
    v[i] = e < E ? (float)logits[(int64_t)tok * E + e] : -INFINITY;
  }
  // softmax denominator over all experts
  float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
  mx = wave_max(mx);
  float den = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) den += (lane + 64 * i < E) ? __expf(v[i] - mx) : 0.f;
  den = wave_sum(den);
  float w_sel[8];
  int e_sel[8];
  float wsum = 0.f;
  for (int k = 0; k < K; ++k) {
    // lane-local best (lowest index among equals), then wave argmax
    float bv = -INFINITY;
    int be = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane + 64 * i;
      if (e < E && (v[i] > bv || (v[i] == bv && e < be))) { bv = v[i]; be = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oe = __shfl_xor(be, o, 64);
      if (ov > bv || (ov == bv && oe < be)) { bv = ov; be = oe; }
    }
    w_sel[k] = __expf(bv - mx) / den;
    e_sel[k] = be;
    wsum += w_sel[k];
    if ((be & 63) == lane) v[be >> 6] = -INFINITY;  // remove it for the next round
  }
  if (lane == 0) {
    for (int k = 0; k < K; ++k) {
      scores[(int64_t)tok * K + k] = renorm ? w_sel[k] / wsum : w_sel[k];
      experts[(int64_t)tok * K + k] = e_sel[k];
      slots[(int64_t)tok * K + k] = atomicAdd(counts + e_sel[k], 1);
    }
  }
}

// exclusive prefix of counts[0..E) into sh[0..E] (sh[E] = total), by wave 0 of the block
__device__ __forceinline__ void block_prefix(const int* __restrict__ counts, int E, int* sh) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int c[4], s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane * 4 + i;
      c[i] = e < E ? counts[e] : 0;
      s += c[i];
    }
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    int run = incl - s;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane * 4 + i;
      if (e <= E) sh[e] = run;
      run += c[i];
    }
    if (lane == 63 && 4 * 64 >= E) sh[E] = incl;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------ scatter / gather
__global__ void __launch_bounds__(256) moe_scatter_kernel(const bf16* __restrict__ x, const int* __restrict__ experts,
                                                          const int* __restrict__ slots, const int* __restrict__ counts,
                                                          bf16* __restrict__ xs, int* __restrict__ rows,
                                                          int64_t* __restrict__ cumsum, int H, int E, int K) {
  __shared__ int pre[MAXE + 1];
  block_prefix(counts, E, pre);
  const int tok = blockIdx.x;
  if (tok == 0 && threadIdx.x < E) cumsum[threadIdx.x] = pre[threadIdx.x + 1];
  const bf16x8* src = reinterpret_cast<const bf16x8*>(x + (int64_t)tok * H);
  for (int k = 0; k < K; ++k) {
    const int e = experts[(int64_t)tok * K + k];
    const int row = pre[e] + slots[(int64_t)tok * K + k];
    if (threadIdx.x == 0) rows[(int64_t)tok * K + k] = row;
    bf16x8* dst = reinterpret_cast<bf16x8*>(xs + (int64_t)row * H);
    for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
  }
}

__global__ void __launch_bounds__(256) moe_gather_kernel(const bf16* __restrict__ y, const float* __restrict__ scores,
                                                         const int* __restrict__ rows, bf16* __restrict__ out, int H,
                                                         int K) {
  const int tok = blockIdx.x;
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float w = scores[(int64_t)tok * K + k];
      float v[8];
      Vec8<bf16>::load(y + (int64_t)rows[(int64_t)tok * K + k] * H + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(w, v[j], acc[j]);
    }
    Vec8<bf16>::store(out + (int64_t)tok * H + i * 8, acc);
  }
}

// ------------------------------------------------------------------------------------------------ grouped GEMM
constexpr int GBM = 128, GBN = 128, GBK = 128, GTHR = 256;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int goff(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// grid.x: upper bound on m-tiles over all experts (sum_e ceil(cnt_e / 128) <= rows/128 + E), grid.y: N / 128.
__global__ void __launch_bounds__(GTHR, 2) grouped_gemm_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                               bf16* __restrict__ Y, const int* __restrict__ counts,
                                                               int E, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  __shared__ int pre[MAXE + 1];
  block_prefix(counts, E, pre);
  // locate (expert, m-tile) of this block
  int mt = blockIdx.x, e = -1, m0 = 0, cnt = 0, tiles_before = 0;
  for (int i = 0; i < E; ++i) {
    const int c = pre[i + 1] - pre[i];
    const int t = (c + GBM - 1) / GBM;
    if (mt < tiles_before + t) { e = i; m0 = (mt - tiles_before) * GBM; cnt = c; break; }
    tiles_before += t;
  }
  if (e < 0) return;  // uniform across the block: past the last real tile
  const int rbase = pre[e];
  const int n0 = blockIdx.y * GBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;  // 2x2 waves, 64x64 each
  const bf16* Xe = X + (int64_t)rbase * K;
  const bf16* We = W + (int64_t)e * N * K + (int64_t)n0 * K;
  char* As = gsm;
  char* Bs = gsm + GBM * GBK * 2;

  u32x4_t ar[8], br[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + i * GTHR, row = c >> 4, ch = c & 15;
      const int mr = min(m0 + row, cnt - 1);
      ar[i] = *reinterpret_cast<const u32x4_t*>(Xe + (int64_t)mr * K + k0 + ch * 8);
      br[i] = *reinterpret_cast<const u32x4_t*>(We + (int64_t)row * K + k0 + ch * 8);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + i * GTHR, row = c >> 4, ch = c & 15;
      *reinterpret_cast<u32x4_t*>(As + goff(row, ch)) = ar[i];
      *reinterpret_cast<u32x4_t*>(Bs + goff(row, ch)) = br[i];
    }
  };
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = K / GBK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // previous tile fully consumed
    store();
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * GBK);  // in flight under this tile's MFMAs
#pragma unroll
    for (int kk = 0; kk < GBK / 16; ++kk) {
      bf16x8_t a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8_t*>(As + goff(wm + 32 * i + l32, 2 * kk + h));
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(Bs + goff(wn + 32 * j + l32, 2 * kk + h));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // C: col = lane&31 (n), row = (r&3) + 8(r>>2) + 4h (m)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < cnt) {
        bf16* yrow = Y + (int64_t)(rbase + m) * N + n0 + wn + l32;
#pragma unroll
        for (int j = 0; j < 2; ++j) yrow[32 * j] = (bf16)acc[i][j][r];
      }
    }
}

// ------------------------------------------------------------------------------------------------ ragged gathers
// out[i] = table[ids[i]] (+ pos_table[pos[i]]), rows of H bf16
__global__ void __launch_bounds__(256) embed_gather_kernel(const bf16* __restrict__ table, const int64_t* __restrict__ ids,
                                                           const bf16* __restrict__ pos_table,
                                                           const int64_t* __restrict__ pos, bf16* __restrict__ out,
                                                           int H) {
  const int64_t t = blockIdx.x;
  const bf16* src = table + ids[t] * H;
  const bf16* ps = pos_table ? pos_table + pos[t] * H : nullptr;
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) {
    float v[8];
    Vec8<bf16>::load(src + i * 8, v);
    if (ps) {
      float p[8];
      Vec8<bf16>::load(ps + i * 8, p);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p[j];
    }
    Vec8<bf16>::store(out + t * H + i * 8, v);
  }
}

// out[s] = x[last[s]] for each sequence s (last-token hidden states of a ragged batch)
__global__ void __launch_bounds__(256) rows_gather_kernel(const bf16* __restrict__ x, const int64_t* __restrict__ idx,
                                                          bf16* __restrict__ out, int H) {
  const int64_t s = blockIdx.x;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(x + idx[s] * H);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out + s * H);
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
}

// full[b, idx[b, j]] = part[b, j] (rows of H) — random-LTD token scatter; gather is rows_gather with flat indices
__global__ void __launch_bounds__(256) rows_scatter_kernel(const bf16* __restrict__ part, const int64_t* __restrict__ idx,
                                                           bf16* __restrict__ full, int H) {
  const int64_t r = blockIdx.x;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(part + r * H);
  bf16x8* dst = reinterpret_cast<bf16x8*>(full + idx[r] * H);
  for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
}

}  // namespace

extern "C" int ds_topk_gating(const void* logits, float* scores, int* experts, int* slots, int* counts, int T, int E,
                              int K, int renorm, int dtype, hipStream_t s) {
  if (E < 1 || E > MAXE || K < 1 || K > 8 || K > E) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  const int grid = (T + 3) / 4;
  if (dtype == DS_BF16)
    hipLaunchKernelGGL(topk_gating_kernel<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)logits, scores, experts,
                       slots, counts, T, E, K, renorm);
  else if (dtype == DS_F32)
    hipLaunchKernelGGL(topk_gating_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)logits, scores, experts,
                       slots, counts, T, E, K, renorm);
  else
    hipLaunchKernelGGL(topk_gating_kernel<fp16>, dim3(grid), dim3(256), 0, s, (const fp16*)logits, scores, experts,
                       slots, counts, T, E, K, renorm);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_moe_scatter(const void* x, const int* experts, const int* slots, const int* counts, void* xs,
                              int* rows, int64_t* cumsum, int T, int H, int E, int K, hipStream_t s) {
  if (E > MAXE || H % 8) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  hipLaunchKernelGGL(moe_scatter_kernel, dim3(T), dim3(256), 0, s, (const bf16*)x, experts, slots, counts, (bf16*)xs,
                     rows, cumsum, H, E, K);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_moe_gather(const void* y, const float* scores, const int* rows, void* out, int T, int H, int K,
                             hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  hipLaunchKernelGGL(moe_gather_kernel, dim3(T), dim3(256), 0, s, (const bf16*)y, scores, rows, (bf16*)out, H, K);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_grouped_gemm_ok(int N, int K) { return N % GBN == 0 && K % GBK == 0; }

extern "C" int ds_grouped_gemm(const void* X, const void* W, void* Y, const int* counts, int total_rows, int E, int N,
                               int K, hipStream_t s) {
  if (!ds_grouped_gemm_ok(N, K) || E > MAXE) return (int)hipErrorInvalidValue;
  if (total_rows == 0) return 0;
  const int lds = 2 * GBM * GBK * 2;  // 64 KB
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&grouped_gemm_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int mtiles = (total_rows + GBM - 1) / GBM + E;
  hipLaunchKernelGGL(grouped_gemm_kernel, dim3(mtiles, N / GBN), dim3(GTHR), lds, s, (const bf16*)X, (const bf16*)W,
                     (bf16*)Y, counts, E, N, K);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_embed_gather(const void* table, const int64_t* ids, const void* pos_table, const int64_t* pos,
                               void* out, int64_t n, int H, hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(embed_gather_kernel, dim3(n), dim3(256), 0, s, (const bf16*)table, ids, (const bf16*)pos_table,
                     pos, (bf16*)out, H);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_rows_gather(const void* x, const int64_t* idx, void* out, int64_t n, int H, hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(rows_gather_kernel, dim3(n), dim3(256), 0, s, (const bf16*)x, idx, (bf16*)out, H);
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_rows_scatter(const void* part, const int64_t* idx, void* full, int64_t n, int H, hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(rows_scatter_kernel, dim3(n), dim3(256), 0, s, (const bf16*)part, idx, (bf16*)full, H);
  DS_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------ random-LTD token sort
// Sort each row of k DISTINCT token positions in [0, S) (reference `csrc/random_ltd/token_sort.cu:28` scan_sort):
// because the values are distinct and bounded, the sorted row is the compaction of a bitmap. One workgroup per row:
// set the row's bits in an LDS bitmap (S/32 words), popcount each thread's contiguous word range, one exclusive scan
// over the 256 per-thread counts, then every thread writes its positions in order. O(S + k) per row, no comparisons.
namespace {
constexpr int TS_THREADS = 256;
__global__ void __launch_bounds__(TS_THREADS) token_sort_kernel(int* __restrict__ idx, int k, int S) {
  extern __shared__ unsigned int bm[];  // [words] bitmap, then [TS_THREADS] scan scratch
  const int words = (S + 31) >> 5;
  unsigned int* scan = bm + words;
  int* row = idx + (int64_t)blockIdx.x * k;
  for (int w = threadIdx.x; w < words; w += TS_THREADS) bm[w] = 0u;
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += TS_THREADS) {
    const int v = row[i];
    if (v >= 0 && v < S) atomicOr(&bm[v >> 5], 1u << (v & 31));
  }
  __syncthreads();
  const int per = (words + TS_THREADS - 1) / TS_THREADS;
  const int w0 = min(threadIdx.x * per, words), w1 = min(w0 + per, words);
  unsigned int cnt = 0;
  for (int w = w0; w < w1; ++w) cnt += __popc(bm[w]);
  scan[threadIdx.x] = cnt;
  __syncthreads();
  // Hillis-Steele inclusive scan over 256 counts (8 steps)
  for (int off = 1; off < TS_THREADS; off <<= 1) {
    const unsigned int add = threadIdx.x >= off ? scan[threadIdx.x - off] : 0u;
    __syncthreads();
    scan[threadIdx.x] += add;
    __syncthreads();
  }
  int pos = (int)(scan[threadIdx.x] - cnt);
  for (int w = w0; w < w1; ++w) {
    unsigned int bits = bm[w];
    while (bits) {
      const int b = __ffs(bits) - 1;
      bits &= bits - 1;
      if (pos < k) row[pos] = (w << 5) + b;
      ++pos;
    }
  }
}
}  // namespace

// idx [rows, k] int32 distinct values in [0, S), sorted in place per row.
extern "C" int ds_token_sort(int* idx, int rows, int k, int S, hipStream_t s) {
  if (rows <= 0 || k <= 0) return 0;
  if (S <= 0 || k > S || S > (1 << 20)) return (int)hipErrorInvalidValue;
  const size_t lds = ((size_t)(S + 31) / 32 + TS_THREADS) * sizeof(unsigned int);
  static bool big = false;
  if (lds > 65536 && !big) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&token_sort_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    big = true;
  }
  hipLaunchKernelGGL(token_sort_kernel, dim3(rows), dim3(TS_THREADS), lds, s, idx, k, S);
  return (int)hipGetLastError();
}
