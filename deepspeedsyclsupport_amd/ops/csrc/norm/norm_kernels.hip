// RMSNorm / LayerNorm forward+backward (optionally fused with the residual add) for CDNA4.
//
// Parity: reference training kernels `csrc/transformer/normalize_kernels.cu` (fused_bias_residual_layer_norm,
// LayerNormBackward1/2) and inference `csrc/transformer/inference/csrc/{layer_norm.cu,rms_norm.cu}`
// (fused_ln, fused_residual_ln, rms_norm, pre_rms_norm).
//
// MI355X design: rows narrower than 1024 give ONE WAVE one row: it keeps the row in NV*8 registers per lane (NV =
// compile-time vectors per lane), so the statistics need only a 64-lane butterfly (no LDS, no __syncthreads) and the
// row is read from HBM exactly once; 256-thread blocks = 4 rows, every access is 16 B/lane. Wider rows give a whole
// block one row, forward (norm_fwd_block_kernel) and backward (norm_bwd_block_kernel).
// Backward: pass 1 over the row accumulates the dot products and the per-lane dgamma/dbeta partials, pass 2
// re-reads the (L1/L2-hot) row to write dx. dgamma/dbeta partials are reduced across the block's 4 waves in LDS
// and written as one fp32 row per block, then summed by a column kernel (deterministic, no float atomics).
#include "../include/ds_hip.h"

namespace {

template <typename T, int NV>
__device__ __forceinline__ void load_row(const T* row, int H, int lane, float (&v)[NV][8]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < H) Vec8<T>::load(row + c, v[k]);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
  }
}

__device__ __forceinline__ void zero8(float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
}

// ------------------------------------------------------------------------------------------------ RMSNorm fwd
template <typename T, int NV, bool RES>
__global__ void __launch_bounds__(256) rms_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                      const T* __restrict__ w, T* __restrict__ y,
                                                      T* __restrict__ res_out, float* __restrict__ rstd_out,
                                                      int64_t rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += wstride) {
    float v[NV][8];
    load_row<T, NV>(x + row * H, H, lane, v);
    if (RES) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < H) {
          float rr[8];
          Vec8<T>::load(r + row * H + c, rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] += rr[j];
          Vec8<T>::store(res_out + row * H + c, v[k]);
        }
      }
    }
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) ss = fmaf(v[k][j], v[k][j], ss);
    ss = wave_sum(ss);
    const float rs = rsqrtf(ss / H + eps);
    if (lane == 0 && rstd_out) rstd_out[row] = rs;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float ww[8], o[8];
        Vec8<T>::load(w + c, ww);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rs * ww[j];
        Vec8<T>::store(y + row * H + c, o);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ RMSNorm bwd
// x is the normalized input (x + r when the forward fused the residual). dx (+ dres if given).
// One wave per row. The row's x and dy are read from HBM ONCE and kept in registers in their storage type (bf16: 4
// VGPRs per 8 elements) across the two passes (dot product, then dx): re-reading them in the second pass missed
// the 4 MB per-XCD L2 (512 rows in flight per XCD x 16 KB) and cost ~25 % extra traffic.
template <typename T> struct Raw8 { typedef bf16x8 type; };
template <> struct Raw8<fp16> { typedef fp16x8 type; };
template <> struct Raw8<float> { struct type { f32x4 lo, hi; }; };
template <typename T> __device__ __forceinline__ typename Raw8<T>::type ld_raw8(const T* p) {
  return *reinterpret_cast<const typename Raw8<T>::type*>(p);
}
template <typename T> __device__ __forceinline__ void raw_to_f(const typename Raw8<T>::type& r, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
}
template <> __device__ __forceinline__ void raw_to_f<float>(const Raw8<float>::type& r, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[i] = r.lo[i]; v[i + 4] = r.hi[i]; }
}

typedef unsigned int raw_u32x4 __attribute__((ext_vector_type(4)));
template <typename T, int NV>
__device__ __forceinline__ void launder_raw(typename Raw8<T>::type (&a)[NV], typename Raw8<T>::type (&b)[NV]) {
  if constexpr (sizeof(typename Raw8<T>::type) == 16) {  // bf16 / fp16 rows (fp32 rows are not register-bound)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      raw_u32x4 ua = __builtin_bit_cast(raw_u32x4, a[k]), ub = __builtin_bit_cast(raw_u32x4, b[k]);
      asm volatile("" : "+v"(ua), "+v"(ub));
      a[k] = __builtin_bit_cast(typename Raw8<T>::type, ua);
      b[k] = __builtin_bit_cast(typename Raw8<T>::type, ub);
    }
  }
}

template <typename T, int NV, bool ADD_DRES>
__global__ void __launch_bounds__(256) rms_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const T* __restrict__ w, const float* __restrict__ rstd,
                                                      const T* __restrict__ dres, T* __restrict__ dx,
                                                      float* __restrict__ dw_part, int64_t rows, int H) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [4][H]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float dwacc[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k) zero8(dwacc[k]);
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += wstride) {
    const float rs = rstd[row];
    const T* xr = x + row * H;
    const T* gr = dy + row * H;
    typename Raw8<T>::type xraw[NV], graw[NV], draw[ADD_DRES ? NV : 1];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        xraw[k] = ld_raw8(xr + c);
        graw[k] = ld_raw8(gr + c);
        if constexpr (ADD_DRES) draw[k] = ld_raw8(dres + row * H + c);  // in flight with x / dy, not after the dot
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float xv[8], gv[8], ww[8];
        raw_to_f<T>(xraw[k], xv);
        raw_to_f<T>(graw[k], gv);
        Vec8<T>::load(w + c, ww);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dwacc[k][j] = fmaf(gv[j], xv[j] * rs, dwacc[k][j]);
          dot = fmaf(gv[j] * ww[j], xv[j], dot);
        }
      }
    }
    dot = wave_sum(dot);
    const float c2 = dot * rs * rs * rs / H;
    // opaque to the optimiser: the second pass re-converts from the packed registers instead of keeping the first
    // pass's fp32 copies alive (that doubles the live registers and drops occupancy to 1 wave per SIMD)
    launder_raw<T, NV>(xraw, graw);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float xv[8], gv[8], ww[8], o[8];
        raw_to_f<T>(xraw[k], xv);
        raw_to_f<T>(graw[k], gv);
        Vec8<T>::load(w + c, ww);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = gv[j] * ww[j] * rs - xv[j] * c2;
        if constexpr (ADD_DRES) {
          float d2[8];
          raw_to_f<T>(draw[k], d2);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d2[j];
        }
        Vec8<T>::store(dx + row * H + c, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < H) {
      *reinterpret_cast<f32x4*>(&sm[wid * H + c]) = f32x4{dwacc[k][0], dwacc[k][1], dwacc[k][2], dwacc[k][3]};
      *reinterpret_cast<f32x4*>(&sm[wid * H + c + 4]) = f32x4{dwacc[k][4], dwacc[k][5], dwacc[k][6], dwacc[k][7]};
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256)
    dw_part[(int64_t)blockIdx.x * H + c] = sm[c] + sm[H + c] + sm[2 * H + c] + sm[3 * H + c];
}

// Column sum of nb partial rows, two deterministic stages so the reduction uses the whole chip:
// stage 1 (grid H/256 x CS): block (x, y) sums rows y, y+CS, ... of its 256 columns into stage[y][c];
// stage 2 (grid H/256): sums the CS stage rows and casts.
constexpr int CS = 32;
__global__ void __launch_bounds__(256) colsum_stage1(const float* __restrict__ part, int nb, int H, int ld,
                                                     float* __restrict__ stage) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= H) return;
  float acc = 0.f;
  for (int b = blockIdx.y; b < nb; b += CS) acc += part[(int64_t)b * ld + c];
  stage[(int64_t)blockIdx.y * H + c] = acc;
}
template <typename T>
__global__ void __launch_bounds__(256) colsum_stage2(const float* __restrict__ stage, int H, T* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= H) return;
  float acc = 0.f;
#pragma unroll
  for (int y = 0; y < CS; ++y) acc += stage[(int64_t)y * H + c];
  out[c] = (T)acc;
}
template <typename T>
static void colsum(const float* part, int nb, int H, int ld, float* stage, T* out, hipStream_t s) {
  hipLaunchKernelGGL(colsum_stage1, dim3((H + 255) / 256, CS), dim3(256), 0, s, part, nb, H, ld, stage);
  hipLaunchKernelGGL((colsum_stage2<T>), dim3((H + 255) / 256), dim3(256), 0, s, stage, H, out);
}

// ------------------------------------------------------------------------------------------------ LayerNorm
template <typename T, int NV, bool RES>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                     const T* __restrict__ gamma, const T* __restrict__ beta,
                                                     T* __restrict__ y, T* __restrict__ res_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += wstride) {
    float v[NV][8];
    load_row<T, NV>(x + row * H, H, lane, v);
    if (RES) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < H) {
          float rr[8];
          Vec8<T>::load(r + row * H + c, rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] += rr[j];
          Vec8<T>::store(res_out + row * H + c, v[k]);
        }
      }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    const float mu = wave_sum(s) / H;
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[k][j] - mu;
          ss = fmaf(d, d, ss);
        }
      }
    }
    const float rs = rsqrtf(wave_sum(ss) / H + eps);
    if (lane == 0) {
      if (mean_out) mean_out[row] = mu;
      if (rstd_out) rstd_out[row] = rs;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float gg[8], bb[8], o[8];
        Vec8<T>::load(gamma + c, gg);
        Vec8<T>::load(beta + c, bb);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mu) * rs * gg[j] + bb[j];
        Vec8<T>::store(y + row * H + c, o);
      }
    }
  }
}

template <typename T, int NV, bool ADD_DRES>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const T* __restrict__ dres,
                                                     T* __restrict__ dx, float* __restrict__ part, int64_t rows,
                                                     int H) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [4][H], used twice (dgamma then dbeta)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k) { zero8(dg[k]); zero8(db[k]); }
  const int64_t wstride = (int64_t)gridDim.x * 4;
  // rows up to 2048 wide (BERT / GPT-2 class) stay in packed registers between the two passes like rms_bwd; wider
  // rows re-read (their dgamma / dbeta accumulators already hold 128 registers)
  constexpr bool KEEP = NV <= 4;
  constexpr int NK = KEEP ? NV : 1;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += wstride) {
    const float mu = mean[row], rs = rstd[row];
    const T* xr = x + row * H;
    const T* gr = dy + row * H;
    typename Raw8<T>::type xraw[NK], graw[NK], draw[(KEEP && ADD_DRES) ? NK : 1];
    if constexpr (KEEP) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 8;
        if (c < H) {
          xraw[k] = ld_raw8(xr + c);
          graw[k] = ld_raw8(gr + c);
          if constexpr (ADD_DRES) draw[k] = ld_raw8(dres + row * H + c);
        }
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float xv[8], gv[8], gm[8];
        if constexpr (KEEP) {
          raw_to_f<T>(xraw[k < NK ? k : 0], xv);
          raw_to_f<T>(graw[k < NK ? k : 0], gv);
        } else {
          Vec8<T>::load(xr + c, xv);
          Vec8<T>::load(gr + c, gv);
        }
        Vec8<T>::load(gamma + c, gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - mu) * rs;
          dg[k][j] = fmaf(gv[j], xh, dg[k][j]);
          db[k][j] += gv[j];
          const float g = gv[j] * gm[j];
          s1 += g;
          s2 = fmaf(g, xh, s2);
        }
      }
    }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
    if constexpr (KEEP) launder_raw<T, NK>(xraw, graw);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float xv[8], gv[8], gm[8], o[8];
        if constexpr (KEEP) {
          raw_to_f<T>(xraw[k < NK ? k : 0], xv);
          raw_to_f<T>(graw[k < NK ? k : 0], gv);
        } else {
          Vec8<T>::load(xr + c, xv);
          Vec8<T>::load(gr + c, gv);
        }
        Vec8<T>::load(gamma + c, gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gv[j] * gm[j] - s1 - (xv[j] - mu) * rs * s2);
        if (ADD_DRES) {
          float d2[8];
          if constexpr (KEEP) raw_to_f<T>(draw[k < NK ? k : 0], d2);
          else Vec8<T>::load(dres + row * H + c, d2);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d2[j];
        }
        Vec8<T>::store(dx + row * H + c, o);
      }
    }
  }
  // dgamma partial -> part[b][0:H], dbeta partial -> part[b][H:2H]
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
        float (&a)[8] = pass == 0 ? dg[k] : db[k];
        *reinterpret_cast<f32x4*>(&sm[wid * H + c]) = f32x4{a[0], a[1], a[2], a[3]};
        *reinterpret_cast<f32x4*>(&sm[wid * H + c + 4]) = f32x4{a[4], a[5], a[6], a[7]};
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 256)
      part[(int64_t)blockIdx.x * 2 * H + pass * H + c] = sm[c] + sm[H + c] + sm[2 * H + c] + sm[3 * H + c];
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------ wide-row forward
// Rows of 1024 - 16384 elements: a 256-thread block owns the row, every thread holds NB <= 8 chunks, the statistics
// go through the 64-lane butterfly and 4 LDS words. (With one wave per row a 14336-wide row is 28 dependent 16-B
// loads per lane and a register file's worth of values: 35 us for ONE BLOOM-176B decode LayerNorm against 5.5 us
// here, and 1.5 - 2.4x slower at training row counts.) LN = LayerNorm (mean + variance, gamma / beta), else RMSNorm.
template <typename T, int NB, bool RES, bool LN>
__global__ void __launch_bounds__(256) norm_fwd_block_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                             const T* __restrict__ gamma, const T* __restrict__ beta,
                                                             T* __restrict__ y, T* __restrict__ res_out,
                                                             float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                             int H, float eps) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t row = blockIdx.x;
  float v[NB][8];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int c = (k * 256 + tid) * 8;
    if (c < H) {
      Vec8<T>::load(x + row * H + c, v[k]);
      if (RES) {
        float rr[8];
        Vec8<T>::load(r + row * H + c, rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += rr[j];
        Vec8<T>::store(res_out + row * H + c, v[k]);
      }
    } else {
      zero8(v[k]);
    }
  }
  float mu = 0.f;
  if (LN) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    s = wave_sum(s);
    if (lane == 0) red[0][wid] = s;
    __syncthreads();
    mu = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / H;
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    if ((k * 256 + tid) * 8 < H) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mu;
        ss = fmaf(d, d, ss);
      }
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[1][wid] = ss;
  __syncthreads();
  const float rs = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / H + eps);
  if (tid == 0) {
    if (LN && mean_out) mean_out[row] = mu;
    if (rstd_out) rstd_out[row] = rs;
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int c = (k * 256 + tid) * 8;
    if (c < H) {
      float gg[8], o[8];
      Vec8<T>::load(gamma + c, gg);
      if (LN) {
        float bb[8];
        Vec8<T>::load(beta + c, bb);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mu) * rs * gg[j] + bb[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rs * gg[j];
      }
      Vec8<T>::store(y + row * H + c, o);
    }
  }
}

// ------------------------------------------------------------------------------------------------ wide-row backward
// Rows of 1024 - 8192 elements: a 256-thread block walks rows blockIdx.x, + gridDim.x, ...; thread t owns the columns
// (k * 256 + t) * 8 .. + 7 of every row it sees, so its dgamma / dbeta sums stay in registers for the whole launch and
// go straight to the partial buffer (no [4][H] LDS staging: at H = 8192 that staging is 128 KB, one block per CU, and
// the wave-per-row kernels above fall to 1.8 - 3.9 TB/s). x, dy, dres and gamma stay packed in registers between the
// reduction pass and the dx pass; the two row sums cross waves through 8 LDS words, double-buffered by row parity so a
// row costs one barrier.
template <typename T, int NB, bool ADD_DRES, bool LN>
__global__ void __launch_bounds__(256) norm_bwd_block_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             const T* __restrict__ gamma,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const T* __restrict__ dres, T* __restrict__ dx,
                                                             float* __restrict__ part, int64_t rows, int H) {
  __shared__ float red[2][2][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float dg[NB][8], db[LN ? NB : 1][8];
  typename Raw8<T>::type wraw[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    zero8(dg[k]);
    if (LN) zero8(db[k < (LN ? NB : 1) ? k : 0]);
    const int c = (k * 256 + tid) * 8;
    if (c < H) wraw[k] = ld_raw8(gamma + c);
  }
  const float invH = 1.f / H;
  int par = 0;
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x, par ^= 1) {
    const float rs = rstd[row], mu = LN ? mean[row] : 0.f;
    const T* xr = x + row * H;
    const T* gr = dy + row * H;
    typename Raw8<T>::type xraw[NB], graw[NB], draw[ADD_DRES ? NB : 1];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int c = (k * 256 + tid) * 8;
      if (c < H) {
        xraw[k] = ld_raw8(xr + c);
        graw[k] = ld_raw8(gr + c);
        if constexpr (ADD_DRES) draw[k] = ld_raw8(dres + row * H + c);
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if ((k * 256 + tid) * 8 < H) {
        float xv[8], gv[8], ww[8];
        raw_to_f<T>(xraw[k], xv);
        raw_to_f<T>(graw[k], gv);
        raw_to_f<T>(wraw[k], ww);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - mu) * rs;
          dg[k][j] = fmaf(gv[j], xh, dg[k][j]);
          if (LN) db[k < (LN ? NB : 1) ? k : 0][j] += gv[j];
          const float g = gv[j] * ww[j];
          if (LN) s1 += g;
          s2 = fmaf(g, xh, s2);
        }
      }
    }
    if (LN) s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      if (LN) red[par][0][wid] = s1;
      red[par][1][wid] = s2;
    }
    __syncthreads();
    const float m1 = LN ? (red[par][0][0] + red[par][0][1] + red[par][0][2] + red[par][0][3]) * invH : 0.f;
    const float m2 = (red[par][1][0] + red[par][1][1] + red[par][1][2] + red[par][1][3]) * invH;
    // opaque to the optimiser: the dx pass re-converts from the packed registers instead of keeping fp32 copies alive
    launder_raw<T, NB>(xraw, graw);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int c = (k * 256 + tid) * 8;
      if (c < H) {
        float xv[8], gv[8], ww[8], o[8];
        raw_to_f<T>(xraw[k], xv);
        raw_to_f<T>(graw[k], gv);
        raw_to_f<T>(wraw[k], ww);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gv[j] * ww[j] - m1 - (xv[j] - mu) * rs * m2);
        if constexpr (ADD_DRES) {
          float d2[8];
          raw_to_f<T>(draw[k], d2);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d2[j];
        }
        Vec8<T>::store(dx + row * H + c, o);
      }
    }
  }
  // this block's column sums: RMSNorm part[b][0:H]; LayerNorm dgamma part[b][0:H], dbeta part[b][H:2H]
  const int64_t ld = LN ? 2 * (int64_t)H : H;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int c = (k * 256 + tid) * 8;
    if (c < H) {
      float* p = part + blockIdx.x * ld + c;
      *reinterpret_cast<f32x4*>(p) = f32x4{dg[k][0], dg[k][1], dg[k][2], dg[k][3]};
      *reinterpret_cast<f32x4*>(p + 4) = f32x4{dg[k][4], dg[k][5], dg[k][6], dg[k][7]};
      if (LN) {
        float (&b)[8] = db[k < (LN ? NB : 1) ? k : 0];
        *reinterpret_cast<f32x4*>(p + H) = f32x4{b[0], b[1], b[2], b[3]};
        *reinterpret_cast<f32x4*>(p + H + 4) = f32x4{b[4], b[5], b[6], b[7]};
      }
    }
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                   \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)

// NV buckets: hidden <= 512*NV
#define DISPATCH_NV(H, ...)                                      \
  do {                                                           \
    const int nv__ = ((H) + 511) / 512;                          \
    if (nv__ <= 1) { constexpr int NV = 1; __VA_ARGS__; }        \
    else if (nv__ <= 2) { constexpr int NV = 2; __VA_ARGS__; }   \
    else if (nv__ <= 4) { constexpr int NV = 4; __VA_ARGS__; }   \
    else if (nv__ <= 6) { constexpr int NV = 6; __VA_ARGS__; }   \
    else if (nv__ <= 8) { constexpr int NV = 8; __VA_ARGS__; }   \
    else if (nv__ <= 12) { constexpr int NV = 12; __VA_ARGS__; } \
    else { constexpr int NV = 16; __VA_ARGS__; }                 \
  } while (0)

// forward-only buckets for very wide rows (BLOOM-176B: 14336): one wave still owns a whole row, up to 256 fp32
// values per lane in registers (one wave per SIMD at that size; the row-per-wave structure avoids a block reduction)


// Rows of 1024+ elements: a block per row at every row count (measured faster than a wave per row from 1 row to
// 32768, 1.1x at hidden 4096 and 1.5 - 2.4x at 8192 / 14336); narrower rows keep the wave-per-row kernels.
static bool block_rows(int H) { return H >= 1024; }

template <typename T, bool LN>
static void launch_block_norm(const void* x, const void* r, const void* g, const void* b, void* y, void* res_out,
                              float* mean, float* rstd, int64_t rows, int H, float eps, hipStream_t s) {
  const int nb = (H + 2047) / 2048;
#define DS_BLOCK_NORM(NB_)                                                                                          \
  do {                                                                                                              \
    if (r)                                                                                                          \
      hipLaunchKernelGGL((norm_fwd_block_kernel<T, NB_, true, LN>), dim3((unsigned)rows), dim3(256), 0, s,          \
                         (const T*)x, (const T*)r, (const T*)g, (const T*)b, (T*)y, (T*)res_out, mean, rstd, H, eps); \
    else                                                                                                            \
      hipLaunchKernelGGL((norm_fwd_block_kernel<T, NB_, false, LN>), dim3((unsigned)rows), dim3(256), 0, s,         \
                         (const T*)x, nullptr, (const T*)g, (const T*)b, (T*)y, nullptr, mean, rstd, H, eps);       \
  } while (0)
  if (nb <= 1) DS_BLOCK_NORM(1);
  else if (nb <= 2) DS_BLOCK_NORM(2);
  else if (nb <= 4) DS_BLOCK_NORM(4);
  else DS_BLOCK_NORM(8);
#undef DS_BLOCK_NORM
}

// Wide-row backward launch (H >= 1024): nb persistent blocks, NB = chunks per thread.
template <typename T, bool LN>
static void launch_block_norm_bwd(const void* dy, const void* x, const void* g, const float* mean, const float* rstd,
                                  const void* dres, void* dx, float* part, int nb, int64_t rows, int H,
                                  hipStream_t s) {
  const int cb = (H + 2047) / 2048;
#define DS_BLOCK_NORM_BWD(NB_)                                                                                     \
  do {                                                                                                             \
    if (dres)                                                                                                      \
      hipLaunchKernelGGL((norm_bwd_block_kernel<T, NB_, true, LN>), dim3(nb), dim3(256), 0, s, (const T*)dy,       \
                         (const T*)x, (const T*)g, mean, rstd, (const T*)dres, (T*)dx, part, rows, H);             \
    else                                                                                                           \
      hipLaunchKernelGGL((norm_bwd_block_kernel<T, NB_, false, LN>), dim3(nb), dim3(256), 0, s, (const T*)dy,      \
                         (const T*)x, (const T*)g, mean, rstd, nullptr, (T*)dx, part, rows, H);                    \
  } while (0)
  if (cb <= 1) DS_BLOCK_NORM_BWD(1);
  else if (cb <= 2) DS_BLOCK_NORM_BWD(2);
  else DS_BLOCK_NORM_BWD(4);
#undef DS_BLOCK_NORM_BWD
}

static bool bwd_wave_rows() {  // measurement switch: DS_NORM_BWD_WAVE=1 keeps the wave-per-row backward at every width
  static const bool v = [] { const char* e = getenv("DS_NORM_BWD_WAVE"); return e && e[0] == '1'; }();
  return v;
}

static constexpr int kMaxHidden = 8192;      // backward kernels
static constexpr int kMaxHiddenFwd = 16384;  // forward kernels
static int norm_grid(int64_t rows) { return ds_grid_for((rows + 3) / 4, 1, 256 * 8); }

// Number of fp32 partial rows the backward writes for `rows`. The host allocates part[(nb + 32) * H] for RMSNorm
// and part[(nb + 32) * 2H] for LayerNorm (the trailing 32 rows are the column-sum stage buffer).
// (512 = two persistent blocks per CU: measured best for the wide-row backward against 256 / 768 / 1024 / 2048)
extern "C" int ds_norm_bwd_blocks(int64_t rows) { return ds_grid_for((rows + 3) / 4, 1, 512); }

extern "C" int ds_rms_fwd(const void* x, const void* r, const void* w, void* y, void* res_out, float* rstd,
                          int64_t rows, int H, float eps, int dtype, hipStream_t s) {
  if (H % 8 != 0 || H > kMaxHiddenFwd) return (int)hipErrorInvalidValue;
  if (r && !res_out) return (int)hipErrorInvalidValue;  // the fused-residual kernel always writes x + r
  if (rows <= 0) return 0;
  if (block_rows(H)) {
    DISPATCH_T(dtype, (launch_block_norm<T, false>(x, r, w, nullptr, y, res_out, nullptr, rstd, rows, H, eps, s)));
    DS_CHECK_LAUNCH();
    return 0;
  }
  const int grid = norm_grid(rows);
  DISPATCH_T(dtype, DISPATCH_NV(H, {
    if (r)
      hipLaunchKernelGGL((rms_fwd_kernel<T, NV, true>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)r,
                         (const T*)w, (T*)y, (T*)res_out, rstd, rows, H, eps);
    else
      hipLaunchKernelGGL((rms_fwd_kernel<T, NV, false>), dim3(grid), dim3(256), 0, s, (const T*)x, nullptr,
                         (const T*)w, (T*)y, nullptr, rstd, rows, H, eps);
  }));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_rms_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                          void* dw, float* part, int64_t rows, int H, int dtype, hipStream_t s) {
  if (H % 8 != 0 || H > kMaxHidden) return (int)hipErrorInvalidValue;
  if (rows <= 0) return 0;
  const int nb = ds_norm_bwd_blocks(rows);
  if (block_rows(H) && !bwd_wave_rows()) {
    DISPATCH_T(dtype, (launch_block_norm_bwd<T, false>(dy, x, w, nullptr, rstd, dres, dx, part, nb, rows, H, s)));
    DS_CHECK_LAUNCH();
    DISPATCH_T(dtype, colsum<T>(part, nb, H, H, part + (int64_t)nb * H, (T*)dw, s));
    DS_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = 4 * (size_t)H * sizeof(float);
  DISPATCH_T(dtype, DISPATCH_NV(H, {
    if (dres)
      hipLaunchKernelGGL((rms_bwd_kernel<T, NV, true>), dim3(nb), dim3(256), lds, s, (const T*)dy, (const T*)x,
                         (const T*)w, rstd, (const T*)dres, (T*)dx, part, rows, H);
    else
      hipLaunchKernelGGL((rms_bwd_kernel<T, NV, false>), dim3(nb), dim3(256), lds, s, (const T*)dy, (const T*)x,
                         (const T*)w, rstd, nullptr, (T*)dx, part, rows, H);
  }));
  DS_CHECK_LAUNCH();
  DISPATCH_T(dtype, colsum<T>(part, nb, H, H, part + (int64_t)nb * H, (T*)dw, s));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_ln_fwd(const void* x, const void* r, const void* g, const void* b, void* y, void* res_out,
                         float* mean, float* rstd, int64_t rows, int H, float eps, int dtype, hipStream_t s) {
  if (H % 8 != 0 || H > kMaxHiddenFwd) return (int)hipErrorInvalidValue;
  if (r && !res_out) return (int)hipErrorInvalidValue;
  if (rows <= 0) return 0;
  if (block_rows(H)) {
    DISPATCH_T(dtype, (launch_block_norm<T, true>(x, r, g, b, y, res_out, mean, rstd, rows, H, eps, s)));
    DS_CHECK_LAUNCH();
    return 0;
  }
  const int grid = norm_grid(rows);
  DISPATCH_T(dtype, DISPATCH_NV(H, {
    if (r)
      hipLaunchKernelGGL((ln_fwd_kernel<T, NV, true>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)r,
                         (const T*)g, (const T*)b, (T*)y, (T*)res_out, mean, rstd, rows, H, eps);
    else
      hipLaunchKernelGGL((ln_fwd_kernel<T, NV, false>), dim3(grid), dim3(256), 0, s, (const T*)x, nullptr,
                         (const T*)g, (const T*)b, (T*)y, nullptr, mean, rstd, rows, H, eps);
  }));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_ln_bwd(const void* dy, const void* x, const void* g, const float* mean, const float* rstd,
                         const void* dres, void* dx, void* dg, void* db, float* part, int64_t rows, int H, int dtype,
                         hipStream_t s) {
  if (H % 8 != 0 || H > kMaxHidden) return (int)hipErrorInvalidValue;
  if (rows <= 0) return 0;
  const int nb = ds_norm_bwd_blocks(rows);
  const bool blk = block_rows(H) && !bwd_wave_rows();
  if (blk)
    DISPATCH_T(dtype, (launch_block_norm_bwd<T, true>(dy, x, g, mean, rstd, dres, dx, part, nb, rows, H, s)));
  const size_t lds = 4 * (size_t)H * sizeof(float);
  if (!blk) DISPATCH_T(dtype, DISPATCH_NV(H, {
    if (dres)
      hipLaunchKernelGGL((ln_bwd_kernel<T, NV, true>), dim3(nb), dim3(256), lds, s, (const T*)dy, (const T*)x,
                         (const T*)g, mean, rstd, (const T*)dres, (T*)dx, part, rows, H);
    else
      hipLaunchKernelGGL((ln_bwd_kernel<T, NV, false>), dim3(nb), dim3(256), lds, s, (const T*)dy, (const T*)x,
                         (const T*)g, mean, rstd, nullptr, (T*)dx, part, rows, H);
  }));
  DS_CHECK_LAUNCH();
  float* stage = part + (int64_t)nb * 2 * H;
  DISPATCH_T(dtype, {
    colsum<T>(part, nb, H, 2 * H, stage, (T*)dg, s);
    colsum<T>(part + H, nb, H, 2 * H, stage + (int64_t)CS * H, (T*)db, s);
  });
  DS_CHECK_LAUNCH();
  return 0;
}
