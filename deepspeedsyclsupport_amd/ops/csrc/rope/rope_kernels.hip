// Rotary position embedding (RoPE) + fused QKV split/layout transform, CDNA4.
//
// Parity: reference `csrc/transformer/inference/csrc/apply_rotary_pos_emb.cu:27` (apply_rotary_pos_half),
// `transform.cu:20-641` (bias_add_transform_0213: split fused QKV, add bias, rotary, write head-major),
// v2 `ragged_ops/linear_blocked_kv_rotary` (rotary on q,k), training `transform_kernels.cu` (transform_0213).
//
// MI355X design: the fused QKV GEMM output [B, S, Hq+2Hk, D] is read once; each lane owns 8 rotary PAIRS
// (elements i..i+7 and i+D/2..i+D/2+7 for rotate_half), applies the rotation with cos/sin read from a host-built
// fp32 table [max_pos, rot/2] (no on-device trig: guide App. B), and writes q/k/v directly in the layout the
// attention kernel consumes ([B, H, S, D]), fusing the 0213 transpose into the same pass. Backward is the same
// kernel with sin -> -sin (inverse rotation) and the layouts swapped.
#include "../include/ds_hip.h"

namespace {

// rotate_half convention (Llama/NeoX): pairs (i, i + rot/2).
template <typename T>
__device__ __forceinline__ void rot_pairs(float (&a)[8], float (&b)[8], const float* cs, const float* sn, int i,
                                          float sgn) {
  float c[8], s[8];
  *reinterpret_cast<f32x4*>(c) = *reinterpret_cast<const f32x4*>(cs + i);
  *reinterpret_cast<f32x4*>(c + 4) = *reinterpret_cast<const f32x4*>(cs + i + 4);
  *reinterpret_cast<f32x4*>(s) = *reinterpret_cast<const f32x4*>(sn + i);
  *reinterpret_cast<f32x4*>(s + 4) = *reinterpret_cast<const f32x4*>(sn + i + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x0 = a[j], x1 = b[j], ss = sgn * s[j];
    a[j] = x0 * c[j] - x1 * ss;
    b[j] = x1 * c[j] + x0 * ss;
  }
}

// element strides (batch, head, seq) of the head-major q / k / v views (unit last stride): [B,H,S,D] contiguous or a
// [B,S,H,D]-memory view (token-major, what the flash kernel and the efficient backward exchange without copies)
struct HmStrides {
  int64_t q[3], k[3], v[3];
};

// Forward: qkv [B,S,NH,D] (NH = Hq + 2*Hk) -> q [B,Hq,S,D], k [B,Hk,S,D], v [B,Hk,S,D]; rope on q,k first `rot` dims.
// Backward (INV): dq,dk,dv [B,H,S,D] -> dqkv [B,S,NH,D] with inverse rotation.
// pos: optional int32 [B*S] position ids (else s + pos_offset).
template <typename T, bool INV>
__global__ void __launch_bounds__(256) qkv_rope_kernel(const T* __restrict__ qkv_in, const T* __restrict__ q_in,
                                                       const T* __restrict__ k_in, const T* __restrict__ v_in,
                                                       T* __restrict__ qkv_out, T* __restrict__ q_out,
                                                       T* __restrict__ k_out, T* __restrict__ v_out,
                                                       const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                       const int* __restrict__ pos, int B, int S, int Hq, int Hk,
                                                       int D, int rot, int pos_offset, HmStrides st) {
  const int NH = Hq + 2 * Hk;
  const int half = rot / 2;
  // work item = (token, head, 16-element chunk): rotary chunks cover pairs, the rest plain 8-wide copies
  const int rot_chunks = half / 8;             // each covers 8 pairs (16 elements)
  const int pass_chunks = (D - rot) / 8;       // non-rotary tail, 8 elements each
  const int per_head = rot_chunks + pass_chunks;
  const int64_t total = (int64_t)B * S * NH * per_head;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int chunk = (int)(t % per_head);
    const int64_t th = t / per_head;
    const int h = (int)(th % NH);
    const int64_t tok = th / NH;
    const int s = (int)(tok % S), b = (int)(tok / S);
    // head-major destination/source
    const T* hm_src;
    T* hm_dst;
    int hh;
    bool do_rot;
    const int64_t* sd;
    if (h < Hq) { hh = h; do_rot = true; hm_src = q_in; hm_dst = q_out; sd = st.q; }
    else if (h < Hq + Hk) { hh = h - Hq; do_rot = true; hm_src = k_in; hm_dst = k_out; sd = st.k; }
    else { hh = h - Hq - Hk; do_rot = false; hm_src = v_in; hm_dst = v_out; sd = st.v; }
    const int64_t tm_off = (tok * NH + h) * (int64_t)D;                       // token-major [B,S,NH,D]
    const int64_t hm_off = b * sd[0] + hh * sd[1] + s * sd[2];              // head-major view [B,H,S,D]
    const T* src = INV ? hm_src + hm_off : qkv_in + tm_off;
    T* dst = INV ? qkv_out + tm_off : hm_dst + hm_off;
    if (chunk < rot_chunks) {
      const int i = chunk * 8;
      float a[8], bb[8];
      Vec8<T>::load(src + i, a);
      Vec8<T>::load(src + i + half, bb);
      if (do_rot) {
        const int p = pos ? pos[tok] : s + pos_offset;
        rot_pairs<T>(a, bb, cos_t + (int64_t)p * half, sin_t + (int64_t)p * half, i, INV ? -1.f : 1.f);
      }
      Vec8<T>::store(dst + i, a);
      Vec8<T>::store(dst + i + half, bb);
    } else {
      const int i = rot + (chunk - rot_chunks) * 8;
      float a[8];
      Vec8<T>::load(src + i, a);
      Vec8<T>::store(dst + i, a);
    }
  }
}

// In-place rotary on a strided [B, S, H, D] view (strides in elements), both conventions:
// interleaved=0: rotate_half pairs (i, i+rot/2); interleaved=1: GPT-J pairs (2i, 2i+1).
template <typename T>
__global__ void __launch_bounds__(256) rope_inplace_kernel(T* __restrict__ x, int B, int S, int H, int D,
                                                           int64_t sb, int64_t ss, int64_t sh,
                                                           const float* __restrict__ cos_t,
                                                           const float* __restrict__ sin_t,
                                                           const int* __restrict__ pos, int rot, int pos_offset,
                                                           int interleaved, float sgn) {
  const int half = rot / 2;
  const int64_t total = (int64_t)B * S * H * half;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int i = (int)(t % half);
    const int64_t r = t / half;
    const int h = (int)(r % H);
    const int64_t tok = r / H;
    const int s = (int)(tok % S), b = (int)(tok / S);
    T* base = x + b * sb + s * ss + h * sh;
    const int p = pos ? pos[tok] : s + pos_offset;
    const float c = cos_t[(int64_t)p * half + i], sn = sgn * sin_t[(int64_t)p * half + i];
    const int i0 = interleaved ? 2 * i : i, i1 = interleaved ? 2 * i + 1 : i + half;
    const float x0 = (float)base[i0], x1 = (float)base[i1];
    base[i0] = (T)(x0 * c - x1 * sn);
    base[i1] = (T)(x1 * c + x0 * sn);
  }
}

}  // namespace

#define DISPATCH_T(dt, ...)                                    \
  do {                                                         \
    if ((dt) == DS_F32) { using T = float; __VA_ARGS__; }      \
    else if ((dt) == DS_BF16) { using T = bf16; __VA_ARGS__; } \
    else { using T = fp16; __VA_ARGS__; }                      \
  } while (0)

extern "C" int ds_qkv_rope_fwd(const void* qkv, void* q, void* k, void* v, const float* cos_t, const float* sin_t,
                               const int* pos, int B, int S, int Hq, int Hk, int D, int rot, int pos_offset,
                               const int64_t* strides9, int dtype, hipStream_t s) {
  HmStrides st;
  for (int i = 0; i < 3; ++i) { st.q[i] = strides9[i]; st.k[i] = strides9[3 + i]; st.v[i] = strides9[6 + i]; }
  if (D % 8 || rot % 16 || rot > D) return (int)hipErrorInvalidValue;
  const int64_t work = (int64_t)B * S * (Hq + 2 * Hk) * (rot / 16 + (D - rot) / 8);
  const int grid = ds_grid_for(work, 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((qkv_rope_kernel<T, false>), dim3(grid), dim3(256), 0, s, (const T*)qkv,
                                       nullptr, nullptr, nullptr, nullptr, (T*)q, (T*)k, (T*)v, cos_t, sin_t, pos, B,
                                       S, Hq, Hk, D, rot, pos_offset, st));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_qkv_rope_bwd(const void* dq, const void* dk, const void* dv, void* dqkv, const float* cos_t,
                               const float* sin_t, const int* pos, int B, int S, int Hq, int Hk, int D, int rot,
                               int pos_offset, const int64_t* strides9, int dtype, hipStream_t s) {
  HmStrides st;
  for (int i = 0; i < 3; ++i) { st.q[i] = strides9[i]; st.k[i] = strides9[3 + i]; st.v[i] = strides9[6 + i]; }
  if (D % 8 || rot % 16 || rot > D) return (int)hipErrorInvalidValue;
  const int64_t work = (int64_t)B * S * (Hq + 2 * Hk) * (rot / 16 + (D - rot) / 8);
  const int grid = ds_grid_for(work, 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((qkv_rope_kernel<T, true>), dim3(grid), dim3(256), 0, s, nullptr,
                                       (const T*)dq, (const T*)dk, (const T*)dv, (T*)dqkv, nullptr, nullptr, nullptr,
                                       cos_t, sin_t, pos, B, S, Hq, Hk, D, rot, pos_offset, st));
  DS_CHECK_LAUNCH();
  return 0;
}

extern "C" int ds_rope_inplace(void* x, int B, int S, int H, int D, int64_t sb, int64_t ss, int64_t sh,
                               const float* cos_t, const float* sin_t, const int* pos, int rot, int pos_offset,
                               int interleaved, int inverse, int dtype, hipStream_t s) {
  if (rot % 2 || rot > D) return (int)hipErrorInvalidValue;
  const int grid = ds_grid_for((int64_t)B * S * H * (rot / 2), 256);
  DISPATCH_T(dtype, hipLaunchKernelGGL((rope_inplace_kernel<T>), dim3(grid), dim3(256), 0, s, (T*)x, B, S, H, D, sb,
                                       ss, sh, cos_t, sin_t, pos, rot, pos_offset, interleaved,
                                       inverse ? -1.f : 1.f));
  DS_CHECK_LAUNCH();
  return 0;
}
