// 16-bit 2-D transpose, CDNA4: out[C, R] = in[R, C]^T (input rows may be strided).
//
// Used to hand hipBLASLt K-major operands for the weight-gradient GEMMs of the training step (dW = dY^T X with the
// token dimension as K): with both operands MN-major the library GEMM runs at ~1.0-1.1 PF/s, with K-major copies at
// ~1.4-1.5 PF/s (`profiles/wgrad_gemm_layouts_r2.jsonl`) — the copies must therefore stream at HBM speed.
//
// One workgroup moves a 64 x 64 tile: 16-B global loads along the input rows (8 lanes per 128-B row segment), the
// tile parked in LDS with rows padded to 33 dwords (column reads by consecutive lanes hit consecutive banks), then
// 16-B global stores along the output rows. Tiles are walked in an order that keeps each XCD on a contiguous band
// of output rows.
#include "../include/ds_hip.h"

namespace {

constexpr int TS = 64;           // tile edge
constexpr int LROW = 33;         // LDS row stride in dwords (64 x 16-bit + 1 dword pad)

__global__ void __launch_bounds__(256) transpose16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                          int R, int Rp, int C, int64_t ld, int tiles_r,
                                                          int tiles_c) {
  __shared__ uint32_t tile[TS * LROW];
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tr = bid % tiles_r, tc = bid / tiles_r;  // consecutive ids walk down the input rows = along out rows
  const int r0 = tr * TS, c0 = tc * TS;
  const int t = threadIdx.x, lr = t >> 3, lc = t & 7;
  // load: rows lr and lr + 32, 8 x 16-bit at column 8 * lc
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = lr + 32 * p, gr = r0 + r, gc = c0 + 8 * lc;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gr < R && gc < C) v = *reinterpret_cast<const uint4*>(in + (int64_t)gr * ld + gc);
    uint32_t* dst = tile + r * LROW + 4 * lc;
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();
  // store: output row oc = c0 + j holds input column j; 8 consecutive output elements = input rows 8 * lc .. + 7
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int j = lr + 32 * p, oc = c0 + j, orow0 = r0 + 8 * lc;
    if (oc >= C || orow0 >= Rp) continue;  // rows R..Rp-1 of the output are the zero padding
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = t16[(8 * lc + 2 * e) * LROW * 2 + j];
      const uint32_t hi = t16[(8 * lc + 2 * e + 1) * LROW * 2 + j];
      w[e] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(out + (int64_t)oc * Rp + orow0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

}  // namespace

// in [R, C] with row stride ld (elements), out [C, Rp] contiguous (Rp >= R: columns R..Rp-1 zero-filled, so a
// GEMM can contract over a padded token dimension); 16-bit elements; R, Rp, C, ld multiples of 8 and 16-B aligned
// bases (whole 16-B chunks are moved).
extern "C" int ds_transpose16(const void* in, void* out, int R, int Rp, int C, int64_t ld, hipStream_t st) {
  if (R <= 0 || C <= 0 || Rp < R || R % 8 || Rp % 8 || C % 8 || ld % 8 || ld < C) return (int)hipErrorInvalidValue;
  const int tiles_r = (Rp + TS - 1) / TS, tiles_c = (C + TS - 1) / TS;
  const int64_t n = (int64_t)tiles_r * tiles_c;
  if (n > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)n), dim3(256), 0, st, (const uint16_t*)in, (uint16_t*)out, R,
                     Rp, C, ld, tiles_r, tiles_c);
  DS_CHECK_LAUNCH();
  return 0;
}
