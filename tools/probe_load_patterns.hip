// HBM read-pattern probe for the int8 decode GEMV: how fast can one wave stream a 16-row weight block when each
// 16-byte-per-lane load instruction covers (A) 16 rows x 64 B (the MFMA operand layout), (B) 4 rows x 256 B,
// (C) 1 row x 1 KB? Loads only (xor-reduced so nothing is dead). Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int PAT, int UNR>
__global__ void __launch_bounds__(256) probe(const int8_t* __restrict__ Q, int* __restrict__ out, int N, int K,
                                             int ksplit) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nblk = N / 16;
  const int wave = blockIdx.x * 4 + wid;
  const int blk = wave % nblk, ks = wave / nblk;
  if (ks >= ksplit) return;
  const int klen = K / ksplit, k0 = ks * klen;
  int r, c, rstep, cstep;  // lane's row / column and the per-sub-load steps
  if (PAT == 0) { r = lane & 15; c = 16 * (lane >> 4); rstep = 0; cstep = 64; }
  else if (PAT == 1) { r = lane >> 4; c = 16 * (lane & 15); rstep = 4; cstep = 256; }
  else { r = 0; c = 16 * lane; rstep = 1; cstep = 1024; }
  // every pattern reads the same 16 rows x 1 KB per "step" with 16 instructions
  const int8_t* base = Q + (int64_t)(blk * 16) * K + k0;
  i32x4 acc = {0, 0, 0, 0};
  for (int kk = 0; kk < klen; kk += 1024 * UNR) {
    i32x4 w[UNR][16];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        int rr, cc;
        if (PAT == 0) { rr = r; cc = kk + u * 1024 + c + i * cstep; }
        else if (PAT == 1) { rr = r + (i & 3) * rstep; cc = kk + u * 1024 + c + (i >> 2) * cstep; }
        else { rr = i; cc = kk + u * 1024 + c; }
        w[u][i] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(base + (int64_t)rr * K + cc));
      }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= w[u][i];
  }
  const int v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x12345678) out[0] = v;  // practically never: keeps the loads live
}

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

// (D) the same 4 rows x 256 B pattern through LDS-DMA: each wave streams its 16-row block through a private ring of
// NS 4-KB slots (16 rows x 256 B), NS-1 slots ahead, reading one 16-B word per lane back from LDS.
template <int NS, int WPB>
__global__ void __launch_bounds__(64 * WPB) probe_dma(const int8_t* __restrict__ Q, int* __restrict__ out, int N, int K,
                                                      int ksplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nblk = N / 16;
  const int wave = blockIdx.x * WPB + wid;
  const int blk = wave % nblk, ks = wave / nblk;
  if (ks >= ksplit) return;
  const int klen = K / ksplit, k0 = ks * klen;
  const int8_t* base = Q + (int64_t)(blk * 16) * K + k0;
  char* ring = smem + wid * NS * 4096;
  const int nsl = klen / 256;
  auto issue = [&](int sl) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * j + (lane >> 4);
      glds16(base + (int64_t)r * K + sl * 256 + 16 * (lane & 15), ring + (sl % NS) * 4096 + j * 1024);
    }
  };
  for (int i = 0; i < NS - 1 && i < nsl; ++i) issue(i);
  i32x4 acc = {0, 0, 0, 0};
  for (int sl = 0; sl < nsl; ++sl) {
    if (sl + NS - 1 <= nsl) {
      if (NS == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (NS == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc ^= *reinterpret_cast<const i32x4*>(ring + (sl % NS) * 4096 + lane * 16);
    acc ^= *reinterpret_cast<const i32x4*>(ring + (sl % NS) * 4096 + 1024 + lane * 16);
    acc ^= *reinterpret_cast<const i32x4*>(ring + (sl % NS) * 4096 + 2048 + lane * 16);
    acc ^= *reinterpret_cast<const i32x4*>(ring + (sl % NS) * 4096 + 3072 + lane * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (sl + NS - 1 < nsl) issue(sl + NS - 1);
  }
  const int v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x12345678) out[0] = v;
}

template <int NS, int WPB>
float run_dma(const int8_t* q, int* o, int N, int K, int ksplit) {
  const int waves = (N / 16) * ksplit;
  const int grid = (waves + WPB - 1) / WPB;
  const int lds = NS * 4096 * WPB;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_dma<NS, WPB>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) probe_dma<NS, WPB><<<grid, 64 * WPB, lds>>>(q, o, N, K, ksplit);
  hipEventRecord(a);
  const int it = 20;
  for (int i = 0; i < it; ++i) probe_dma<NS, WPB><<<grid, 64 * WPB, lds>>>(q, o, N, K, ksplit);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return (double)N * K / (ms / it * 1e-3) / 1e12;
}

// (E) 1-KB-per-instruction streams as the pre-shuffled int8 GEMV issues them. MODE 0: wave w reads chunks
// w*L .. (w+1)*L-1 in order (blocked, sequential per wave); MODE 1: chunks w, w+W, w+2W, ... (interleaved: at any
// time the waves together read one contiguous window); MODE 2: blocked, but FB=4 streams per wave spaced L/4 apart.
template <int MODE, int UNR>
__global__ void __launch_bounds__(256) probe_stream(const int8_t* __restrict__ Q, int* __restrict__ out,
                                                     int64_t nchunks) {
  const int lane = threadIdx.x & 63;
  const int64_t w = blockIdx.x * 4 + (threadIdx.x >> 6), W = gridDim.x * 4;
  const int64_t L = nchunks / W;
  i32x4 acc = {0, 0, 0, 0};
  for (int64_t j = 0; j + UNR <= L; j += UNR) {  // whole batches only: never past this wave's range
    i32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      int64_t c;
      if (MODE == 0) c = w * L + j + u;
      else if (MODE == 1) c = w + (j + u) * W;
      else c = w * L + (u & 3) * (L / 4) + (j + u) / 4;
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(Q + c * 1024 + lane * 16));
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= v[u];
  }
  const int r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (r == 0x12345678) out[0] = r;
}

template <int MODE, int UNR>
float run_stream(const int8_t* q, int* o, int64_t bytes, int waves) {
  const int64_t nchunks = bytes / 1024;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) probe_stream<MODE, UNR><<<waves / 4, 256>>>(q, o, nchunks);
  hipEventRecord(a);
  const int it = 20;
  for (int i = 0; i < it; ++i) probe_stream<MODE, UNR><<<waves / 4, 256>>>(q, o, nchunks);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const int64_t used = (nchunks / waves) / UNR * UNR * waves * 1024;
  return (double)used / (ms / it * 1e-3) / 1e12;
}

template <int PAT, int UNR>
float run(const int8_t* q, int* o, int N, int K, int ksplit) {
  const int waves = (N / 16) * ksplit;
  const int grid = (waves + 3) / 4;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) probe<PAT, UNR><<<grid, 256>>>(q, o, N, K, ksplit);
  hipEventRecord(a);
  const int it = 20;
  for (int i = 0; i < it; ++i) probe<PAT, UNR><<<grid, 256>>>(q, o, N, K, ksplit);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return (double)N * K / (ms / it * 1e-3) / 1e12;
}

int main() {
  const int shapes[][2] = {{57344, 14336}, {14336, 57344}, {22016, 4096}, {4096, 4096}};
  int8_t* q;
  int* o;
  hipMalloc(&q, (size_t)57344 * 14336);
  hipMalloc(&o, 64);
  hipMemset(q, 1, (size_t)57344 * 14336);
  const int64_t bytes = (int64_t)57344 * 14336;
  for (int waves : {1024, 2048, 3072, 4096}) {
    printf("{\"stream_waves\": %d, \"blocked_u8\": %.2f, \"blocked_u16\": %.2f, \"interleaved_u8\": %.2f, "
           "\"interleaved_u16\": %.2f, \"blocked4_u8\": %.2f, \"blocked4_u16\": %.2f}\n",
           waves, run_stream<0, 8>(q, o, bytes, waves), run_stream<0, 16>(q, o, bytes, waves),
           run_stream<1, 8>(q, o, bytes, waves), run_stream<1, 16>(q, o, bytes, waves),
           run_stream<2, 8>(q, o, bytes, waves), run_stream<2, 16>(q, o, bytes, waves));
    fflush(stdout);
  }
  for (auto& s : shapes) {
    const int N = s[0], K = s[1];
    for (int ksplit : {1, 2, 4, 8}) {
      if (K / ksplit < 1024 * 2 || (K / ksplit) % 2048) continue;
      printf("{\"N\": %d, \"K\": %d, \"ksplit\": %d, \"A16x64\": %.2f, \"B4x256\": %.2f, \"C1x1k\": %.2f, "
             "\"dma3_w4\": %.2f, \"dma4_w4\": %.2f, \"dma4_w1\": %.2f, \"dma5_w2\": %.2f}\n",
             N, K, ksplit, run<0, 2>(q, o, N, K, ksplit), run<1, 2>(q, o, N, K, ksplit),
             run<2, 2>(q, o, N, K, ksplit), run_dma<3, 4>(q, o, N, K, ksplit), run_dma<4, 4>(q, o, N, K, ksplit),
             run_dma<4, 1>(q, o, N, K, ksplit), run_dma<5, 2>(q, o, N, K, ksplit));
      fflush(stdout);
    }
  }
  return 0;
}
