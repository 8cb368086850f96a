// Peer-mapped one-shot / two-shot all-reduce for small tensor-parallel messages (decode), over xGMI.
//
// Reference counterpart (behaviour): `inference_all_reduce` (`deepspeed/comm/comm.py`, `csrc/cpu/comm/ccl.cpp:540-611`
// POSIX-shm + AVX-512 N-way reduce for the CPU accelerator). On a GPU node the reference falls back to NCCL, whose
// small-message all-reduce costs tens of microseconds of protocol latency; TP decode issues two of them per layer.
//
// MI355X design: every GPU pair of a node has its own xGMI link, so a rank can store straight into its peers' HBM.
// Each rank owns one uncached buffer + one uncached flag array, exported once with hipIpc handles and mapped by every
// peer (comm/xgmi.py does the exchange over the process group).
//  * push, not pull: a rank WRITES its data into each peer's receive slot (posted writes, no round trip), raises a
//    per-(block, source) flag in the peer's flag array, waits for its own flags and reduces from local memory;
//  * one-shot (small): each block pushes its whole chunk to every peer, then sums world copies -> out;
//    two-shot (larger): reduce-scatter by push (peer p receives sub-chunk p from everyone), reduce, push the reduced
//    sub-chunk to everyone, gather -> 2 (N-1)/N of the bytes per link instead of (N-1);
//  * no host involvement per call: the epoch of every block lives in device memory (incremented by the block
//    itself), so a call is one kernel launch and is capturable in a HIP graph;
//  * block b always uses its own private slot, double-buffered by epoch parity: a rank can only reach epoch e+2 of
//    block b after every peer signalled e+1 of block b, i.e. after every peer finished reading epoch e's slot;
//  * flags are compared wrap-safe (a fast peer may already have written e+2 when a slow one looks for e+1);
//  * every wait is bounded (5 s of the 100 MHz wall clock by default): on timeout the block records a sticky error
//    word (in device memory and in a host-mapped word the launcher reads without synchronising), fills its part of
//    the output with NaN and leaves — a broken or late peer can never leave waves spinning on the GPU, and a partial
//    sum is never returned as if it were a result: the NaNs poison the consumer and the next call raises.
// Stores to peers are ordinary vector stores; the flag release / acquire use system-scope atomics.
#include "ds_hip.h"

#include <cstring>

namespace {

constexpr int XAR_MAX_WORLD = 8;
constexpr int XAR_BLOCKS = 64;       // fixed block -> slot mapping (see above)
constexpr int XAR_THREADS = 512;
constexpr long long XAR_TIMEOUT = 500000000LL;  // default wait limit in wall_clock64 ticks (100 MHz): 5 s

struct XarCtx {
  char* buf[XAR_MAX_WORLD];          // every rank's exchange buffer (own at [rank])
  unsigned* flags[XAR_MAX_WORLD];    // every rank's flag array
  unsigned* meta;                    // own: epoch per block, then error word
  unsigned* err_host;                // host-mapped copy of the error word (sticky)
  int rank, world;
  long long slot;                    // bytes of one (block, source) slot
  long long timeout;                 // wait limit in wall-clock ticks
};

// buffer layout: [parity 2][block][area 2 (recv, gather)][source world][slot]
__device__ __forceinline__ long long xar_off(const XarCtx& c, int par, int b, int area, int src) {
  return ((((long long)par * XAR_BLOCKS + b) * 2 + area) * c.world + src) * c.slot;
}
// flag layout: [phase 2][block][source]
__device__ __forceinline__ int xar_flag(const XarCtx& c, int phase, int b, int src) {
  return (phase * XAR_BLOCKS + b) * c.world + src;
}

// raise flag (phase, b, my rank) in every peer, then wait for every peer's flag in my array; returns false (for
// the whole block) if a peer did not arrive within the limit
__device__ __forceinline__ bool xar_barrier(const XarCtx& c, int phase, int b, unsigned v) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < c.world) {
    __hip_atomic_store(c.flags[t] + xar_flag(c, phase, b, c.rank), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine = c.flags[c.rank] + xar_flag(c, phase, b, t);
    const long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - v) < 0) {
      if (wall_clock64() - t0 > c.timeout) {
        __hip_atomic_store(c.meta + XAR_BLOCKS, 1u + (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(c.err_host, 1u + (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return timed_out == 0;
}

// all-ones is a NaN in fp32, bf16 and fp16: the output of a call whose peers did not all arrive
__device__ __forceinline__ void xar_poison(uint4* dst, long long cnt) {
  const uint4 nan = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
  for (long long i = threadIdx.x; i < cnt; i += XAR_THREADS) dst[i] = nan;
}

// one 16-byte unit of T: 4 fp32 or 8 bf16 / fp16 elements, summed in fp32
template <typename T>
struct U16 {
  static constexpr int E = 16 / sizeof(T);
  __device__ __forceinline__ static void add(float (&acc)[8], const char* p) {
    const uint4 raw = *reinterpret_cast<const uint4*>(p);
    const T* v = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] += (float)v[j];
  }
  __device__ __forceinline__ static uint4 pack(const float (&acc)[8]) {
    uint4 raw;
    T* v = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = (T)acc[j];
    return raw;
  }
};

// n elements, 16-B units: each block owns `per` consecutive units
template <typename T>
__global__ void __launch_bounds__(XAR_THREADS) xar_oneshot(XarCtx c, const T* in, T* out, long long nu,
                                                            long long per) {
  const int b = blockIdx.x;
  const long long lo = (long long)b * per, cnt = max(0LL, min(nu, lo + per) - lo);
  const unsigned e = c.meta[b];
  const int par = e & 1;
  const unsigned v = e + 1;
  const uint4* src = reinterpret_cast<const uint4*>(in) + lo;
  for (long long i = threadIdx.x; i < cnt; i += XAR_THREADS) {
    const uint4 val = src[i];
    for (int p = 0; p < c.world; ++p)
      *reinterpret_cast<uint4*>(c.buf[p] + xar_off(c, par, b, 0, c.rank) + 16 * i) = val;
  }
  const bool ok = xar_barrier(c, 0, b, v);
  const char* mine = c.buf[c.rank];
  uint4* dst = reinterpret_cast<uint4*>(out) + lo;
  if (ok) {
    for (long long i = threadIdx.x; i < cnt; i += XAR_THREADS) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < c.world; ++s) U16<T>::add(acc, mine + xar_off(c, par, b, 0, s) + 16 * i);
      dst[i] = U16<T>::pack(acc);
    }
  } else {
    xar_poison(dst, cnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) c.meta[b] = v;
}

template <typename T>
__global__ void __launch_bounds__(XAR_THREADS) xar_twoshot(XarCtx c, const T* in, T* out, long long nu,
                                                            long long per) {
  const int b = blockIdx.x;
  const long long lo = (long long)b * per, cnt = max(0LL, min(nu, lo + per) - lo);
  const unsigned e = c.meta[b];
  const int par = e & 1;
  const unsigned v = e + 1;
  // sub-chunk s of this block: units [s * sub, min(cnt, (s + 1) * sub))
  const long long sub = (cnt + c.world - 1) / c.world;
  auto sub_lo = [&](int s) { return min(cnt, (long long)s * sub); };
  auto sub_n = [&](int s) { return min(cnt, (long long)(s + 1) * sub) - sub_lo(s); };
  const uint4* src = reinterpret_cast<const uint4*>(in) + lo;
  uint4* dst = reinterpret_cast<uint4*>(out) + lo;
  // reduce-scatter by push: peer p receives my sub-chunk p in its slot [recv][my rank]
  for (int p = 0; p < c.world; ++p) {
    const long long s0 = sub_lo(p), nv = sub_n(p);
    char* d = c.buf[p] + xar_off(c, par, b, 0, c.rank);
    for (long long i = threadIdx.x; i < nv; i += XAR_THREADS) *reinterpret_cast<uint4*>(d + 16 * i) = src[s0 + i];
  }
  bool ok = xar_barrier(c, 0, b, v);
  {  // reduce my sub-chunk, push it to every peer's gather slot [gather][my rank], keep it in out
    const char* mine = c.buf[c.rank];
    const long long s0 = sub_lo(c.rank), nv = sub_n(c.rank);
    for (long long i = threadIdx.x; i < nv; i += XAR_THREADS) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < c.world; ++s) U16<T>::add(acc, mine + xar_off(c, par, b, 0, s) + 16 * i);
      const uint4 val = U16<T>::pack(acc);
      dst[s0 + i] = val;
      for (int p = 0; p < c.world; ++p)
        if (p != c.rank) *reinterpret_cast<uint4*>(c.buf[p] + xar_off(c, par, b, 1, c.rank) + 16 * i) = val;
    }
  }
  ok = xar_barrier(c, 1, b, v) && ok;
  for (int s = 0; s < c.world; ++s) {
    if (s == c.rank) continue;
    const long long s0 = sub_lo(s), nv = sub_n(s);
    const char* g = c.buf[c.rank] + xar_off(c, par, b, 1, s);
    for (long long i = threadIdx.x; i < nv; i += XAR_THREADS) dst[s0 + i] = *reinterpret_cast<const uint4*>(g + 16 * i);
  }
  __syncthreads();
  if (!ok) xar_poison(dst, cnt);  // (peers that did get this rank's partial sub-chunk poison theirs as well: they
                                  // waited for the same missing flags)
  __syncthreads();
  if (threadIdx.x == 0) c.meta[b] = v;
}

struct XarComm {
  int rank = 0, world = 0;
  long long slot = 0, cap = 0;
  char* buf = nullptr;
  unsigned* flags = nullptr;
  unsigned* meta = nullptr;
  unsigned* err_host = nullptr;      // pinned, device-mapped: sticky error word readable without synchronising
  long long timeout = XAR_TIMEOUT;
  char* peer_buf[XAR_MAX_WORLD] = {};
  unsigned* peer_flags[XAR_MAX_WORLD] = {};
};

size_t buf_bytes(const XarComm* m) { return (size_t)2 * XAR_BLOCKS * 2 * m->world * m->slot; }
size_t flag_bytes(const XarComm* m) { return (size_t)2 * XAR_BLOCKS * m->world * sizeof(unsigned); }

}  // namespace

extern "C" int ds_xar_max_world() { return XAR_MAX_WORLD; }
extern "C" int ds_xar_handle_bytes() { return (int)(2 * sizeof(hipIpcMemHandle_t)); }

// Allocate this rank's exchange buffer / flags (uncached) and epoch words; messages up to cap_bytes.
extern "C" int ds_xar_create(int world, int rank, long long cap_bytes, void** out) {
  if (world < 2 || world > XAR_MAX_WORLD || rank < 0 || rank >= world || cap_bytes <= 0)
    return (int)hipErrorInvalidValue;
  auto* m = new XarComm();
  m->world = world;
  m->rank = rank;
  // one (block, source) slot holds a block's whole chunk: cap / blocks, rounded to 256 B
  m->slot = ((cap_bytes + XAR_BLOCKS - 1) / XAR_BLOCKS + 255) / 256 * 256;
  m->cap = m->slot * XAR_BLOCKS;
  hipError_t rc = hipExtMallocWithFlags((void**)&m->buf, buf_bytes(m), hipDeviceMallocUncached);
  if (rc == hipSuccess) rc = hipExtMallocWithFlags((void**)&m->flags, flag_bytes(m), hipDeviceMallocUncached);
  if (rc == hipSuccess) rc = hipMalloc((void**)&m->meta, (XAR_BLOCKS + 1) * sizeof(unsigned));
  if (rc == hipSuccess) rc = hipHostMalloc((void**)&m->err_host, sizeof(unsigned), hipHostMallocMapped);
  if (rc == hipSuccess) *m->err_host = 0;
  if (rc == hipSuccess) rc = hipMemset(m->flags, 0, flag_bytes(m));
  if (rc == hipSuccess) rc = hipMemset(m->meta, 0, (XAR_BLOCKS + 1) * sizeof(unsigned));
  if (rc == hipSuccess) rc = hipDeviceSynchronize();
  if (rc != hipSuccess) {
    (void)hipFree(m->buf);
    (void)hipFree(m->flags);
    (void)hipFree(m->meta);
    if (m->err_host) (void)hipHostFree(m->err_host);
    delete m;
    return (int)rc;
  }
  m->peer_buf[rank] = m->buf;
  m->peer_flags[rank] = m->flags;
  *out = m;
  return 0;
}

extern "C" long long ds_xar_cap(void* h) { return static_cast<XarComm*>(h)->cap; }

// IPC handles of this rank's buffer and flags, back to back (ds_xar_handle_bytes() bytes)
extern "C" int ds_xar_handles(void* h, void* dst) {
  auto* m = static_cast<XarComm*>(h);
  hipIpcMemHandle_t hb, hf;
  hipError_t rc = hipIpcGetMemHandle(&hb, m->buf);
  if (rc == hipSuccess) rc = hipIpcGetMemHandle(&hf, m->flags);
  if (rc != hipSuccess) return (int)rc;
  std::memcpy(dst, &hb, sizeof(hb));
  std::memcpy(static_cast<char*>(dst) + sizeof(hb), &hf, sizeof(hf));
  return 0;
}

// Map peer `p`'s buffer and flags from its handles.
extern "C" int ds_xar_open(void* h, int p, const void* handles) {
  auto* m = static_cast<XarComm*>(h);
  if (p < 0 || p >= m->world || p == m->rank) return (int)hipErrorInvalidValue;
  hipIpcMemHandle_t hb, hf;
  std::memcpy(&hb, handles, sizeof(hb));
  std::memcpy(&hf, static_cast<const char*>(handles) + sizeof(hb), sizeof(hf));
  void* b = nullptr;
  void* f = nullptr;
  hipError_t rc = hipIpcOpenMemHandle(&b, hb, hipIpcMemLazyEnablePeerAccess);
  if (rc == hipSuccess) rc = hipIpcOpenMemHandle(&f, hf, hipIpcMemLazyEnablePeerAccess);
  if (rc != hipSuccess) return (int)rc;
  m->peer_buf[p] = static_cast<char*>(b);
  m->peer_flags[p] = static_cast<unsigned*>(f);
  return 0;
}

// in / out: n elements of dtype (DS_F32 / DS_BF16 / DS_F16), n * size a multiple of 16 B and <= cap; out may alias in.
// mode 1 one-shot, 2 two-shot.
extern "C" int ds_xar_allreduce(void* h, const void* in, void* out, long long n, int dtype, int mode,
                                hipStream_t st) {
  auto* m = static_cast<XarComm*>(h);
  for (int p = 0; p < m->world; ++p)
    if (!m->peer_buf[p] || !m->peer_flags[p]) return (int)hipErrorNotInitialized;
  const int es = dtype == DS_F32 ? 4 : 2;
  if (n <= 0 || (n * es) % 16 || n * es > m->cap || (mode != 1 && mode != 2)) return (int)hipErrorInvalidValue;
  // a wait of an earlier call timed out (its output was poisoned): refuse to go on until the caller resets
  if (*static_cast<volatile unsigned*>(m->err_host) != 0) return (int)hipErrorLaunchTimeOut;
  XarCtx c;
  for (int p = 0; p < XAR_MAX_WORLD; ++p) {
    c.buf[p] = m->peer_buf[p];
    c.flags[p] = m->peer_flags[p];
  }
  c.meta = m->meta;
  c.err_host = m->err_host;
  c.timeout = m->timeout;
  c.rank = m->rank;
  c.world = m->world;
  c.slot = m->slot;
  // 16-B units; blocks of at least ~8 KB, at most XAR_BLOCKS
  const long long nu = n * es / 16;
  const int blocks = (int)std::max(1LL, std::min<long long>(XAR_BLOCKS, nu * 16 / 8192));
  const long long per = (nu + blocks - 1) / blocks;
  const int grid = (int)((nu + per - 1) / per);
  if (per * 16 > m->slot || grid > XAR_BLOCKS) return (int)hipErrorInvalidValue;
#define XAR_GO(T)                                                                                            \
  if (mode == 1)                                                                                             \
    hipLaunchKernelGGL(xar_oneshot<T>, dim3(grid), dim3(XAR_THREADS), 0, st, c, (const T*)in, (T*)out, nu, per); \
  else                                                                                                       \
    hipLaunchKernelGGL(xar_twoshot<T>, dim3(grid), dim3(XAR_THREADS), 0, st, c, (const T*)in, (T*)out, nu, per);
  if (dtype == DS_F32) {
    XAR_GO(float)
  } else if (dtype == DS_BF16) {
    XAR_GO(bf16)
  } else {
    XAR_GO(fp16)
  }
#undef XAR_GO
  DS_CHECK_LAUNCH();
  return 0;
}

// error word: 0 ok, 1 + peer index of a wait that timed out (sticky until reset)
extern "C" int ds_xar_error(void* h, int reset) {
  auto* m = static_cast<XarComm*>(h);
  unsigned e = 0;
  if (hipMemcpy(&e, m->meta + XAR_BLOCKS, sizeof(e), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (e == 0) e = *static_cast<volatile unsigned*>(m->err_host);
  if (reset) {
    (void)hipMemset(m->meta + XAR_BLOCKS, 0, sizeof(unsigned));
    *m->err_host = 0;
  }
  return (int)e;
}

// wait limit of every later call, in milliseconds (tests of the failure path use a few ms)
extern "C" void ds_xar_set_timeout_ms(void* h, double ms) {
  static_cast<XarComm*>(h)->timeout = (long long)(ms * 1e5);  // 100 MHz wall clock
}

extern "C" void ds_xar_destroy(void* h) {
  auto* m = static_cast<XarComm*>(h);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < m->world; ++p) {
    if (p == m->rank) continue;
    if (m->peer_buf[p]) (void)hipIpcCloseMemHandle(m->peer_buf[p]);
    if (m->peer_flags[p]) (void)hipIpcCloseMemHandle(m->peer_flags[p]);
  }
  (void)hipFree(m->buf);
  (void)hipFree(m->flags);
  (void)hipFree(m->meta);
  (void)hipHostFree(m->err_host);
  delete m;
}
