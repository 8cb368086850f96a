// Single-node shared-memory all-reduce for HOST tensors (CPU inference / gloo plumbing path).
//
// Parity: reference `csrc/cpu/comm/ccl.cpp:37-66,146-270,309-367,540-611` (POSIX shm + AVX-512 N-way reduce used by
// `inference_all_reduce` on the CPU accelerator). Used by `comm.inference_all_reduce` for host tensors
// (comm/xgmi.py ShmAllReduce; device tensors take the xGMI peer-mapped path, csrc/comm/xgmi_allreduce.hip): ranks of
// one node map one POSIX shm segment per process group, each rank owns a slot, a generation-counter barrier in
// shared memory orders the phases, and every rank reduces its 1/world slice of the vector (reduce-scatter) and then
// gathers the full result (all-gather) — 2(N-1)/N of the bytes per rank instead of the naive N-way read.
#include <torch/extension.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

struct ShmHeader {
  std::atomic<int64_t> arrive[2];
  std::atomic<int64_t> gen;
  int64_t world;
  int64_t slot_bytes;
};

struct ShmState {
  int rank = -1, world = 0;
  int64_t slot_bytes = 0;
  char* base = nullptr;
  size_t map_bytes = 0;
  int64_t my_gen = 0;
  std::string name;
};

// one segment per process group; `cur` is the one the current call works on
std::vector<ShmState*> segments;
thread_local ShmState* cur = nullptr;

ShmState* seg(int64_t h) {
  if (h < 0 || h >= (int64_t)segments.size() || !segments[h]) throw std::runtime_error("shm: bad handle");
  return segments[h];
}

ShmHeader* hdr() { return reinterpret_cast<ShmHeader*>(cur->base); }
char* slot(int r) { return cur->base + 4096 + (size_t)r * cur->slot_bytes; }

void barrier() {
  ShmHeader* h = hdr();
  const int64_t gen = cur->my_gen;
  const int idx = gen & 1;
  const int64_t arrived = h->arrive[idx].fetch_add(1, std::memory_order_acq_rel) + 1;
  if (arrived == cur->world) {
    h->arrive[idx].store(0, std::memory_order_relaxed);
    h->gen.store(gen + 1, std::memory_order_release);
  } else {
    int64_t spins = 0;
    while (h->gen.load(std::memory_order_acquire) <= gen) {
      if (++spins > 1000) sched_yield();
    }
  }
  cur->my_gen = gen + 1;
}

inline float bf(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t tobf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__attribute__((target_clones("avx512f", "avx2", "default"))) void reduce_f32(float* out, int world, int64_t off,
                                                                             int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    float acc = 0.f;
    for (int r = 0; r < world; ++r) acc += reinterpret_cast<float*>(slot(r))[off + i];
    out[i] = acc;
  }
}

}  // namespace

// Create (rank 0) / open (others) the segment. All ranks must call; rank 0 first or concurrently (open retries).
// Returns the segment handle.
int64_t shm_init(const std::string& name, int64_t rank, int64_t world, int64_t max_bytes) {
  segments.push_back(new ShmState());
  cur = segments.back();
  cur->rank = (int)rank;
  cur->world = (int)world;
  cur->slot_bytes = (max_bytes + 4095) / 4096 * 4096;
  cur->map_bytes = 4096 + (size_t)world * cur->slot_bytes;
  cur->name = name;
  int fd = -1;
  if (rank == 0) {
    shm_unlink(name.c_str());
    fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)cur->map_bytes) != 0) throw std::runtime_error("shm_init: create failed");
  } else {
    for (int tries = 0; tries < 200000 && fd < 0; ++tries) {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) usleep(100);
    }
    if (fd < 0) throw std::runtime_error("shm_init: open failed");
    struct stat st;
    for (int tries = 0; tries < 200000; ++tries) {
      if (fstat(fd, &st) == 0 && (size_t)st.st_size >= cur->map_bytes) break;
      usleep(100);
    }
  }
  void* p = mmap(nullptr, cur->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("shm_init: mmap failed");
  cur->base = static_cast<char*>(p);
  cur->my_gen = 0;
  if (rank == 0) {
    // ftruncate zero-filled the segment, so the counters already read 0 (no re-init: peers may be arriving)
    hdr()->world = world;
    hdr()->slot_bytes = cur->slot_bytes;
  }
  return (int64_t)segments.size() - 1;
}

// In-place sum all-reduce of a contiguous fp32 or bf16 host tensor across the segment's ranks.
void shm_allreduce(int64_t handle, torch::Tensor t) {
  cur = seg(handle);
  TORCH_CHECK(cur->base != nullptr, "shm_allreduce: call shm_init first");
  TORCH_CHECK(t.device().is_cpu() && t.is_contiguous(), "shm_allreduce: host contiguous tensor required");
  const bool isbf = t.scalar_type() == at::kBFloat16;
  TORCH_CHECK(isbf || t.scalar_type() == at::kFloat, "shm_allreduce: fp32/bf16 only");
  const int64_t n = t.numel();
  const int64_t elems_per_slot = cur->slot_bytes / 4 / 2;  // slot = [fp32 input | fp32 reduced]
  for (int64_t base = 0; base < n; base += elems_per_slot) {
    const int64_t cnt = std::min(elems_per_slot, n - base);
    float* mine = reinterpret_cast<float*>(slot(cur->rank));
    if (isbf) {
      const uint16_t* s = reinterpret_cast<const uint16_t*>(t.data_ptr()) + base;
      for (int64_t i = 0; i < cnt; ++i) mine[i] = bf(s[i]);
    } else {
      std::memcpy(mine, t.data_ptr<float>() + base, cnt * 4);
    }
    barrier();
    // reduce-scatter: rank r reduces slice r into the "reduced" half of its own slot
    const int64_t per = (cnt + cur->world - 1) / cur->world;
    const int64_t lo = std::min(cnt, per * cur->rank), hi = std::min(cnt, lo + per);
    float* red = mine + elems_per_slot;
    if (hi > lo) reduce_f32(red + lo, cur->world, lo, hi - lo);
    barrier();
    // all-gather the reduced slices
    for (int r = 0; r < cur->world; ++r) {
      const int64_t rlo = std::min(cnt, per * r), rhi = std::min(cnt, rlo + per);
      const float* src = reinterpret_cast<float*>(slot(r)) + elems_per_slot;
      if (isbf) {
        uint16_t* d = reinterpret_cast<uint16_t*>(t.data_ptr()) + base;
        for (int64_t i = rlo; i < rhi; ++i) d[i] = tobf(src[i]);
      } else {
        std::memcpy(t.data_ptr<float>() + base + rlo, src + rlo, (rhi - rlo) * 4);
      }
    }
    barrier();
  }
}

void shm_barrier(int64_t handle) {
  cur = seg(handle);
  barrier();
}

// Drop the segment's name once every rank has mapped it: the mappings stay valid and nothing is left in /dev/shm
// when the job ends, however it ends.
void shm_release_name(int64_t handle) {
  cur = seg(handle);
  shm_unlink(cur->name.c_str());
}

void shm_finalize(int64_t handle) {
  cur = seg(handle);
  if (cur->base) {
    munmap(cur->base, cur->map_bytes);
    cur->base = nullptr;
  }
  delete cur;
  segments[handle] = nullptr;
  cur = nullptr;
}

void register_shm_comm(pybind11::module& m) {
  m.def("shm_init", &shm_init);
  m.def("shm_allreduce", &shm_allreduce);
  m.def("shm_barrier", &shm_barrier);
  m.def("shm_finalize", &shm_finalize);
  m.def("shm_release_name", &shm_release_name);
}
