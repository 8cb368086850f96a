// Host-code sanitizer harness for the native CPU ops (SURVEY §5.2 [design]: run the C++ kernels under
// -fsanitize=address,undefined host builds; GPU-side ASan / XNACK is not available on the MI355X pool).
//
// The three host translation units of `ds_cpu_ops` are compiled INTO this executable (so their internal-linkage
// helpers are reachable and the sanitizer runtime is linked the normal way, no preloading), and `main` drives each
// with ragged sizes that hit tile tails / partial I/O blocks:
//   optim : CPU Adam / AdamW / Adagrad / Lion with fp32 / bf16 / fp16 grads and low-precision copies, bf16 cast
//   aio   : async tensor writes + reads through the thread pool (unaligned sizes, several in flight), data check
//   shm   : two forked ranks run the POSIX-shm all-reduce (fp32 + bf16) and barrier, result check
// Built and run by tests/unit/ops/test_host_sanitizers.py (ASan + UBSan, runtimes linked statically).
#include "../../deepspeedsyclsupport_amd/ops/csrc/cpu/cpu_optim.cpp"
#include "../../deepspeedsyclsupport_amd/ops/csrc/cpu/aio.cpp"
#include "../../deepspeedsyclsupport_amd/ops/csrc/cpu/shm_comm.cpp"

#include <sys/wait.h>

#include <cstdio>
#include <cstdlib>

#define EXPECT(c)                                                              \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "EXPECT failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(3);                                                            \
    }                                                                          \
  } while (0)

static void run_optim() {
  const int64_t sizes[] = {1, 7, (1 << 16) + 5, 3 * (1 << 16) + 129};
  for (int64_t n : sizes) {
    for (auto gdt : {at::kFloat, at::kBFloat16, at::kHalf}) {
      auto p = torch::randn({n});
      auto m = torch::zeros({n});
      auto v = torch::zeros({n});
      auto g = torch::randn({n}).to(gdt);
      auto lp = torch::empty({n}, torch::TensorOptions().dtype(at::kBFloat16));
      auto p0 = p.clone();
      cpu_adam_update(p, m, v, g, lp, 1, 1e-3, 0.9, 0.999, 1e-8, 0.01, true, true, 1.0);
      EXPECT(!p.isnan().any().item<bool>());
      EXPECT((lp.to(at::kFloat) - p).abs().max().item<float>() < 1e-2f * (1.f + p.abs().max().item<float>()));
      EXPECT(!torch::equal(p, p0));
      auto s = torch::zeros({n});
      cpu_adagrad_update(p, s, g, c10::nullopt, 1e-2, 1e-10, 0.0, 1.0);
      auto lph = torch::empty({n}, torch::TensorOptions().dtype(at::kHalf));
      cpu_lion_update(p, m, g, lph, 1e-4, 0.9, 0.99, 0.1, 1.0);
      auto dst = torch::empty({n}, torch::TensorOptions().dtype(at::kBFloat16));
      cpu_to_bf16(p, dst);
      EXPECT((dst.to(at::kFloat) - p).abs().max().item<float>() <= 1e-2f * (1.f + p.abs().max().item<float>()));
    }
  }
  std::printf("optim ok (%s)\n", simd_level().c_str());
}

static void run_aio(const std::string& dir) {
  AioHandle h(1 << 16, 8, false, true, 4);
  std::vector<torch::Tensor> src, dst;
  const int64_t sizes[] = {1, 1000, (1 << 16) + 3, 5 * (1 << 16) - 17, 1 << 20};
  int i = 0;
  for (int64_t n : sizes) {
    src.push_back(torch::randn({n}));
    const std::string f = dir + "/aio_" + std::to_string(i++) + ".bin";
    h.async_pwrite(src.back(), f);
  }
  h.wait();
  i = 0;
  for (int64_t n : sizes) {
    dst.push_back(torch::empty({n}));
    const std::string f = dir + "/aio_" + std::to_string(i++) + ".bin";
    h.async_pread(dst.back(), f);
  }
  h.wait();
  for (size_t k = 0; k < src.size(); ++k) EXPECT(torch::equal(src[k], dst[k]));
  auto a = torch::randn({12345});
  auto b = torch::empty({12345});
  deepspeed_memcpy(b, a);
  EXPECT(torch::equal(a, b));
  std::printf("aio ok\n");
}

static int shm_rank(const std::string& name, int rank) {
  const int64_t h = shm_init(name, rank, 2, 1 << 20);
  shm_barrier(h);
  if (rank == 0) shm_release_name(h);
  for (int it = 0; it < 3; ++it) {
    auto t = torch::full({100003}, (float)(rank + 1 + it));
    shm_allreduce(h, t);
    if (!torch::allclose(t, torch::full({100003}, (float)(3 + 2 * it)))) return 4;
    auto tb = torch::full({4099}, (float)(rank + 1), torch::TensorOptions().dtype(at::kBFloat16));
    shm_allreduce(h, tb);
    if (!torch::allclose(tb.to(at::kFloat), torch::full({4099}, 3.f))) return 5;
    shm_barrier(h);
  }
  shm_finalize(h);
  return 0;
}

static void run_shm() {
  const std::string name = "/ds_amd_sanitize_" + std::to_string(getpid());
  pid_t pid = fork();
  if (pid == 0) std::_Exit(shm_rank(name, 1));
  const int rc0 = shm_rank(name, 0);
  int status = 0;
  waitpid(pid, &status, 0);
  EXPECT(rc0 == 0);
  EXPECT(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  std::printf("shm ok\n");
}

int main(int argc, char** argv) {
  torch::manual_seed(0);
  const std::string dir = argc > 2 ? argv[2] : "/tmp";
  const std::string what = argc > 1 ? argv[1] : "optim,aio,shm";
  if (what.find("optim") != std::string::npos) run_optim();
  if (what.find("aio") != std::string::npos) run_aio(dir);
  if (what.find("shm") != std::string::npos) run_shm();
  std::printf("all ok\n");
  return 0;
}
