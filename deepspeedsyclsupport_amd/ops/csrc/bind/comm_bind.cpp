// Bindings: peer-mapped xGMI all-reduce (comm/xgmi_allreduce.hip) used by comm.inference_all_reduce.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <mutex>
#include <vector>

extern "C" {
int ds_xar_max_world();
int ds_xar_handle_bytes();
int ds_xar_create(int, int, long long, void**);
long long ds_xar_cap(void*);
int ds_xar_handles(void*, void*);
int ds_xar_open(void*, int, const void*);
int ds_xar_allreduce(void*, const void*, void*, long long, int, int, hipStream_t);
int ds_xar_error(void*, int);
void ds_xar_set_timeout_ms(void*, double);
void ds_xar_destroy(void*);
}

namespace {

std::mutex mu;
std::vector<void*> comms;

void* get(int64_t id) {
  std::lock_guard<std::mutex> g(mu);
  TORCH_CHECK(id >= 0 && id < (int64_t)comms.size() && comms[id], "xar: bad communicator id ", id);
  return comms[id];
}
void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", hipGetErrorString((hipError_t)rc)); }

int64_t xar_create(int64_t world, int64_t rank, int64_t cap_bytes) {
  void* h = nullptr;
  check(ds_xar_create((int)world, (int)rank, cap_bytes, &h), "xar_create");
  std::lock_guard<std::mutex> g(mu);
  comms.push_back(h);
  return (int64_t)comms.size() - 1;
}

py::bytes xar_handles(int64_t id) {
  std::string s(ds_xar_handle_bytes(), '\0');
  check(ds_xar_handles(get(id), s.data()), "xar_handles");
  return py::bytes(s);
}

void xar_open(int64_t id, int64_t peer, py::bytes handles) {
  std::string s = handles;
  TORCH_CHECK((int)s.size() == ds_xar_handle_bytes(), "xar_open: handle size");
  check(ds_xar_open(get(id), (int)peer, s.data()), "xar_open");
}

// in-place when out is in; mode 1 one-shot, 2 two-shot
void xar_allreduce(int64_t id, torch::Tensor in, torch::Tensor out, int64_t mode) {
  TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_cuda() && out.is_contiguous(), "xar: contiguous device");
  TORCH_CHECK(in.numel() == out.numel() && in.scalar_type() == out.scalar_type(), "xar: in/out mismatch");
  int dt = 0;
  if (in.scalar_type() == at::kBFloat16) dt = 1;
  else if (in.scalar_type() == at::kHalf) dt = 2;
  else TORCH_CHECK(in.scalar_type() == at::kFloat, "xar: fp32/bf16/fp16 only");
  const int rc = ds_xar_allreduce(get(id), in.data_ptr(), out.data_ptr(), in.numel(), dt, (int)mode,
                                  at::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(rc != (int)hipErrorLaunchTimeOut,
              "xGMI all-reduce: a peer did not arrive within the wait limit in an earlier call (error word ",
              ds_xar_error(get(id), 0), " = 1 + peer index); that call's output was filled with NaN. The ranks "
              "are out of step: fix the straggler, or raise DS_XGMI_AR_TIMEOUT_MS, then reset the communicator");
  check(rc, "xar_allreduce");
}
void xar_set_timeout_ms(int64_t id, double ms) { ds_xar_set_timeout_ms(get(id), ms); }

int64_t xar_error(int64_t id, bool reset) { return ds_xar_error(get(id), reset ? 1 : 0); }
int64_t xar_cap(int64_t id) { return ds_xar_cap(get(id)); }

void xar_destroy(int64_t id) {
  void* h = get(id);
  {
    std::lock_guard<std::mutex> g(mu);
    comms[id] = nullptr;
  }
  ds_xar_destroy(h);
}

}  // namespace

void register_comm_ops(pybind11::module& m) {
  m.def("xar_max_world", &ds_xar_max_world);
  m.def("xar_create", &xar_create);
  m.def("xar_handles", &xar_handles);
  m.def("xar_open", &xar_open);
  m.def("xar_allreduce", &xar_allreduce);
  m.def("xar_error", &xar_error, py::arg("id"), py::arg("reset") = false);
  m.def("xar_cap", &xar_cap);
  m.def("xar_set_timeout_ms", &xar_set_timeout_ms);
  m.def("xar_destroy", &xar_destroy);
}
