// Exact-size pinned host buffers (reference `inference/v2/ragged/csrc/fast_host_buffer.cu:9-17`
// `allocate_fast_host_buffer`, and the pinned swap buffers of `csrc/aio`).
//
// torch's pinned allocator rounds every request up to a power of two (a 52 GB Twin-Flow master partition would
// take 64 GB), which caps how much of the host a ZeRO-Offload++ / ZeRO-Infinity run can use. These buffers are
// allocated with hipHostMalloc at their exact size and freed by the tensor's deleter. `coherent=false` requests
// write-combined memory (fast host->device streaming of ragged-batch metadata, slow host reads).
#include <torch/extension.h>
#include <hip/hip_runtime_api.h>

namespace {

torch::Tensor alloc_pinned(int64_t numel, py::object dtype_obj, bool coherent) {
  TORCH_CHECK(numel >= 0, "alloc_pinned: negative size");
  const at::ScalarType dt = torch::python::detail::py_object_to_dtype(dtype_obj);
  const size_t bytes = std::max<size_t>(1, (size_t)numel * c10::elementSize(dt));
  void* p = nullptr;
  unsigned flags = coherent ? hipHostMallocDefault : (hipHostMallocWriteCombined | hipHostMallocMapped);
  hipError_t rc = hipHostMalloc(&p, bytes, flags);
  TORCH_CHECK(rc == hipSuccess, "hipHostMalloc(", bytes, " B) failed: ", hipGetErrorString(rc));
  auto opts = torch::TensorOptions().dtype(dt).device(torch::kCPU);
  return torch::from_blob(p, {numel}, [](void* q) { (void)hipHostFree(q); }, opts);
}

}  // namespace

void register_host_mem_ops(pybind11::module& m) {
  m.def("alloc_pinned", &alloc_pinned, py::arg("numel"), py::arg("dtype"), py::arg("coherent") = true);
}
