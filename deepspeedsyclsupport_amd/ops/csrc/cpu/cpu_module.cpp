// Module definition for the host extension `ds_cpu_ops` (optimizers, async I/O, shm collectives).
#include <torch/extension.h>

void register_cpu_optim(pybind11::module& m);
void register_aio(pybind11::module& m);
void register_shm_comm(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "deepspeedsyclsupport_amd host ops";
  register_cpu_optim(m);
  register_aio(m);
  register_shm_comm(m);
}
