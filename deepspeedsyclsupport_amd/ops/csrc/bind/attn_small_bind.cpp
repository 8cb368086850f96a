// Bindings: small-head-dim flash attention with additive biases and attention dropout (attn/flash_small.hip), used
// by DS4Sci_EvoformerAttention and the BERT training layer (DeepSpeedTransformerLayer).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <optional>
#include <vector>

extern "C" {
int ds_flash_small_fwd(const void*, const void*, const void*, void*, float*, const void*, const void*,
                       const int64_t*, int64_t, int, int, int, int, int, int, float, float, uint64_t, int, int,
                       hipStream_t);
int ds_flash_small_bwd(const void*, const void*, const void*, const void*, const void*, const float*, const void*,
                       const void*, void*, void*, void*, float*, float*, float*, const int64_t*, int64_t, int, int, int, int,
                       int, float, float, uint64_t, int, int, hipStream_t);
}

using torch::Tensor;
using OptT = std::optional<Tensor>;

namespace {

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", hipGetErrorString((hipError_t)rc)); }

int dcode(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 1;
  if (t.scalar_type() == at::kHalf) return 2;
  TORCH_CHECK(false, "flash_small: bf16 / fp16 only, got ", t.scalar_type());
  return -1;
}

bool aligned(const void* p, int bytes) { return reinterpret_cast<uintptr_t>(p) % bytes == 0; }

// [Z, S, H, D] operand: device, dtype, unit last stride, 16-B rows (the kernel reads 16-B chunks). any_s: the
// sequence length may differ from q's (keys / values of a cross-attention context).
void operand(const Tensor& t, const Tensor& q, const char* name, bool any_s = false) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, "flash_small: ", name, " must be a 4-D device tensor [Z,S,H,D]");
  TORCH_CHECK(t.size(0) == q.size(0) && t.size(2) == q.size(2) && t.size(3) == q.size(3) &&
                  (any_s || t.size(1) == q.size(1)),
              "flash_small: ", name, " shape ", t.sizes(), " does not match q ", q.sizes());
  TORCH_CHECK(t.scalar_type() == q.scalar_type(), "flash_small: ", name, " dtype mismatch");
  TORCH_CHECK(t.stride(3) == 1, "flash_small: ", name, " needs a unit last stride");
  for (int d = 0; d < 3; ++d) TORCH_CHECK(t.stride(d) % 8 == 0, "flash_small: ", name, " strides must be multiples of 8");
  TORCH_CHECK(aligned(t.data_ptr(), 16), "flash_small: ", name, " must be 16-B aligned");
}

struct Bias {
  const void* b1 = nullptr;
  const void* b2 = nullptr;
  int64_t b1_zs = 0;
  int vec = 1;
};

Bias biases(const OptT& b1, const OptT& b2, const Tensor& q, int64_t Sk, int64_t b2_div) {
  const int64_t Z = q.size(0), S = q.size(1), H = q.size(2);
  Bias r;
  r.vec = Sk % 8 == 0;  // bias rows are read in whole 16-B chunks of 8 keys
  if (b1.has_value() && b1->defined()) {
    TORCH_CHECK(b1->is_cuda() && b1->dim() == 2 && b1->size(0) == Z && b1->size(1) == Sk && b1->stride(1) == 1,
                "flash_small: bias1 must be [Z, Sk] with a unit last stride");
    TORCH_CHECK(b1->scalar_type() == q.scalar_type(), "flash_small: bias1 dtype mismatch");
    r.b1 = b1->data_ptr();
    r.b1_zs = b1->stride(0);
    r.vec &= aligned(r.b1, 16) && r.b1_zs % 8 == 0;
  }
  if (b2.has_value() && b2->defined()) {
    TORCH_CHECK(b2_div >= 1 && Z % b2_div == 0, "flash_small: b2_div must divide Z");
    TORCH_CHECK(b2->is_cuda() && b2->is_contiguous() && b2->dim() == 4 && b2->size(0) == Z / b2_div &&
                    b2->size(1) == H && b2->size(2) == S && b2->size(3) == Sk,
                "flash_small: bias2 must be contiguous [Z / b2_div, H, S, Sk]");
    TORCH_CHECK(b2->scalar_type() == q.scalar_type(), "flash_small: bias2 dtype mismatch");
    r.b2 = b2->data_ptr();
    r.vec &= aligned(r.b2, 16);
  }
  return r;
}

void push(std::vector<int64_t>& st, const Tensor& t) {
  st.push_back(t.stride(0));
  st.push_back(t.stride(1));
  st.push_back(t.stride(2));
}

// q [Z, S, H, D], k/v [Z, Sk, H, D] (D in {32, 64}); returns o [Z, S, H, D] (contiguous) and lse [Z, H, S] fp32
std::vector<Tensor> flash_small_fwd(Tensor q, Tensor k, Tensor v, OptT b1, OptT b2, int64_t b2_div, double scale,
                                    double pdrop, int64_t seed) {
  operand(q, q, "q");
  operand(k, q, "k", true);
  operand(v, k, "v");
  const int64_t Z = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3), Sk = k.size(1);
  TORCH_CHECK(D == 32 || D == 64, "flash_small: head dim 32 or 64 only, got ", D);
  TORCH_CHECK(pdrop >= 0.0 && pdrop < 1.0, "flash_small: dropout must be in [0, 1)");
  const Bias bs = biases(b1, b2, q, Sk, b2_div);
  auto o = torch::empty({Z, S, H, D}, q.options());
  auto lse = torch::empty({Z, H, S}, q.options().dtype(at::kFloat));
  std::vector<int64_t> st;
  push(st, q); push(st, k); push(st, v); push(st, o);
  check(ds_flash_small_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), bs.b1,
                           bs.b2, st.data(), bs.b1_zs, (int)Z, (int)H, (int)S, (int)Sk, (int)D, (int)b2_div, (float)scale,
                           (float)pdrop, (uint64_t)seed, bs.vec, dcode(q), at::hip::getCurrentHIPStream().stream()),
        "flash_small_fwd");
  return {o, lse};
}

// Returns dq (contiguous, q dtype), dk, dv (q dtype), db1 [Z, S] fp32 / db2 [Z / b2_div, H, S, S] fp32 (empty when
// not requested).
std::vector<Tensor> flash_small_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, OptT b1,
                                    OptT b2, int64_t b2_div, double scale, double pdrop, int64_t seed, bool want_db1,
                                    bool want_db2) {
  operand(q, q, "q");
  operand(k, q, "k");
  operand(v, q, "v");
  operand(o, q, "o");
  operand(dout, q, "dout");
  const int64_t Z = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3);
  TORCH_CHECK(D == 32 || D == 64, "flash_small: head dim 32 or 64 only, got ", D);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == Z * H * S,
              "flash_small: lse must be the forward's [Z, H, S] fp32");
  const Bias bs = biases(b1, b2, q, S, b2_div);
  TORCH_CHECK(!want_db1 || bs.b1, "flash_small: dB1 requested without bias1");
  TORCH_CHECK(!want_db2 || bs.b2, "flash_small: dB2 requested without bias2");
  auto dq = torch::empty({Z, S, H, D}, q.options());
  auto f32 = q.options().dtype(at::kFloat);
  auto dk = torch::empty({Z, S, H, D}, q.options());
  auto dv = torch::empty({Z, S, H, D}, q.options());
  auto delta = torch::empty({Z, H, S}, f32);
  Tensor db1 = want_db1 ? torch::zeros({Z, S}, f32) : torch::empty({0}, f32);
  Tensor db2 = want_db2 ? torch::zeros({Z / b2_div, H, S, S}, f32) : torch::empty({0}, f32);
  std::vector<int64_t> st;
  push(st, q); push(st, k); push(st, v); push(st, o); push(st, dout); push(st, dq);
  check(ds_flash_small_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                           lse.data_ptr<float>(), bs.b1, bs.b2, dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                           delta.data_ptr<float>(), want_db1 ? db1.data_ptr<float>() : nullptr,
                           want_db2 ? db2.data_ptr<float>() : nullptr, st.data(), bs.b1_zs, (int)Z, (int)H, (int)S,
                           (int)D, (int)b2_div, (float)scale, (float)pdrop, (uint64_t)seed, bs.vec, dcode(q),
                           at::hip::getCurrentHIPStream().stream()),
        "flash_small_bwd");
  return {dq, dk, dv, db1, db2};
}

}  // namespace

void register_attn_small_ops(pybind11::module& m) {
  m.def("flash_small_fwd", &flash_small_fwd, pybind11::arg("q"), pybind11::arg("k"), pybind11::arg("v"),
        pybind11::arg("b1") = pybind11::none(), pybind11::arg("b2") = pybind11::none(), pybind11::arg("b2_div") = 1,
        pybind11::arg("scale"), pybind11::arg("pdrop") = 0.0, pybind11::arg("seed") = 0);
  m.def("flash_small_bwd", &flash_small_bwd, pybind11::arg("dout"), pybind11::arg("q"), pybind11::arg("k"),
        pybind11::arg("v"), pybind11::arg("o"), pybind11::arg("lse"), pybind11::arg("b1") = pybind11::none(),
        pybind11::arg("b2") = pybind11::none(), pybind11::arg("b2_div") = 1, pybind11::arg("scale"),
        pybind11::arg("pdrop") = 0.0, pybind11::arg("seed") = 0, pybind11::arg("want_db1") = false,
        pybind11::arg("want_db2") = false);
}
