// Bindings: inference decode attention over the paged KV cache, KV append, group quantisation (ZeRO++ / MoQ /
// weight-only inference).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <optional>

extern "C" {
int ds_paged_decode_splits(int, int, int);
int ds_paged_decode(const void*, const void*, const void*, const int*, const int*, const float*, float*, float*, void*,
                    int, int, int, int, int, int, int, int, float, int, hipStream_t);
int ds_kv_append(const void*, const void*, void*, void*, const int*, const int*, int, int, int, int, int, int,
                 hipStream_t);
int ds_quantize(const void*, int8_t*, float*, float*, int64_t, int, int, int, int, unsigned, int, hipStream_t);
int ds_dequantize(const int8_t*, const float*, const float*, void*, int64_t, int, int, int, int, hipStream_t);
int ds_dequant_reduce(const int8_t*, const float*, void*, int64_t, int, int, float, int, hipStream_t);
}

using torch::Tensor;
using OptT = std::optional<Tensor>;

namespace {
hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }
void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", hipGetErrorString((hipError_t)rc)); }
int dcode(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  if (t.scalar_type() == at::kHalf) return 2;
  TORCH_CHECK(false, "unsupported dtype");
  return -1;
}
void need(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), n, " must be a contiguous device tensor");
}

// q [B, Hq, D] bf16; caches [NB, Hk, BS, D] bf16; block_table [B, max_blocks] int32; seq_lens [B] int32
Tensor paged_decode(Tensor q, Tensor kc, Tensor vc, Tensor block_table, Tensor seq_lens, int64_t max_len, double scale,
                    OptT alibi, int64_t window) {
  need(q, "q"); need(kc, "k_cache"); need(vc, "v_cache"); need(block_table, "block_table"); need(seq_lens, "seq_lens");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && kc.scalar_type() == at::kBFloat16, "bf16 q/cache");
  TORCH_CHECK(block_table.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt, "int32 tables");
  const int B = (int)q.size(0), Hq = (int)q.size(1), D = (int)q.size(2);
  const int Hk = (int)kc.size(1), BS = (int)kc.size(2);
  TORCH_CHECK(kc.size(3) == D, "head dim mismatch");
  const int max_blocks = (int)block_table.size(1);
  TORCH_CHECK((int64_t)max_blocks * BS >= max_len, "block table too small for max_len");
  const int splits = ds_paged_decode_splits(B, Hk, (int)max_len);
  auto out = torch::empty_like(q);
  auto fo = q.options().dtype(at::kFloat);
  Tensor pacc, pml;
  if (splits > 1) {
    pacc = torch::empty({B, Hq, splits, D}, fo);
    pml = torch::empty({B, Hq, splits, 2}, fo);
  }
  const float* al = nullptr;
  if (alibi.has_value()) { need(*alibi, "alibi"); al = alibi->data_ptr<float>(); }
  check(ds_paged_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_table.data_ptr<int>(),
                        seq_lens.data_ptr<int>(), al, splits > 1 ? pacc.data_ptr<float>() : nullptr,
                        splits > 1 ? pml.data_ptr<float>() : nullptr, out.data_ptr(), B, Hq, Hk, D, BS, max_blocks,
                        (int)max_len, splits, (float)scale, (int)window, stream()),
        "paged_decode");
  return out;
}

// k, v [B, n_new, Hk, D] -> caches at positions start_pos[b] + j
void kv_append(Tensor k, Tensor v, Tensor kc, Tensor vc, Tensor block_table, Tensor start_pos) {
  need(k, "k"); need(v, "v"); need(kc, "kc"); need(vc, "vc");
  check(ds_kv_append(k.data_ptr(), v.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_table.data_ptr<int>(),
                     start_pos.data_ptr<int>(), (int)k.size(0), (int)k.size(1), (int)k.size(2), (int)k.size(3),
                     (int)kc.size(2), (int)block_table.size(1), stream()),
        "kv_append");
}

// returns (q int8 [n or n/2], scales fp32 [n/gs], zeros fp32 [n/gs] or empty)
std::vector<Tensor> quantize(Tensor x, int64_t gs, int64_t bits, bool asym, bool stochastic, int64_t seed) {
  need(x, "x");
  const int64_t n = x.numel();
  auto q = torch::empty({bits == 8 ? n : n / 2}, x.options().dtype(at::kChar));
  auto fo = x.options().dtype(at::kFloat);
  auto scales = torch::empty({n / gs}, fo);
  auto zeros = asym ? torch::empty({n / gs}, fo) : torch::empty({0}, fo);
  check(ds_quantize(x.data_ptr(), q.data_ptr<int8_t>(), scales.data_ptr<float>(),
                    asym ? zeros.data_ptr<float>() : nullptr, n, (int)gs, (int)bits, asym ? 1 : 0, stochastic ? 1 : 0,
                    (unsigned)seed, dcode(x), stream()),
        "quantize");
  return {q, scales, zeros};
}

Tensor dequantize(Tensor q, Tensor scales, OptT zeros, int64_t n, int64_t gs, int64_t bits, at::ScalarType dtype) {
  need(q, "q"); need(scales, "scales");
  auto out = torch::empty({n}, q.options().dtype(dtype));
  const bool asym = zeros.has_value() && zeros->numel() > 0;
  check(ds_dequantize(q.data_ptr<int8_t>(), scales.data_ptr<float>(), asym ? zeros->data_ptr<float>() : nullptr,
                      out.data_ptr(), n, (int)gs, (int)bits, asym ? 1 : 0, dcode(out), stream()),
        "dequantize");
  return out;
}

// q [nsrc * n] int8 (sym), scales [nsrc * n/gs] -> sum over sources, scaled
Tensor dequant_reduce(Tensor q, Tensor scales, int64_t nsrc, int64_t gs, double out_scale, at::ScalarType dtype) {
  need(q, "q"); need(scales, "scales");
  const int64_t n = q.numel() / nsrc;
  auto out = torch::empty({n}, q.options().dtype(dtype));
  check(ds_dequant_reduce(q.data_ptr<int8_t>(), scales.data_ptr<float>(), out.data_ptr(), n, (int)gs, (int)nsrc,
                          (float)out_scale, dcode(out), stream()),
        "dequant_reduce");
  return out;
}
}  // namespace

void register_inference_ops(pybind11::module& m) {
  m.def("paged_decode", &paged_decode);
  m.def("kv_append", &kv_append);
  m.def("quantize", &quantize);
  m.def("dequantize", &dequantize);
  m.def("dequant_reduce", &dequant_reduce);
}
