// Bindings: MoE routing (top-k gating, expert scatter/gather), grouped expert GEMM, ragged-batch row gathers
// (inference v2 embed / logits gather, random-LTD token gather/scatter). Kernels: csrc/moe/moe_kernels.hip.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <optional>

extern "C" {
int ds_topk_gating(const void*, float*, int*, int*, int*, int, int, int, int, int, hipStream_t);
int ds_moe_scatter(const void*, const int*, const int*, const int*, void*, int*, int64_t*, int, int, int, int,
                   hipStream_t);
int ds_moe_gather(const void*, const float*, const int*, void*, int, int, int, hipStream_t);
int ds_grouped_gemm_ok(int, int);
int ds_grouped_gemm(const void*, const void*, void*, const int*, int, int, int, int, hipStream_t);
int ds_embed_gather(const void*, const int64_t*, const void*, const int64_t*, void*, int64_t, int, hipStream_t);
int ds_rows_gather(const void*, const int64_t*, void*, int64_t, int, hipStream_t);
int ds_rows_scatter(const void*, const int64_t*, void*, int64_t, int, hipStream_t);
int ds_token_sort(int*, int, int, int, hipStream_t);
}

using torch::Tensor;

namespace {
hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }
void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", hipGetErrorString((hipError_t)rc)); }
void need(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), n, " must be a contiguous device tensor");
}
void need_bf16(const Tensor& t, const char* n) {
  need(t, n);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, n, " must be bf16");
}
int dcode(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  if (t.scalar_type() == at::kHalf) return 2;
  TORCH_CHECK(false, "unsupported dtype");
  return -1;
}

// logits [T, E] -> (scores fp32 [T, k], experts int32 [T, k], slots int32 [T, k], counts int32 [E])
std::vector<Tensor> topk_gating(Tensor logits, int64_t k, bool renormalize) {
  need(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [T, E]");
  const int T = (int)logits.size(0), E = (int)logits.size(1);
  TORCH_CHECK(E >= 1 && E <= 256 && k >= 1 && k <= 8 && k <= E, "top-k gating supports E <= 256, k <= 8");
  auto io = logits.options().dtype(at::kInt);
  auto scores = torch::empty({T, k}, logits.options().dtype(at::kFloat));
  auto experts = torch::empty({T, k}, io);
  auto slots = torch::empty({T, k}, io);
  auto counts = torch::zeros({E}, io);
  check(ds_topk_gating(logits.data_ptr(), scores.data_ptr<float>(), experts.data_ptr<int>(), slots.data_ptr<int>(),
                       counts.data_ptr<int>(), T, E, (int)k, renormalize ? 1 : 0, dcode(logits), stream()),
        "topk_gating");
  return {scores, experts, slots, counts};
}

// x [T, H] -> (expert-sorted rows xs [T*k, H], row of each (t, j) [T, k], inclusive expert cumsum int64 [E])
std::vector<Tensor> moe_scatter(Tensor x, Tensor experts, Tensor slots, Tensor counts) {
  need_bf16(x, "x"); need(experts, "experts"); need(slots, "slots"); need(counts, "counts");
  const int T = (int)x.size(0), H = (int)x.size(1), K = (int)experts.size(1), E = (int)counts.numel();
  TORCH_CHECK(experts.size(0) == T && slots.sizes() == experts.sizes(), "routing shape mismatch");
  TORCH_CHECK(H % 8 == 0 && E <= 256, "moe_scatter: H % 8 == 0, E <= 256");
  auto xs = torch::empty({(int64_t)T * K, H}, x.options());
  auto rows = torch::empty({T, K}, experts.options());
  auto cumsum = torch::empty({E}, experts.options().dtype(at::kLong));
  if (T == 0) cumsum.zero_();
  check(ds_moe_scatter(x.data_ptr(), experts.data_ptr<int>(), slots.data_ptr<int>(), counts.data_ptr<int>(),
                       xs.data_ptr(), rows.data_ptr<int>(), cumsum.data_ptr<int64_t>(), T, H, E, K, stream()),
        "moe_scatter");
  return {xs, rows, cumsum};
}

// y [T*k, H] expert outputs, scores [T, k], rows [T, k] -> out [T, H] = sum_j scores[t, j] * y[rows[t, j]]
Tensor moe_gather(Tensor y, Tensor scores, Tensor rows) {
  need_bf16(y, "y"); need(scores, "scores"); need(rows, "rows");
  const int T = (int)rows.size(0), K = (int)rows.size(1), H = (int)y.size(1);
  TORCH_CHECK(y.size(0) == (int64_t)T * K && scores.sizes() == rows.sizes(), "moe_gather shape mismatch");
  auto out = torch::empty({T, H}, y.options());
  check(ds_moe_gather(y.data_ptr(), scores.data_ptr<float>(), rows.data_ptr<int>(), out.data_ptr(), T, H, K, stream()),
        "moe_gather");
  return out;
}

bool grouped_gemm_ok(int64_t n, int64_t k) { return ds_grouped_gemm_ok((int)n, (int)k) != 0; }

// X [R, K] expert-sorted rows, W [E, N, K], counts int32 [E] (sum = R) -> Y [R, N], Y[rows of e] = X . W_e^T
Tensor grouped_gemm(Tensor X, Tensor W, Tensor counts) {
  need_bf16(X, "X"); need_bf16(W, "W"); need(counts, "counts");
  TORCH_CHECK(W.dim() == 3 && X.dim() == 2 && X.size(1) == W.size(2), "grouped_gemm shapes");
  const int E = (int)W.size(0), N = (int)W.size(1), K = (int)W.size(2), R = (int)X.size(0);
  TORCH_CHECK(counts.numel() == E && counts.scalar_type() == at::kInt, "counts must be int32 [E]");
  TORCH_CHECK(ds_grouped_gemm_ok(N, K), "grouped_gemm needs N % 128 == 0 and K % 128 == 0");
  auto Y = torch::empty({R, N}, X.options());
  check(ds_grouped_gemm(X.data_ptr(), W.data_ptr(), Y.data_ptr(), counts.data_ptr<int>(), R, E, N, K, stream()),
        "grouped_gemm");
  return Y;
}

// out[i] = table[ids[i]] (+ pos_table[pos[i]])
Tensor embed_gather(Tensor table, Tensor ids, std::optional<Tensor> pos_table, std::optional<Tensor> pos) {
  need_bf16(table, "table"); need(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids must be int64");
  const int64_t n = ids.numel();
  const int H = (int)table.size(1);
  const bool has_pos = pos_table.has_value() && pos.has_value();
  if (has_pos) {
    need_bf16(*pos_table, "pos_table"); need(*pos, "pos");
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->numel() == n && pos_table->size(1) == H, "pos shapes");
  }
  auto out = torch::empty({n, H}, table.options());
  check(ds_embed_gather(table.data_ptr(), ids.data_ptr<int64_t>(), has_pos ? pos_table->data_ptr() : nullptr,
                        has_pos ? pos->data_ptr<int64_t>() : nullptr, out.data_ptr(), n, H, stream()),
        "embed_gather");
  return out;
}

// out[i] = x[idx[i]] rows
// In-place per-row sort of distinct int32 token positions in [0, S) (random-LTD token_sort_).
Tensor token_sort_(Tensor idx, int64_t S) {
  need(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.dim() >= 1, "token_sort_: int32 indices");
  const int64_t k = idx.size(-1);
  TORCH_CHECK(k <= S && S <= (1 << 20), "token_sort_: need k <= S <= 2^20");
  check(ds_token_sort(idx.data_ptr<int>(), (int)(idx.numel() / k), (int)k, (int)S, stream()), "token_sort_");
  return idx;
}

Tensor rows_gather(Tensor x, Tensor idx) {
  need_bf16(x, "x"); need(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong, "idx must be int64");
  const int H = (int)x.size(-1);
  auto out = torch::empty({idx.numel(), H}, x.options());
  check(ds_rows_gather(x.data_ptr(), idx.data_ptr<int64_t>(), out.data_ptr(), idx.numel(), H, stream()),
        "rows_gather");
  return out;
}

// full[idx[i]] = part[i] rows (in place on full)
void rows_scatter(Tensor part, Tensor idx, Tensor full) {
  need_bf16(part, "part"); need(idx, "idx"); need_bf16(full, "full");
  TORCH_CHECK(idx.scalar_type() == at::kLong && part.size(-1) == full.size(-1), "rows_scatter shapes");
  check(ds_rows_scatter(part.data_ptr(), idx.data_ptr<int64_t>(), full.data_ptr(), idx.numel(), (int)part.size(-1),
                        stream()),
        "rows_scatter");
}
}  // namespace

void register_moe_ops(pybind11::module& m) {
  m.def("topk_gating", &topk_gating);
  m.def("moe_scatter", &moe_scatter);
  m.def("moe_gather", &moe_gather);
  m.def("grouped_gemm_ok", &grouped_gemm_ok);
  m.def("grouped_gemm", &grouped_gemm);
  m.def("embed_gather", &embed_gather);
  m.def("token_sort_", &token_sort_);
  m.def("rows_gather", &rows_gather);
  m.def("rows_scatter", &rows_scatter);
}
