// Bindings: inference decode attention over the paged KV cache, KV append, group quantisation (ZeRO++ / MoQ /
// weight-only inference).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime_api.h>

#include <map>
#include <optional>
#include <utility>

extern "C" {
int ds_paged_decode_splits(int, int, int);
int ds_skinny_gemm(const void*, const void*, const void*, const void*, const void*, const void*, void*, void*, int, int,
                   int, int, int, int, float, hipStream_t);
int ds_skinny_fits_lds(int, int);
int ds_skinny_mfma_ok(int, int, int);
int ds_skinny_mfma(const void*, const void*, const void*, const void*, const void*, const void*, void*, void*, int, int,
                   int, int, int, int, float, hipStream_t);
int ds_rms_fwd(const void*, const void*, const void*, void*, void*, float*, int64_t, int, float, int, hipStream_t);
int ds_qkv_rope_append(const void*, const float*, const float*, const int*, void*, void*, void*, void*, void*,
                       const int*, const int*, const int*, int, int, int, int, int, int, int, int, int, float*,
                       const void*, int, hipStream_t);
int ds_paged_prefill(const void*, const void*, const void*, void*, const int*, const int*, const int*, const int*, int,
                     const float*, int, int, int, int, int, int, float, hipStream_t);
int ds_paged_decode(const void*, const void*, const void*, const int*, const int*, const float*, float*, float*, void*,
                    int, int, int, int, int, int, int, int, float, int, hipStream_t);
int ds_kv_append(const void*, const void*, void*, void*, const int*, const int*, int, int, int, int, int, int,
                 hipStream_t);
int ds_skinny_i8_ok(int, int, int);
int ds_skinny_i8_mfma_ok(int, int, int);
int ds_skinny_i8_mfma(const void*, const int8_t*, const float*, const void*, void*, float*, int, int, int, int,
                      hipStream_t);
int64_t ds_skinny_i8_mfma_ws_floats(int);
void ds_skinny_i8_tune(int, int, int);
int ds_skinny_b16_mfma_ok(int, int);
int ds_skinny_b16_mfma(const void*, const void*, const void*, void*, float*, int, int, int, hipStream_t);
int ds_unshuffle_sh16(const void*, void*, int, int, hipStream_t);
void ds_skinny_b16_tune(int, int);
int ds_dequant_sh(const int8_t*, const float*, void*, int, int, int, hipStream_t);
int ds_skinny_i8(const void*, const int8_t*, const float*, const void*, void*, int, int, int, int, hipStream_t);
int ds_skinny_i4_mfma_ok(int, int, int);
int ds_skinny_i4_mfma(const void*, const int8_t*, const float*, const void*, void*, float*, int, int, int, int,
                      hipStream_t);
int64_t ds_skinny_i4_mfma_ws_floats(int);
void ds_skinny_i4_tune(int, int, int);
int ds_dequant_sh4(const int8_t*, const float*, void*, int, int, int, hipStream_t);
int ds_skinny_finalize_rms(float*, const void*, const void*, const void*, void*, void*, int, int, int, float, hipStream_t);
int ds_skinny_finalize_gated(float*, const void*, void*, int, int, int, int, hipStream_t);
int ds_skinny_finalize_plain(float*, const void*, void*, int, int, int, hipStream_t);
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

// Skinny-GEMM path policy: 0 = auto, 1 = VALU kernel only, 2 = MFMA kernel only (A/B testing; DS_SKINNY_PATH).
int skinny_path = getenv("DS_SKINNY_PATH") ? atoi(getenv("DS_SKINNY_PATH")) : 0;
void skinny_set_path(int64_t p) { skinny_path = (int)p; }
void skinny_force_valu(bool v) { skinny_path = v ? 1 : 0; }

// auto policy (measured on MI355X, tools/bench_skinny.py): M <= 2 -> VALU kernel (its fused RMSNorm staging and
// gated epilogue are cheapest there); M > 2 -> RMSNorm once, then the MFMA kernel (per-workgroup normalisation
// cost grows with M, and VALU FMA throughput runs out)
static bool use_mfma(int M, int K, int in_mode) {
  if (skinny_path == 1) return false;
  if (skinny_path == 2) return ds_skinny_mfma_ok(M, K, in_mode);
  if (M <= 2 && K % 8 == 0 && (in_mode == 0 || ds_skinny_fits_lds(M, K))) return false;
  return in_mode == 0 && ds_skinny_mfma_ok(M, K, 0);
}

// y [M, N] = X . W^T for M <= 16 rows (decode). in_mode 0: X = x; 1: X = RMSNorm(x (+ r)) * nw (res_out <- x + r).
// gated: W is a fused [gate; up] weight (N = 2I) and y = act(X.gate^T) * (X.up^T) of width I.
Tensor skinny_gemm(Tensor x, Tensor w, OptT bias, OptT add, int64_t in_mode, bool gated, int64_t act, OptT r, OptT nw,
                   double eps, OptT res_out) {
  need(x, "x"); need(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "skinny_gemm: bf16 only");
  const int N = (int)w.size(0), K = (int)w.size(1);
  TORCH_CHECK(x.size(-1) == K, "skinny_gemm: inner dim mismatch");
  const int M = (int)(x.numel() / K);
  TORCH_CHECK(M >= 1 && M <= 16, "skinny_gemm: M must be in [1, 16]");
  TORCH_CHECK(!gated || N % 2 == 0, "gated skinny_gemm needs an even N");
  auto sizes = x.sizes().vec();
  sizes.back() = gated ? N / 2 : N;
  auto y = torch::empty(sizes, x.options());
  auto ptr = [](const OptT& t) -> const void* { return t.has_value() ? t->data_ptr() : nullptr; };
  for (auto* t : {&bias, &add, &r, &nw, &res_out})
    if (t->has_value()) need(**t, "skinny_gemm operand");
  const void* xin = x.data_ptr();
  const void* rin = ptr(r);
  Tensor normed;
  bool mfma = use_mfma(M, K, (int)in_mode);
  const bool valu_fused = skinny_path != 2 && M <= 8 && ds_skinny_fits_lds(M, K) && (skinny_path == 1 || M <= 2);
  if (in_mode == 1 && !mfma && !valu_fused) {
    // activations too large to stage in LDS: normalise with the RMSNorm kernel, then a plain skinny GEMM
    normed = torch::empty_like(x);
    auto rstd = torch::empty({M}, x.options().dtype(at::kFloat));
    // the fused-residual RMSNorm kernel always writes x + r: give it a scratch buffer when the caller wants none
    Tensor res_scratch;
    void* rdst = nullptr;
    if (rin) {
      if (res_out.has_value()) {
        rdst = res_out->data_ptr();
      } else {
        res_scratch = torch::empty_like(x);
        rdst = res_scratch.data_ptr();
      }
    }
    check(ds_rms_fwd(x.data_ptr(), rin, nw->data_ptr(), normed.data_ptr(), rdst, rstd.data_ptr<float>(), M, K,
                     (float)eps, 1, stream()), "rms_fwd");
    if (res_out.has_value() && !r.has_value()) res_out->copy_(x);
    xin = normed.data_ptr();
    rin = nullptr;
    in_mode = 0;
    mfma = use_mfma(M, K, 0);
  }
  TORCH_CHECK(mfma || M <= 8, "skinny_gemm: M > 8 needs K % 256 == 0 (MFMA path)");
  void* ro = in_mode == 1 && res_out.has_value() ? res_out->data_ptr() : nullptr;
  auto fn = mfma ? ds_skinny_mfma : ds_skinny_gemm;
  check(fn(w.data_ptr(), xin, rin, ptr(nw), ptr(bias), ptr(add), y.data_ptr(), ro, M, N, K, (int)in_mode,
           gated ? 1 : 0, (int)act, (float)eps, stream()),
        "skinny_gemm");
  return y;
}

// qkv [T, (Hq+2Hk)*D] -> q [T, Hq, D] roped; k (roped) / v scattered into the paged cache; optional k/v copies.
// `qkv` is either the bf16 projection or — with `acc_rows` > 0 — the fp32 workspace view [16, NP] a weight-only GEMV left
// un-finalized (skinny_q_raw): then the kernel adds `acc_bias`, and re-zeroes the workspace rows it consumed.
std::vector<Tensor> qkv_rope_append(Tensor qkv, OptT cos, OptT sin, Tensor pos, Tensor kc, Tensor vc,
                                    Tensor block_table, Tensor start_pos, int64_t n_new, int64_t Hq, int64_t Hk,
                                    int64_t rot, bool interleaved, bool want_kv, OptT seq_ids, int64_t acc_rows,
                                    OptT acc_bias) {
  need(qkv, "qkv"); need(pos, "pos"); need(kc, "kc"); need(vc, "vc"); need(block_table, "block_table");
  need(start_pos, "start_pos");
  const bool from_acc = acc_rows > 0;
  TORCH_CHECK(kc.scalar_type() == at::kBFloat16 && (from_acc ? qkv.scalar_type() == at::kFloat
                                                             : qkv.scalar_type() == at::kBFloat16),
              "bf16 qkv (or fp32 GEMV workspace) / bf16 cache");
  const int D = (int)kc.size(3);
  const int64_t N3 = (Hq + 2 * Hk) * D;
  const int64_t T = from_acc ? acc_rows : qkv.numel() / N3;
  const bool ragged = seq_ids.has_value() && seq_ids->defined();
  if (from_acc)
    TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == 16 && qkv.size(1) >= N3 && T <= 16, "workspace view [16, NP >= N]");
  TORCH_CHECK((from_acc || T * N3 == qkv.numel()) && (ragged || T % n_new == 0), "qkv shape");
  const void* abp = nullptr;
  if (from_acc && acc_bias.has_value() && acc_bias->defined()) {
    need(*acc_bias, "acc_bias");
    TORCH_CHECK(acc_bias->scalar_type() == at::kBFloat16 && acc_bias->numel() == N3, "acc_bias bf16 [N]");
    abp = acc_bias->data_ptr();
  }
  if (ragged) {
    need(*seq_ids, "seq_ids");
    TORCH_CHECK(seq_ids->scalar_type() == at::kInt && seq_ids->numel() == T && pos.numel() == T, "seq_ids / pos [T]");
  }
  TORCH_CHECK(kc.size(1) == Hk, "cache kv heads");
  TORCH_CHECK(rot == 0 || (cos.has_value() && sin.has_value()), "rope tables required");
  auto bopt = kc.options();
  auto q = torch::empty({T, Hq, D}, bopt);
  Tensor k, v;
  if (want_kv) {
    k = torch::empty({T, Hk, D}, bopt);
    v = torch::empty({T, Hk, D}, bopt);
  }
  check(ds_qkv_rope_append(from_acc ? nullptr : qkv.data_ptr(), rot ? cos->data_ptr<float>() : nullptr,
                           rot ? sin->data_ptr<float>() : nullptr, pos.data_ptr<int>(), q.data_ptr(),
                           want_kv ? k.data_ptr() : nullptr, want_kv ? v.data_ptr() : nullptr, kc.data_ptr(),
                           vc.data_ptr(), block_table.data_ptr<int>(), start_pos.data_ptr<int>(),
                           ragged ? seq_ids->data_ptr<int>() : nullptr, (int)T, (int)n_new,
                           (int)Hq, (int)Hk, D, (int)rot, interleaved ? 1 : 0, (int)kc.size(2),
                           (int)block_table.size(1), from_acc ? qkv.data_ptr<float>() : nullptr, abp,
                           from_acc ? (int)qkv.size(1) : 0, stream()),
        "qkv_rope_append");
  if (want_kv) return {q, k, v};
  return {q};
}

// Self-cleaning split-K workspace of the MFMA path (zero between calls: the kernel re-zeroes what it used), one per
// (device, stream) so concurrent streams never share partial sums; grown (never shrunk) on demand.
struct I8Workspace {
  Tensor acc;
};
std::map<std::pair<int, hipStream_t>, I8Workspace>& i8_workspaces() {
  static std::map<std::pair<int, hipStream_t>, I8Workspace> m;
  return m;
}
I8Workspace& i8_workspace(const Tensor& like, int64_t N) {
  auto& ws = i8_workspaces()[{like.get_device(), stream()}];
  const int64_t nf = ds_skinny_i8_mfma_ws_floats((int)N);
  if (!ws.acc.defined() || ws.acc.numel() < nf) ws.acc = torch::zeros({nf}, like.options().dtype(at::kFloat));
  return ws;
}

bool skinny_i8_ok(int64_t M, int64_t K, int64_t gs) { return ds_skinny_i8_ok((int)M, (int)K, (int)gs) != 0; }
bool skinny_i8_sh_ok(int64_t M, int64_t K, int64_t gs) { return ds_skinny_i8_mfma_ok((int)M, (int)K, (int)gs) != 0; }

// VALU stream over a row-major weight: x [M, K] bf16 (M <= 8), q int8 [N * K] (symmetric), scales fp32
// [N * K / gs] -> y [M, N] bf16
Tensor skinny_i8(Tensor x, Tensor q, Tensor scales, OptT bias, int64_t N, int64_t gs) {
  need(x, "x"); need(q, "q"); need(scales, "scales");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "skinny_i8: x must be bf16 [M, K]");
  TORCH_CHECK(q.scalar_type() == at::kChar && scales.scalar_type() == at::kFloat, "skinny_i8: int8 q, fp32 scales");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(ds_skinny_i8_ok((int)M, (int)K, (int)gs) != 0, "skinny_i8: unsupported shape (M ", M, ", K ", K,
              ", gs ", gs, ")");
  TORCH_CHECK(q.numel() == N * K && scales.numel() == N * K / gs, "skinny_i8: q / scales size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_i8: 16-B aligned x / q");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    need(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "skinny_i8: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  auto y = torch::empty({M, N}, x.options());
  check(ds_skinny_i8(x.data_ptr(), q.data_ptr<int8_t>(), scales.data_ptr<float>(), bp, y.data_ptr(), (int)M, (int)N,
                     (int)K, (int)gs, stream()),
        "skinny_i8");
  return y;
}

// MFMA stream over the pre-shuffled layout (ops/int8_gemv.py: preshuffle): x [M, K] bf16 (M <= 16),
// qsh int8 [ceil(N/16), K/64, 64, 16], ssh fp32 [ceil(N/16), K/gs, 16] -> y [M, N] bf16
Tensor skinny_i8_sh(Tensor x, Tensor qsh, Tensor ssh, OptT bias, int64_t N, int64_t gs) {
  need(x, "x"); need(qsh, "qsh"); need(ssh, "ssh");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "skinny_i8_sh: x must be bf16 [M, K]");
  TORCH_CHECK(qsh.scalar_type() == at::kChar && ssh.scalar_type() == at::kFloat, "skinny_i8_sh: int8 q, fp32 scales");
  const int64_t M = x.size(0), K = x.size(1), NB = (N + 15) / 16;
  TORCH_CHECK(ds_skinny_i8_mfma_ok((int)M, (int)K, (int)gs) != 0, "skinny_i8_sh: unsupported shape (M ", M, ", K ", K,
              ", gs ", gs, ")");
  TORCH_CHECK(qsh.numel() == NB * 16 * K && ssh.numel() == NB * 16 * (K / gs), "skinny_i8_sh: qsh / ssh size");
  TORCH_CHECK(NB * K < ((int64_t)1 << 40) && N < ((int64_t)1 << 31) / 16, "skinny_i8_sh: matrix too large");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(qsh.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_i8_sh: 16-B aligned x / q");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    need(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "skinny_i8_sh: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  auto y = torch::empty({M, N}, x.options());
  auto& ws = i8_workspace(x, N);
  check(ds_skinny_i8_mfma(x.data_ptr(), qsh.data_ptr<int8_t>(), ssh.data_ptr<float>(), bp, y.data_ptr(),
                          ws.acc.data_ptr<float>(), (int)M, (int)N, (int)K, (int)gs, stream()),
        "skinny_i8_sh");
  return y;
}

// pre-shuffled int8 (ops/int8_gemv.py) -> row-major bf16 [N, K]
Tensor dequant_sh(Tensor qsh, Tensor ssh, int64_t N, int64_t gs) {
  need(qsh, "qsh"); need(ssh, "ssh");
  TORCH_CHECK(qsh.scalar_type() == at::kChar && ssh.scalar_type() == at::kFloat && qsh.dim() == 4, "dequant_sh: layout");
  const int64_t K = qsh.size(1) * 64;
  TORCH_CHECK(qsh.size(0) == (N + 15) / 16 && ssh.numel() == qsh.size(0) * 16 * (K / gs), "dequant_sh: sizes");
  auto w = torch::empty({N, K}, qsh.options().dtype(at::kBFloat16));
  check(ds_dequant_sh(qsh.data_ptr<int8_t>(), ssh.data_ptr<float>(), w.data_ptr(), (int)N, (int)K, (int)gs, stream()),
        "dequant_sh");
  return w;
}

bool skinny_i4_ok(int64_t M, int64_t K, int64_t gs) { return ds_skinny_i4_mfma_ok((int)M, (int)K, (int)gs) != 0; }

// int4 MFMA stream over the packed layout (ops/int4_gemv.py: pack_int4_operands): x [M, K] bf16 (M <= 16),
// q4 int8 bytes [ceil(N/16), K/128, 64, 16], s4 fp32 [ceil(N/16), K/gs, 16] -> y [M, N] bf16
Tensor skinny_i4(Tensor x, Tensor q4, Tensor s4, OptT bias, int64_t N, int64_t gs) {
  need(x, "x"); need(q4, "q4"); need(s4, "s4");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "skinny_i4: x must be bf16 [M, K]");
  TORCH_CHECK(q4.scalar_type() == at::kChar && s4.scalar_type() == at::kFloat, "skinny_i4: packed int8 bytes, fp32 scales");
  const int64_t M = x.size(0), K = x.size(1), NB = (N + 15) / 16;
  TORCH_CHECK(ds_skinny_i4_mfma_ok((int)M, (int)K, (int)gs) != 0, "skinny_i4: unsupported shape (M ", M, ", K ", K,
              ", gs ", gs, ")");
  TORCH_CHECK(q4.numel() == NB * 16 * K / 2 && s4.numel() == NB * 16 * (K / gs), "skinny_i4: q4 / s4 size");
  TORCH_CHECK(NB * K < ((int64_t)1 << 40) && N < ((int64_t)1 << 31) / 16, "skinny_i4: matrix too large");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(q4.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_i4: 16-B aligned x / q4");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    need(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "skinny_i4: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  auto y = torch::empty({M, N}, x.options());
  auto& ws = i8_workspace(x, N);  // same fp32 scratch contract as the int8 stream (zero between calls)
  TORCH_CHECK(ws.acc.numel() >= ds_skinny_i4_mfma_ws_floats((int)N), "skinny_i4: workspace");
  check(ds_skinny_i4_mfma(x.data_ptr(), q4.data_ptr<int8_t>(), s4.data_ptr<float>(), bp, y.data_ptr(),
                          ws.acc.data_ptr<float>(), (int)M, (int)N, (int)K, (int)gs, stream()),
        "skinny_i4");
  return y;
}

// The int8 / int4 stream WITHOUT its finalize pass: returns the fp32 workspace view [16, NP] holding the sums of the M
// token rows (no bias). The caller must hand it to one of the skinny_finalize* ops before the next weight-only GEMV on
// this stream (they convert, fuse the consumer's element-wise work and re-zero the workspace).
Tensor skinny_q_raw(Tensor x, Tensor wq, Tensor ws_s, int64_t N, int64_t gs, int64_t bits) {
  need(x, "x"); need(wq, "wq"); need(ws_s, "scales");
  TORCH_CHECK(bits == 4 || bits == 8, "skinny_q_raw: 4 or 8 bits");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "skinny_q_raw: x must be bf16 [M, K]");
  TORCH_CHECK(wq.scalar_type() == at::kChar && ws_s.scalar_type() == at::kFloat, "skinny_q_raw: int8 bytes, fp32 scales");
  const int64_t M = x.size(0), K = x.size(1), NB = (N + 15) / 16;
  const bool ok = bits == 4 ? ds_skinny_i4_mfma_ok((int)M, (int)K, (int)gs) != 0 : ds_skinny_i8_mfma_ok((int)M, (int)K, (int)gs) != 0;
  TORCH_CHECK(ok, "skinny_q_raw: unsupported shape (M ", M, ", K ", K, ", gs ", gs, ")");
  TORCH_CHECK(wq.numel() == NB * 16 * K * bits / 8 && ws_s.numel() == NB * 16 * (K / gs), "skinny_q_raw: weight / scale size");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(wq.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_q_raw: 16-B aligned x / weights");
  auto& ws = i8_workspace(x, N);
  const int64_t NP = ds_skinny_i8_mfma_ws_floats((int)N) / 16;
  TORCH_CHECK(NP == ds_skinny_i4_mfma_ws_floats((int)N) / 16, "workspace layouts differ");
  if (bits == 4)
    check(ds_skinny_i4_mfma(x.data_ptr(), wq.data_ptr<int8_t>(), ws_s.data_ptr<float>(), nullptr, nullptr,
                            ws.acc.data_ptr<float>(), (int)M, (int)N, (int)K, (int)gs, stream()), "skinny_i4 (raw)");
  else
    check(ds_skinny_i8_mfma(x.data_ptr(), wq.data_ptr<int8_t>(), ws_s.data_ptr<float>(), nullptr, nullptr,
                            ws.acc.data_ptr<float>(), (int)M, (int)N, (int)K, (int)gs, stream()), "skinny_i8 (raw)");
  return ws.acc.narrow(0, 0, 16 * NP).view({16, NP});
}

// bf16 MFMA stream over the pre-shuffled weight (ops/bf16_gemv.py: preshuffle16): x [M, K] bf16 (M <= 16),
// wsh bf16 [ceil(N/16), K/64, 2, 64, 8] -> y [M, N] bf16; `raw`: the un-finalized fp32 workspace view [16, NP] instead
// (same contract as skinny_q_raw).
Tensor skinny_b16_impl(Tensor x, Tensor wsh, OptT bias, int64_t N, bool raw) {
  need(x, "x"); need(wsh, "wsh");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && wsh.scalar_type() == at::kBFloat16,
              "skinny_b16: bf16 x [M, K] and bf16 shuffled weight");
  const int64_t M = x.size(0), K = x.size(1), NB = (N + 15) / 16;
  TORCH_CHECK(ds_skinny_b16_mfma_ok((int)M, (int)K) != 0, "skinny_b16: unsupported shape (M ", M, ", K ", K, ")");
  TORCH_CHECK(wsh.numel() == NB * 16 * K && wsh.is_contiguous(), "skinny_b16: shuffled weight size");
  TORCH_CHECK(NB * K < ((int64_t)1 << 40) && N < ((int64_t)1 << 31) / 16, "skinny_b16: matrix too large");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(wsh.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_b16: 16-B aligned x / weight");
  const void* bp = nullptr;
  if (!raw && bias.has_value() && bias->defined()) {
    need(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "skinny_b16: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  auto& ws = i8_workspace(x, N);
  if (raw) {
    check(ds_skinny_b16_mfma(x.data_ptr(), wsh.data_ptr(), nullptr, nullptr, ws.acc.data_ptr<float>(), (int)M, (int)N,
                             (int)K, stream()), "skinny_b16 (raw)");
    const int64_t NP = ds_skinny_i8_mfma_ws_floats((int)N) / 16;
    return ws.acc.narrow(0, 0, 16 * NP).view({16, NP});
  }
  auto y = torch::empty({M, N}, x.options());
  check(ds_skinny_b16_mfma(x.data_ptr(), wsh.data_ptr(), bp, y.data_ptr(), ws.acc.data_ptr<float>(), (int)M, (int)N,
                           (int)K, stream()), "skinny_b16");
  return y;
}
Tensor skinny_b16_sh(Tensor x, Tensor wsh, OptT bias, int64_t N) { return skinny_b16_impl(x, wsh, bias, N, false); }
Tensor skinny_b16_raw(Tensor x, Tensor wsh, int64_t N) { return skinny_b16_impl(x, wsh, c10::nullopt, N, true); }
bool skinny_b16_ok(int64_t M, int64_t K) { return ds_skinny_b16_mfma_ok((int)M, (int)K) != 0; }

// pre-shuffled bf16 -> row-major bf16 [N, K]
Tensor unshuffle_sh16(Tensor wsh, int64_t N) {
  need(wsh, "wsh");
  TORCH_CHECK(wsh.scalar_type() == at::kBFloat16 && wsh.dim() == 5 && wsh.is_contiguous(), "unshuffle_sh16: layout");
  const int64_t K = wsh.size(1) * 64;
  TORCH_CHECK(wsh.size(0) == (N + 15) / 16, "unshuffle_sh16: sizes");
  auto w = torch::empty({N, K}, wsh.options());
  check(ds_unshuffle_sh16(wsh.data_ptr(), w.data_ptr(), (int)N, (int)K, stream()), "unshuffle_sh16");
  return w;
}

const void* opt_bf16(const OptT& t, int64_t numel, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  need(*t, what);
  TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->numel() == numel, what, ": bf16 with ", numel, " elements");
  return t->data_ptr();
}
void check_acc(const Tensor& acc, int64_t M, int64_t N) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat && acc.dim() == 2 && acc.size(0) == 16 &&
                  acc.is_contiguous() && acc.size(1) >= N && M >= 1 && M <= 16, "skinny_finalize: fp32 workspace view [16, NP]");
}

// (acc + bias + residual) -> res_out; RMSNorm(res_out) * w -> y   (both [M, N] bf16)
std::vector<Tensor> skinny_finalize_rms(Tensor acc, int64_t M, int64_t N, OptT bias, OptT residual, Tensor w, double eps) {
  check_acc(acc, M, N);
  const void* bp = opt_bf16(bias, N, "bias");
  const void* rp = opt_bf16(residual, M * N, "residual");
  OptT wo = w;
  const void* wp = opt_bf16(wo, N, "norm weight");
  auto y = torch::empty({M, N}, acc.options().dtype(at::kBFloat16));
  auto res = torch::empty({M, N}, acc.options().dtype(at::kBFloat16));
  check(ds_skinny_finalize_rms(acc.data_ptr<float>(), bp, rp, wp, y.data_ptr(), res.data_ptr(), (int)M, (int)N,
                               (int)acc.size(1), (float)eps, stream()), "skinny_finalize_rms");
  return {y, res};
}

// act(acc[:, :I] + b) * (acc[:, I:] + b) -> [M, N / 2] bf16
Tensor skinny_finalize_gated(Tensor acc, int64_t M, int64_t N, OptT bias, int64_t act) {
  check_acc(acc, M, N);
  const void* bp = opt_bf16(bias, N, "bias");
  auto out = torch::empty({M, N / 2}, acc.options().dtype(at::kBFloat16));
  check(ds_skinny_finalize_gated(acc.data_ptr<float>(), bp, out.data_ptr(), (int)M, (int)N, (int)acc.size(1), (int)act,
                                 stream()), "skinny_finalize_gated");
  return out;
}

Tensor skinny_finalize(Tensor acc, int64_t M, int64_t N, OptT bias) {
  check_acc(acc, M, N);
  const void* bp = opt_bf16(bias, N, "bias");
  auto y = torch::empty({M, N}, acc.options().dtype(at::kBFloat16));
  check(ds_skinny_finalize_plain(acc.data_ptr<float>(), bp, y.data_ptr(), (int)M, (int)N, (int)acc.size(1), stream()),
        "skinny_finalize");
  return y;
}

// packed int4 (ops/int4_gemv.py) -> row-major bf16 [N, K]
Tensor dequant_sh4(Tensor q4, Tensor s4, int64_t N, int64_t gs) {
  need(q4, "q4"); need(s4, "s4");
  TORCH_CHECK(q4.scalar_type() == at::kChar && s4.scalar_type() == at::kFloat && q4.dim() == 4, "dequant_sh4: layout");
  const int64_t K = q4.size(1) * 128;
  TORCH_CHECK(q4.size(0) == (N + 15) / 16 && q4.size(2) == 64 && q4.size(3) == 16 &&
                  s4.numel() == q4.size(0) * 16 * (K / gs), "dequant_sh4: sizes");
  auto w = torch::empty({N, K}, q4.options().dtype(at::kBFloat16));
  check(ds_dequant_sh4(q4.data_ptr<int8_t>(), s4.data_ptr<float>(), w.data_ptr(), (int)N, (int)K, (int)gs, stream()),
        "dequant_sh4");
  return w;
}

// Ragged paged flash prefill (attn/paged_prefill.hip): q [T, Hq, D] bf16, caches [blocks, Hk, BS, D], D in {64, 80,
// 96, 128, 256},
// block_table [nseq, max_blocks], start [nseq], cu_q [nseq + 1], work [nwork, 2] int32 built by the caller from the
// same lengths (every (sequence, 128-row block) with block * 128 < that sequence's new tokens).
Tensor paged_prefill(Tensor q, Tensor kc, Tensor vc, Tensor block_table, Tensor start, Tensor cu_q, Tensor work,
                     OptT alibi, int64_t window, double scale) {
  need(q, "q"); need(kc, "k_cache"); need(vc, "v_cache"); need(block_table, "block_table"); need(start, "start");
  need(cu_q, "cu_q"); need(work, "work");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && kc.scalar_type() == at::kBFloat16 && q.dim() == 3,
              "paged_prefill: bf16 q [T, Hq, D]");
  const int D = (int)q.size(2);
  TORCH_CHECK(D == 64 || D == 80 || D == 96 || D == 128 || D == 256, "paged_prefill: head dim 64/80/96/128/256");
  TORCH_CHECK(kc.dim() == 4 && kc.size(3) == D && vc.sizes() == kc.sizes(), "paged_prefill: caches [NB, Hk, BS, D]");
  TORCH_CHECK(block_table.scalar_type() == at::kInt && start.scalar_type() == at::kInt && cu_q.scalar_type() == at::kInt &&
              work.scalar_type() == at::kInt, "paged_prefill: int32 tables");
  const int64_t nseq = start.numel();
  TORCH_CHECK(block_table.dim() == 2 && block_table.size(0) == nseq && cu_q.numel() == nseq + 1, "paged_prefill: tables");
  TORCH_CHECK(work.dim() == 2 && work.size(1) == 2, "paged_prefill: work [nwork, 2]");
  const int Hq = (int)q.size(1), Hk = (int)kc.size(1);
  TORCH_CHECK(Hq % Hk == 0, "paged_prefill: GQA ratio");
  const float* al = nullptr;
  if (alibi.has_value() && alibi->defined()) {
    need(*alibi, "alibi");
    TORCH_CHECK(alibi->scalar_type() == at::kFloat && alibi->numel() == Hq, "paged_prefill: alibi [Hq] fp32");
    al = alibi->data_ptr<float>();
  }
  auto o = torch::empty_like(q);
  check(ds_paged_prefill(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), o.data_ptr(), block_table.data_ptr<int>(),
                         start.data_ptr<int>(), cu_q.data_ptr<int>(), work.data_ptr<int>(), (int)work.size(0), al, Hq,
                         Hk, D, (int)kc.size(2), (int)block_table.size(1), (int)window, (float)scale, stream()),
        "paged_prefill");
  return o;
}

void register_inference_ops(pybind11::module& m) {
  m.def("paged_prefill", &paged_prefill);
  m.def("dequant_sh", &dequant_sh);
  m.def("skinny_i8_ok", &skinny_i8_ok);
  m.def("skinny_i8_sh_ok", &skinny_i8_sh_ok);
  m.def("skinny_i8_tune", [](int64_t cfg, int64_t wpc, int64_t dbg) { ds_skinny_i8_tune((int)cfg, (int)wpc, (int)dbg); },
        py::arg("cfg"), py::arg("wpc"), py::arg("dbg") = 0);
  m.def("skinny_i8", &skinny_i8, py::arg("x"), py::arg("q"), py::arg("scales"), py::arg("bias"), py::arg("N"),
        py::arg("gs"));
  m.def("skinny_i8_sh", &skinny_i8_sh, py::arg("x"), py::arg("qsh"), py::arg("ssh"), py::arg("bias"), py::arg("N"),
        py::arg("gs"));
  m.def("skinny_i4_ok", &skinny_i4_ok);
  m.def("skinny_i4", &skinny_i4, py::arg("x"), py::arg("q4"), py::arg("s4"), py::arg("bias"), py::arg("N"),
        py::arg("gs"));
  m.def("skinny_i4_tune", [](int64_t p, int64_t wpc, int64_t rounds) { ds_skinny_i4_tune((int)p, (int)wpc, (int)rounds); },
        py::arg("p"), py::arg("wpc"), py::arg("rounds") = 0);
  m.def("dequant_sh4", &dequant_sh4);
  m.def("skinny_q_raw", &skinny_q_raw);
  m.def("skinny_b16_ok", &skinny_b16_ok);
  m.def("skinny_b16_sh", &skinny_b16_sh, py::arg("x"), py::arg("wsh"), py::arg("bias"), py::arg("N"));
  m.def("skinny_b16_raw", &skinny_b16_raw);
  m.def("unshuffle_sh16", &unshuffle_sh16);
  m.def("skinny_b16_tune", [](int64_t cfg, int64_t wpc) { ds_skinny_b16_tune((int)cfg, (int)wpc); }, py::arg("cfg"),
        py::arg("wpc") = 0);
  m.def("skinny_finalize_rms", &skinny_finalize_rms);
  m.def("skinny_finalize_gated", &skinny_finalize_gated);
  m.def("skinny_finalize", &skinny_finalize);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("skinny_force_valu", &skinny_force_valu);
  m.def("skinny_set_path", &skinny_set_path);
  m.def("qkv_rope_append", &qkv_rope_append, py::arg("qkv"), py::arg("cos"), py::arg("sin"), py::arg("pos"),
        py::arg("kc"), py::arg("vc"), py::arg("block_table"), py::arg("start_pos"), py::arg("n_new"), py::arg("Hq"),
        py::arg("Hk"), py::arg("rot"), py::arg("interleaved"), py::arg("want_kv"), py::arg("seq_ids") = py::none(), py::arg("acc_rows") = 0,
        py::arg("acc_bias") = py::none());
  m.def("paged_decode", &paged_decode);
  m.def("kv_append", &kv_append);
  m.def("quantize", &quantize);
  m.def("dequantize", &dequantize);
  m.def("dequant_reduce", &dequant_reduce);
}
