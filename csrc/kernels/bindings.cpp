// PyTorch <-> HIP kernel glue for flexflow_amd._C. Only this translation unit includes torch
// headers; the kernels themselves are torch-free .hip files. Every entry point launches on the
// caller's current HIP stream (so the executor can route ops to its compute / comm streams and
// capture whole steps into hipGraphs) and checks shapes before launching.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "attention.h"
#include "blaslt.h"
#include "gemm.h"
#include "ops.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtcode(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return ffk::DT_BF16;
  if (t.scalar_type() == at::kFloat) return ffk::DT_F32;
  TORCH_CHECK(false, "flexflow_amd kernels support bf16/fp32 only, got ", t.scalar_type());
  return -1;
}
void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
}
template <typename T = void>
T* ptr(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void gemm(Tensor A, Tensor B, Tensor C, optional<Tensor> bias, optional<Tensor> Z, int64_t M, int64_t N,
          int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC, int64_t batch,
          bool a_k, bool b_k, double alpha, double beta, int64_t act, int64_t splitk, optional<Tensor> ws,
          int64_t impl, bool skip_reduce) {
  check_dev(A, "A"); check_dev(B, "B"); check_dev(C, "C");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm: A/B must be bf16");
  TORCH_CHECK(C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat, "gemm: C must be bf16/fp32");
  // bounds: the furthest element touched must lie inside each storage
  auto last = [](int64_t rows, int64_t cols, int64_t ld, int64_t stride, int64_t nb) {
    return (nb - 1) * stride + (rows - 1) * ld + cols;
  };
  TORCH_CHECK(last(a_k ? M : K, a_k ? K : M, lda, sA, batch) <= A.numel(), "gemm: A too small");
  TORCH_CHECK(last(b_k ? N : K, b_k ? K : N, ldb, sB, batch) <= B.numel(), "gemm: B too small");
  TORCH_CHECK(last(M, N, ldc, sC, batch) <= C.numel(), "gemm: C too small");
  ffk::GemmArgs p;
  p.A = reinterpret_cast<const uint16_t*>(A.data_ptr());
  p.B = reinterpret_cast<const uint16_t*>(B.data_ptr());
  p.C = C.data_ptr();
  p.Z = ptr(Z);
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N, "gemm: bias too small");
    p.bias = bias->data_ptr();
    p.bias_bf16 = bias->scalar_type() == at::kBFloat16;
  }
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC; p.batch = batch;
  p.alpha = alpha; p.beta = beta; p.act = act;
  p.a_kcontig = a_k; p.b_kcontig = b_k;
  p.out_f32 = C.scalar_type() == at::kFloat;
  p.a_bytes = A.numel() * 2;
  p.b_bytes = B.numel() * 2;
  p.impl = (int)impl;
  p.splitk = 1;
  if (splitk > 1 && ws.has_value() && ws->defined()) {
    TORCH_CHECK(ws->numel() * ws->element_size() >= ffk::gemm_workspace_bytes(M, N, K, batch, splitk),
                "gemm: split-K workspace too small");
    p.splitk = splitk;
    p.ws = reinterpret_cast<float*>(ws->data_ptr());
    p.skip_reduce = skip_reduce;
  }
  ffk::gemm_bf16(p, cur_stream());
}

// C = (A.B) * act'(zin) [+ dbias += colsum] in one 256-row MFMA GEMM; false if the shape does not fit
bool gemm_dact(Tensor A, Tensor B, Tensor C, Tensor zin, optional<Tensor> dbias, int64_t M, int64_t N, int64_t K,
               int64_t lda, int64_t ldb, int64_t ldc, bool a_k, bool b_k, int64_t act, int64_t impl) {
  check_dev(A, "A"); check_dev(B, "B"); check_dev(C, "C"); check_dev(zin, "zin");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
              C.scalar_type() == at::kBFloat16 && zin.scalar_type() == at::kBFloat16, "gemm_dact: bf16 operands");
  TORCH_CHECK((a_k ? (M - 1) * lda + K : (K - 1) * lda + M) <= A.numel(), "gemm_dact: A too small");
  TORCH_CHECK((b_k ? (N - 1) * ldb + K : (K - 1) * ldb + N) <= B.numel(), "gemm_dact: B too small");
  TORCH_CHECK((M - 1) * ldc + N <= C.numel() && (M - 1) * ldc + N <= zin.numel(), "gemm_dact: C / zin too small");
  const bool has_db = dbias.has_value() && dbias->defined();
  if (has_db) TORCH_CHECK(dbias->scalar_type() == at::kFloat && dbias->numel() >= N, "gemm_dact: dbias");
  ffk::GemmArgs p;
  p.A = reinterpret_cast<const uint16_t*>(A.data_ptr());
  p.B = reinterpret_cast<const uint16_t*>(B.data_ptr());
  p.C = C.data_ptr();
  p.zin = zin.data_ptr();
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.act = act;
  p.a_kcontig = a_k; p.b_kcontig = b_k;
  p.a_bytes = A.numel() * 2;
  p.b_bytes = B.numel() * 2;
  const int64_t rows = 2 * ((M + 255) / 256);
  Tensor part;
  if (has_db) {
    part = at::empty({rows * N}, C.options().dtype(at::kFloat));
    p.colpart = part.data_ptr<float>();
  }
  p.impl = (int)impl;  // 6: the ping-pong kernel's DACT epilogue; else the 256-row kernel's
  if (!ffk::gemm_dact_bf16(p, cur_stream())) return false;
  if (has_db) ffk::col_reduce_add(p.colpart, dbias->data_ptr<float>(), (int)rows, (int)N, cur_stream());
  return true;
}

void box_copy(std::vector<Tensor> srcs, Tensor dst, Tensor desc, int64_t nbox, int64_t max_n, int64_t vec_bytes,
              bool add, bool idx32) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= ffk::kBoxSrcs, "box_copy: 1..16 sources");
  check_dev(dst, "dst"); check_dev(desc, "desc");
  TORCH_CHECK(desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.numel() >= nbox * ffk::box_words(),
              "box_copy: descriptors");
  TORCH_CHECK(nbox >= 0 && nbox <= 65535, "box_copy: at most 65535 boxes per launch");
  std::vector<const void*> ptrs;
  for (auto& t : srcs) {
    check_dev(t, "src");
    TORCH_CHECK(t.scalar_type() == dst.scalar_type(), "box_copy: one dtype");
    TORCH_CHECK(add || (reinterpret_cast<uintptr_t>(t.data_ptr()) % vec_bytes) == 0,
                "box_copy: source not aligned to the vector width");
    ptrs.push_back(t.data_ptr());
  }
  int dt = 0;
  if (add) {
    TORCH_CHECK(dst.scalar_type() == at::kFloat || dst.scalar_type() == at::kBFloat16, "box_copy add: fp32 / bf16");
    dt = dst.scalar_type() == at::kFloat ? ffk::DT_F32 : ffk::DT_BF16;
  } else {
    TORCH_CHECK(vec_bytes == 1 || vec_bytes == 2 || vec_bytes == 4 || vec_bytes == 8 || vec_bytes == 16,
                "box_copy: vector width");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(dst.data_ptr()) % vec_bytes) == 0,
                "box_copy: destination not aligned to the vector width");
  }
  ffk::box_copy(ptrs.data(), (int)ptrs.size(), dst.data_ptr(), desc.data_ptr<int64_t>(), (int)nbox, max_n,
                (int)vec_bytes, add ? 1 : 0, dt, idx32 ? 1 : 0, cur_stream());
}

// out [outer][sum lens] (vec units) = concat of srcs [outer][lens[i]]; sizes and alignment checked here
void concat_rows(std::vector<Tensor> srcs, std::vector<int64_t> lens, Tensor out, int64_t outer, int64_t vec_bytes) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= ffk::kBoxSrcs && srcs.size() == lens.size(), "concat_rows: 1..16 inputs");
  TORCH_CHECK(vec_bytes == 2 || vec_bytes == 4 || vec_bytes == 8 || vec_bytes == 16, "concat_rows: vector width");
  check_dev(out, "out");
  const int64_t esz = out.element_size();
  TORCH_CHECK(vec_bytes % esz == 0 && (reinterpret_cast<uintptr_t>(out.data_ptr()) % vec_bytes) == 0,
              "concat_rows: output alignment");
  int64_t row = 0;
  std::vector<const void*> ptrs;
  std::vector<int> l32;
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& t = srcs[i];
    check_dev(t, "src");
    TORCH_CHECK(t.scalar_type() == out.scalar_type(), "concat_rows: one dtype");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) % vec_bytes) == 0, "concat_rows: input alignment");
    TORCH_CHECK(lens[i] > 0 && t.numel() * esz == outer * lens[i] * vec_bytes, "concat_rows: input size");
    // 32-bit grid-stride index: the last step (at most 8192 x 256 past the end) stays below 2^31
    TORCH_CHECK(outer * lens[i] + 8192LL * 256 < (1LL << 31), "concat_rows: input too large for 32-bit indexing");
    row += lens[i];
    ptrs.push_back(t.data_ptr());
    l32.push_back((int)lens[i]);
  }
  TORCH_CHECK(out.numel() * esz == outer * row * vec_bytes && outer < (1LL << 31), "concat_rows: output size");
  ffk::concat_rows(ptrs.data(), l32.data(), (int)ptrs.size(), out.data_ptr(), (int)outer, (int)vec_bytes, cur_stream());
}

// dst [cols][rows] = src [rows][cols]^T (2-byte elements, both contiguous, dims multiples of 8)
void transpose2d(Tensor src, Tensor dst) {
  check_dev(src, "src"); check_dev(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.is_contiguous() && dst.is_contiguous() &&
              src.element_size() == 2 && dst.scalar_type() == src.scalar_type(), "transpose2d: contiguous 2-D 16-bit");
  const int64_t r = src.size(0), c = src.size(1);
  TORCH_CHECK(dst.size(0) == c && dst.size(1) == r, "transpose2d: dst must be [cols][rows]");
  TORCH_CHECK(r % 8 == 0 && c % 8 == 0 && r * c < (1LL << 31), "transpose2d: dims multiples of 8, < 2^31 elements");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(src.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16) == 0,
              "transpose2d: 16-B aligned");
  ffk::transpose16(src.data_ptr(), dst.data_ptr(), (int)r, (int)c, cur_stream());
}
// desc: int64 device tensor [n][5] = {src, dst, rows, cols, first tile}, built by the caller from
// tensors it validated with transpose2d's rules (kernels.wt_refresh_all)
void transpose2d_batch(Tensor desc, int64_t n, int64_t tiles) {
  check_dev(desc, "desc");
  TORCH_CHECK(desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.numel() >= n * 5 && n > 0 &&
              tiles > 0 && tiles < (1LL << 31), "transpose2d_batch: descriptors");
  ffk::transpose16_batch(desc.data_ptr<int64_t>(), (int)n, tiles, cur_stream());
}

// x [.., xd, inner] and idx / out [.., dsz, inner], contiguous, other dims equal (checked by caller)
void gather_fwd(Tensor x, Tensor idx, Tensor out, int64_t dsz, int64_t inner, int64_t xd) {
  check_dev(x, "x"); check_dev(idx, "idx"); check_dev(out, "out");
  TORCH_CHECK(x.is_contiguous() && idx.is_contiguous() && out.is_contiguous() && out.numel() == idx.numel() &&
              out.scalar_type() == x.scalar_type(), "gather_fwd: contiguous x / idx / out");
  TORCH_CHECK(idx.scalar_type() == at::kInt || idx.scalar_type() == at::kLong, "gather_fwd: int32 / int64 indices");
  TORCH_CHECK(dsz > 0 && inner > 0 && xd > 0 && idx.numel() % (dsz * inner) == 0 &&
              x.numel() == idx.numel() / dsz * xd, "gather_fwd: geometry");
  ffk::gather_fwd(dtcode(x), idx.scalar_type() == at::kLong, x.data_ptr(), idx.data_ptr(), out.data_ptr(),
                  idx.numel(), dsz, inner, xd, cur_stream());
}
void gather_bwd(Tensor dy, Tensor idx, Tensor dx, int64_t dsz, int64_t inner, int64_t xd) {
  check_dev(dy, "dy"); check_dev(idx, "idx"); check_dev(dx, "dx");
  TORCH_CHECK(dy.is_contiguous() && idx.is_contiguous() && dx.is_contiguous() && dy.numel() == idx.numel() &&
              dx.scalar_type() == at::kFloat, "gather_bwd: contiguous dy / idx, fp32 dx");
  TORCH_CHECK(idx.scalar_type() == at::kInt || idx.scalar_type() == at::kLong, "gather_bwd: int32 / int64 indices");
  TORCH_CHECK(dsz > 0 && inner > 0 && xd > 0 && idx.numel() % (dsz * inner) == 0 &&
              dx.numel() == idx.numel() / dsz * xd, "gather_bwd: geometry");
  ffk::gather_bwd(dtcode(dy), idx.scalar_type() == at::kLong, dy.data_ptr(), idx.data_ptr(), dx.data_ptr<float>(),
                  idx.numel(), dsz, inner, xd, cur_stream());
}

int64_t gemm_pick_splitk(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t impl) {
  return ffk::gemm_pick_splitk(M, N, K, batch, (int)impl);
}

// two tensors whose elements sit at the same offsets of dense memory (both NCHW-contiguous or both
// channel-last-contiguous): elementwise kernels index them flat
bool same_dense(const Tensor& a, const Tensor& b) {
  if (a.numel() != b.numel()) return false;
  if (a.is_contiguous() && b.is_contiguous()) return true;
  return a.dim() == 4 && b.dim() == 4 && a.sizes() == b.sizes() && a.is_contiguous(at::MemoryFormat::ChannelsLast) &&
         b.is_contiguous(at::MemoryFormat::ChannelsLast);
}

void unary_fwd(Tensor x, Tensor y, int64_t op, double s) {
  check_dev(x, "x");
  TORCH_CHECK(x.numel() == y.numel() && same_dense(x, y), "unary_fwd: x / y must be dense in one memory order");
  ffk::unary_fwd(dtcode(x), x.data_ptr(), y.data_ptr(), x.numel(), op, s, cur_stream());
}
void bias_act_fwd(Tensor z, optional<Tensor> bias, optional<Tensor> zout, Tensor y, int64_t rows, int64_t cols,
                  int64_t act) {
  check_dev(z, "z");
  TORCH_CHECK(z.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 && cols % 8 == 0);
  TORCH_CHECK(z.numel() >= rows * cols && y.numel() >= rows * cols && z.is_contiguous() && y.is_contiguous());
  TORCH_CHECK(!bias || bias->numel() >= cols);
  ffk::bias_act_fwd(z.data_ptr(), ptr(bias), bias && bias->scalar_type() == at::kBFloat16, ptr(zout), y.data_ptr(),
                    rows, cols, act, cur_stream());
}
void unary_bwd(Tensor x, Tensor y, Tensor dy, Tensor dx, int64_t op, double s, bool acc) {
  TORCH_CHECK(x.numel() == dx.numel() && dy.numel() == dx.numel() && y.numel() == dx.numel());
  TORCH_CHECK(same_dense(x, dx) && same_dense(y, dx) && same_dense(dy, dx),
              "unary_bwd: x / y / dy / dx must be dense in one memory order");
  ffk::unary_bwd(dtcode(x), x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), op, s, acc,
                 cur_stream());
}
void binary_fwd(Tensor a, Tensor b, Tensor c, int64_t op, std::vector<int64_t> shape, std::vector<int64_t> sa,
                std::vector<int64_t> sb, bool same) {
  TORCH_CHECK(shape.size() <= 6 && sa.size() == shape.size() && sb.size() == shape.size());
  TORCH_CHECK(!same || (same_dense(a, c) && same_dense(b, c)), "binary_fwd: flat operands must share a memory order");
  TORCH_CHECK(same || c.is_contiguous(), "binary_fwd: broadcast output must be contiguous");
  ffk::binary_fwd(dtcode(c), a.data_ptr(), b.data_ptr(), c.data_ptr(), c.numel(), op, shape.size(), shape.data(),
                  sa.data(), sb.data(), same, cur_stream());
}
void binary_bwd(Tensor a, Tensor b, Tensor dc, optional<Tensor> da, optional<Tensor> db, int64_t op,
                std::vector<int64_t> shape, std::vector<int64_t> sa, std::vector<int64_t> sb, bool same) {
  TORCH_CHECK(shape.size() <= 6);
  TORCH_CHECK(!same || (same_dense(a, dc) && same_dense(b, dc) && (!da || same_dense(*da, dc)) &&
                        (!db || same_dense(*db, dc))),
              "binary_bwd: flat operands must share a memory order");
  TORCH_CHECK(same || (dc.is_contiguous() && (!da || da->is_contiguous()) && (!db || db->is_contiguous())),
              "binary_bwd: broadcast gradients must be contiguous");
  ffk::binary_bwd(dtcode(dc), a.data_ptr(), b.data_ptr(), dc.data_ptr(), ptr(da), ptr(db), dc.numel(), op,
                  shape.size(), shape.data(), sa.data(), sb.data(), same, cur_stream());
}
void cast(Tensor x, Tensor y) {
  TORCH_CHECK(x.numel() == y.numel());
  ffk::cast(dtcode(x), dtcode(y), x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
}
void dropout_fwd(Tensor x, Tensor y, Tensor mask, double rate, int64_t seed, int64_t offset) {
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() == x.numel());
  ffk::dropout_fwd(dtcode(x), x.data_ptr(), y.data_ptr(), mask.data_ptr<uint8_t>(), x.numel(), rate, seed, offset,
                   cur_stream());
}
void dropout_bwd(Tensor dy, Tensor mask, Tensor dx, double rate, bool acc) {
  ffk::dropout_bwd(dtcode(dy), dy.data_ptr(), mask.data_ptr<uint8_t>(), dx.data_ptr(), dy.numel(), rate, acc,
                   cur_stream());
}
int64_t bias_act_bwd_ws(int64_t rows, int64_t cols) { return (int64_t)ffk::bias_act_bwd_chunks(rows, cols) * cols; }

// stage 0: row pass + slab fold; 1: row pass into `ws_in`; 2: slab fold of `ws_in` into dbias
void bias_act_bwd(Tensor dy, optional<Tensor> z, optional<Tensor> dz, optional<Tensor> dbias, int64_t rows,
                  int64_t cols, int64_t act, optional<Tensor> ws_in, int64_t stage) {
  TORCH_CHECK(dy.numel() == rows * cols);
  if (dbias.has_value() && dbias->defined()) TORCH_CHECK(dbias->scalar_type() == at::kFloat && dbias->numel() >= cols);
  Tensor ws;
  float* wsp = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    if (ws_in.has_value() && ws_in->defined()) {
      TORCH_CHECK(ws_in->scalar_type() == at::kFloat && ws_in->numel() >= bias_act_bwd_ws(rows, cols), "bias_act_bwd: ws");
      ws = *ws_in;
    } else {
      TORCH_CHECK(stage == 0, "bias_act_bwd: a staged call needs its workspace");
      ws = at::empty({bias_act_bwd_ws(rows, cols)}, dy.options().dtype(at::kFloat));
    }
    wsp = ws.data_ptr<float>();
  }
  ffk::bias_act_bwd(dtcode(dy), dy.data_ptr(), ptr(z), ptr(dz), ptr<float>(dbias), wsp, rows, cols, act,
                    cur_stream(), (int)stage);
}
void layernorm_fwd(Tensor x, optional<Tensor> res, optional<Tensor> sum_out, optional<Tensor> gamma,
                   optional<Tensor> beta, Tensor y, Tensor mean, Tensor rstd, int64_t rows, int64_t cols,
                   double eps) {
  TORCH_CHECK(x.numel() == rows * cols && y.numel() == rows * cols && mean.numel() >= rows && rstd.numel() >= rows);
  ffk::layernorm_fwd(dtcode(x), x.data_ptr(), ptr(res), ptr(sum_out), ptr(gamma), ptr(beta), y.data_ptr(),
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, cols, eps, cur_stream());
}
int64_t layernorm_bwd_ws(int64_t rows, int64_t cols) {
  return 3 * (int64_t)ffk::layernorm_bwd_waves(rows) * cols + (int64_t)ffk::bias_act_bwd_chunks(rows, cols) * cols;
}

// stage as bias_act_bwd's (the slab folds of dgamma / dbeta / dsum run in stage 2)
void layernorm_bwd(Tensor dy, Tensor x, optional<Tensor> gamma, Tensor mean, Tensor rstd, Tensor dx,
                   optional<Tensor> dres, optional<Tensor> dgamma, optional<Tensor> dbeta, int64_t rows,
                   int64_t cols, bool acc, optional<Tensor> dsum, optional<Tensor> ws_in, int64_t stage) {
  TORCH_CHECK(dy.numel() == rows * cols && dx.numel() == rows * cols);
  TORCH_CHECK(!dsum || (dsum->scalar_type() == at::kFloat && dsum->numel() >= cols), "layernorm_bwd: dsum");
  Tensor ws;
  if (ws_in.has_value() && ws_in->defined()) {
    TORCH_CHECK(ws_in->scalar_type() == at::kFloat && ws_in->numel() >= layernorm_bwd_ws(rows, cols), "layernorm_bwd: ws");
    ws = *ws_in;
  } else {
    TORCH_CHECK(stage == 0, "layernorm_bwd: a staged call needs its workspace");
    ws = at::empty({layernorm_bwd_ws(rows, cols)}, dy.options().dtype(at::kFloat));
  }
  ffk::layernorm_bwd(dtcode(dy), dy.data_ptr(), x.data_ptr(), ptr(gamma), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), dx.data_ptr(), ptr(dres), ptr<float>(dgamma), ptr<float>(dbeta),
                     ptr<float>(dsum), ws.data_ptr<float>(), rows, cols, acc, cur_stream(), (int)stage);
}
void softmax_fwd(Tensor x, Tensor y, int64_t rows, int64_t cols, double scale) {
  TORCH_CHECK(x.numel() == rows * cols);
  ffk::softmax_fwd(dtcode(x), x.data_ptr(), y.data_ptr(), rows, cols, scale, cur_stream());
}
void softmax_bwd(Tensor y, Tensor dy, Tensor dx, int64_t rows, int64_t cols, double scale, bool acc) {
  ffk::softmax_bwd(dtcode(y), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), rows, cols, scale, acc, cur_stream());
}
void softmax_xent(Tensor logits, Tensor labels, optional<Tensor> loss, optional<Tensor> dlogits, int64_t rows,
                  int64_t cols, double gscale, optional<Tensor> acc3) {
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.numel() >= rows);
  TORCH_CHECK(!acc3 || (acc3->scalar_type() == at::kFloat && acc3->numel() >= 3));
  ffk::softmax_xent_fwd_bwd(dtcode(logits), logits.data_ptr(), labels.data_ptr<int>(), ptr<float>(loss),
                            ptr(dlogits), rows, cols, gscale, ptr<float>(acc3), cur_stream());
}
void xent_grad(Tensor probs, optional<Tensor> labels, optional<Tensor> onehot, Tensor dprobs, optional<Tensor> loss,
               int64_t rows, int64_t cols, double gscale, bool sparse) {
  ffk::xent_grad(dtcode(probs), probs.data_ptr(), ptr<int>(labels), ptr(onehot), dprobs.data_ptr(),
                 ptr<float>(loss), rows, cols, gscale, sparse, cur_stream());
}
void mse_grad(Tensor pred, Tensor label, Tensor dpred, optional<Tensor> loss, double gscale) {
  TORCH_CHECK(pred.numel() == label.numel());
  ffk::mse_grad(dtcode(pred), pred.data_ptr(), label.data_ptr(), dpred.data_ptr(), ptr<float>(loss), pred.numel(),
                gscale, cur_stream());
}
void metrics_classify(Tensor probs, Tensor labels, int64_t rows, int64_t cols, Tensor out) {
  ffk::metrics_classify(dtcode(probs), probs.data_ptr(), labels.data_ptr<int>(), rows, cols, out.data_ptr<float>(),
                        cur_stream());
}
void reduce_rows(Tensor x, Tensor y, int64_t outer, int64_t red, int64_t inner, bool mean) {
  ffk::reduce_rows(dtcode(x), x.data_ptr(), y.data_ptr(), outer, red, inner, mean, cur_stream());
}
void sgd_sparse_rows(Tensor idx, Tensor mark, Tensor master, Tensor grad, optional<Tensor> lowp, double lr) {
  check_dev(idx, "idx"); check_dev(master, "master");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous(), "sgd_sparse_rows: int64 contiguous ids");
  TORCH_CHECK(master.dim() == 2 && grad.sizes() == master.sizes() && master.is_contiguous() && grad.is_contiguous() &&
              master.scalar_type() == at::kFloat && grad.scalar_type() == at::kFloat, "sgd_sparse_rows: fp32 [rows, dim]");
  TORCH_CHECK(mark.scalar_type() == at::kInt && mark.numel() >= master.size(0), "sgd_sparse_rows: mark");
  if (lowp.has_value() && lowp->defined())
    TORCH_CHECK(lowp->scalar_type() == at::kBFloat16 && lowp->numel() == master.numel() && lowp->is_contiguous());
  TORCH_CHECK(idx.numel() < (1LL << 31));
  ffk::sgd_sparse_rows(idx.data_ptr<int64_t>(), (int)idx.numel(), master.size(0), (int)master.size(1),
                       mark.data_ptr<int>(), master.data_ptr<float>(), grad.data_ptr<float>(), ptr(lowp), lr,
                       cur_stream());
}
void sgd_update(Tensor master, Tensor grad, optional<Tensor> mom, optional<Tensor> lowp, double lr,
                double momentum, bool nesterov, double wd, double gscale, int64_t max_blocks) {
  TORCH_CHECK(master.scalar_type() == at::kFloat && grad.scalar_type() == at::kFloat);
  TORCH_CHECK(master.numel() == grad.numel());
  if (momentum > 0) TORCH_CHECK(mom.has_value() && mom->numel() == master.numel());
  if (lowp.has_value() && lowp->defined())
    TORCH_CHECK(lowp->scalar_type() == at::kBFloat16 && lowp->numel() == master.numel());
  ffk::sgd_update(master.data_ptr<float>(), grad.data_ptr<float>(), ptr<float>(mom), ptr(lowp), master.numel(), lr,
                  momentum, nesterov, wd, gscale, cur_stream(), (int)max_blocks);
}
void adam_update(Tensor master, Tensor grad, Tensor m, Tensor v, optional<Tensor> lowp, double alpha_t, double b1,
                 double b2, double wd, double eps, double gscale, int64_t max_blocks, optional<Tensor> alpha_dev) {
  if (alpha_dev) TORCH_CHECK(alpha_dev->scalar_type() == at::kFloat && alpha_dev->numel() == 1 && alpha_dev->is_cuda(),
                             "adam_update: alpha_dev must be a one-element fp32 device tensor");
  TORCH_CHECK(master.numel() == grad.numel() && m.numel() == master.numel() && v.numel() == master.numel());
  if (lowp.has_value() && lowp->defined())
    TORCH_CHECK(lowp->scalar_type() == at::kBFloat16 && lowp->numel() == master.numel());
  ffk::adam_update(master.data_ptr<float>(), grad.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                   ptr(lowp), master.numel(), alpha_t, b1, b2, wd, eps, gscale, cur_stream(), (int)max_blocks,
                   alpha_dev ? alpha_dev->data_ptr<float>() : nullptr);
}
void embedding_fwd(Tensor idx, Tensor table, Tensor out, int64_t n_rows, int64_t bag, int64_t dim, bool avg) {
  TORCH_CHECK(idx.numel() == n_rows * bag && out.numel() == n_rows * dim && table.size(-1) == dim);
  const bool i64 = idx.scalar_type() == at::kLong;
  ffk::embedding_fwd(dtcode(table), i64, idx.data_ptr(), table.data_ptr(), out.data_ptr(), n_rows, bag, dim,
                     table.numel() / dim, avg, cur_stream());
}
void embedding_bwd(Tensor idx, Tensor dout, Tensor dtable, int64_t n_rows, int64_t bag, int64_t dim, bool avg) {
  TORCH_CHECK(dtable.scalar_type() == at::kFloat && dout.numel() == n_rows * dim);
  const bool i64 = idx.scalar_type() == at::kLong;
  ffk::embedding_bwd(dtcode(dout), i64, idx.data_ptr(), dout.data_ptr(), dtable.data_ptr<float>(), n_rows, bag, dim,
                     dtable.numel() / dim, avg, cur_stream());
}
void init_uniform(Tensor out, double lo, double hi, int64_t seed, int64_t offset) {
  ffk::init_uniform(dtcode(out), out.data_ptr(), out.numel(), lo, hi, seed, offset, cur_stream());
}
void init_normal(Tensor out, double mean, double stdv, int64_t seed, int64_t offset) {
  ffk::init_normal(dtcode(out), out.data_ptr(), out.numel(), mean, stdv, seed, offset, cur_stream());
}
void fill(Tensor out, double v) { ffk::fill(dtcode(out), out.data_ptr(), out.numel(), v, cur_stream()); }
void slab_sum(Tensor slabs, Tensor out, int64_t S, double beta) {
  TORCH_CHECK(slabs.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat && slabs.is_contiguous() &&
              out.is_contiguous());
  TORCH_CHECK(slabs.numel() == out.numel() * S && out.numel() % 4 == 0);
  TORCH_CHECK(((uintptr_t)slabs.data_ptr() % 16) == 0 && ((uintptr_t)out.data_ptr() % 16) == 0);
  ffk::slab_sum(slabs.data_ptr<float>(), out.data_ptr<float>(), out.numel(), (int)S, (float)beta, cur_stream());
}

void gemm_f32(Tensor A, Tensor B, Tensor C, optional<Tensor> bias, optional<Tensor> Z, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC, int64_t batch,
              bool a_k, bool b_k, double alpha, double beta, int64_t act) {
  check_dev(A, "A"); check_dev(B, "B"); check_dev(C, "C");
  TORCH_CHECK(A.scalar_type() == at::kFloat && B.scalar_type() == at::kFloat && C.scalar_type() == at::kFloat,
              "gemm_f32: A/B/C must be fp32");
  auto last = [](int64_t rows, int64_t cols, int64_t ld, int64_t stride, int64_t nb) {
    return (nb - 1) * stride + (rows - 1) * ld + cols;
  };
  TORCH_CHECK(last(a_k ? M : K, a_k ? K : M, lda, sA, batch) <= A.numel(), "gemm_f32: A too small");
  TORCH_CHECK(last(b_k ? N : K, b_k ? K : N, ldb, sB, batch) <= B.numel(), "gemm_f32: B too small");
  TORCH_CHECK(last(M, N, ldc, sC, batch) <= C.numel(), "gemm_f32: C too small");
  ffk::GemmArgs p;
  p.A = reinterpret_cast<const uint16_t*>(A.data_ptr());
  p.B = reinterpret_cast<const uint16_t*>(B.data_ptr());
  p.C = C.data_ptr();
  if (Z.has_value() && Z->defined()) {
    TORCH_CHECK(Z->scalar_type() == at::kFloat && Z->numel() >= last(M, N, ldc, sC, batch), "gemm_f32: Z");
    p.Z = Z->data_ptr();
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() >= N, "gemm_f32: bias too small");
    p.bias = bias->data_ptr();
    p.bias_bf16 = bias->scalar_type() == at::kBFloat16;
  }
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC; p.batch = batch;
  p.alpha = alpha; p.beta = beta; p.act = act;
  p.a_kcontig = a_k; p.b_kcontig = b_k; p.out_f32 = true;
  ffk::gemm_f32(p, cur_stream());
}

void causal_mask_f32(Tensor s, int64_t Sq, int64_t Sk) {
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.is_contiguous() && s.numel() % Sk == 0);
  ffk::causal_mask_f32(s.data_ptr<float>(), s.numel() / Sk, (int)Sq, (int)Sk, cur_stream());
}

// ------------------------------------------------------------------ mixture of experts (moe.hip)
std::vector<void*> ptr_list(const std::vector<optional<Tensor>>& ts, at::ScalarType dt, int64_t numel) {
  TORCH_CHECK((int)ts.size() <= ffk::kMoeMaxExperts, "moe: at most ", ffk::kMoeMaxExperts, " experts");
  std::vector<void*> out;
  for (auto& t : ts) {
    if (t.has_value() && t->defined()) {
      check_dev(*t, "expert tensor");
      TORCH_CHECK(t->scalar_type() == dt && t->is_contiguous() && t->numel() == numel, "moe: expert tensor shape/dtype");
      out.push_back(t->data_ptr());
    } else {
      out.push_back(nullptr);
    }
  }
  return out;
}

void topk_fwd(Tensor x, Tensor vals, Tensor idx, int64_t k) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && vals.is_contiguous() && idx.is_contiguous() && idx.scalar_type() == at::kInt);
  const int64_t n = x.size(-1), rows = x.numel() / n;
  TORCH_CHECK(k >= 1 && k <= n && vals.numel() == rows * k && idx.numel() == rows * k && vals.scalar_type() == x.scalar_type());
  ffk::topk_fwd(dtcode(x), x.data_ptr(), vals.data_ptr(), idx.data_ptr<int>(), (int)rows, (int)n, (int)k, cur_stream());
}

void topk_bwd(Tensor dvals, Tensor idx, Tensor dx) {
  const int64_t n = dx.size(-1), rows = dx.numel() / n, k = idx.size(-1);
  TORCH_CHECK(dvals.is_contiguous() && idx.is_contiguous() && dx.is_contiguous() && idx.scalar_type() == at::kInt &&
              dvals.numel() == rows * k && idx.numel() == rows * k && dvals.scalar_type() == dx.scalar_type());
  ffk::topk_bwd(dtcode(dx), dvals.data_ptr(), idx.data_ptr<int>(), dx.data_ptr(), (int)rows, (int)n, (int)k, cur_stream());
}

int64_t moe_route_ws_ints(int64_t L, int64_t n) { return ffk::moe_route_ws_ints((int)L, (int)n); }

void moe_route(Tensor assign, int64_t n, int64_t cap, Tensor expert, Tensor pos, Tensor load, Tensor ws) {
  check_dev(assign, "assign");
  const int64_t L = assign.numel();
  TORCH_CHECK(assign.scalar_type() == at::kInt && assign.is_contiguous() && expert.numel() == L && pos.numel() == L &&
              load.numel() == n && expert.scalar_type() == at::kInt && pos.scalar_type() == at::kInt &&
              load.scalar_type() == at::kInt && ws.scalar_type() == at::kInt &&
              ws.numel() >= ffk::moe_route_ws_ints((int)L, (int)n) && n >= 1);
  ffk::moe_route(assign.data_ptr<int>(), (int)L, (int)n, (int)cap, expert.data_ptr<int>(), pos.data_ptr<int>(),
                 load.data_ptr<int>(), ws.data_ptr<int>(), cur_stream());
}

void groupby_fwd(Tensor data, Tensor expert, Tensor pos, std::vector<optional<Tensor>> outs, int64_t cap, int64_t k) {
  check_dev(data, "data");
  TORCH_CHECK(data.is_contiguous());
  const int64_t B = data.size(0), D = data.numel() / B, L = expert.numel();
  TORCH_CHECK(L == B * k && pos.numel() == L);
  auto ptrs = ptr_list(outs, data.scalar_type(), cap * D);
  ffk::groupby_fwd(dtcode(data), data.data_ptr(), expert.data_ptr<int>(), pos.data_ptr<int>(), ptrs.data(),
                   (int)ptrs.size(), (int)cap, (int)L, (int)k, (int)D, cur_stream());
}

void groupby_bwd(std::vector<optional<Tensor>> douts, Tensor expert, Tensor pos, Tensor dx, int64_t cap, int64_t k) {
  TORCH_CHECK(dx.is_contiguous());
  const int64_t B = dx.size(0), D = dx.numel() / B;
  TORCH_CHECK(expert.numel() == B * k && pos.numel() == B * k);
  auto ptrs = ptr_list(douts, dx.scalar_type(), cap * D);
  ffk::groupby_bwd(dtcode(dx), ptrs.data(), (int)ptrs.size(), expert.data_ptr<int>(), pos.data_ptr<int>(),
                   dx.data_ptr(), (int)B, (int)k, (int)D, cur_stream());
}

void aggregate_fwd(optional<Tensor> gate, std::vector<optional<Tensor>> exps, Tensor expert, Tensor pos, Tensor out,
                   int64_t cap, int64_t k) {
  TORCH_CHECK(out.is_contiguous());
  const int64_t B = out.size(0), D = out.numel() / B;
  TORCH_CHECK(expert.numel() == B * k && pos.numel() == B * k);
  if (gate.has_value() && gate->defined())
    TORCH_CHECK(gate->numel() == B * k && gate->is_contiguous() && gate->scalar_type() == out.scalar_type());
  auto ptrs = ptr_list(exps, out.scalar_type(), cap * D);
  for (void* q : ptrs) TORCH_CHECK(q != nullptr, "aggregate: every expert prediction is needed");
  ffk::aggregate_fwd(dtcode(out), ptr(gate), ptrs.data(), (int)ptrs.size(), expert.data_ptr<int>(),
                     pos.data_ptr<int>(), out.data_ptr(), (int)B, (int)k, (int)D, cur_stream());
}

void aggregate_bwd(Tensor dout, optional<Tensor> gate, std::vector<optional<Tensor>> exps,
                   std::vector<optional<Tensor>> dexps, Tensor expert, Tensor pos, optional<Tensor> assign,
                   optional<Tensor> true_assign, Tensor load, double lambda_bal, optional<Tensor> dgate,
                   optional<Tensor> dfull, int64_t cap, int64_t k) {
  TORCH_CHECK(dout.is_contiguous());
  const int64_t B = dout.size(0), D = dout.numel() / B;
  const int64_t n = (int64_t)exps.size();
  TORCH_CHECK(expert.numel() == B * k && pos.numel() == B * k && load.numel() == n && dexps.size() == exps.size());
  TORCH_CHECK(k >= 1 && k <= 64, "aggregate_bwd: at most 64 choices per row (the kernel's per-row LDS dot array)");
  if (dgate.has_value() && dgate->defined()) TORCH_CHECK(dgate->numel() == B * k && dgate->scalar_type() == dout.scalar_type());
  if (dfull.has_value() && dfull->defined()) TORCH_CHECK(dfull->numel() == B * n && dfull->scalar_type() == dout.scalar_type());
  auto pe = ptr_list(exps, dout.scalar_type(), cap * D);
  auto pd = ptr_list(dexps, dout.scalar_type(), cap * D);
  ffk::aggregate_bwd(dtcode(dout), dout.data_ptr(), ptr(gate), pe.data(), pd.data(), (int)n, (int)cap,
                     expert.data_ptr<int>(), pos.data_ptr<int>(), ptr<int>(assign), ptr<int>(true_assign),
                     load.data_ptr<int>(), (float)lambda_bal, ptr(dgate), ptr(dfull), (int)B, (int)k, (int)D,
                     cur_stream());
}

// q/k/v/o given with explicit [b,h,s] element strides (d contiguous)
void attn_fwd(Tensor q, std::vector<int64_t> qs, Tensor k, std::vector<int64_t> ks, Tensor v,
              std::vector<int64_t> vs, Tensor o, std::vector<int64_t> os, Tensor lse, int64_t B, int64_t H,
              int64_t Sq, int64_t Sk, int64_t D, double scale, bool causal) {
  TORCH_CHECK(D == 64 || D == 128, "flash attention supports head_dim 64/128");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && o.scalar_type() == at::kBFloat16);
  TORCH_CHECK(lse.numel() >= B * H * Sq && lse.scalar_type() == at::kFloat);
  for (auto* s : {&qs, &ks, &vs, &os}) TORCH_CHECK(s->size() == 3 && (*s)[2] % 8 == 0, "attn: row stride % 8");
  ffk::AttnArgs a;
  a.q = (const uint16_t*)q.data_ptr(); a.q_sb = qs[0]; a.q_sh = qs[1]; a.q_ss = qs[2];
  a.k = (const uint16_t*)k.data_ptr(); a.k_sb = ks[0]; a.k_sh = ks[1]; a.k_ss = ks[2];
  a.v = (const uint16_t*)v.data_ptr(); a.v_sb = vs[0]; a.v_sh = vs[1]; a.v_ss = vs[2];
  a.o = (uint16_t*)o.data_ptr(); a.o_sb = os[0]; a.o_sh = os[1]; a.o_ss = os[2];
  a.lse = lse.data_ptr<float>();
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.D = D; a.scale = scale; a.causal = causal;
  ffk::attn_fwd(a, cur_stream());
}
int64_t attn_bwd_ws(int64_t B, int64_t H, int64_t Sq, int64_t Sk, int64_t D) {
  return ffk::attn_bwd_workspace_floats(B, H, Sq, Sk, D);
}
bool attn_bwd(Tensor q, std::vector<int64_t> qs, Tensor k, std::vector<int64_t> ks, Tensor v,
              std::vector<int64_t> vs, Tensor o, std::vector<int64_t> os, Tensor dout, std::vector<int64_t> dos,
              Tensor lse, Tensor dq, std::vector<int64_t> dqs, Tensor dk, std::vector<int64_t> dks, Tensor dv,
              std::vector<int64_t> dvs, Tensor ws, int64_t B, int64_t H, int64_t Sq, int64_t Sk, int64_t D,
              double scale, bool causal, optional<Tensor> dbias) {
  TORCH_CHECK(D == 64 || D == 128, "flash attention supports head_dim 64/128");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= ffk::attn_bwd_workspace_floats(B, H, Sq, Sk, D),
              "attn_bwd: workspace too small");
  ffk::AttnArgs a;
  a.q = (const uint16_t*)q.data_ptr(); a.q_sb = qs[0]; a.q_sh = qs[1]; a.q_ss = qs[2];
  a.k = (const uint16_t*)k.data_ptr(); a.k_sb = ks[0]; a.k_sh = ks[1]; a.k_ss = ks[2];
  a.v = (const uint16_t*)v.data_ptr(); a.v_sb = vs[0]; a.v_sh = vs[1]; a.v_ss = vs[2];
  a.o = (uint16_t*)o.data_ptr(); a.o_sb = os[0]; a.o_sh = os[1]; a.o_ss = os[2];
  a.dout = (const uint16_t*)dout.data_ptr(); a.do_sb = dos[0]; a.do_sh = dos[1]; a.do_ss = dos[2];
  a.dq = (uint16_t*)dq.data_ptr(); a.dq_sb = dqs[0]; a.dq_sh = dqs[1]; a.dq_ss = dqs[2];
  a.dk = (uint16_t*)dk.data_ptr(); a.dk_sb = dks[0]; a.dk_sh = dks[1]; a.dk_ss = dks[2];
  a.dv = (uint16_t*)dv.data_ptr(); a.dv_sb = dvs[0]; a.dv_sh = dvs[1]; a.dv_ss = dvs[2];
  a.lse = lse.data_ptr<float>();
  a.dq_acc = ws.data_ptr<float>();
  // layout: [nkb partial dQ slabs][delta][lse2][bias-gradient partials]
  a.delta = a.dq_acc + ffk::attn_bwd_slab_floats(B, H, Sq, Sk, D);
  a.lse2 = a.delta + (int64_t)B * H * Sq;
  if (dbias) {  // [3*H*D] fp32, accumulated into
    TORCH_CHECK(dbias->scalar_type() == at::kFloat && dbias->is_contiguous() && dbias->numel() == 3 * H * D,
                "attn_bwd: dbias must be a contiguous fp32 [3*H*D] tensor");
    a.dbp = a.lse2 + (int64_t)B * H * Sq;
    a.dbias = dbias->data_ptr<float>();
  }
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.D = D; a.scale = scale; a.causal = causal;
  return ffk::attn_bwd(a, cur_stream());
}


// ---- hipBLASLt with fused epilogues (blaslt.h)
std::tuple<int64_t, int64_t> lt_plan(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                                     int64_t batch, int64_t sA, int64_t sB, int64_t sC, bool a_k, bool b_k,
                                     bool out_f32, bool bias_f32, bool beta_nz, int64_t epi, int64_t aux_ld,
                                     int64_t max_algos, bool all_algos, int64_t max_ws, optional<Tensor> bias,
                                     optional<Tensor> aux) {
  ffk::lt::PlanKey k{M, N, K, lda, ldb, ldc, batch, sA, sB, sC, a_k, b_k, out_f32, bias_f32, beta_nz, (int)epi, aux_ld};
  int n = 0;
  int64_t id = ffk::lt::plan(k, (int)max_algos, all_algos, (size_t)max_ws, ptr(bias), ptr(aux), &n);
  return {id, n};
}

int64_t lt_run(int64_t plan, int64_t algo, Tensor A, Tensor B, Tensor C, optional<Tensor> bias, optional<Tensor> aux,
               double alpha, double beta, optional<Tensor> ws) {
  check_dev(A, "A"); check_dev(B, "B"); check_dev(C, "C");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "lt_run: A/B must be bf16");
  size_t wsb = (ws.has_value() && ws->defined()) ? (size_t)ws->numel() * ws->element_size() : 0;
  return ffk::lt::run(plan, (int)algo, A.data_ptr(), B.data_ptr(), C.data_ptr(), ptr(bias), ptr(aux), (float)alpha,
                      (float)beta, ptr(ws), wsb, cur_stream());
}


// ---- LSTM step (rnn.hip); tensors may be strided views: pointers + explicit row strides
void lstm_fwd_cell(Tensor G, int64_t ldg, Tensor c_prev, Tensor c_out, Tensor h_out, int64_t ldh, int64_t B,
                   int64_t H) {
  check_dev(G, "G");
  TORCH_CHECK(c_prev.scalar_type() == at::kFloat && c_out.scalar_type() == at::kFloat, "lstm: c must be fp32");
  TORCH_CHECK(c_prev.numel() >= B * H && c_out.numel() >= B * H, "lstm: c too small");
  TORCH_CHECK(G.scalar_type() == h_out.scalar_type(), "lstm: G / h dtype");
  ffk::lstm_fwd_cell(dtcode(G), G.data_ptr(), ldg, c_prev.data_ptr<float>(), c_out.data_ptr<float>(), h_out.data_ptr(),
                     ldh, B, H, cur_stream());
}
void lstm_bwd_cell(Tensor G, int64_t ldg, Tensor c, Tensor c_prev, optional<Tensor> dy, int64_t lddy,
                   optional<Tensor> dh_rec, Tensor dc, Tensor dG, int64_t B, int64_t H) {
  check_dev(G, "G");
  TORCH_CHECK(c.scalar_type() == at::kFloat && c_prev.scalar_type() == at::kFloat && dc.scalar_type() == at::kFloat,
              "lstm: c / dc must be fp32");
  TORCH_CHECK(dc.numel() >= B * H && c.numel() >= B * H && c_prev.numel() >= B * H, "lstm: state too small");
  ffk::lstm_bwd_cell(dtcode(G), G.data_ptr(), ldg, c.data_ptr<float>(), c_prev.data_ptr<float>(), ptr(dy), lddy,
                     ptr(dh_rec), dc.data_ptr<float>(), dG.data_ptr(), B, H, cur_stream());
}

// layout of a 4-D activation operand: NCHW-contiguous, or (nhwc) channel-last-contiguous bf16
// with C % 8 == 0
void check_layout(const Tensor& t, bool nhwc, int64_t C, const char* what) {
  if (!nhwc) {
    TORCH_CHECK(t.is_contiguous(), what, ": NCHW-contiguous tensor expected");
    return;
  }
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && C % 8 == 0, what, ": channel-last path needs bf16 and C % 8 == 0");
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast), what,
              ": channel-last-contiguous tensor expected");
}

void batchnorm_fwd(Tensor x, Tensor y, Tensor g, Tensor b, Tensor mean, Tensor rstd, Tensor run_mean,
                   Tensor run_var, Tensor ws, int64_t N, int64_t C, int64_t HW, double eps, double momentum,
                   bool training, bool relu, bool nhwc) {
  check_dev(x, "x");
  check_layout(x, nhwc, C, "batchnorm_fwd x");
  check_layout(y, nhwc, C, "batchnorm_fwd y");
  TORCH_CHECK(x.numel() == N * C * HW && y.numel() == x.numel(), "batchnorm_fwd: x/y size");
  TORCH_CHECK(g.numel() >= C && b.numel() >= C && g.scalar_type() == x.scalar_type() &&
              b.scalar_type() == x.scalar_type(), "batchnorm_fwd: scale/bias");
  TORCH_CHECK(mean.numel() >= C && rstd.numel() >= C && run_mean.numel() >= C && run_var.numel() >= C,
              "batchnorm_fwd: statistics");
  TORCH_CHECK(ws.numel() >= ffk::bn_partial_floats(N, C, HW), "batchnorm_fwd: workspace too small");
  ffk::batchnorm_fwd(dtcode(x), x.data_ptr(), y.data_ptr(), g.data_ptr(), b.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), run_mean.data_ptr<float>(), run_var.data_ptr<float>(),
                     ws.data_ptr<float>(), N, C, HW, eps, momentum, training, relu, nhwc, cur_stream());
}
void batchnorm_bwd(Tensor x, Tensor dy, Tensor g, Tensor b, Tensor mean, Tensor rstd, Tensor dx,
                   optional<Tensor> dg, optional<Tensor> db, Tensor ws, int64_t N, int64_t C, int64_t HW, bool relu,
                   bool nhwc) {
  check_dev(x, "x");
  check_layout(x, nhwc, C, "batchnorm_bwd x");
  check_layout(dy, nhwc, C, "batchnorm_bwd dy");
  check_layout(dx, nhwc, C, "batchnorm_bwd dx");
  TORCH_CHECK(x.numel() == N * C * HW && dy.numel() == x.numel() && dx.numel() == x.numel(), "batchnorm_bwd: size");
  TORCH_CHECK(ws.numel() >= ffk::bn_partial_floats(N, C, HW), "batchnorm_bwd: workspace too small");
  TORCH_CHECK(!dg.has_value() || (dg->scalar_type() == at::kFloat && dg->numel() >= C), "batchnorm_bwd: dg fp32");
  TORCH_CHECK(!db.has_value() || (db->scalar_type() == at::kFloat && db->numel() >= C), "batchnorm_bwd: db fp32");
  ffk::batchnorm_bwd(dtcode(x), x.data_ptr(), dy.data_ptr(), g.data_ptr(), b.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), dx.data_ptr(), ptr<float>(dg), ptr<float>(db), ws.data_ptr<float>(), N,
                     C, HW, relu, nhwc, cur_stream());
}
int64_t bn_ws(int64_t N, int64_t C, int64_t HW) { return ffk::bn_partial_floats(N, C, HW); }
void rmsnorm_fwd(Tensor x, Tensor w, Tensor y, Tensor rstd, int64_t rows, int64_t d, double eps) {
  check_dev(x, "x");
  TORCH_CHECK(d <= 8192, "rmsnorm: last dimension > 8192");
  TORCH_CHECK(x.is_contiguous() && x.numel() == rows * d && y.numel() == x.numel() && w.numel() == d &&
              w.scalar_type() == x.scalar_type() && rstd.numel() >= rows, "rmsnorm_fwd: shapes");
  ffk::rmsnorm_fwd(dtcode(x), x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr<float>(), rows, d, eps,
                   cur_stream());
}
void rmsnorm_bwd(Tensor x, Tensor w, Tensor dy, Tensor rstd, Tensor dx, optional<Tensor> dw, int64_t rows, int64_t d) {
  check_dev(x, "x");
  TORCH_CHECK(d <= 8192, "rmsnorm: last dimension > 8192");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous() && x.numel() == rows * d && dy.numel() == x.numel() &&
              dx.numel() == x.numel() && w.numel() == d && rstd.numel() >= rows, "rmsnorm_bwd: shapes");
  TORCH_CHECK(!dw.has_value() || (dw->scalar_type() == at::kFloat && dw->numel() >= d), "rmsnorm_bwd: dw fp32");
  ffk::rmsnorm_bwd(dtcode(x), x.data_ptr(), w.data_ptr(), dy.data_ptr(), rstd.data_ptr<float>(), dx.data_ptr(),
                   ptr<float>(dw), rows, d, cur_stream());
}
void channel_sum(Tensor dy, optional<Tensor> y, optional<Tensor> dz, optional<Tensor> db, Tensor ws, int64_t N,
                 int64_t C, int64_t HW, bool nhwc) {
  check_dev(dy, "dy");
  TORCH_CHECK(dy.numel() == N * C * HW, "channel_sum: dy");
  check_layout(dy, nhwc, C, "channel_sum dy");
  if (y.has_value()) check_layout(*y, nhwc, C, "channel_sum y");
  if (dz.has_value()) check_layout(*dz, nhwc, C, "channel_sum dz");
  TORCH_CHECK(!y.has_value() || (y->numel() == dy.numel() && y->scalar_type() == dy.scalar_type()), "channel_sum: y");
  TORCH_CHECK(!dz.has_value() || (dz->numel() == dy.numel() && dz->scalar_type() == dy.scalar_type()),
              "channel_sum: dz");
  TORCH_CHECK(!db.has_value() || (db->scalar_type() == at::kFloat && db->numel() >= C), "channel_sum: db fp32");
  TORCH_CHECK(ws.numel() >= ffk::bn_partial_floats(N, C, HW), "channel_sum: workspace too small");
  ffk::channel_sum(dtcode(dy), dy.data_ptr(), ptr(y), ptr(dz), ptr<float>(db), ws.data_ptr<float>(), N, C, HW,
                   nhwc, cur_stream());
}
std::vector<int> pool_geom(const std::vector<int64_t>& g) {
  TORCH_CHECK(g.size() == 14, "pool2d: geometry is N C H W OH OW kh kw sh sw pad_t pad_b pad_l pad_r");
  TORCH_CHECK(g[6] * g[7] <= 256, "pool2d: window larger than 256 (byte winner index)");
  TORCH_CHECK(g[8] > 0 && g[9] > 0 && g[10] < g[6] && g[12] < g[7], "pool2d: stride > 0, pad < window");
  // every output window must start inside the padded input
  TORCH_CHECK((g[4] - 1) * g[8] - g[10] < g[2] + g[11] && (g[5] - 1) * g[9] - g[12] < g[3] + g[13],
              "pool2d: output larger than the padded input");
  return std::vector<int>(g.begin(), g.end());
}
void pool2d_fwd(Tensor x, Tensor y, optional<Tensor> idx, std::vector<int64_t> g, bool is_max, bool include_pad,
                bool relu, bool nhwc) {
  check_dev(x, "x");
  const auto gi = pool_geom(g);
  check_layout(x, nhwc, g[1], "pool2d_fwd x");
  check_layout(y, nhwc, g[1], "pool2d_fwd y");
  TORCH_CHECK(x.numel() == g[0] * g[1] * g[2] * g[3] && y.numel() == g[0] * g[1] * g[4] * g[5], "pool2d_fwd: size");
  TORCH_CHECK(!idx.has_value() || idx->numel() >= y.numel(), "pool2d_fwd: idx");
  ffk::pool2d_fwd(dtcode(x), x.data_ptr(), y.data_ptr(), ptr<uint8_t>(idx), gi.data(), is_max, include_pad, relu,
                  nhwc, cur_stream());
}
void pool2d_bwd(Tensor x, optional<Tensor> y, Tensor dy, optional<Tensor> idx, Tensor dx, std::vector<int64_t> g,
                bool is_max, bool include_pad, bool relu, bool nhwc) {
  check_dev(x, "x");
  const auto gi = pool_geom(g);
  check_layout(x, nhwc, g[1], "pool2d_bwd x");
  check_layout(dy, nhwc, g[1], "pool2d_bwd dy");
  check_layout(dx, nhwc, g[1], "pool2d_bwd dx");
  if (y.has_value()) check_layout(*y, nhwc, g[1], "pool2d_bwd y");
  TORCH_CHECK(dx.numel() == x.numel() && x.numel() == g[0] * g[1] * g[2] * g[3] &&
              dy.numel() == g[0] * g[1] * g[4] * g[5], "pool2d_bwd: size");
  TORCH_CHECK(!is_max || (idx.has_value() && idx->numel() >= dy.numel()), "pool2d_bwd: max pooling needs idx");
  TORCH_CHECK(is_max || !relu || (y.has_value() && y->numel() == dy.numel()), "pool2d_bwd: avg + relu needs y");
  ffk::pool2d_bwd(dtcode(x), x.data_ptr(), ptr(y), dy.data_ptr(), ptr<uint8_t>(idx), dx.data_ptr(), gi.data(), is_max,
                  include_pad, relu, nhwc, cur_stream());
}

std::vector<int> conv_geom(const std::vector<int64_t>& g) {
  TORCH_CHECK(g.size() == 14, "conv2d: geometry is N C H W K OH OW KH KW sh sw ph pw G");
  TORCH_CHECK(g[13] >= 1 && g[1] % g[13] == 0 && g[4] % g[13] == 0, "conv2d: groups must divide C and K");
  TORCH_CHECK(g[9] > 0 && g[10] > 0 && g[11] >= 0 && g[12] >= 0, "conv2d: stride > 0, pad >= 0");
  TORCH_CHECK(g[5] == (g[2] + 2 * g[11] - g[7]) / g[9] + 1 && g[6] == (g[3] + 2 * g[12] - g[8]) / g[10] + 1,
              "conv2d: output size does not match the geometry");
  return std::vector<int>(g.begin(), g.end());
}
int64_t conv_ws(std::vector<int64_t> g) {
  const auto gi = conv_geom(g);
  return ffk::conv_ws_elems(gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[13]);
}
int64_t conv_wpack(std::vector<int64_t> g) {
  const auto gi = conv_geom(g);
  return ffk::conv_wpack_elems(gi[1], gi[4], gi[7], gi[8], gi[13]);
}
void conv2d_fwd(Tensor x, Tensor w, optional<Tensor> bias, Tensor y, Tensor ws, std::vector<int64_t> g, bool relu,
                bool x_nhwc, bool y_nhwc, optional<Tensor> wpack_bwd) {
  check_dev(x, "x");
  const auto gi = conv_geom(g);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
              "conv2d: bf16 tensors");
  TORCH_CHECK(w.is_contiguous(), "conv2d: contiguous weights");
  check_layout(x, x_nhwc, g[1] / g[13], "conv2d_fwd x");
  check_layout(y, y_nhwc, g[4] / g[13], "conv2d_fwd y");
  TORCH_CHECK(x.numel() == g[0] * g[1] * g[2] * g[3] && y.numel() == g[0] * g[4] * g[5] * g[6] &&
              w.numel() == g[4] * (g[1] / g[13]) * g[7] * g[8], "conv2d_fwd: sizes");
  TORCH_CHECK(!bias.has_value() || (bias->scalar_type() == at::kBFloat16 && bias->numel() >= g[4]), "conv2d: bias");
  TORCH_CHECK(ws.numel() * ws.element_size() >= 2 * conv_ws(g), "conv2d_fwd: workspace too small");
  TORCH_CHECK(!wpack_bwd.has_value() || (wpack_bwd->scalar_type() == at::kBFloat16 && wpack_bwd->numel() >= conv_wpack(g)),
              "conv2d_fwd: wpack_bwd");
  ffk::conv2d_fwd(x.data_ptr(), w.data_ptr(), ptr(bias), y.data_ptr(), ws.data_ptr(), gi.data(), relu, x_nhwc, y_nhwc,
                  cur_stream(), ptr(wpack_bwd));
}
void conv2d_bwd(Tensor x, Tensor w, Tensor dy, optional<Tensor> dx, optional<Tensor> dw, Tensor ws,
                std::vector<int64_t> g, bool x_nhwc, bool dy_nhwc, bool accum_dx, optional<Tensor> wpack,
                optional<Tensor> dmask, optional<Tensor> dpart) {
  check_dev(x, "x");
  const auto gi = conv_geom(g);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "conv2d: bf16 tensors");
  TORCH_CHECK(w.is_contiguous(), "conv2d: contiguous weights");
  check_layout(x, x_nhwc, g[1] / g[13], "conv2d_bwd x");
  check_layout(dy, dy_nhwc, g[4] / g[13], "conv2d_bwd dy");
  if (dx.has_value()) check_layout(*dx, x_nhwc, g[1] / g[13], "conv2d_bwd dx (x's layout)");
  TORCH_CHECK(x.numel() == g[0] * g[1] * g[2] * g[3] && dy.numel() == g[0] * g[4] * g[5] * g[6], "conv2d_bwd: sizes");
  TORCH_CHECK(!dx.has_value() || (dx->numel() == x.numel() && dx->scalar_type() == at::kBFloat16), "conv2d_bwd: dx");
  TORCH_CHECK(!dw.has_value() || (dw->numel() == w.numel() && dw->scalar_type() == at::kFloat && dw->is_contiguous()),
              "conv2d_bwd: dw must be fp32 like w");
  TORCH_CHECK(ws.numel() * ws.element_size() >= 2 * conv_ws(g), "conv2d_bwd: workspace too small");
  TORCH_CHECK(!wpack.has_value() || (wpack->scalar_type() == at::kBFloat16 && wpack->numel() >= conv_wpack(g)),
              "conv2d_bwd: wpack");
  if (dmask.has_value()) {  // the producer's channel-last output, x's geometry; the partial slab
    TORCH_CHECK(x_nhwc && dx.has_value() && !accum_dx && (g[1] / g[13]) % 8 == 0, "conv2d_bwd dmask: channel-last dx");
    TORCH_CHECK(dmask->scalar_type() == at::kBFloat16 && dmask->numel() == x.numel(), "conv2d_bwd dmask: x's size");
    check_layout(*dmask, true, g[1] / g[13], "conv2d_bwd dmask");
    TORCH_CHECK(!dpart.has_value() || (dpart->scalar_type() == at::kFloat && dpart->is_contiguous() &&
                                        dpart->numel() >= ffk::conv_dact_rows(gi.data()) * g[1]),
                "conv2d_bwd dpart: rows x C fp32");
  }
  ffk::conv2d_bwd(x.data_ptr(), w.data_ptr(), dy.data_ptr(), ptr(dx), ptr<float>(dw), ws.data_ptr(), gi.data(),
                  dx.has_value(), x_nhwc, dy_nhwc, accum_dx && dx.has_value(), cur_stream(), ptr(wpack),
                  dmask.has_value() ? dmask->data_ptr() : nullptr, dmask.has_value() ? ptr<float>(dpart) : nullptr);
}
int64_t conv_dact_rows(std::vector<int64_t> g) {
  const auto gi = conv_geom(g);
  return ffk::conv_dact_rows(gi.data());
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "flexflow_amd HIP/CDNA4 kernels (gfx950)";
  m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("Z"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("sA"), py::arg("sB"),
        py::arg("sC"), py::arg("batch"), py::arg("a_k"), py::arg("b_k"), py::arg("alpha"), py::arg("beta"),
        py::arg("act"), py::arg("splitk"), py::arg("ws"), py::arg("impl") = 2, py::arg("skip_reduce") = false);
  m.def("gemm_dact", &gemm_dact);
  m.def("box_copy", &box_copy);
  m.def("gather_fwd", &gather_fwd);
  m.def("gather_bwd", &gather_bwd);
  m.def("box_words", []() { return ffk::box_words(); });
  m.def("box_dims", []() { return ffk::box_dims(); });
  m.def("lstm_fwd_cell", &lstm_fwd_cell);
  m.def("lstm_bwd_cell", &lstm_bwd_cell);
  m.def("lt_plan", &lt_plan);
  m.def("lt_run", &lt_run);
  m.def("lt_num_algos", [](int64_t p) { return ffk::lt::num_algos(p); });
  m.def("lt_algo_index", [](int64_t p, int64_t a) { return ffk::lt::algo_index(p, (int)a); });
  m.def("lt_find_algo", [](int64_t p, int64_t sol, int64_t max_ws) { return ffk::lt::find_algo(p, (int)sol, (size_t)max_ws); });
  m.def("lt_algo_ws", [](int64_t p, int64_t a) { return (int64_t)ffk::lt::algo_ws(p, (int)a); });
  m.def("lt_algo_name", [](int64_t p, int64_t a) { return ffk::lt::algo_name(p, (int)a); });
  m.def("gemm_pick_splitk", &gemm_pick_splitk, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("batch"),
        py::arg("impl") = 2);
  m.def("unary_fwd", &unary_fwd);
  m.def("unary_bwd", &unary_bwd);
  m.def("binary_fwd", &binary_fwd);
  m.def("binary_bwd", &binary_bwd);
  m.def("cast", &cast);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("bias_act_bwd", &bias_act_bwd, py::arg("dy"), py::arg("z"), py::arg("dz"), py::arg("dbias"), py::arg("rows"),
        py::arg("cols"), py::arg("act"), py::arg("ws") = py::none(), py::arg("stage") = 0);
  m.def("bias_act_bwd_ws", &bias_act_bwd_ws);
  m.def("col_reduce_add3", [](Tensor part, c10::optional<Tensor> o0, c10::optional<Tensor> o1, c10::optional<Tensor> o2,
                              int64_t R, int64_t C) {
    TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= 3 * R * C || part.numel() >= R * C, "col_reduce_add3: part");
    auto fp = [](c10::optional<Tensor>& t) { return t ? t->data_ptr<float>() : (float*)nullptr; };
    ffk::col_reduce_add3(part.data_ptr<float>(), fp(o0), fp(o1), fp(o2), (int)R, (int)C, cur_stream());
  });
  m.def("col_reduce_set_gy", [](int64_t g) { ffk::col_reduce_set_gy((int)g); });
  m.def("col_reduce_gy", []() { return ffk::col_reduce_gy(); });
  m.def("fold_record", [](bool on) { ffk::fold_record(on); });
  m.def("fold_pending", []() { return ffk::fold_pending(); });
  m.def("fold_flush", []() { ffk::fold_flush(cur_stream()); });
  m.def("layernorm_bwd_ws", &layernorm_bwd_ws);
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("dx"), py::arg("dres"), py::arg("dgamma"), py::arg("dbeta"), py::arg("rows"),
        py::arg("cols"), py::arg("acc"), py::arg("dsum") = py::none(), py::arg("ws") = py::none(),
        py::arg("stage") = 0);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.def("softmax_xent", &softmax_xent, py::arg("logits"), py::arg("labels"), py::arg("loss"), py::arg("dlogits"),
        py::arg("rows"), py::arg("cols"), py::arg("gscale"), py::arg("acc3") = py::none());
  m.def("xent_grad", &xent_grad);
  m.def("mse_grad", &mse_grad);
  m.def("metrics_classify", &metrics_classify);
  m.def("reduce_rows", &reduce_rows);
  m.def("sgd_update", &sgd_update, py::arg("master"), py::arg("grad"), py::arg("mom"), py::arg("lowp"), py::arg("lr"),
        py::arg("momentum"), py::arg("nesterov"), py::arg("wd"), py::arg("gscale"), py::arg("max_blocks") = 0);
  m.def("sgd_sparse_rows", &sgd_sparse_rows);
  m.def("adam_update", &adam_update, py::arg("master"), py::arg("grad"), py::arg("m"), py::arg("v"), py::arg("lowp"),
        py::arg("alpha_t"), py::arg("b1"), py::arg("b2"), py::arg("wd"), py::arg("eps"), py::arg("gscale"),
        py::arg("max_blocks") = 0, py::arg("alpha_dev") = py::none());
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("init_uniform", &init_uniform);
  m.def("init_normal", &init_normal);
  m.def("fill", &fill);
  m.def("slab_sum", &slab_sum);
  m.def("concat_rows", &concat_rows);
  m.def("transpose2d", &transpose2d);
  m.def("transpose2d_batch", &transpose2d_batch);
  m.def("gemm_f32", &gemm_f32);
  m.def("causal_mask_f32", &causal_mask_f32);
  m.def("topk_fwd", &topk_fwd);
  m.def("topk_bwd", &topk_bwd);
  m.def("moe_route_ws_ints", &moe_route_ws_ints);
  m.def("moe_route", &moe_route);
  m.def("groupby_fwd", &groupby_fwd);
  m.def("groupby_bwd", &groupby_bwd);
  m.def("aggregate_fwd", &aggregate_fwd);
  m.def("aggregate_bwd", &aggregate_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd, py::arg("q"), py::arg("qs"), py::arg("k"), py::arg("ks"), py::arg("v"), py::arg("vs"),
        py::arg("o"), py::arg("os"), py::arg("dout"), py::arg("dos"), py::arg("lse"), py::arg("dq"), py::arg("dqs"),
        py::arg("dk"), py::arg("dks"), py::arg("dv"), py::arg("dvs"), py::arg("ws"), py::arg("B"), py::arg("H"),
        py::arg("Sq"), py::arg("Sk"), py::arg("D"), py::arg("scale"), py::arg("causal"),
        py::arg("dbias") = py::none());
  m.def("attn_bwd_ws", &attn_bwd_ws);
  m.def("attn_set_bwd_variant", [](int v) { ffk::attn_set_bwd_variant(v); });
  m.def("attn_fwd_variant", []() { return ffk::attn_fwd_variant(); });
  m.def("attn_set_fwd_variant", [](int v) { ffk::attn_set_fwd_variant(v); });
  m.def("attn_bwd_variant", []() { return ffk::attn_bwd_variant(); });
  m.def("attn_stagger", []() { return ffk::attn_stagger(); });
  m.def("attn_set_stagger", [](int v) { ffk::attn_set_stagger(v); });
  m.def("attn_rescale_thr", []() { return ffk::attn_rescale_thr(); });
  m.def("attn_set_rescale_thr", [](double t) { ffk::attn_set_rescale_thr((float)t); });
  m.def("batchnorm_fwd", &batchnorm_fwd);
  m.def("batchnorm_bwd", &batchnorm_bwd);
  m.def("bn_ws", &bn_ws);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("channel_sum", &channel_sum);
  m.def("pool2d_fwd", &pool2d_fwd);
  m.def("pool2d_bwd", &pool2d_bwd);
  m.def("conv_ws", &conv_ws);
  m.def("conv_wpack", &conv_wpack);
  m.def("conv2d_fwd", &conv2d_fwd);
  m.def("conv2d_bwd", &conv2d_bwd, py::arg("x"), py::arg("w"), py::arg("dy"), py::arg("dx"), py::arg("dw"),
        py::arg("ws"), py::arg("g"), py::arg("x_nhwc"), py::arg("dy_nhwc"), py::arg("accum_dx"), py::arg("wpack"),
        py::arg("dmask") = py::none(), py::arg("dpart") = py::none());
  m.def("conv_dact_rows", &conv_dact_rows);
}
