// Host-side launcher declarations of the flexflow_amd HIP kernel library. Every launcher takes raw
// device pointers and a hipStream_t so that it can be captured into a hipGraph (no allocation or
// synchronisation inside: Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ffk {

enum DType : int { DT_F32 = 0, DT_BF16 = 1 };

enum UnaryOp : int {
  U_RELU = 0, U_SIGMOID, U_TANH, U_ELU, U_GELU, U_EXP, U_SIN, U_COS, U_RSQRT, U_POW, U_IDENTITY,
  U_SCALAR_MUL, U_SCALAR_ADD, U_SCALAR_SUB, U_SCALAR_TRUEDIV, U_SCALAR_FLOORDIV, U_LOG, U_SQRT, U_NEG,
  U_LEAKY_RELU
};
enum BinaryOp : int { B_ADD = 0, B_SUB, B_MUL, B_DIV, B_MAX, B_MIN };

// elementwise.hip
void unary_fwd(int dt, const void* x, void* y, int64_t n, int op, float s, hipStream_t st);
void unary_bwd(int dt, const void* x, const void* y, const void* dy, void* dx, int64_t n, int op, float s,
               int accumulate, hipStream_t st);
void binary_fwd(int dt, const void* a, const void* b, void* c, int64_t n, int op, int ndim, const int64_t* shape,
                const int64_t* sa, const int64_t* sb, int same, hipStream_t st);
void binary_bwd(int dt, const void* a, const void* b, const void* dc, void* da, void* db, int64_t n, int op,
                int ndim, const int64_t* shape, const int64_t* sa, const int64_t* sb, int same, hipStream_t st);
void cast(int dt_in, int dt_out, const void* x, void* y, int64_t n, hipStream_t st);
void dropout_fwd(int dt, const void* x, void* y, uint8_t* mask, int64_t n, float rate, uint64_t seed,
                 uint64_t offset, hipStream_t st);
void dropout_bwd(int dt, const void* dy, const uint8_t* mask, void* dx, int64_t n, float rate, int accumulate,
                 hipStream_t st);
// dbias += colsum(dz); ws: fp32 slab of bias_act_bwd_chunks(rows, cols) * cols floats
// y = act(z + bias) (bf16, cols % 8 == 0); zout (may be z) receives z + bias when bias is given
void bias_act_fwd(const void* z, const void* bias, int bias_bf16, void* zout, void* y, int64_t rows, int cols,
                  int act, hipStream_t st);
void bias_act_bwd(int dt, const void* dy, const void* z, void* dz, float* dbias, float* ws, int rows, int cols,
                  int act, hipStream_t st, int stage = 0);
int bias_act_bwd_chunks(int rows, int cols);
void col_reduce_add(const float* part, float* out, int R, int C, hipStream_t st);
void slab_sum(const float* slabs, float* out, int64_t n, int S, float beta, hipStream_t st);
// out0 += colsum(part[0:R]); out1 += colsum(part[R:2R]) (out1 may be null)
void col_reduce_add2(const float* part, float* out0, float* out1, int R, int C, hipStream_t st);
// out_k += colsum(part[k*R:(k+1)*R]) for each non-null out_k, k < 3 (slab k at offset k*R*C)
int col_reduce_gy();
void col_reduce_set_gy(int g);
void col_reduce_add3(const float* part, float* out0, float* out1, float* out2, int R, int C, hipStream_t st);
// queue (record on) / launch (flush) the deterministic column folds, see elementwise.hip
void fold_record(bool on);
int fold_pending();
void fold_flush(hipStream_t st);
// out[c] += sum_r part[r][c] queued when recording (true), else nothing done (false)
bool fold_queue(const float* part, float* out, int R, int C, hipStream_t st);

// transfer.hip: one launch over a list of boxes (pack / unpack / local re-layout of activation
// shards); desc: device int64 [nbox][box_words()] (see transfer.hip), units of vec_bytes (copy)
// or elements of dt (add: dst += src)
void gather_fwd(int dt, int idx64, const void* x, const void* idx, void* out, int64_t n, int64_t dsz, int64_t inner,
                int64_t xd, hipStream_t st);
void gather_bwd(int dt, int idx64, const void* dy, const void* idx, float* dx, int64_t n, int64_t dsz, int64_t inner,
                int64_t xd, hipStream_t st);
constexpr int kBoxSrcs = 16;  // source tensors per launch
int box_words();
int box_dims();
void box_copy(const void* const* srcs, int nsrc, void* dst, const int64_t* desc, int nbox, int64_t max_n,
              int vec_bytes, int add, int dt, int idx32, hipStream_t st);
// out [outer][sum lens] = concat of x_i [outer][lens[i]] (units of vec_bytes; transfer.hip)
void concat_rows(const void* const* srcs, const int* lens, int nsrc, void* out, int outer, int vec_bytes,
                 hipStream_t st);
// dst [cols][rows] = src [rows][cols]^T, 2-byte elements, rows % 8 == cols % 8 == 0 (transfer.hip)
void transpose16(const void* src, void* dst, int rows, int cols, hipStream_t st);
// desc[i] = {src, dst, rows, cols, first tile} (int64, device), tiles = 64 x 64 tiles in all
void transpose16_batch(const int64_t* desc, int n, int64_t tiles, hipStream_t st);

// moe.hip: TopK and the mixture-of-experts routing (GroupBy / Aggregate / AggregateSpec), fully
// on the device. Expert tensors are passed as arrays of up to kMoeMaxExperts device pointers.
constexpr int kMoeMaxExperts = 64;
void topk_fwd(int dt, const void* x, void* vals, int* idx, int rows, int n, int k, hipStream_t st);
void topk_bwd(int dt, const void* dvals, const int* idx, void* dx, int rows, int n, int k, hipStream_t st);
int64_t moe_route_ws_ints(int L, int n);
// expert[i] (clamped id), pos[i] (row in the expert's tensor, -1 = dropped) of the L = B*k
// flattened (sample, choice) pairs in reference order; load[e] = pairs routed to e
void moe_route(const int* assign, int L, int n, int cap, int* expert, int* pos, int* load, int* ws, hipStream_t st);
void groupby_fwd(int dt, const void* data, const int* expert, const int* pos, void* const* outs, int n, int cap,
                 int L, int k, int D, hipStream_t st);
void groupby_bwd(int dt, void* const* douts, int n, const int* expert, const int* pos, void* dx, int B, int k, int D,
                 hipStream_t st);
void aggregate_fwd(int dt, const void* gate, void* const* exps, int n, const int* expert, const int* pos, void* out,
                   int B, int k, int D, hipStream_t st);
void aggregate_bwd(int dt, const void* dout, const void* gate, void* const* exps, void* const* dexps, int n,
                   int cap, const int* expert, const int* pos, const int* assign, const int* true_assign,
                   const int* load, float lambda_bal, void* dgate, void* dfull, int B, int k, int D, hipStream_t st);

// norm.hip
void layernorm_fwd(int dt, const void* x, const void* res, void* sum_out, const void* gamma, const void* beta,
                   void* y, float* mean, float* rstd, int rows, int cols, float eps, hipStream_t st);
// ws: fp32 slab of 3 * layernorm_bwd_waves(rows) * cols floats (dgamma / dbeta / dsum partials).
// dsum (optional) += colsum(dx): the bias gradient of the Linear that produced the LN input.
void layernorm_bwd(int dt, const void* dy, const void* x, const void* gamma, const float* mean, const float* rstd,
                   void* dx, const void* dres_in, float* dgamma, float* dbeta, float* dsum, float* ws, int rows,
                   int cols, int accumulate, hipStream_t st, int stage = 0);
int layernorm_bwd_waves(int rows);

// softmax.hip
void softmax_fwd(int dt, const void* x, void* y, int rows, int cols, float scale, hipStream_t st);
void softmax_bwd(int dt, const void* y, const void* dy, void* dx, int rows, int cols, float scale, int accumulate,
                 hipStream_t st);
// Fused softmax + sparse categorical cross-entropy: writes per-row loss (fp32) and dlogits = (p - onehot)*gscale.
void softmax_xent_fwd_bwd(int dt, const void* logits, const int* labels, float* loss, void* dlogits, int rows,
                          int cols, float gscale, float* acc3 /*[3] or null*/, hipStream_t st);
// Loss on already-normalised probabilities (reference semantics: loss follows a Softmax op)
void xent_grad(int dt, const void* probs, const int* labels, const void* onehot, void* dprobs, float* loss, int rows,
               int cols, float gscale, int sparse, hipStream_t st);
void mse_grad(int dt, const void* pred, const void* label, void* dpred, float* loss, int64_t n, float gscale,
              hipStream_t st);

// optimizer.hip (flat multi-tensor buffers)
// row-sparse SGD (momentum 0, no weight decay) over the rows named in idx, clearing their gradient;
// mark: int32 [rows] scratch
void sgd_sparse_rows(const int64_t* idx, int n, int64_t rows, int dim, int* mark, float* master, float* grad,
                     void* lowp, float lr, hipStream_t st);
void sgd_update(float* master, const float* grad, float* mom, void* param_lowp, int64_t n, float lr, float momentum,
                int nesterov, float wd, float gscale, hipStream_t st, int max_blocks = 0);
void adam_update(float* master, const float* grad, float* m, float* v, void* param_lowp, int64_t n, float alpha_t,
                 float beta1, float beta2, float wd, float eps, float gscale, hipStream_t st, int max_blocks = 0, const float* alpha_dev = nullptr);

// embedding.hip
void embedding_fwd(int dt, int idx64, const void* idx, const void* table, void* out, int64_t n_out_rows, int bag,
                   int dim, int64_t num_rows, int aggr_avg, hipStream_t st);
void embedding_bwd(int dt, int idx64, const void* idx, const void* dout, float* dtable, int64_t n_out_rows, int bag,
                   int dim, int64_t num_rows, int aggr_avg, hipStream_t st);

// init.hip
void init_uniform(int dt, void* out, int64_t n, float lo, float hi, uint64_t seed, int64_t offset, hipStream_t st);
void init_normal(int dt, void* out, int64_t n, float mean, float stdv, uint64_t seed, int64_t offset, hipStream_t st);
void fill(int dt, void* out, int64_t n, float v, hipStream_t st);

// attention.hip (flash attention, bf16, head_dim 64 or 128)
// q,k,v,o: [B, H, S, D] contiguous (bf16); lse: [B, H, Sq] fp32
void flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk,
                    int D, float scale, int causal, hipStream_t st);
void flash_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                    float* delta_ws, float* dq_acc, void* dq, void* dk, void* dv, int B, int H, int Sq, int Sk, int D,
                    float scale, int causal, hipStream_t st);

// reduce.hip
void reduce_rows(int dt, const void* x, void* y, int64_t outer, int64_t red, int64_t inner, int mean,
                 hipStream_t st);
void metrics_classify(int dt, const void* probs, const int* labels, int rows, int cols, float* out /*[3]*/,
                      hipStream_t st);

// rnn.hip: pointwise LSTM step (gate order i, f, g, o; G rows of stride ldg; c in fp32)
void lstm_fwd_cell(int dt, void* G, int64_t ldg, const float* c_prev, float* c_out, void* h_out, int64_t ldh, int B,
                   int H, hipStream_t st);
void lstm_bwd_cell(int dt, const void* G, int64_t ldg, const float* c, const float* c_prev, const void* dy,
                   int64_t lddy, const void* dh_rec, float* dc, void* dG, int B, int H, hipStream_t st);

// norm.hip: RMS norm over the last dimension (d <= 8192); rstd [rows] saved for the backward;
// dw (fp32) += the weight gradient
void rmsnorm_fwd(int dt, const void* x, const void* w, void* y, float* rstd, int rows, int d, float eps,
                 hipStream_t st);
void rmsnorm_bwd(int dt, const void* x, const void* w, const void* dy, const float* rstd, void* dx, float* dw,
                 int rows, int d, hipStream_t st);
// cnn.hip: batch norm (split Welford statistics, fused ReLU) and 2-D pooling of NCHW tensors, or
// (nhwc = 1: bf16, C % 8 == 0) of channel-last tensors
int bn_partial_floats(int N, int C, int HW);  // ws floats for batchnorm_fwd / batchnorm_bwd
void batchnorm_fwd(int dt, const void* x, void* y, const void* g, const void* b, float* mean, float* rstd,
                   float* run_mean, float* run_var, float* ws, int N, int C, int HW, float eps, float momentum,
                   int training, int relu, int nhwc, hipStream_t st);
void batchnorm_bwd(int dt, const void* x, const void* dy, const void* g, const void* b, const float* mean,
                   const float* rstd, void* dx, float* dg, float* db, float* ws, int N, int C, int HW, int relu,
                   int nhwc, hipStream_t st);
// db (fp32) += per-channel sum of dy; with y, dy is ReLU-masked by y > 0 (written to dz if given)
void channel_sum(int dt, const void* dy, const void* y, void* dz, float* db, float* ws, int N, int C, int HW,
                 int nhwc, hipStream_t st);
// geom: N C H W OH OW kh kw sh sw pad_top pad_bottom pad_left pad_right
void pool2d_fwd(int dt, const void* x, void* y, uint8_t* idx, const int* geom, int is_max, int include_pad, int relu,
                int nhwc, hipStream_t st);
void pool2d_bwd(int dt, const void* x, const void* y, const void* dy, const uint8_t* idx, void* dx, const int* geom,
                int is_max, int include_pad, int relu, int nhwc, hipStream_t st);

// conv.hip: bf16 convolution as implicit GEMMs on MFMA. x / y / dy / dx are NCHW or (*_nhwc = 1)
// channel-last; a channel-last operand with channels per group % 8 == 0 is read in place, others are
// staged through channel-last padded copies in ws; dx takes x's layout. geom: N C H W K OH OW KH KW
// sh sw ph pw G
int64_t conv_ws_elems(int N, int C, int H, int W, int K, int OH, int OW, int KH, int KW, int G);  // bf16 elems
// wpack_bwd (optional, conv_wpack_elems): the forward also packs the backward-data weight operand,
// which conv2d_bwd then takes as wpack instead of packing it again
int64_t conv_wpack_elems(int C, int K, int KH, int KW, int G);
void conv2d_fwd(const void* x, const void* w, const void* bias, void* y, void* ws, const int* geom, int relu,
                int x_nhwc, int y_nhwc, hipStream_t st, void* wpack_bwd = nullptr);
// accum_dx: dx +=; dmask / dpart: fused producer ReLU mask + bias-gradient partials (conv.hip
// IGemmArgs), dpart of conv_dact_rows(geom) x C floats
void conv2d_bwd(const void* x, const void* w, const void* dy, void* dx, float* dw, void* ws, const int* geom,
                int need_dx, int x_nhwc, int dy_nhwc, int accum_dx, hipStream_t st,
                const void* wpack = nullptr, const void* dmask = nullptr, float* dpart = nullptr);
int64_t conv_dact_rows(const int* geom);

}  // namespace ffk
