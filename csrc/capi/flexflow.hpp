// flexflow_amd C++ API: value-semantic FFConfig / FFModel / Tensor / optimizer classes over the
// C API (flexflow_c.h), with the reference's C++ builder names (include/flexflow/model.h:326-958:
// ff.dense, ff.conv2d, ff.pool2d, ff.split, ff.top_k, ff.group_by, ff.aggregate, ...) and enum
// values (include/flexflow/ffconst.h). Header-only; link with -lflexflow_c.
//
// Differences from the reference's C++ API, on purpose: a program is an ordinary main() (no Legion
// top_level_task / register_custom_tasks); tensors are shared handles (no Tensor* / ->); failures
// throw flexflow::Error with the runtime's message instead of asserting; dims are listed outermost
// first (batch first), as in the Python API.
#ifndef FLEXFLOW_AMD_HPP
#define FLEXFLOW_AMD_HPP

#include <chrono>
#include <iterator>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "flexflow_c.h"

namespace flexflow {

enum ActiMode { AC_MODE_NONE = 10, AC_MODE_RELU = 11, AC_MODE_SIGMOID = 12, AC_MODE_TANH = 13, AC_MODE_GELU = 14 };
enum AggrMode { AGGR_MODE_NONE = 20, AGGR_MODE_SUM = 21, AGGR_MODE_AVG = 22 };
enum PoolType { POOL_MAX = 30, POOL_AVG = 31 };
enum DataType {
  DT_BOOLEAN = 40, DT_INT32 = 41, DT_INT64 = 42, DT_HALF = 43, DT_FLOAT = 44, DT_DOUBLE = 45, DT_BF16 = 46, DT_NONE = 49
};
enum LossType {
  LOSS_CATEGORICAL_CROSSENTROPY = 50,
  LOSS_SPARSE_CATEGORICAL_CROSSENTROPY = 51,
  LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE = 52,
  LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE = 53,
  LOSS_IDENTITY = 54
};
enum CompMode { COMP_MODE_TRAINING = 70, COMP_MODE_INFERENCE = 71 };
enum MetricsType {
  METRICS_ACCURACY = 1001,
  METRICS_CATEGORICAL_CROSSENTROPY = 1002,
  METRICS_SPARSE_CATEGORICAL_CROSSENTROPY = 1004,
  METRICS_MEAN_SQUARED_ERROR = 1008,
  METRICS_ROOT_MEAN_SQUARED_ERROR = 1016,
  METRICS_MEAN_ABSOLUTE_ERROR = 1032
};

struct Error : std::runtime_error {
  explicit Error(const std::string& what) : std::runtime_error(what) {}
};

namespace detail {
inline void check(bool ok, const char* what) {
  if (!ok) throw Error(std::string(what) + ": " + flexflow_last_error());
}
// shared ownership of one C handle; the deleter is the matching *_destroy
template <typename H, void (*Destroy)(H)>
class Handle {
 public:
  Handle() = default;
  Handle(H h, const char* what) {
    check(h.impl != nullptr, what);
    p_ = std::shared_ptr<void>(h.impl, [](void* impl) {
      H x;
      x.impl = impl;
      Destroy(x);
    });
  }
  H raw() const {
    H h;
    h.impl = p_.get();
    return h;
  }
  bool valid() const { return p_ != nullptr; }

 private:
  std::shared_ptr<void> p_;
};
}  // namespace detail

class Tensor {
 public:
  Tensor() = default;
  Tensor(flexflow_tensor_t h, const char* what) : h_(h, what) {}
  flexflow_tensor_t raw() const { return h_.raw(); }
  bool valid() const { return h_.valid(); }
  int num_dims() const { return flexflow_tensor_get_num_dims(raw()); }
  std::vector<int> dims() const {  // outermost first (the C API reports Legion order)
    const int n = flexflow_tensor_get_num_dims(raw());
    const int* d = flexflow_tensor_get_dims(raw());
    detail::check(n >= 0 && d != nullptr, "Tensor::dims");
    return std::vector<int>(std::reverse_iterator<const int*>(d + n), std::reverse_iterator<const int*>(d));
  }
  int dim(int i) const {
    const auto d = dims();
    return d[i < 0 ? i + (int)d.size() : i];
  }

 private:
  detail::Handle<flexflow_tensor_t, flexflow_tensor_destroy> h_;
};

class FFConfig {
 public:
  FFConfig() : h_(flexflow_config_create(), "FFConfig") {}
  // FlexFlow flags (-b, -e, --search, --only-data-parallel, ...); unknown flags are ignored
  FFConfig(int argc, char** argv) : FFConfig() { flexflow_config_parse_args(raw(), argv + 1, argc - 1); }
  flexflow_config_t raw() const { return h_.raw(); }
  int batch_size() const { return flexflow_config_get_batch_size(raw()); }
  void set_batch_size(int b) { flexflow_config_set_batch_size(raw(), b); }
  int epochs() const { return flexflow_config_get_epochs(raw()); }
  int workers_per_node() const { return flexflow_config_get_workers_per_node(raw()); }
  int num_nodes() const { return flexflow_config_get_num_nodes(raw()); }

 private:
  detail::Handle<flexflow_config_t, flexflow_config_destroy> h_;
};

class FFModel;

class Optimizer {
 public:
  flexflow_optimizer_t raw() const {
    flexflow_optimizer_t o;
    o.impl = h_.raw().impl;
    return o;
  }
  // the typed C handles share one implementation (a Python optimizer object), so the SGD entry
  // points serve both kinds here
  void set_learning_rate(double lr) { flexflow_sgd_optimizer_set_lr(h_.raw(), lr); }

 protected:
  template <typename H>
  Optimizer(H h, const char* what) : h_(as_sgd(h.impl), what) {}

 private:
  static flexflow_sgd_optimizer_t as_sgd(void* impl) {
    flexflow_sgd_optimizer_t s;
    s.impl = impl;
    return s;
  }
  detail::Handle<flexflow_sgd_optimizer_t, flexflow_sgd_optimizer_destroy> h_;
};

// weight initializers (reference include/flexflow/initializer.h); a default-constructed one is the
// op's default initializer
class Initializer {
 public:
  Initializer() = default;
  flexflow_initializer_t raw() const {
    flexflow_initializer_t i;
    i.impl = h_.valid() ? h_.raw().impl : nullptr;
    return i;
  }

 protected:
  template <typename H>
  Initializer(H h, const char* what) : h_(as_generic(h.impl), what) {}

 private:
  static flexflow_norm_initializer_t as_generic(void* impl) {
    flexflow_norm_initializer_t n;
    n.impl = impl;
    return n;
  }
  detail::Handle<flexflow_norm_initializer_t, flexflow_norm_initializer_destroy> h_;
};
struct GlorotUniformInitializer : Initializer {
  explicit GlorotUniformInitializer(int seed) : Initializer(flexflow_glorot_uniform_initializer_create(seed), "glorot") {}
};
struct ZeroInitializer : Initializer {
  ZeroInitializer() : Initializer(flexflow_zero_initializer_create(), "zero") {}
};
struct UniformInitializer : Initializer {
  UniformInitializer(int seed, float mn, float mx)
      : Initializer(flexflow_uniform_initializer_create(seed, mn, mx), "uniform") {}
};
struct NormInitializer : Initializer {
  NormInitializer(int seed, float mean, float stddev)
      : Initializer(flexflow_norm_initializer_create(seed, mean, stddev), "norm") {}
};

class FFModel {
 public:
  explicit FFModel(const FFConfig& cfg) : config_(cfg), h_(flexflow_model_create(cfg.raw()), "FFModel") {}
  flexflow_model_t raw() const { return h_.raw(); }
  const FFConfig& config() const { return config_; }

  // ------------------------------------------------------------------ tensors
  Tensor create_tensor(const std::vector<int>& dims, DataType dt = DT_FLOAT, bool create_grad = true) {
    return Tensor(flexflow_tensor_create(raw(), (int)dims.size(), dims.data(), dt, create_grad), "create_tensor");
  }
  void set_tensor(const Tensor& t, const std::vector<float>& v) {
    detail::check(flexflow_tensor_set_data_float(t.raw(), raw(), v.data(), (int64_t)v.size()), "set_tensor");
  }
  void set_tensor(const Tensor& t, const std::vector<int32_t>& v) {
    detail::check(flexflow_tensor_set_data_int(t.raw(), raw(), v.data(), (int64_t)v.size()), "set_tensor");
  }
  void set_tensor(const Tensor& t, const std::vector<int64_t>& v) {
    detail::check(flexflow_tensor_set_data_int64(t.raw(), raw(), v.data(), (int64_t)v.size()), "set_tensor");
  }
  std::vector<float> get_tensor(const Tensor& t) {
    int64_t n = 1;
    for (int d : t.dims()) n *= d;
    std::vector<float> v((size_t)n);
    detail::check(flexflow_tensor_get_data_float(t.raw(), raw(), v.data(), n), "get_tensor");
    return v;
  }
  Tensor label_tensor() { return Tensor(flexflow_model_get_label_tensor(raw()), "label_tensor"); }

  // ------------------------------------------------------------------ layers
  Tensor dense(const Tensor& x, int out_dim, ActiMode act = AC_MODE_NONE, bool use_bias = true,
               const char* name = nullptr, const Initializer& kernel_init = Initializer(),
               const Initializer& bias_init = Initializer()) {
    return Tensor(flexflow_model_add_dense(raw(), x.raw(), out_dim, act, use_bias, DT_FLOAT, no_op(), kernel_init.raw(),
                                           bias_init.raw(), 17 /* REG_MODE_NONE */, 0.f, name),
                  "dense");
  }
  Tensor conv2d(const Tensor& x, int out_channels, int kh, int kw, int sh, int sw, int ph, int pw,
                ActiMode act = AC_MODE_NONE, int groups = 1, bool use_bias = true, const char* name = nullptr,
                const Initializer& kernel_init = Initializer(), const Initializer& bias_init = Initializer()) {
    return Tensor(flexflow_model_add_conv2d(raw(), x.raw(), out_channels, kh, kw, sh, sw, ph, pw, act, groups,
                                            use_bias, no_op(), kernel_init.raw(), bias_init.raw(), name),
                  "conv2d");
  }
  Tensor pool2d(const Tensor& x, int kh, int kw, int sh, int sw, int ph, int pw, PoolType type = POOL_MAX,
                ActiMode act = AC_MODE_NONE, const char* name = nullptr) {
    return Tensor(flexflow_model_add_pool2d(raw(), x.raw(), kh, kw, sh, sw, ph, pw, type, act, name), "pool2d");
  }
  Tensor batch_norm(const Tensor& x, bool relu = true, const char* name = nullptr) {
    return Tensor(flexflow_model_add_batch_norm(raw(), x.raw(), relu, name), "batch_norm");
  }
  Tensor layer_norm(const Tensor& x, const std::vector<int>& axes, bool affine = true, float eps = 1e-5f,
                    const char* name = nullptr) {
    std::vector<int> a(axes);
    return Tensor(flexflow_model_add_layer_norm(raw(), x.raw(), (int)a.size(), a.data(), affine, eps, name),
                  "layer_norm");
  }
  Tensor rms_norm(const Tensor& x, float eps = 1e-6f, const char* name = nullptr) {
    return Tensor(flexflow_model_add_rms_norm(raw(), x.raw(), eps, name), "rms_norm");
  }
  Tensor embedding(const Tensor& x, int num_entries, int out_dim, AggrMode aggr = AGGR_MODE_NONE,
                   DataType dt = DT_FLOAT, const char* name = nullptr) {
    return Tensor(flexflow_model_add_embedding_typed(raw(), x.raw(), num_entries, out_dim, aggr, dt, name),
                  "embedding");
  }
  Tensor multihead_attention(const Tensor& q, const Tensor& k, const Tensor& v, int embed_dim, int num_heads,
                             int kdim = 0, int vdim = 0, float dropout = 0.f, bool bias = true,
                             const char* name = nullptr) {
    return Tensor(flexflow_model_add_multihead_attention(raw(), q.raw(), k.raw(), v.raw(), embed_dim, num_heads,
                                                         kdim, vdim, dropout, bias, false, false,
                                                         Initializer().raw(), name),
                  "multihead_attention");
  }
  Tensor batch_matmul(const Tensor& a, const Tensor& b, int a_seq_length_dim = -1, int b_seq_length_dim = -1) {
    return Tensor(flexflow_model_add_batch_matmul(raw(), a.raw(), b.raw(), a_seq_length_dim, b_seq_length_dim),
                  "batch_matmul");
  }
  Tensor flat(const Tensor& x, const char* name = nullptr) {
    return Tensor(flexflow_model_add_flat(raw(), x.raw(), name), "flat");
  }
  Tensor softmax(const Tensor& x, int axis = -1, const char* name = nullptr) {
    return Tensor(flexflow_model_add_softmax(raw(), x.raw(), axis, name), "softmax");
  }
  Tensor dropout(const Tensor& x, float rate, unsigned long long seed = 0, const char* name = nullptr) {
    return Tensor(flexflow_model_add_dropout(raw(), x.raw(), rate, seed, name), "dropout");
  }
  Tensor reshape(const Tensor& x, const std::vector<int>& shape, const char* name = nullptr) {
    std::vector<int> v(shape);
    return Tensor(flexflow_model_add_reshape(raw(), x.raw(), (int)v.size(), v.data(), name), "reshape");
  }
  Tensor transpose(const Tensor& x, const std::vector<int>& perm, const char* name = nullptr) {
    std::vector<int> v(perm);
    return Tensor(flexflow_model_add_transpose(raw(), x.raw(), (int)v.size(), v.data(), name), "transpose");
  }
  Tensor concat(const std::vector<Tensor>& xs, int axis, const char* name = nullptr) {
    auto r = raws(xs);
    return Tensor(flexflow_model_add_concat(raw(), (int)r.size(), r.data(), axis, name), "concat");
  }
  std::vector<Tensor> split(const Tensor& x, const std::vector<int>& sizes, int axis, const char* name = nullptr) {
    std::vector<flexflow_tensor_t> out(sizes.size());
    std::vector<int> v(sizes);
    for (auto& o : out) o.impl = nullptr;
    flexflow_model_add_split(raw(), x.raw(), (int)v.size(), out.data(), v.data(), axis, name);
    return adopt(out, out.empty() || out.back().impl ? (int)out.size() : -1, "split");
  }
  Tensor mean(const Tensor& x, const std::vector<int>& dims, bool keepdims = false, const char* name = nullptr) {
    std::vector<int> v(dims);
    return Tensor(flexflow_model_add_mean(raw(), x.raw(), v.data(), (int)v.size(), keepdims, name), "mean");
  }
  Tensor reduce_sum(const Tensor& x, const std::vector<int>& axes, bool keepdims = false,
                    const char* name = nullptr) {
    std::vector<int> v(axes);
    return Tensor(flexflow_model_add_reduce_sum(raw(), x.raw(), v.data(), (int)v.size(), keepdims, name),
                  "reduce_sum");
  }
  Tensor gather(const Tensor& x, const Tensor& index, int dim, const char* name = nullptr) {
    return Tensor(flexflow_model_add_gather(raw(), x.raw(), index.raw(), dim, name), "gather");
  }
  Tensor cast(const Tensor& x, DataType dt, const char* name = nullptr) {
    return Tensor(flexflow_model_add_cast(raw(), x.raw(), dt, name), "cast");
  }
  Tensor reverse(const Tensor& x, int axis, const char* name = nullptr) {
    return Tensor(flexflow_model_add_reverse(raw(), x.raw(), axis, name), "reverse");
  }
  // mixture of experts: top_k -> {values, indices}; group_by -> n expert batches
  std::vector<Tensor> top_k(const Tensor& x, int k, bool sorted = false, const char* name = nullptr) {
    std::vector<flexflow_tensor_t> out(2);
    return adopt(out, flexflow_model_add_top_k(raw(), x.raw(), k, sorted, out.data(), name), "top_k");
  }
  std::vector<Tensor> group_by(const Tensor& data, const Tensor& assign, int n, float alpha,
                               const char* name = nullptr) {
    std::vector<flexflow_tensor_t> out(n);
    return adopt(out, flexflow_model_add_group_by(raw(), data.raw(), assign.raw(), n, alpha, out.data(), name),
                 "group_by");
  }
  Tensor aggregate(const std::vector<Tensor>& xs, int n, float lambda_bal, const char* name = nullptr) {
    const auto r = raws(xs);
    return Tensor(flexflow_model_add_aggregate(raw(), (int)r.size(), r.data(), n, lambda_bal, name), "aggregate");
  }
  Tensor aggregate_spec(const std::vector<Tensor>& xs, int n, float lambda_bal, const char* name = nullptr) {
    const auto r = raws(xs);
    return Tensor(flexflow_model_add_aggregate_spec(raw(), (int)r.size(), r.data(), n, lambda_bal, name),
                  "aggregate_spec");
  }
  Tensor moe(const Tensor& x, int num_exp, int num_select, int expert_hidden_size, float alpha, float lambda_bal) {
    return Tensor(flexflow_model_add_moe(raw(), x.raw(), num_exp, num_select, expert_hidden_size, alpha, lambda_bal),
                  "moe");
  }

#define FF_UNARY(fn)                                                         \
  Tensor fn(const Tensor& x, const char* name = nullptr) {                   \
    return Tensor(flexflow_model_add_##fn(raw(), x.raw(), name), #fn);      \
  }
  FF_UNARY(gelu)
  FF_UNARY(sigmoid)
  FF_UNARY(tanh)
  FF_UNARY(identity)
  FF_UNARY(exp)
  FF_UNARY(sin)
  FF_UNARY(cos)
  FF_UNARY(rsqrt)
#undef FF_UNARY
  Tensor relu(const Tensor& x, const char* name = nullptr) {
    return Tensor(flexflow_model_add_relu(raw(), x.raw(), false, name), "relu");
  }
  Tensor elu(const Tensor& x, const char* name = nullptr) {
    return Tensor(flexflow_model_add_elu(raw(), x.raw(), false, name), "elu");
  }
#define FF_BINARY(fn)                                                                    \
  Tensor fn(const Tensor& a, const Tensor& b, const char* name = nullptr) {              \
    return Tensor(flexflow_model_add_##fn(raw(), a.raw(), b.raw(), false, name), #fn);  \
  }
  FF_BINARY(add)
  FF_BINARY(subtract)
  FF_BINARY(multiply)
  FF_BINARY(divide)
  FF_BINARY(max)
  FF_BINARY(min)
#undef FF_BINARY
  Tensor scalar_multiply(const Tensor& x, float s, const char* name = nullptr) {
    return Tensor(flexflow_model_add_scalar_multiply(raw(), x.raw(), s, false, name), "scalar_multiply");
  }
  Tensor scalar_add(const Tensor& x, float s, const char* name = nullptr) {
    return Tensor(flexflow_model_add_scalar_add(raw(), x.raw(), s, false, name), "scalar_add");
  }
  Tensor pow(const Tensor& x, float e, const char* name = nullptr) {
    return Tensor(flexflow_model_add_pow(raw(), x.raw(), e, name), "pow");
  }

  // ------------------------------------------------------------------ training
  void compile(const Optimizer& opt, LossType loss, const std::vector<MetricsType>& metrics,
               CompMode mode = COMP_MODE_TRAINING) {
    flexflow_model_set_optimizer(raw(), opt.raw());
    std::vector<int> m(metrics.begin(), metrics.end());
    flexflow_model_compile(raw(), loss, m.data(), (int)m.size(), mode);
    detail::check(flexflow_model_get_num_layers(raw()) >= 0, "compile");
  }
  void init_operators() { flexflow_model_init_layers(raw()); }
  void forward() { flexflow_model_forward(raw(), -1); }
  void backward() { flexflow_model_backward(raw(), -1); }
  void update() { flexflow_model_update(raw()); }
  void zero_gradients() { flexflow_model_zero_gradients(raw()); }
  void reset_metrics() { flexflow_model_reset_metrics(raw()); }
  void compute_metrics() { flexflow_model_compute_metrics(raw()); }
  // forward + zero_gradients + backward + update, replayed as one captured HIP graph when enabled
  void train_step() { flexflow_model_train_step(raw()); }
  float accuracy() { return flexflow_model_get_accuracy(raw()); }  // reads back: waits for the device
  float loss() { return flexflow_model_get_loss(raw()); }
  void print_layers(int id = -1) { flexflow_model_print_layers(raw(), id); }
  int num_layers() { return flexflow_model_get_num_layers(raw()); }
  std::string strategy_name() { return flexflow_model_get_strategy_name(raw()); }

 private:
  static flexflow_op_t no_op() {
    flexflow_op_t o;
    o.impl = nullptr;
    return o;
  }
  static std::vector<flexflow_tensor_t> raws(const std::vector<Tensor>& xs) {
    std::vector<flexflow_tensor_t> r;
    r.reserve(xs.size());
    for (const auto& x : xs) r.push_back(x.raw());
    return r;
  }
  static std::vector<Tensor> adopt(const std::vector<flexflow_tensor_t>& hs, int n, const char* what) {
    detail::check(n >= 0, what);
    std::vector<Tensor> out;
    for (int i = 0; i < n; ++i) out.emplace_back(hs[i], what);
    return out;
  }

  FFConfig config_;
  detail::Handle<flexflow_model_t, flexflow_model_destroy> h_;
};

class SGDOptimizer : public Optimizer {
 public:
  explicit SGDOptimizer(const FFModel& m, double lr = 0.01, double momentum = 0.0, bool nesterov = false,
                        double weight_decay = 0.0)
      : Optimizer(flexflow_sgd_optimizer_create(m.raw(), lr, momentum, nesterov, weight_decay), "SGDOptimizer") {}
};

class AdamOptimizer : public Optimizer {
 public:
  explicit AdamOptimizer(const FFModel& m, double alpha = 0.001, double beta1 = 0.9, double beta2 = 0.999,
                         double weight_decay = 0.0, double epsilon = 1e-8)
      : Optimizer(flexflow_adam_optimizer_create(m.raw(), alpha, beta1, beta2, weight_decay, epsilon),
                  "AdamOptimizer") {}
};

// wall-clock microseconds (reference Realm::Clock::current_time_in_microseconds)
inline double current_time_in_microseconds() {
  using namespace std::chrono;
  return (double)duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace flexflow

#endif
