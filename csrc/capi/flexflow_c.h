/* flexflow_amd C API. Source-compatible with the reference's include/flexflow/flexflow_c.h: the same
 * 144 entry points with the same parameter lists, opaque handles over FFConfig / FFModel / Tensor /
 * Op / optimizers / initializers / data loaders / metrics, plus the extensions at the end (layers
 * the reference reaches only from Python: MoE, top-k, group-by, aggregate, RMS norm, cast).
 *
 * Implemented in flexflow_c.cc by an embedded CPython runtime that drives the flexflow_amd package,
 * so C and C++ programs build, train and query models with the same strategy search, HIP kernels
 * and RCCL collectives as the Python API. Enum arguments take the reference's numeric values
 * (flexflow_amd/type.py). A failing call prints the error to stderr and returns a null handle
 * (false, -1, or leaves outputs untouched); flexflow_last_error() reports the message.
 *
 * Semantics that differ from the Legion-based reference, by design:
 *   - `inplace` flags of element-wise builders are accepted and ignored: the executor plans
 *     in-place execution itself (runtime/executor.py _plan_inplace);
 *   - flexflow_tensor_inline_map() copies the tensor's value into a host buffer owned by the
 *     handle; raw pointers stay valid until flexflow_tensor_inline_unmap(), which writes the buffer
 *     back into an input / label tensor (weights: use flexflow_parameter_set_weights_float);
 *   - flexflow_tensor_attach_raw_ptr() makes a host array the tensor's value without a copy
 *     (read at every compile / feed); column_major = true is rejected;
 *   - flexflow_tensor_get_dims() returns dims innermost-first (Legion order, as the reference);
 *     flexflow_tensor_get_dim(t, legion_axis) indexes that order;
 *   - begin/end_trace delimit a hipGraph-captured region (runtime/graph.py) instead of a Legion
 *     trace; flexflow_perform_registration() is a no-op (there are no Legion tasks). */
#ifndef FLEXFLOW_AMD_C_H
#define FLEXFLOW_AMD_C_H
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FF_AMD_HANDLE(T) typedef struct T { void* impl; } T
FF_AMD_HANDLE(flexflow_config_t);
FF_AMD_HANDLE(flexflow_model_t);
FF_AMD_HANDLE(flexflow_tensor_t);
FF_AMD_HANDLE(flexflow_parallel_tensor_t);
FF_AMD_HANDLE(flexflow_sgd_optimizer_t);
FF_AMD_HANDLE(flexflow_adam_optimizer_t);
FF_AMD_HANDLE(flexflow_initializer_t);
FF_AMD_HANDLE(flexflow_glorot_uniform_initializer_t);
FF_AMD_HANDLE(flexflow_zero_initializer_t);
FF_AMD_HANDLE(flexflow_uniform_initializer_t);
FF_AMD_HANDLE(flexflow_norm_initializer_t);
FF_AMD_HANDLE(flexflow_op_t);
FF_AMD_HANDLE(flexflow_perf_metrics_t);
FF_AMD_HANDLE(flexflow_net_config_t);
FF_AMD_HANDLE(flexflow_dlrm_config_t);
FF_AMD_HANDLE(flexflow_dataloader_4d_t);
FF_AMD_HANDLE(flexflow_dataloader_2d_t);
FF_AMD_HANDLE(flexflow_single_dataloader_t);
#undef FF_AMD_HANDLE
typedef flexflow_tensor_t flexflow_parameter_t;
/* a generic optimizer handle (either kind) for flexflow_model_set_optimizer */
typedef struct flexflow_optimizer_t { void* impl; } flexflow_optimizer_t;

int flexflow_initialize(void); /* idempotent; called implicitly by every entry point */
const char* flexflow_last_error(void);

/* ------------------------------------------------------------------ FFConfig */
flexflow_config_t flexflow_config_create(void);
void flexflow_config_destroy(flexflow_config_t handle);
void flexflow_config_parse_args(flexflow_config_t handle, char** argv, int argc);
void flexflow_config_parse_args_default(flexflow_config_t handle); /* the process's own argv */
int flexflow_config_get_batch_size(flexflow_config_t handle);
int flexflow_config_get_workers_per_node(flexflow_config_t handle);
int flexflow_config_get_num_nodes(flexflow_config_t handle);
int flexflow_config_get_epochs(flexflow_config_t handle);
bool flexflow_config_get_enable_control_replication(flexflow_config_t handle);
int flexflow_config_get_python_data_loader_type(flexflow_config_t handle);

/* ------------------------------------------------------------------ FFModel */
flexflow_model_t flexflow_model_create(flexflow_config_t config);
void flexflow_model_destroy(flexflow_model_t handle);
void flexflow_model_reset_metrics(flexflow_model_t handle);
void flexflow_model_init_layers(flexflow_model_t handle);
void flexflow_model_prefetch(flexflow_model_t handle);
void flexflow_model_forward(flexflow_model_t handle, int seq_length);
void flexflow_model_backward(flexflow_model_t handle, int seq_length);
void flexflow_model_compute_metrics(flexflow_model_t handle);
void flexflow_model_update(flexflow_model_t handle);
void flexflow_model_compile(flexflow_model_t handle, int loss_type, int* metrics, int nb_metrics, int comp_mode);
flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t handle);
void flexflow_model_zero_gradients(flexflow_model_t handle);

flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
flexflow_tensor_t flexflow_model_add_add(flexflow_model_t handle, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t handle, const flexflow_tensor_t x,
                                              const flexflow_tensor_t y, bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t handle, const flexflow_tensor_t x,
                                              const flexflow_tensor_t y, bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t handle, const flexflow_tensor_t x,
                                            const flexflow_tensor_t y, bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_max(flexflow_model_t handle, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_min(flexflow_model_t handle, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool inplace_a, const char* name);
flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t handle, const flexflow_tensor_t input, int* axes, int n,
                                                bool keepdims, const char* name);
flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t handle, const flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t handle, const flexflow_tensor_t input, const float exponent,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t handle, const flexflow_tensor_t input, int* dims, int n,
                                          bool keepdims, const char* name);
flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t handle, const flexflow_tensor_t input, int out_channels,
                                            int kernel_h, int kernel_w, int stride_h, int stride_w, int padding_h,
                                            int padding_w, int activation, int groups, bool use_bias,
                                            flexflow_op_t shared_op, flexflow_initializer_t kernel_initializer,
                                            flexflow_initializer_t bias_initializer, const char* name);
flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t handle, const flexflow_tensor_t input, int num_entries,
                                               int out_dim, int aggr, flexflow_op_t shared_op,
                                               flexflow_initializer_t kernel_initializer, const char* name);
flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t handle, flexflow_tensor_t input, int kernel_h,
                                            int kernel_w, int stride_h, int stride_w, int padding_h, int padding_w,
                                            int type, int activation, const char* name);
flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t handle, const flexflow_tensor_t input, bool relu,
                                                const char* name);
flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t handle, const flexflow_tensor_t input, int n,
                                                int* axes, bool elementwise_affine, float eps, const char* name);
flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t handle, const flexflow_tensor_t a,
                                                  const flexflow_tensor_t b, int a_seq_length_dim,
                                                  int b_seq_length_dim);
flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t handle, const flexflow_tensor_t input, int out_dim,
                                           int activation, bool use_bias, int data_type, flexflow_op_t shared_op,
                                           flexflow_initializer_t kernel_initializer,
                                           flexflow_initializer_t bias_initializer, int kernel_reg_type,
                                           float kernel_reg_lambda, const char* name);
flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t handle, int n, flexflow_tensor_t* input, int axis,
                                            const char* name);
void flexflow_model_add_split(flexflow_model_t handle, flexflow_tensor_t input, int n, flexflow_tensor_t* outputs,
                              int* split, int axis, const char* name);
flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t handle, const flexflow_tensor_t input,
                                            const flexflow_tensor_t index, int dim, const char* name);
flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t handle, const flexflow_tensor_t input, int dim,
                                             const char* name);
flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t handle, const flexflow_tensor_t input, int n, int* perm,
                                               const char* name);
flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t handle, const flexflow_tensor_t input, int n, int* shape,
                                             const char* name);
flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t handle, const flexflow_tensor_t input, int axis,
                                             const char* name);
flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t handle, const flexflow_tensor_t input, bool inplace,
                                          const char* name);
flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t handle, const flexflow_tensor_t input,
                                                     const float scalar, bool inplace, const char* name);
flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t handle, const flexflow_tensor_t input,
                                                const float scalar, bool inplace, const char* name);
flexflow_tensor_t flexflow_model_add_scalar_sub(flexflow_model_t handle, const flexflow_tensor_t input,
                                                const float scalar, bool inplace, const char* name);
flexflow_tensor_t flexflow_model_add_scalar_truediv(flexflow_model_t handle, const flexflow_tensor_t input,
                                                    const float scalar, bool inplace, const char* name);
flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t handle, const flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t handle, const flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t handle, const flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t handle, const flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t handle, const flexflow_tensor_t input, bool inplace,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t handle, const flexflow_tensor_t input, float rate,
                                             unsigned long long seed, const char* name);
flexflow_tensor_t flexflow_model_add_multihead_attention(flexflow_model_t handle, const flexflow_tensor_t query,
                                                         const flexflow_tensor_t key, const flexflow_tensor_t value,
                                                         int embed_dim, int num_heads, int kdim, int vdim,
                                                         float dropout, bool bias, bool add_bias_kv,
                                                         bool add_zero_attn, flexflow_initializer_t kernel_initializer,
                                                         const char* name);
void flexflow_model_set_sgd_optimizer(flexflow_model_t handle, flexflow_sgd_optimizer_t optimizer);
void flexflow_model_set_adam_optimizer(flexflow_model_t handle, flexflow_adam_optimizer_t optimizer);
void flexflow_model_print_layers(flexflow_model_t handle, int id);
flexflow_op_t flexflow_model_get_layer_by_id(flexflow_model_t handle, int layer_id);
flexflow_op_t flexflow_model_get_last_layer(flexflow_model_t handle);
flexflow_tensor_t flexflow_model_get_parameter_by_id(flexflow_model_t handle, int layer_id);
flexflow_perf_metrics_t flexflow_model_get_perf_metrics(flexflow_model_t handle);

/* ------------------------------------------------------------------ Tensor */
flexflow_tensor_t flexflow_tensor_create(flexflow_model_t model, int num_dims, const int* dims, int data_type,
                                         bool create_grad);
void flexflow_tensor_map(flexflow_model_t model, flexflow_tensor_t tensor, flexflow_op_t op);
flexflow_tensor_t flexflow_constant_create(flexflow_model_t model, int num_dims, const int* dims, float value,
                                           int data_type);
void flexflow_tensor_destroy(flexflow_tensor_t handle);
void flexflow_tensor_inline_map(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
void flexflow_tensor_inline_unmap(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
float* flexflow_tensor_get_raw_ptr_float(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
int32_t* flexflow_tensor_get_raw_ptr_int32(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
int flexflow_tensor_get_num_dims(flexflow_tensor_t handle);
int flexflow_tensor_get_dim(flexflow_tensor_t handle, int legion_axis);
int* flexflow_tensor_get_dims(flexflow_tensor_t handle); /* innermost first; valid while the handle lives */
int flexflow_tensor_get_data_type(flexflow_tensor_t handle);
flexflow_op_t flexflow_tensor_get_owner_op(flexflow_tensor_t handle);
void flexflow_tensor_attach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config,
                                    void* raw_ptr, bool column_major);
void flexflow_tensor_detach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
bool flexflow_tensor_is_mapped(flexflow_tensor_t handle);
bool flexflow_tensor_set_tensor_float(flexflow_tensor_t handle, flexflow_model_t model, int num_dim, int* dims,
                                      const float* data);
bool flexflow_tensor_get_tensor_float(flexflow_tensor_t handle, flexflow_model_t model, float* data,
                                      bool get_gradients);
bool flexflow_tensor_set_tensor_int(flexflow_tensor_t handle, flexflow_model_t model, int num_dim, int* dims,
                                    const int* data);
bool flexflow_tensor_get_tensor_int(flexflow_tensor_t handle, flexflow_model_t model, int* data, bool get_gradients);
bool flexflow_tensor_set_tensor_int64(flexflow_tensor_t handle, flexflow_model_t model, int num_dim, int* dims,
                                      const int64_t* data, int comm_type);
bool flexflow_tensor_get_tensor_int64(flexflow_tensor_t handle, flexflow_model_t model, int64_t* data,
                                      bool get_gradients);
bool flexflow_model_get_output_tensor_float(flexflow_model_t model, flexflow_tensor_t handle, float* data,
                                            bool get_gradients);

/* ------------------------------------------------------------------ Parameter */
bool flexflow_parameter_set_weights_float(flexflow_parameter_t handle, flexflow_model_t model, int num_dim, int* dims,
                                          const float* data);
bool flexflow_parameter_get_weights_float(flexflow_parameter_t handle, flexflow_model_t model, float* data);

/* ------------------------------------------------------------------ optimizers */
flexflow_sgd_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t model, double lr, double momentum,
                                                       bool nesterov, double weight_decay);
void flexflow_sgd_optimizer_destroy(flexflow_sgd_optimizer_t handle);
void flexflow_sgd_optimizer_set_lr(flexflow_sgd_optimizer_t handle, double lr);
flexflow_adam_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t model, double alpha, double beta1,
                                                         double beta2, double weight_decay, double epsilon);
void flexflow_adam_optimizer_destroy(flexflow_adam_optimizer_t handle);
void flexflow_adam_optimizer_set_lr(flexflow_adam_optimizer_t handle, double lr);

/* ------------------------------------------------------------------ initializers */
flexflow_initializer_t flexflow_initializer_create_null(void);
flexflow_glorot_uniform_initializer_t flexflow_glorot_uniform_initializer_create(int seed);
void flexflow_glorot_uniform_initializer_destroy(flexflow_glorot_uniform_initializer_t handle);
flexflow_zero_initializer_t flexflow_zero_initializer_create(void);
void flexflow_zero_initializer_destroy(flexflow_zero_initializer_t handle);
flexflow_uniform_initializer_t flexflow_uniform_initializer_create(int seed, float min, float max);
void flexflow_uniform_initializer_destroy(flexflow_uniform_initializer_t handle);
flexflow_norm_initializer_t flexflow_norm_initializer_create(int seed, float mean, float stddev);
void flexflow_norm_initializer_destroy(flexflow_norm_initializer_t handle);
/* the typed initializer handles convert to the generic one the builders take */
#define FF_AS_INITIALIZER(h) ((flexflow_initializer_t){(h).impl})

/* ------------------------------------------------------------------ PerfMetrics */
void flexflow_per_metrics_destroy(flexflow_perf_metrics_t handle);
float flexflow_per_metrics_get_accuracy(flexflow_perf_metrics_t handle);

/* ------------------------------------------------------------------ example configs */
flexflow_net_config_t flexflow_net_config_create(void);
void flexflow_net_config_destroy(flexflow_net_config_t handle);
const char* flexflow_net_config_get_dataset_path(flexflow_net_config_t handle);
flexflow_dlrm_config_t flexflow_dlrm_config_create(void);
void flexflow_dlrm_config_destroy(flexflow_dlrm_config_t handle);
const char* flexflow_dlrm_config_get_dataset_path(flexflow_dlrm_config_t handle);
const char* flexflow_dlrm_config_get_arch_interaction_op(flexflow_dlrm_config_t handle);
int flexflow_dlrm_config_get_sparse_feature_size(flexflow_dlrm_config_t handle);
int flexflow_dlrm_config_get_sigmoid_bot(flexflow_dlrm_config_t handle);
int flexflow_dlrm_config_get_sigmoid_top(flexflow_dlrm_config_t handle);
int flexflow_dlrm_config_get_embedding_bag_size(flexflow_dlrm_config_t handle);
float flexflow_dlrm_config_get_loss_threshold(flexflow_dlrm_config_t handle);
/* arrays: element 0 is the count, elements 1..count the values (reference layout) */
int* flexflow_dlrm_config_get_mlp_bot(flexflow_dlrm_config_t handle);
int* flexflow_dlrm_config_get_mlp_top(flexflow_dlrm_config_t handle);
int* flexflow_dlrm_config_get_embedding_size(flexflow_dlrm_config_t handle);

/* ------------------------------------------------------------------ SingleDataLoader */
flexflow_single_dataloader_t flexflow_single_dataloader_create(flexflow_model_t ffmodel, flexflow_tensor_t input,
                                                               flexflow_tensor_t full_input, int num_samples,
                                                               int data_type);
/* full_input_ptr: host array of num_samples x (input dims without the batch dim), not copied */
flexflow_single_dataloader_t flexflow_single_dataloader_create2(flexflow_model_t ffmodel, flexflow_tensor_t input,
                                                                void* full_input_ptr, int num_samples, int data_type);
void flexflow_single_dataloader_destroy(flexflow_single_dataloader_t handle);
void flexflow_single_dataloader_set_num_samples(flexflow_single_dataloader_t handle, int samples);
int flexflow_single_dataloader_get_num_samples(flexflow_single_dataloader_t handle);
void flexflow_single_dataloader_reset(flexflow_single_dataloader_t handle);
/* stage the next batch into the loader's input tensor (reference SingleDataLoader::next_batch) */
void flexflow_single_dataloader_next_batch(flexflow_single_dataloader_t handle, flexflow_model_t model);

/* ------------------------------------------------------------------ timing / tracing / ops */
double flexflow_get_current_time(flexflow_config_t config); /* microseconds */
void flexflow_begin_trace(flexflow_config_t config, int trace_id);
void flexflow_end_trace(flexflow_config_t config, int trace_id);
int flexflow_op_get_num_parameters(flexflow_op_t handle);
flexflow_tensor_t flexflow_op_get_parameter_by_id(flexflow_op_t handle, int id);
int flexflow_op_get_num_inputs(flexflow_op_t handle);
flexflow_tensor_t flexflow_op_get_input_by_id(flexflow_op_t handle, int id);
int flexflow_op_get_num_outputs(flexflow_op_t handle);
flexflow_tensor_t flexflow_op_get_output_by_id(flexflow_op_t handle, int id);
void flexflow_op_init(flexflow_op_t handle, flexflow_model_t model);
void flexflow_op_forward(flexflow_op_t handle, flexflow_model_t model);
void flexflow_op_destroy(flexflow_op_t handle);
void flexflow_perform_registration(void);

/* ================================================================== extensions */
void flexflow_config_set_batch_size(flexflow_config_t handle, int batch_size);
void flexflow_model_train_step(flexflow_model_t handle);
float flexflow_model_get_accuracy(flexflow_model_t handle);
float flexflow_model_get_loss(flexflow_model_t handle);
float flexflow_per_metrics_get_loss(flexflow_perf_metrics_t handle);
/* generic optimizer view of either typed handle */
#define FF_AS_OPTIMIZER(h) ((flexflow_optimizer_t){(h).impl})
void flexflow_model_set_optimizer(flexflow_model_t model, flexflow_optimizer_t optimizer);
/* flat host buffers of exactly n elements */
bool flexflow_tensor_set_data_float(flexflow_tensor_t handle, flexflow_model_t model, const float* data, int64_t n);
bool flexflow_tensor_set_data_int(flexflow_tensor_t handle, flexflow_model_t model, const int32_t* data, int64_t n);
bool flexflow_tensor_set_data_int64(flexflow_tensor_t handle, flexflow_model_t model, const int64_t* data, int64_t n);
bool flexflow_tensor_get_data_float(flexflow_tensor_t handle, flexflow_model_t model, float* data, int64_t n);
flexflow_tensor_t flexflow_model_add_embedding_typed(flexflow_model_t handle, flexflow_tensor_t input, int num_entries,
                                                     int out_dim, int aggr, int data_type, const char* name);
flexflow_tensor_t flexflow_model_add_cast(flexflow_model_t handle, flexflow_tensor_t input, int data_type,
                                          const char* name);
flexflow_tensor_t flexflow_model_add_rms_norm(flexflow_model_t handle, flexflow_tensor_t input, float eps,
                                              const char* name);
/* multi-output layers write their outputs to outputs[] (top_k: 2 = values, indices; group_by: n)
 * and return how many they wrote, or -1 on error */
int flexflow_model_add_top_k(flexflow_model_t handle, flexflow_tensor_t input, int k, bool sorted,
                             flexflow_tensor_t* outputs, const char* name);
int flexflow_model_add_group_by(flexflow_model_t handle, flexflow_tensor_t data, flexflow_tensor_t assign, int n,
                                float alpha, flexflow_tensor_t* outputs, const char* name);
/* inputs: gate values, gate assignment, [gate predictions,] then n expert outputs */
flexflow_tensor_t flexflow_model_add_aggregate(flexflow_model_t handle, int n_inputs, const flexflow_tensor_t* inputs,
                                               int n, float lambda_bal, const char* name);
flexflow_tensor_t flexflow_model_add_aggregate_spec(flexflow_model_t handle, int n_inputs,
                                                    const flexflow_tensor_t* inputs, int n, float lambda_bal,
                                                    const char* name);
/* composite mixture-of-experts layer: gate dense -> top_k -> group_by -> expert denses -> aggregate */
flexflow_tensor_t flexflow_model_add_moe(flexflow_model_t handle, flexflow_tensor_t input, int num_exp, int num_select,
                                         int expert_hidden_size, float alpha, float lambda_bal);
int flexflow_model_get_num_layers(flexflow_model_t handle);
/* name of the parallelization strategy chosen at compile ("" before compile); valid until the next call */
const char* flexflow_model_get_strategy_name(flexflow_model_t handle);

#ifdef __cplusplus
}
#endif
#endif
