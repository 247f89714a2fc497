/* flexflow_amd C API (reference include/flexflow/flexflow_c.h: opaque handles over FFConfig /
 * FFModel / Tensor / optimizers). Implemented in flexflow_c.cc by an embedded CPython runtime
 * that drives the flexflow_amd package, so C and C++ programs build, train and query models
 * with the same strategy search, HIP kernels and RCCL collectives as the Python API.
 * Enum arguments take the reference's numeric values (flexflow_amd/type.py).
 * Every function returns / accepts handles; a failing call prints the Python error to stderr and
 * returns a null handle (or leaves outputs untouched); flexflow_last_error() reports it. */
#ifndef FLEXFLOW_AMD_C_H
#define FLEXFLOW_AMD_C_H
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { void* impl; } flexflow_config_t;
typedef struct { void* impl; } flexflow_model_t;
typedef struct { void* impl; } flexflow_tensor_t;
typedef struct { void* impl; } flexflow_optimizer_t;

int flexflow_initialize(void);  /* idempotent; called implicitly by every entry point */
const char* flexflow_last_error(void);

/* FFConfig */
flexflow_config_t flexflow_config_create(void);
void flexflow_config_destroy(flexflow_config_t handle);
void flexflow_config_parse_args(flexflow_config_t handle, char** argv, int argc);
int flexflow_config_get_batch_size(flexflow_config_t handle);
void flexflow_config_set_batch_size(flexflow_config_t handle, int batch_size);
int flexflow_config_get_workers_per_node(flexflow_config_t handle);
int flexflow_config_get_num_nodes(flexflow_config_t handle);
int flexflow_config_get_epochs(flexflow_config_t handle);

/* FFModel */
flexflow_model_t flexflow_model_create(flexflow_config_t config);
void flexflow_model_destroy(flexflow_model_t handle);
void flexflow_model_compile(flexflow_model_t handle, int loss_type, const int* metrics, int nb_metrics, int comp_mode);
void flexflow_model_forward(flexflow_model_t handle, int seq_length);
void flexflow_model_backward(flexflow_model_t handle, int seq_length);
void flexflow_model_update(flexflow_model_t handle);
void flexflow_model_zero_gradients(flexflow_model_t handle);
void flexflow_model_reset_metrics(flexflow_model_t handle);
void flexflow_model_compute_metrics(flexflow_model_t handle);
void flexflow_model_init_layers(flexflow_model_t handle);
void flexflow_model_train_step(flexflow_model_t handle);
flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t handle);
float flexflow_model_get_accuracy(flexflow_model_t handle);
float flexflow_model_get_loss(flexflow_model_t handle);

/* optimizers */
flexflow_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t model, double lr, double momentum, bool nesterov,
                                                   double weight_decay);
flexflow_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t model, double alpha, double beta1, double beta2,
                                                    double weight_decay, double epsilon);
void flexflow_optimizer_destroy(flexflow_optimizer_t handle);
void flexflow_model_set_optimizer(flexflow_model_t model, flexflow_optimizer_t optimizer);
void flexflow_optimizer_set_lr(flexflow_optimizer_t handle, double lr);

/* tensors */
flexflow_tensor_t flexflow_tensor_create(flexflow_model_t model, int num_dims, const int* dims, int data_type,
                                         bool create_grad);
void flexflow_tensor_destroy(flexflow_tensor_t handle);
int flexflow_tensor_get_num_dims(flexflow_tensor_t handle);
int flexflow_tensor_get_dims(flexflow_tensor_t handle, int* dims /* >= num_dims */);
bool flexflow_tensor_set_data_float(flexflow_tensor_t handle, flexflow_model_t model, const float* data, int64_t n);
bool flexflow_tensor_set_data_int(flexflow_tensor_t handle, flexflow_model_t model, const int32_t* data, int64_t n);
bool flexflow_tensor_get_data_float(flexflow_tensor_t handle, flexflow_model_t model, float* data, int64_t n);

/* layers (reference FFModel builders) */
flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t handle, flexflow_tensor_t input, int out_dim,
                                           int activation, bool use_bias, const char* name);
flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t handle, flexflow_tensor_t input, int out_channels,
                                            int kernel_h, int kernel_w, int stride_h, int stride_w, int padding_h,
                                            int padding_w, int activation, int groups, bool use_bias, const char* name);
flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t handle, flexflow_tensor_t input, int kernel_h,
                                            int kernel_w, int stride_h, int stride_w, int padding_h, int padding_w,
                                            int pool_type, int activation, const char* name);
flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t handle, flexflow_tensor_t input, bool relu,
                                                const char* name);
flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t handle, flexflow_tensor_t input, int n_axes,
                                                const int* axes, bool elementwise_affine, float eps,
                                                const char* name);
flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t handle, flexflow_tensor_t input, int num_entries,
                                               int out_dim, int aggr, const char* name);
flexflow_tensor_t flexflow_model_add_multihead_attention(flexflow_model_t handle, flexflow_tensor_t query,
                                                         flexflow_tensor_t key, flexflow_tensor_t value,
                                                         int embed_dim, int num_heads, int kdim, int vdim,
                                                         float dropout, bool bias, const char* name);
flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t handle, flexflow_tensor_t input, int axis,
                                             const char* name);
flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t handle, flexflow_tensor_t input, const char* name);
flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t handle, flexflow_tensor_t input, float scalar,
                                                     const char* name);
flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t handle, flexflow_tensor_t input, float scalar,
                                                const char* name);
flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t handle, flexflow_tensor_t input, float exponent,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_add(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                              const char* name);
flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                              const char* name);
flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                            const char* name);
flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t handle, flexflow_tensor_t a, flexflow_tensor_t b,
                                                  const char* name);
flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t handle, int n, const flexflow_tensor_t* inputs, int axis,
                                            const char* name);
flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t handle, flexflow_tensor_t input, float rate,
                                             unsigned long long seed, const char* name);
flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t handle, flexflow_tensor_t input, int num_dims,
                                             const int* shape, const char* name);
flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t handle, flexflow_tensor_t input, int num_dims,
                                               const int* perm, const char* name);

flexflow_tensor_t flexflow_model_add_embedding_typed(flexflow_model_t handle, flexflow_tensor_t input, int num_entries,
                                                     int out_dim, int aggr, int data_type, const char* name);
flexflow_tensor_t flexflow_model_add_max(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_min(flexflow_model_t handle, flexflow_tensor_t x, flexflow_tensor_t y,
                                         const char* name);
flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t handle, flexflow_tensor_t input, int n_dims,
                                          const int* dims, bool keepdims, const char* name);
flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t handle, flexflow_tensor_t input, int n_axes,
                                                const int* axes, bool keepdims, const char* name);
flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t handle, flexflow_tensor_t input, flexflow_tensor_t index,
                                            int dim, const char* name);
flexflow_tensor_t flexflow_model_add_cast(flexflow_model_t handle, flexflow_tensor_t input, int data_type,
                                          const char* name);
flexflow_tensor_t flexflow_model_add_rms_norm(flexflow_model_t handle, flexflow_tensor_t input, float eps,
                                              const char* name);
flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t handle, flexflow_tensor_t input, int axis,
                                             const char* name);
/* multi-output layers write their outputs to outputs[] (split: n, top_k: 2 = values, indices,
 * group_by: n) and return how many they wrote, or -1 on error */
int flexflow_model_add_split(flexflow_model_t handle, flexflow_tensor_t input, int n, const int* sizes, int axis,
                             flexflow_tensor_t* outputs, const char* name);
int flexflow_model_add_top_k(flexflow_model_t handle, flexflow_tensor_t input, int k, bool sorted,
                             flexflow_tensor_t* outputs, const char* name);
int flexflow_model_add_group_by(flexflow_model_t handle, flexflow_tensor_t data, flexflow_tensor_t assign, int n,
                                float alpha, flexflow_tensor_t* outputs, const char* name);
/* inputs: gate values, gate assignment, [gate predictions,] then n expert outputs (reference
 * FFModel::aggregate / aggregate_spec) */
flexflow_tensor_t flexflow_model_add_aggregate(flexflow_model_t handle, int n_inputs, const flexflow_tensor_t* inputs,
                                               int n, float lambda_bal, const char* name);
flexflow_tensor_t flexflow_model_add_aggregate_spec(flexflow_model_t handle, int n_inputs,
                                                    const flexflow_tensor_t* inputs, int n, float lambda_bal,
                                                    const char* name);
/* composite mixture-of-experts layer: gate dense -> top_k -> group_by -> expert denses -> aggregate */
flexflow_tensor_t flexflow_model_add_moe(flexflow_model_t handle, flexflow_tensor_t input, int num_exp, int num_select,
                                         int expert_hidden_size, float alpha, float lambda_bal);
bool flexflow_tensor_set_data_int64(flexflow_tensor_t handle, flexflow_model_t model, const int64_t* data, int64_t n);
void flexflow_model_print_layers(flexflow_model_t handle, int id /* -1 = all */);
int flexflow_model_get_num_layers(flexflow_model_t handle);
/* name of the parallelization strategy chosen at compile ("" before compile); valid until the next call */
const char* flexflow_model_get_strategy_name(flexflow_model_t handle);

#ifdef __cplusplus
}
#endif
#endif
