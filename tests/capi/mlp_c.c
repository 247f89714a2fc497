/* Train a 2-layer MLP through the flexflow_amd C API the way a program written against the
 * reference's include/flexflow/flexflow_c.h does: initializers on the dense layers, the full
 * dataset in SingleDataLoaders (one from a tensor, one from a raw host pointer), per-op
 * accessors, parameter get/set, inline-mapped raw pointers and PerfMetrics. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flexflow_c.h"

#define B 16
#define IN 8
#define NS 64 /* samples in the dataset: 4 batches */

#define CHECK(c, code)                                                          \
  do {                                                                          \
    if (!(c)) {                                                                 \
      fprintf(stderr, "check failed (%s): %s\n", #c, flexflow_last_error());    \
      return code;                                                              \
    }                                                                           \
  } while (0)

int main(void) {
  CHECK(flexflow_initialize() == 0, 1);
  char* argv[] = {"--no-hip-graphs", "-b", "16"};
  flexflow_config_t cfg = flexflow_config_create();
  flexflow_config_parse_args(cfg, argv, 3);
  CHECK(flexflow_config_get_batch_size(cfg) == B, 2);
  flexflow_model_t m = flexflow_model_create(cfg);

  int dims[2] = {B, IN};
  flexflow_tensor_t x = flexflow_tensor_create(m, 2, dims, 44 /* DT_FLOAT */, true);
  CHECK(flexflow_tensor_get_dim(x, 0) == IN && flexflow_tensor_get_dim(x, 1) == B, 3); /* Legion order */

  flexflow_glorot_uniform_initializer_t glorot = flexflow_glorot_uniform_initializer_create(7);
  flexflow_zero_initializer_t zero = flexflow_zero_initializer_create();
  flexflow_norm_initializer_t norm = flexflow_norm_initializer_create(3, 0.f, 0.05f);
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t h = flexflow_model_add_dense(m, x, 32, 11 /* RELU */, true, 44, no_op,
                                                 FF_AS_INITIALIZER(glorot), FF_AS_INITIALIZER(zero),
                                                 17 /* REG_MODE_NONE */, 0.f, "fc1");
  flexflow_tensor_t o = flexflow_model_add_dense(m, h, 4, 10 /* NONE */, true, 44, no_op, FF_AS_INITIALIZER(norm),
                                                 flexflow_initializer_create_null(), 17, 0.f, "fc2");
  o = flexflow_model_add_softmax(m, o, -1, "sm");
  flexflow_sgd_optimizer_t opt = flexflow_sgd_optimizer_create(m, 0.2, 0.0, false, 0.0);
  flexflow_model_set_sgd_optimizer(m, opt);
  int metrics[1] = {1001 /* METRICS_ACCURACY */};
  flexflow_model_compile(m, 51 /* LOSS_SPARSE_CATEGORICAL_CROSSENTROPY */, metrics, 1, 70 /* TRAINING */);

  /* op accessors: fc1 has 2 parameters, 1 input, 1 output; its zero-initialised bias reads back 0 */
  flexflow_op_t fc1 = flexflow_model_get_layer_by_id(m, 0);
  CHECK(flexflow_op_get_num_parameters(fc1) == 2 && flexflow_op_get_num_inputs(fc1) == 1, 4);
  CHECK(flexflow_op_get_num_outputs(fc1) == 1, 4);
  flexflow_tensor_t bias = flexflow_op_get_parameter_by_id(fc1, 1);
  float b[32];
  CHECK(flexflow_parameter_get_weights_float(bias, m, b), 5);
  for (int i = 0; i < 32; ++i) CHECK(b[i] == 0.f, 5);
  flexflow_tensor_t kernel = flexflow_model_get_parameter_by_id(m, 0);
  CHECK(flexflow_tensor_get_num_dims(kernel) == 2, 5);

  /* dataset: features in a tensor (loader 1), labels from a raw pointer (loader 2) */
  static float xs[NS * IN];
  static int lab[NS];
  for (int i = 0; i < NS; ++i) {
    lab[i] = i % 4;
    for (int j = 0; j < IN; ++j) xs[i * IN + j] = (j % 4 == lab[i]) ? 1.0f : 0.1f * (float)((i * 7 + j) % 5);
  }
  int full_dims[2] = {NS, IN};
  flexflow_tensor_t full_x = flexflow_tensor_create(m, 2, full_dims, 44, false);
  flexflow_tensor_attach_raw_ptr(full_x, m, cfg, xs, false);
  CHECK(flexflow_tensor_is_mapped(full_x), 6);
  flexflow_single_dataloader_t dl_x = flexflow_single_dataloader_create(m, x, full_x, NS, 44);
  flexflow_tensor_t label = flexflow_model_get_label_tensor(m);
  flexflow_single_dataloader_t dl_y = flexflow_single_dataloader_create2(m, label, lab, NS, 41 /* DT_INT32 */);
  CHECK(dl_x.impl && dl_y.impl, 6);
  CHECK(flexflow_single_dataloader_get_num_samples(dl_x) == NS, 6);

  float first = 0.f, last = 0.f;
  double t0 = flexflow_get_current_time(cfg);
  for (int epoch = 0; epoch < 10; ++epoch) {
    flexflow_single_dataloader_reset(dl_x);
    flexflow_single_dataloader_reset(dl_y);
    flexflow_model_reset_metrics(m);
    for (int it = 0; it < NS / B; ++it) {
      flexflow_single_dataloader_next_batch(dl_x, m);
      flexflow_single_dataloader_next_batch(dl_y, m);
      flexflow_model_forward(m, -1);
      flexflow_model_zero_gradients(m);
      flexflow_model_backward(m, -1);
      flexflow_model_update(m);
    }
    flexflow_perf_metrics_t pm = flexflow_model_get_perf_metrics(m);
    last = flexflow_per_metrics_get_loss(pm);
    if (epoch == 0) first = last;
    if (epoch == 9) printf("epoch %d accuracy %.1f%%\n", epoch, flexflow_per_metrics_get_accuracy(pm));
    flexflow_per_metrics_destroy(pm);
  }
  CHECK(flexflow_get_current_time(cfg) > t0, 7);

  /* the model output through an inline-mapped raw pointer */
  flexflow_tensor_inline_map(o, m, cfg);
  float* p = flexflow_tensor_get_raw_ptr_float(o, m, cfg);
  CHECK(p != NULL, 8);
  float row = p[0] + p[1] + p[2] + p[3];
  flexflow_tensor_inline_unmap(o, m, cfg);
  float probs[B * 4];
  CHECK(flexflow_tensor_get_tensor_float(o, m, probs, false), 8);
  CHECK(fabsf(row - 1.f) < 1e-3f && fabsf(probs[0] - p[0]) < 1e-6f, 8);

  /* parameter set / get round trip */
  for (int i = 0; i < 32; ++i) b[i] = 0.01f * (float)i;
  int bdims[1] = {32};
  CHECK(flexflow_parameter_set_weights_float(bias, m, 1, bdims, b), 9);
  float b2[32];
  CHECK(flexflow_parameter_get_weights_float(bias, m, b2) && b2[31] == b[31], 9);

  printf("loss %.4f -> %.4f  out dims %d\n", first, last, flexflow_tensor_get_num_dims(o));
  flexflow_single_dataloader_destroy(dl_x);
  flexflow_single_dataloader_destroy(dl_y);
  flexflow_tensor_destroy(full_x);
  flexflow_tensor_destroy(bias);
  flexflow_tensor_destroy(kernel);
  flexflow_op_destroy(fc1);
  flexflow_tensor_destroy(label);
  flexflow_glorot_uniform_initializer_destroy(glorot);
  flexflow_zero_initializer_destroy(zero);
  flexflow_norm_initializer_destroy(norm);
  flexflow_sgd_optimizer_destroy(opt);
  flexflow_model_destroy(m);
  flexflow_config_destroy(cfg);
  return (last < first && isfinite(last)) ? 0 : 10;
}
