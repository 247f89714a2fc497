/* Train a 2-layer MLP for a few SGD steps through the flexflow_amd C API (reference usage:
 * python/flexflow/core/flexflow_cffi.py drives the same entry points through cffi). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "flexflow_c.h"

int main(void) {
  if (flexflow_initialize() != 0) {
    fprintf(stderr, "init failed: %s\n", flexflow_last_error());
    return 1;
  }
  char* argv[] = {"--no-hip-graphs"};
  flexflow_config_t cfg = flexflow_config_create();
  flexflow_config_parse_args(cfg, argv, 1);
  flexflow_config_set_batch_size(cfg, 16);
  flexflow_model_t m = flexflow_model_create(cfg);
  int dims[2] = {16, 8};
  flexflow_tensor_t x = flexflow_tensor_create(m, 2, dims, 44 /* DT_FLOAT */, true);
  flexflow_tensor_t h = flexflow_model_add_dense(m, x, 32, 11 /* AC_MODE_RELU */, true, "fc1");
  flexflow_tensor_t o = flexflow_model_add_dense(m, h, 4, 10 /* AC_MODE_NONE */, true, "fc2");
  o = flexflow_model_add_softmax(m, o, -1, "sm");
  flexflow_optimizer_t opt = flexflow_sgd_optimizer_create(m, 0.2, 0.0, false, 0.0);
  flexflow_model_set_optimizer(m, opt);
  int metrics[1] = {1001 /* METRICS_ACCURACY */};
  flexflow_model_compile(m, 51 /* LOSS_SPARSE_CATEGORICAL_CROSSENTROPY */, metrics, 1, 70 /* TRAINING */);
  float xs[16 * 8];
  int lab[16];
  for (int i = 0; i < 16; ++i) {
    lab[i] = i % 4;
    for (int j = 0; j < 8; ++j) xs[i * 8 + j] = (j % 4 == lab[i]) ? 1.0f : 0.1f * (float)((i * 7 + j) % 5);
  }
  if (!flexflow_tensor_set_data_float(x, m, xs, 16 * 8)) return 2;
  flexflow_tensor_t label = flexflow_model_get_label_tensor(m);
  if (!flexflow_tensor_set_data_int(label, m, lab, 16)) return 3;
  float first = 0.f, last = 0.f;
  for (int s = 0; s < 30; ++s) {
    flexflow_model_reset_metrics(m);
    flexflow_model_train_step(m);
    last = flexflow_model_get_loss(m);
    if (s == 0) first = last;
  }
  float probs[16 * 4];
  if (!flexflow_tensor_get_data_float(o, m, probs, 16 * 4)) return 4;
  int nd = flexflow_tensor_get_num_dims(o);
  printf("loss %.4f -> %.4f  accuracy %.1f%%  out dims %d  p00 %.3f\n", first, last, flexflow_model_get_accuracy(m), nd,
         probs[0]);
  flexflow_tensor_destroy(label);
  flexflow_optimizer_destroy(opt);
  flexflow_model_destroy(m);
  flexflow_config_destroy(cfg);
  return (last < first && isfinite(last) && nd == 2) ? 0 : 5;
}
