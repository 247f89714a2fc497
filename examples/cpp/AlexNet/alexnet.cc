// AlexNet on synthetic 229x229 images (reference examples/cpp/AlexNet/alexnet.cc:61-79).
//   ./alexnet -b 64 --iterations 20 [--small] [--search unity]
#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size(), hw = args.small ? 67 : 229;
  Tensor x = ff.create_tensor({b, 3, hw, hw});
  Tensor t = ff.conv2d(x, 64, 11, 11, 4, 4, 2, 2, AC_MODE_RELU);
  t = ff.pool2d(t, 3, 3, 2, 2, 0, 0);
  t = ff.conv2d(t, 192, 5, 5, 1, 1, 2, 2, AC_MODE_RELU);
  t = ff.pool2d(t, 3, 3, 2, 2, 0, 0);
  t = ff.conv2d(t, 384, 3, 3, 1, 1, 1, 1, AC_MODE_RELU);
  t = ff.conv2d(t, 256, 3, 3, 1, 1, 1, 1, AC_MODE_RELU);
  t = ff.conv2d(t, 256, 3, 3, 1, 1, 1, 1, AC_MODE_RELU);
  t = ff.pool2d(t, 3, 3, 2, 2, 0, 0);
  t = ff.flat(t);
  t = ff.dense(t, 4096, AC_MODE_RELU);
  t = ff.dense(t, 4096, AC_MODE_RELU);
  t = ff.dense(t, 10);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, 10, rng);
  train_loop(ff, "alexnet", args);
  return 0;
}
