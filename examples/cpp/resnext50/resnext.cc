// ResNeXt-50 (grouped 3x3 bottlenecks, 32 groups) on synthetic images (reference
// examples/cpp/resnext50/resnext.cc:12-87).
//   ./resnext -b 32 --iterations 10 [--small]
#include "../common.hpp"

using namespace ffx;

static Tensor block(FFModel& ff, Tensor x, int stride, int ch, int groups, bool residual) {
  Tensor t = ff.conv2d(x, ch, 1, 1, 1, 1, 0, 0, AC_MODE_RELU);
  t = ff.conv2d(t, ch, 3, 3, stride, stride, 1, 1, AC_MODE_RELU, groups);
  t = ff.conv2d(t, 2 * ch, 1, 1, 1, 1, 0, 0);
  if ((stride > 1 || x.dim(1) != 2 * ch) && residual) {
    x = ff.conv2d(x, 2 * ch, 1, 1, stride, stride, 0, 0, AC_MODE_RELU);
    t = ff.relu(ff.add(x, t));
  }
  return t;
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size(), hw = args.small ? 64 : 224, groups = args.small ? 4 : 32;
  const int classes = args.small ? 10 : 1000;
  Tensor x = ff.create_tensor({b, 3, hw, hw});
  Tensor t = ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3, AC_MODE_RELU);
  t = ff.pool2d(t, 3, 3, 2, 2, 1, 1);
  const int stages[4][3] = {{128, 3, 1}, {256, 4, 2}, {512, 6, 2}, {1024, 3, 2}};
  for (auto& s : stages)
    for (int i = 0; i < s[1]; ++i) t = block(ff, t, i == 0 ? s[2] : 1, s[0], groups, false);
  t = ff.relu(t);
  t = ff.pool2d(t, t.dim(2), t.dim(3), 1, 1, 0, 0, POOL_AVG);
  t = ff.flat(t);
  t = ff.dense(t, classes);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, classes, rng);
  train_loop(ff, "resnext50", args);
  return 0;
}
