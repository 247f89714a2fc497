// ResNet-50 (3-4-6-3 bottlenecks) on synthetic 224x224 images (reference
// examples/cpp/ResNet/resnet.cc:39-113). The reference comments its batch norms out; --batch-norm
// builds the standard network.
//   ./resnet -b 64 --iterations 20 [--small] [--batch-norm]
#include <cstring>

#include "../common.hpp"

using namespace ffx;

static Tensor bottleneck(FFModel& ff, Tensor x, int ch, int stride, bool bn) {
  Tensor t = ff.conv2d(x, ch, 1, 1, 1, 1, 0, 0);
  if (bn) t = ff.batch_norm(t);
  t = ff.conv2d(t, ch, 3, 3, stride, stride, 1, 1);
  if (bn) t = ff.batch_norm(t);
  t = ff.conv2d(t, 4 * ch, 1, 1, 1, 1, 0, 0);
  if (bn) t = ff.batch_norm(t, false);
  if (stride > 1 || x.dim(1) != 4 * ch) {
    x = ff.conv2d(x, 4 * ch, 1, 1, stride, stride, 0, 0);
    if (bn) x = ff.batch_norm(x, false);
  }
  return ff.relu(ff.add(x, t));
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  bool bn = false;
  for (int i = 1; i < argc; ++i) bn |= !std::strcmp(argv[i], "--batch-norm");
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size(), hw = args.small ? 64 : 224;
  Tensor x = ff.create_tensor({b, 3, hw, hw});
  Tensor t = ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3);
  if (bn) t = ff.batch_norm(t);
  t = ff.pool2d(t, 3, 3, 2, 2, 1, 1);
  const int stages[4][2] = {{64, 3}, {128, 4}, {256, 6}, {512, 3}};
  for (int s = 0; s < 4; ++s)
    for (int i = 0; i < stages[s][1]; ++i) t = bottleneck(ff, t, stages[s][0], (i == 0 && s > 0) ? 2 : 1, bn);
  const int fh = t.dim(2);
  t = ff.pool2d(t, fh, fh, 1, 1, 0, 0, POOL_AVG);
  t = ff.flat(t);
  t = ff.dense(t, 10);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, 10, rng);
  train_loop(ff, "resnet50", args);
  return 0;
}
