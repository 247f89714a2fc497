// Inception-v3 (3xA, B, 4xC, D, 2xE) on synthetic 299x299 images (reference
// examples/cpp/InceptionV3/inception.cc:26-174).
//   ./inception -b 64 --iterations 10 [--small]
#include "../common.hpp"

using namespace ffx;

// stem and A blocks use fused ReLU convolutions, blocks B-E plain ones (as the reference)
static Tensor conv(FFModel& ff, const Tensor& x, int oc, int kh, int kw, int s, int ph, int pw) {
  return ff.conv2d(x, oc, kh, kw, s, s, ph, pw, AC_MODE_RELU);
}
static Tensor convn(FFModel& ff, const Tensor& x, int oc, int kh, int kw, int s, int ph, int pw) {
  return ff.conv2d(x, oc, kh, kw, s, s, ph, pw, AC_MODE_NONE);
}

static Tensor inception_a(FFModel& ff, const Tensor& x, int pool_features) {
  Tensor t1 = conv(ff, x, 64, 1, 1, 1, 0, 0);
  Tensor t2 = conv(ff, conv(ff, x, 48, 1, 1, 1, 0, 0), 64, 5, 5, 1, 2, 2);
  Tensor t3 = conv(ff, conv(ff, conv(ff, x, 64, 1, 1, 1, 0, 0), 96, 3, 3, 1, 1, 1), 96, 3, 3, 1, 1, 1);
  Tensor t4 = conv(ff, ff.pool2d(x, 3, 3, 1, 1, 1, 1, POOL_AVG), pool_features, 1, 1, 1, 0, 0);
  return ff.concat({t1, t2, t3, t4}, 1);
}

static Tensor inception_b(FFModel& ff, const Tensor& x) {
  Tensor t1 = convn(ff, x, 384, 3, 3, 2, 0, 0);
  Tensor t2 = convn(ff, convn(ff, convn(ff, x, 64, 1, 1, 1, 0, 0), 96, 3, 3, 1, 1, 1), 96, 3, 3, 2, 0, 0);
  Tensor t3 = ff.pool2d(x, 3, 3, 2, 2, 0, 0);
  return ff.concat({t1, t2, t3}, 1);
}

static Tensor inception_c(FFModel& ff, const Tensor& x, int ch) {
  Tensor t1 = convn(ff, x, 192, 1, 1, 1, 0, 0);
  Tensor t2 = convn(ff, x, ch, 1, 1, 1, 0, 0);
  t2 = convn(ff, t2, ch, 1, 7, 1, 0, 3);
  t2 = convn(ff, t2, 192, 7, 1, 1, 3, 0);
  Tensor t3 = convn(ff, x, ch, 1, 1, 1, 0, 0);
  t3 = convn(ff, t3, ch, 7, 1, 1, 3, 0);
  t3 = convn(ff, t3, ch, 1, 7, 1, 0, 3);
  t3 = convn(ff, t3, ch, 7, 1, 1, 3, 0);
  t3 = convn(ff, t3, 192, 1, 7, 1, 0, 3);
  Tensor t4 = convn(ff, ff.pool2d(x, 3, 3, 1, 1, 1, 1, POOL_AVG), 192, 1, 1, 1, 0, 0);
  return ff.concat({t1, t2, t3, t4}, 1);
}

static Tensor inception_d(FFModel& ff, const Tensor& x) {
  Tensor t1 = convn(ff, convn(ff, x, 192, 1, 1, 1, 0, 0), 320, 3, 3, 2, 0, 0);
  Tensor t2 = convn(ff, x, 192, 1, 1, 1, 0, 0);
  t2 = convn(ff, t2, 192, 1, 7, 1, 0, 3);
  t2 = convn(ff, t2, 192, 7, 1, 1, 3, 0);
  t2 = convn(ff, t2, 192, 3, 3, 2, 0, 0);
  Tensor t3 = ff.pool2d(x, 3, 3, 2, 2, 0, 0);
  return ff.concat({t1, t2, t3}, 1);
}

static Tensor inception_e(FFModel& ff, const Tensor& x) {
  Tensor t1 = convn(ff, x, 320, 1, 1, 1, 0, 0);
  Tensor t2i = convn(ff, x, 384, 1, 1, 1, 0, 0);
  Tensor t2 = convn(ff, t2i, 384, 1, 3, 1, 0, 1);
  Tensor t3 = convn(ff, t2i, 384, 3, 1, 1, 1, 0);
  Tensor t3i = convn(ff, convn(ff, x, 448, 1, 1, 1, 0, 0), 384, 3, 3, 1, 1, 1);
  Tensor t4 = convn(ff, t3i, 384, 1, 3, 1, 0, 1);
  Tensor t5 = convn(ff, t3i, 384, 3, 1, 1, 1, 0);
  Tensor t6 = convn(ff, ff.pool2d(x, 3, 3, 1, 1, 1, 1, POOL_AVG), 192, 1, 1, 1, 0, 0);
  return ff.concat({t1, t2, t3, t4, t5, t6}, 1);
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size(), hw = args.small ? 139 : 299;
  Tensor x = ff.create_tensor({b, 3, hw, hw});
  Tensor t = conv(ff, x, 32, 3, 3, 2, 0, 0);
  t = conv(ff, t, 32, 3, 3, 1, 0, 0);
  t = conv(ff, t, 64, 3, 3, 1, 1, 1);
  t = ff.pool2d(t, 3, 3, 2, 2, 0, 0);
  t = conv(ff, t, 80, 1, 1, 1, 0, 0);
  t = conv(ff, t, 192, 3, 3, 1, 1, 1);
  t = ff.pool2d(t, 3, 3, 2, 2, 0, 0);
  t = inception_a(ff, t, 32);
  t = inception_a(ff, t, 64);
  t = inception_a(ff, t, 64);
  t = inception_b(ff, t);
  for (int ch : {128, 160, 160, 192}) t = inception_c(ff, t, ch);
  t = inception_d(ff, t);
  t = inception_e(ff, t);
  t = inception_e(ff, t);
  t = ff.pool2d(t, t.dim(2), t.dim(3), 1, 1, 0, 0, POOL_AVG);
  t = ff.flat(t);
  t = ff.dense(t, 10);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, 10, rng);
  train_loop(ff, "inception_v3", args);
  return 0;
}
