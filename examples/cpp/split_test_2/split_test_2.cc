// Strided-convolution stack -> flat -> relu -> softmax, plus a split / concat round trip of the
// flattened features (reference examples/cpp/split_test_2/split_test_2.cc:20-55, which prints the
// shape after every convolution).
//   ./split_test_2 -b 64 --iterations 16
#include "../common.hpp"

using namespace ffx;

static void print_dims(const char* what, const Tensor& t) {
  std::printf("%s:", what);
  for (int d : t.dims()) std::printf(" %d", d);
  std::printf("\n");
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int channels[3] = {4, 8, 16};
  Tensor x = ff.create_tensor({cfg.batch_size(), 4, 32, 32});
  Tensor t = x;
  for (int i = 0; i < 3; ++i) {
    t = ff.conv2d(t, channels[1], 3, 3, 2, 2, 0, 0);
    print_dims(("Iteration " + std::to_string(i)).c_str(), t);
  }
  print_dims("Post-conv shape", t);
  t = ff.flat(t);
  const int f = t.dim(1);
  auto parts = ff.split(t, {f / 2, f - f / 2}, 1);
  t = ff.concat({ff.relu(parts[0]), ff.relu(parts[1])}, 1);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, f, rng);
  train_loop(ff, "split_test_2", args);
  return 0;
}
