// Branch-and-merge MLP: a dense layer feeding two parallel denses whose outputs are added, twice
// (reference examples/cpp/split_test/split_test.cc:20-45).
//   ./split_test -b 64 --iterations 128
#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int dims[4] = {256, 128, 64, 32};
  Tensor x = ff.create_tensor({1, cfg.batch_size(), dims[0]});
  Tensor t = ff.relu(ff.dense(x, dims[1]));
  t = ff.relu(ff.add(ff.dense(t, dims[2]), ff.dense(t, dims[2])));
  t = ff.relu(ff.add(ff.dense(t, dims[3]), ff.dense(t, dims[3])));
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, dims[3], rng);
  train_loop(ff, "split_test", args);
  return 0;
}
