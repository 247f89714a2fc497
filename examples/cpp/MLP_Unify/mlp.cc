// MLP_Unify: two dense towers over two inputs, summed, softmax (reference
// examples/cpp/MLP_Unify/mlp.cc:38-57; the reference times forward only, this trains).
//   ./mlp -b 64 --iterations 20 [--small]
#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size(), in_dim = args.small ? 64 : 1024;
  const std::vector<int> hidden(args.small ? 3 : 8, args.small ? 128 : 8192);
  Tensor x1 = ff.create_tensor({b, in_dim}), x2 = ff.create_tensor({b, in_dim});
  Tensor t1 = x1, t2 = x2;
  for (size_t i = 0; i < hidden.size(); ++i) {
    const ActiMode act = i + 1 == hidden.size() ? AC_MODE_NONE : AC_MODE_RELU;
    t1 = ff.dense(t1, hidden[i], act, false);
    t2 = ff.dense(t2, hidden[i], act, false);
  }
  Tensor t = ff.softmax(ff.add(t1, t2));
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x1, rng);
  feed_normal(ff, x2, rng);
  feed_labels(ff, true, hidden.back(), rng);
  train_loop(ff, "mlp_unify", args);
  return 0;
}
