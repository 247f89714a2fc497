// Transformer encoder stack: (self-attention -> dense relu -> dense) x num_layers, dense -> 1, MSE
// loss (reference examples/cpp/Transformer/transformer.cc:33-163, same defaults and flags).
//   ./transformer -b 8 [--num-layers 12] [--hidden-size 1024] [--num-heads 16] [--sequence-length 512] [--small]
#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size();
  const int hidden = args.get_int("--hidden-size", args.small ? 64 : 1024);
  const int heads = args.get_int("--num-heads", args.small ? 4 : 16);
  const int layers = args.get_int("--num-layers", args.small ? 2 : 12);
  const int seq = args.get_int("--sequence-length", args.small ? 16 : 512);
  Tensor x = ff.create_tensor({b, seq, hidden});
  Tensor t = x;
  for (int l = 0; l < layers; ++l) {
    t = ff.multihead_attention(t, t, t, hidden, heads, hidden / heads, hidden / heads);
    t = ff.dense(t, hidden, AC_MODE_RELU, false);
    t = ff.dense(t, hidden, AC_MODE_NONE, false);
  }
  t = ff.dense(t, 1, AC_MODE_NONE, false);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, {METRICS_MEAN_SQUARED_ERROR});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, false, 0, rng);
  train_loop(ff, "transformer", args);
  return 0;
}
