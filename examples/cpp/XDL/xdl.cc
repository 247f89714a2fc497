// XDL: embedding bags -> concat -> MLP, MSE loss (reference examples/cpp/XDL/xdl.cc:24-141).
//   ./xdl -b 2048 --arch-sparse-feature-size 64 --arch-embedding-size 1000000-1000000-1000000-1000000
//         --arch-mlp-top 256-256-256-2 [--small]
#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size();
  const int feat = args.get_int("--arch-sparse-feature-size", 64);
  const int bag = args.get_int("--embedding-bag-size", 1);
  const auto emb = parse_dash_list(args.get("--arch-embedding-size"),
                                   std::vector<int>(4, args.small ? 1000 : 1000000));
  const auto top = parse_dash_list(args.get("--arch-mlp-top"), {256, 256, 256, 2});

  std::vector<Tensor> sparse, ly;
  for (size_t i = 0; i < emb.size(); ++i) {
    sparse.push_back(ff.create_tensor({b, bag}, DT_INT64));
    ly.push_back(ff.embedding(sparse.back(), emb[i], feat, AGGR_MODE_SUM));
  }
  Tensor t = ff.concat(ly, -1);
  for (size_t i = 0; i < top.size(); ++i)
    t = ff.dense(t, top[i], i + 2 == top.size() ? AC_MODE_SIGMOID : (i + 1 == top.size() ? AC_MODE_NONE : AC_MODE_RELU),
                 false);

  SGDOptimizer opt(ff, 0.01);
  ff.compile(opt, LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, {METRICS_MEAN_SQUARED_ERROR});
  std::mt19937 rng(0);
  for (size_t i = 0; i < emb.size(); ++i) feed_indices(ff, sparse[i], emb[i], rng);
  feed_labels(ff, false, 0, rng);
  train_loop(ff, "xdl", args);
  return 0;
}
