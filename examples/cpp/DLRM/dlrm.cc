// DLRM: bottom MLP over dense features, one embedding bag per sparse feature, "cat" interaction,
// top MLP, MSE loss (reference examples/cpp/DLRM/dlrm.cc:26-175, same --arch-* flags).
//   ./dlrm -b 2048 --arch-sparse-feature-size 64 --arch-embedding-size 1000000-1000000-1000000-1000000
//          --arch-mlp-bot 4-64-64 --arch-mlp-top 64-64-2 [--embedding-bag-size 1] [--small]
#include "../common.hpp"

using namespace ffx;

// create_mlp: dense stack without bias; layer `sigmoid_layer` uses a sigmoid, the rest ReLU
static Tensor mlp(FFModel& ff, Tensor t, const std::vector<int>& ln, int sigmoid_layer) {
  for (size_t i = 0; i + 1 < ln.size(); ++i)
    t = ff.dense(t, ln[i + 1], (int)i == sigmoid_layer ? AC_MODE_SIGMOID : AC_MODE_RELU, false);
  return t;
}

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size();
  const int feat = args.get_int("--arch-sparse-feature-size", 64);
  const int bag = args.get_int("--embedding-bag-size", 1);
  const auto emb = parse_dash_list(args.get("--arch-embedding-size"),
                                   std::vector<int>(4, args.small ? 1000 : 1000000));
  const auto bot = parse_dash_list(args.get("--arch-mlp-bot"), {4, 64, 64});
  const auto top = parse_dash_list(args.get("--arch-mlp-top"), {64, 64, 2});
  const int sigmoid_bot = args.get_int("--sigmoid-bot", -1);
  const int sigmoid_top = args.get_int("--sigmoid-top", (int)top.size() - 2);

  std::vector<Tensor> sparse;
  for (size_t i = 0; i < emb.size(); ++i) sparse.push_back(ff.create_tensor({b, bag}, DT_INT64));
  Tensor dense = ff.create_tensor({b, bot[0]});
  std::vector<Tensor> ly{mlp(ff, dense, bot, sigmoid_bot)};
  for (size_t i = 0; i < emb.size(); ++i) ly.push_back(ff.embedding(sparse[i], emb[i], feat, AGGR_MODE_SUM));
  Tensor z = ff.concat(ly, -1);
  std::vector<int> top_ln{z.dim(-1)};
  top_ln.insert(top_ln.end(), top.begin() + 1, top.end());
  Tensor p = mlp(ff, z, top_ln, sigmoid_top);

  SGDOptimizer opt(ff, 0.01);
  ff.compile(opt, LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, {METRICS_MEAN_SQUARED_ERROR});
  std::mt19937 rng(0);
  for (size_t i = 0; i < emb.size(); ++i) feed_indices(ff, sparse[i], emb[i], rng);
  feed_normal(ff, dense, rng);
  feed_labels(ff, false, 0, rng);
  train_loop(ff, "dlrm", args);
  return 0;
}
