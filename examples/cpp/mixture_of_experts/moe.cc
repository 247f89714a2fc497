// Mixture of experts on MNIST-shaped synthetic data, composed from the primitive layers: gate
// dense -> top_k -> group_by -> expert denses -> aggregate -> dense relu -> softmax (reference
// examples/cpp/mixture_of_experts/moe.cc:150-173; --composite uses the one-call ff.moe).
//   ./moe -b 64 [--num-exp 5] [--num-select 2] [--small] [--composite]
#include <cstring>

#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  bool composite = false;
  for (int i = 1; i < argc; ++i) composite |= !std::strcmp(argv[i], "--composite");
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size();
  const int data_dims = args.small ? 64 : 28 * 28, hidden = args.small ? 32 : 28 * 28, out_dim = 10;
  const int num_exp = args.get_int("--num-exp", 5), num_select = args.get_int("--num-select", 2);
  const float alpha = 2.0f, lambda_bal = 0.04f;
  Tensor x = ff.create_tensor({b, data_dims});
  Tensor t;
  if (composite) {
    t = ff.moe(x, num_exp, num_select, hidden, alpha, lambda_bal);
  } else {
    Tensor gate = ff.dense(x, num_exp, AC_MODE_RELU);
    auto topk = ff.top_k(gate, num_select, false);  // {values, indices}
    auto grouped = ff.group_by(x, topk[1], num_exp, alpha);
    // aggregate inputs: gate weights, assignment, true assignment (no spec here), full gate, experts
    std::vector<Tensor> agg{ff.softmax(topk[0]), topk[1], topk[1], gate};
    for (int e = 0; e < num_exp; ++e) agg.push_back(ff.softmax(ff.dense(grouped[e], hidden, AC_MODE_RELU)));
    t = ff.aggregate(agg, num_exp, lambda_bal);
  }
  t = ff.dense(t, out_dim, AC_MODE_RELU);
  t = ff.softmax(t);
  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, {METRICS_ACCURACY, METRICS_SPARSE_CATEGORICAL_CROSSENTROPY});
  std::mt19937 rng(0);
  feed_normal(ff, x, rng);
  feed_labels(ff, true, out_dim, rng);
  train_loop(ff, "moe", args);
  return 0;
}
