// CANDLE-Uno: one dense encoder stack per cell.* / drug.* input feature, concat with the dose
// inputs, dense head -> 1, MSE loss (reference examples/cpp/candle_uno/candle_uno.cc:24-141;
// inputs in sorted-name order like its std::map).
//   ./candle_uno -b 256 [--dense-layers 4192-4192-4192-4192] [--dense-feature-layers 4192-...] [--small]
#include <map>

#include "../common.hpp"

using namespace ffx;

int main(int argc, char** argv) {
  Args args(argc, argv);
  FFConfig cfg(argc, argv);
  FFModel ff(cfg);
  const int b = cfg.batch_size();
  const auto dense_layers =
      parse_dash_list(args.get("--dense-layers"), std::vector<int>(args.small ? 2 : 4, args.small ? 64 : 4192));
  const auto feature_layers = parse_dash_list(args.get("--dense-feature-layers"),
                                              std::vector<int>(args.small ? 2 : 8, args.small ? 64 : 4192));
  const std::map<std::string, int> feature_shapes = {
      {"dose", 1}, {"cell.rnaseq", 942}, {"drug.descriptors", 5270}, {"drug.fingerprints", 2048}};
  const std::map<std::string, std::string> input_features = {
      {"dose1", "dose"},
      {"dose2", "dose"},
      {"cell.rnaseq", "cell.rnaseq"},
      {"drug1.descriptors", "drug.descriptors"},
      {"drug1.fingerprints", "drug.fingerprints"},
      {"drug2.descriptors", "drug.descriptors"},
      {"drug2.fingerprints", "drug.fingerprints"}};

  std::vector<Tensor> inputs, encoded;
  for (const auto& kv : input_features) {
    const std::string& fea = kv.second;
    Tensor x = ff.create_tensor({b, feature_shapes.at(fea)});
    inputs.push_back(x);
    const bool encode = fea.rfind("cell.", 0) == 0 || fea.rfind("drug.", 0) == 0;
    Tensor t = x;
    if (encode)
      for (int d : feature_layers) t = ff.dense(t, d, AC_MODE_RELU, false);
    encoded.push_back(t);
  }
  Tensor t = ff.concat(encoded, -1);
  for (int d : dense_layers) t = ff.dense(t, d, AC_MODE_RELU, false);
  t = ff.dense(t, 1, AC_MODE_NONE, false);

  SGDOptimizer opt(ff, 0.001);
  ff.compile(opt, LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, {METRICS_MEAN_SQUARED_ERROR});
  std::mt19937 rng(0);
  for (auto& x : inputs) feed_normal(ff, x, rng);
  feed_labels(ff, false, 0, rng);
  train_loop(ff, "candle_uno", args);
  return 0;
}
