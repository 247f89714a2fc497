// Shared driver pieces for the C++ examples: example-only flags, synthetic inputs of the model's
// shapes, and the timed training loop of the reference examples (examples/cpp/*/ top_level_task:
// fixed synthetic batch, forward / zero_gradients / backward / update per iteration, then
// "ELAPSED TIME = ..., THROUGHPUT = ... samples/s").
#ifndef FF_EXAMPLES_COMMON_HPP
#define FF_EXAMPLES_COMMON_HPP

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "flexflow.hpp"

namespace ffx {

using namespace flexflow;

struct Args {
  int iterations = 10;
  bool small = false;  // reduced widths / image sizes (CPU runs)
  int argc = 0;
  char** argv = nullptr;

  Args(int c, char** v) : argc(c), argv(v) {
    for (int i = 1; i < c; ++i) {
      if (!std::strcmp(v[i], "--iterations") && i + 1 < c) iterations = std::atoi(v[++i]);
      else if (!std::strcmp(v[i], "--small")) small = true;
    }
  }
  // value of an example-specific "--flag value" (nullptr when absent)
  const char* get(const char* flag) const {
    for (int i = 1; i + 1 < argc; ++i)
      if (!std::strcmp(argv[i], flag)) return argv[i + 1];
    return nullptr;
  }
  int get_int(const char* flag, int def) const {
    const char* s = get(flag);
    return s ? std::atoi(s) : def;
  }
};

// "64-64-2" -> {64, 64, 2} (the reference's --arch-mlp-* / --arch-embedding-size format)
inline std::vector<int> parse_dash_list(const char* s, std::vector<int> def) {
  if (!s) return def;
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, '-'))
    if (!tok.empty()) out.push_back(std::atoi(tok.c_str()));
  return out;
}

inline int64_t volume(const Tensor& t) {
  int64_t n = 1;
  for (int d : t.dims()) n *= d;
  return n;
}

inline void feed_normal(FFModel& ff, const Tensor& t, std::mt19937& rng) {
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> v((size_t)volume(t));
  for (auto& x : v) x = nd(rng);
  ff.set_tensor(t, v);
}

inline void feed_indices(FFModel& ff, const Tensor& t, int hi, std::mt19937& rng) {
  std::uniform_int_distribution<int64_t> ud(0, hi - 1);
  std::vector<int64_t> v((size_t)volume(t));
  for (auto& x : v) x = ud(rng);
  ff.set_tensor(t, v);
}

// class labels for sparse categorical cross-entropy, or N(0,1) targets for MSE
inline void feed_labels(FFModel& ff, bool sparse, int num_classes, std::mt19937& rng) {
  Tensor lab = ff.label_tensor();
  if (sparse) {
    std::uniform_int_distribution<int32_t> ud(0, num_classes - 1);
    std::vector<int32_t> v((size_t)volume(lab));
    for (auto& x : v) x = ud(rng);
    ff.set_tensor(lab, v);
  } else {
    feed_normal(ff, lab, rng);
  }
}

// one warm-up step (kernel autotuning, HIP-graph capture), then `iterations` timed steps
inline void train_loop(FFModel& ff, const char* name, const Args& args) {
  ff.init_operators();
  ff.train_step();
  ff.reset_metrics();
  const double t0 = current_time_in_microseconds();
  for (int it = 0; it < args.iterations; ++it) ff.train_step();
  const float loss = ff.loss();  // host read-back: waits for the device
  const double run_time = 1e-6 * (current_time_in_microseconds() - t0);
  std::printf("%s: ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s, loss %.5f, strategy %s\n", name, run_time,
              ff.config().batch_size() * args.iterations / run_time, loss, ff.strategy_name().c_str());
}

}  // namespace ffx

#endif
