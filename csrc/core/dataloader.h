#pragma once
#include <condition_variable>
#include <cstdint>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

namespace ffcore {

class BatchRing {
 public:
  BatchRing(const char* data, int64_t num_samples, int64_t sample_bytes, int64_t batch, std::vector<char*> bufs);
  ~BatchRing();
  int next();              // blocks until the next batch is in a buffer; returns the slot
  void release(int slot);  // slot may be refilled (its H2D copy has completed)
  void reset(int64_t start);
  int depth() const { return (int)bufs_.size(); }

 private:
  enum State { FREE, FILLING, READY, IN_USE };
  void loop();
  void fill(int slot, int64_t pos);
  const char* data_;
  int64_t n_, sb_, batch_;
  std::vector<char*> bufs_;
  std::vector<State> state_;
  std::vector<int64_t> seq_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread worker_;
  bool stop_ = false;
  int64_t start_ = 0, produced_ = 0, consumed_ = 0;
  int64_t epoch_limit_ = std::numeric_limits<int64_t>::max();
  uint64_t gen_ = 0;
};

}  // namespace ffcore
