// Dynamic batching queue for the inference server (flexflow_amd/serving).
//
// The reference serves through a Triton backend (triton/src/backend.cc, instance.cc) and leaves
// batching to Triton's dynamic batcher. Here the server is ours, so is the batcher: requests
// (id, rows) are pushed by the HTTP threads; the model's executor thread pops a batch when
//   * the queued rows reach a preferred batch size (largest first) or max_rows, or
//   * the oldest queued request has waited max_delay_us,
// never splitting a request and never exceeding max_rows. Waiting releases the Python GIL (the
// binding drops it), so HTTP threads keep accepting while the executor sleeps.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <vector>

namespace ffcore {

class RequestQueue {
 public:
  RequestQueue(int64_t max_rows, int64_t max_delay_us, std::vector<int64_t> preferred);
  // false if the queue is closed or the request alone exceeds max_rows
  bool push(int64_t id, int64_t rows);
  // Blocks up to timeout_us (<0: forever) for a batch; returns its request ids in arrival order
  // (empty on timeout or when closed and drained).
  std::vector<int64_t> pop(int64_t timeout_us);
  void close();
  int64_t queued_requests();
  int64_t queued_rows();
  // stats: batches popped, requests popped, rows popped
  std::vector<int64_t> stats();

 private:
  using clock = std::chrono::steady_clock;
  struct Req {
    int64_t id, rows;
    clock::time_point t;
  };
  bool ready_locked(clock::time_point now, int64_t* take) const;
  int64_t max_rows_, max_delay_us_;
  std::vector<int64_t> preferred_;  // descending
  std::deque<Req> q_;
  int64_t rows_ = 0;
  bool closed_ = false;
  int64_t n_batches_ = 0, n_reqs_ = 0, n_rows_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace ffcore
