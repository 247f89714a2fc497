// Native data-loader ring (reference src/dataloader/dataloader.cc SingleDataLoader: full dataset in
// zero-copy host memory + per-iteration copy task). A background thread gathers the next batches
// of the host dataset into caller-provided PINNED buffers (torch pin_memory tensors) ahead of
// time, so the per-step work on the training thread is only an asynchronous H2D copy.
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "dataloader.h"

namespace ffcore {

BatchRing::BatchRing(const char* data, int64_t num_samples, int64_t sample_bytes, int64_t batch,
                     std::vector<char*> bufs)
    : data_(data), n_(num_samples), sb_(sample_bytes), batch_(batch), bufs_(std::move(bufs)) {
  state_.assign(bufs_.size(), FREE);
  seq_.assign(bufs_.size(), -1);
  worker_ = std::thread([this] { loop(); });
}

BatchRing::~BatchRing() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
}

void BatchRing::fill(int slot, int64_t pos) {
  char* dst = bufs_[slot];
  int64_t done = 0;
  while (done < batch_) {
    const int64_t p = (pos + done) % n_;
    const int64_t take = std::min(batch_ - done, n_ - p);
    std::memcpy(dst + done * sb_, data_ + p * sb_, (size_t)(take * sb_));
    done += take;
  }
}

void BatchRing::loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    int slot = -1;
    for (size_t i = 0; i < state_.size(); ++i)
      if (state_[i] == FREE) { slot = (int)i; break; }
    if (slot < 0 || produced_ >= epoch_limit_) {
      cv_.wait(lk);
      continue;
    }
    const int64_t seq = produced_++;
    const int64_t pos = (start_ + seq * batch_) % n_;
    const uint64_t gen = gen_;
    state_[slot] = FILLING;
    lk.unlock();
    fill(slot, pos);
    lk.lock();
    if (gen != gen_) {  // reset() happened meanwhile: discard
      state_[slot] = FREE;
      continue;
    }
    state_[slot] = READY;
    seq_[slot] = seq;
    cv_.notify_all();
  }
}

int BatchRing::next() {
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t want = consumed_;
  while (true) {
    for (size_t i = 0; i < state_.size(); ++i)
      if (state_[i] == READY && seq_[i] == want) {
        state_[i] = IN_USE;
        ++consumed_;
        cv_.notify_all();
        return (int)i;
      }
    cv_.wait(lk);
  }
}

void BatchRing::release(int slot) {
  std::lock_guard<std::mutex> g(mu_);
  state_[slot] = FREE;
  seq_[slot] = -1;
  cv_.notify_all();
}

void BatchRing::reset(int64_t start) {
  std::lock_guard<std::mutex> g(mu_);
  ++gen_;
  start_ = start;
  produced_ = 0;
  consumed_ = 0;
  for (size_t i = 0; i < state_.size(); ++i)
    if (state_[i] != FILLING) { state_[i] = FREE; seq_[i] = -1; }
  cv_.notify_all();
}

}  // namespace ffcore
