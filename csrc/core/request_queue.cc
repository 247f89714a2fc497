#include "request_queue.h"

#include <algorithm>

namespace ffcore {

RequestQueue::RequestQueue(int64_t max_rows, int64_t max_delay_us, std::vector<int64_t> preferred)
    : max_rows_(std::max<int64_t>(1, max_rows)), max_delay_us_(std::max<int64_t>(0, max_delay_us)),
      preferred_(std::move(preferred)) {
  preferred_.erase(std::remove_if(preferred_.begin(), preferred_.end(),
                                  [&](int64_t p) { return p <= 0 || p > max_rows_; }),
                   preferred_.end());
  std::sort(preferred_.rbegin(), preferred_.rend());
}

bool RequestQueue::push(int64_t id, int64_t rows) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_ || rows <= 0 || rows > max_rows_) return false;
    q_.push_back({id, rows, clock::now()});
    rows_ += rows;
  }
  cv_.notify_all();
  return true;
}

// How many requests (from the front) form the batch, if one is due now.
bool RequestQueue::ready_locked(clock::time_point now, int64_t* take) const {
  if (q_.empty()) return false;
  // greedy prefix that fits max_rows
  int64_t rows = 0, n = 0;
  for (const auto& r : q_) {
    if (rows + r.rows > max_rows_) break;
    rows += r.rows;
    ++n;
  }
  const bool full = rows == max_rows_ || n < (int64_t)q_.size();  // the next request would not fit
  // a preferred size reached exactly by some prefix
  int64_t pref_n = 0;
  if (!preferred_.empty()) {
    int64_t acc = 0;
    for (int64_t i = 0; i < n; ++i) {
      acc += q_[i].rows;
      if (std::find(preferred_.begin(), preferred_.end(), acc) != preferred_.end()) pref_n = i + 1;
    }
  }
  const bool due = std::chrono::duration_cast<std::chrono::microseconds>(now - q_.front().t).count() >= max_delay_us_;
  if (full || due || closed_) {
    *take = n;
    return true;
  }
  if (pref_n > 0 && pref_n == n) {  // the whole fitting prefix is a preferred size: no reason to wait
    *take = pref_n;
    return true;
  }
  return false;
}

std::vector<int64_t> RequestQueue::pop(int64_t timeout_us) {
  std::unique_lock<std::mutex> lk(mu_);
  const auto deadline = clock::now() + std::chrono::microseconds(timeout_us < 0 ? 0 : timeout_us);
  for (;;) {
    const auto now = clock::now();
    int64_t take = 0;
    if (ready_locked(now, &take)) {
      std::vector<int64_t> ids;
      int64_t rows = 0;
      for (int64_t i = 0; i < take; ++i) {
        ids.push_back(q_.front().id);
        rows += q_.front().rows;
        q_.pop_front();
      }
      rows_ -= rows;
      ++n_batches_;
      n_reqs_ += take;
      n_rows_ += rows;
      return ids;
    }
    if (closed_ && q_.empty()) return {};
    if (timeout_us >= 0 && now >= deadline) return {};
    // wake at the earlier of: the oldest request's delay expiry, the caller's deadline
    auto wake = timeout_us >= 0 ? deadline : now + std::chrono::hours(1);
    if (!q_.empty()) wake = std::min(wake, q_.front().t + std::chrono::microseconds(max_delay_us_));
    cv_.wait_until(lk, wake);
  }
}

void RequestQueue::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

int64_t RequestQueue::queued_requests() {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)q_.size();
}

int64_t RequestQueue::queued_rows() {
  std::lock_guard<std::mutex> g(mu_);
  return rows_;
}

std::vector<int64_t> RequestQueue::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return {n_batches_, n_reqs_, n_rows_};
}

}  // namespace ffcore
