#include "gol/parallel.hpp"
#include "gol/tuning.hpp"

#include <atomic>

#include "gol/trace.hpp"

#include <algorithm>
#include <cstdlib>

namespace gol {

ThreadPool::ThreadPool(int threads) {
  int n = std::max(1, threads) - 1;
  for (int i = 0; i < n; ++i) workers_.emplace_back([this, i] { worker_loop(i); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_start_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::parallel_for(int64_t n, const std::function<void(int64_t, int64_t)>& fn,
                              int64_t min_chunk) {
  if (n <= 0) return;
  int64_t max_chunks = int64_t(size()) * 4;
  int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(max_chunks, n / std::max<int64_t>(1, min_chunk)));
  if (chunks == 1 || workers_.empty()) {
    fn(0, n);
    return;
  }
  std::lock_guard<std::mutex> call(call_mu_);
  std::unique_lock<std::mutex> lk(mu_);
  job_ = &fn;
  job_n_ = n;
  job_chunks_ = chunks;
  next_chunk_ = 0;
  done_chunks_ = 0;
  ++epoch_;
  cv_start_.notify_all();
  // Caller participates.
  while (next_chunk_ < job_chunks_) {
    int64_t c = next_chunk_++;
    lk.unlock();
    int64_t b = c * job_n_ / job_chunks_, e = (c + 1) * job_n_ / job_chunks_;
    fn(b, e);
    lk.lock();
    ++done_chunks_;
  }
  cv_done_.wait(lk, [this] { return done_chunks_ == job_chunks_; });
  job_ = nullptr;
}

void ThreadPool::worker_loop(int) {
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_start_.wait(lk, [&] { return stop_ || (epoch_ != seen && job_ && next_chunk_ < job_chunks_); });
    if (stop_) return;
    seen = epoch_;
    while (job_ && next_chunk_ < job_chunks_) {
      int64_t c = next_chunk_++;
      const auto* fn = job_;
      int64_t n = job_n_, chunks = job_chunks_;
      lk.unlock();
      (*fn)(c * n / chunks, (c + 1) * n / chunks);
      lk.lock();
      if (++done_chunks_ == job_chunks_) cv_done_.notify_all();
    }
  }
}

int default_host_threads() {
  if (const int v = Tuning::from_env().i("host_threads"); v > 0) return v;
  unsigned hc = std::thread::hardware_concurrency();
  return int(std::min<unsigned>(hc ? hc : 4, 16));
}

ThreadPool& global_pool() {
  static ThreadPool pool(default_host_threads());
  return pool;
}

namespace trace {
namespace {
std::atomic<PushFn> g_push{nullptr};
std::atomic<PopFn> g_pop{nullptr};
}  // namespace

void set_hooks(PushFn push, PopFn pop) {
  g_push.store(push);
  g_pop.store(pop);
}
void push(const char* name) {
  if (PushFn f = g_push.load(std::memory_order_relaxed)) f(name);
}
void pop() {
  if (PopFn f = g_pop.load(std::memory_order_relaxed)) f();
}
}  // namespace trace

}  // namespace gol
