// Minimal persistent host thread pool.  Replaces the reference's
// `#pragma omp parallel for num_threads(THREADS)` loops (THREADS=4 hard-coded,
// src/game_openmp.c:11,34) for the CPU backend, the text parser/formatter
// and the file I/O workers.  No OpenMP runtime is linked, so the library can
// share a process with PyTorch's own libgomp without conflicts.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gol {

class ThreadPool {
 public:
  explicit ThreadPool(int threads);
  ~ThreadPool();
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  int size() const { return int(workers_.size()) + 1; }
  // Runs fn(begin, end) over [0, n) split into contiguous chunks; the caller
  // thread participates.  Blocks until all chunks are done.
  void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)>& fn,
                    int64_t min_chunk = 1);

 private:
  void worker_loop(int id);
  std::vector<std::thread> workers_;
  std::mutex call_mu_;  // serialises concurrent parallel_for callers
  std::mutex mu_;
  std::condition_variable cv_start_, cv_done_;
  const std::function<void(int64_t, int64_t)>* job_ = nullptr;
  int64_t job_n_ = 0, job_chunks_ = 0;
  int64_t next_chunk_ = 0, done_chunks_ = 0;
  uint64_t epoch_ = 0;
  bool stop_ = false;
};

int default_host_threads();
ThreadPool& global_pool();

}  // namespace gol
