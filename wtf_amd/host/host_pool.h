// host_pool.h — the node's host worker pool (per-lane loops of the gpu
// backend: uploads, exit classification, module calls, harvests).
//
// The batch mutator runs on its own threads at the same time as these loops
// (runner.cc MakeBatch), so idle pool workers must give their core back
// quickly: each worker spins briefly (kSpin pause iterations, a few
// microseconds) for the next loop, then sleeps on a condition variable.
// (OpenMP's default wait policy spins for milliseconds after every parallel
// region; on the node that stole most of the mutator's CPU time.)
//
// For(n, grain, f) runs f(i) for every i in [0, n): chunks of `grain`
// indices, handed out dynamically; the calling thread takes part. A call from
// inside a loop, from a second thread while another loop runs, or with
// parallel = false runs serially on the caller.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace wtfgpu_host {

// host threads of the node (pool loops, batch mutation): OMP_NUM_THREADS when
// set (the GPU box sets the job's CPU share there), else up to 16
unsigned host_threads();

class HostPool {
 public:
  // the process-wide pool: host_threads() threads (workers + the caller)
  static HostPool &Get();
  explicit HostPool(unsigned Threads);
  ~HostPool();
  HostPool(const HostPool &) = delete;
  HostPool &operator=(const HostPool &) = delete;

  unsigned Threads() const { return (unsigned)workers_.size() + 1; }
  // the calling thread's index: 0 outside loops and for a loop's caller,
  // 1 .. Threads() - 1 for workers (per-thread arenas)
  static unsigned ThreadIndex();
  static bool InLoop();

  template <typename F>
  void For(size_t n, size_t grain, F &&f, bool parallel = true) {
    auto chunk = [](void *ctx, size_t b, size_t e) {
      F &fn = *static_cast<F *>(ctx);
      for (size_t i = b; i < e; i++) fn(i);
    };
    run(n, grain ? grain : 1, &f, chunk, parallel);
  }

 private:
  struct Job {
    size_t n, grain;
    void *ctx;
    void (*fn)(void *, size_t, size_t);
    std::atomic<size_t> next{0}, done{0};
    std::atomic<int> active{0};
  };
  void run(size_t n, size_t grain, void *ctx, void (*fn)(void *, size_t, size_t), bool parallel);
  static void work(Job &J);
  void worker(unsigned Index);

  std::vector<std::thread> workers_;
  std::mutex mu_, caller_mu_;
  std::condition_variable cv_;
  Job *job_ = nullptr;                 // the loop workers may join (under mu_)
  uint64_t gen_ = 0;                   // loops started (under mu_)
  std::atomic<uint64_t> gen_seen_{0};  // gen_, readable without the lock (spin phase)
  bool stop_ = false;
};

}  // namespace wtfgpu_host
