// host_pool.cc — see host_pool.h.
#include "host_pool.h"

#include <immintrin.h>

#include <algorithm>
#include <cstdlib>

namespace wtfgpu_host {

unsigned host_threads() {
  if (const char *E = getenv("OMP_NUM_THREADS"))
    if (atoi(E) > 0) return (unsigned)atoi(E);
  const unsigned H = std::thread::hardware_concurrency();
  return H == 0 ? 1 : std::min(H, 16u);
}

namespace {
// pause iterations before a worker sleeps (~10-40 us; WTFGPU_POOL_SPIN for A/Bs)
const int kSpin = [] {
  const char *e = getenv("WTFGPU_POOL_SPIN");
  return e ? atoi(e) : 4000;
}();
thread_local unsigned t_index = 0;
thread_local bool t_in_loop = false;
}  // namespace

HostPool &HostPool::Get() {
  static HostPool P(host_threads());
  return P;
}

HostPool::HostPool(unsigned Threads) {
  for (unsigned i = 1; i < std::max(1u, Threads); i++) workers_.emplace_back([this, i] { worker(i); });
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    gen_++;
    gen_seen_.store(gen_, std::memory_order_release);
  }
  cv_.notify_all();
  for (std::thread &t : workers_) t.join();
}

unsigned HostPool::ThreadIndex() { return t_index; }
bool HostPool::InLoop() { return t_in_loop; }

void HostPool::work(Job &J) {
  for (;;) {
    const size_t b = J.next.fetch_add(J.grain, std::memory_order_relaxed);
    if (b >= J.n) break;
    const size_t e = std::min(J.n, b + J.grain);
    J.fn(J.ctx, b, e);
    J.done.fetch_add(e - b, std::memory_order_acq_rel);
  }
}

void HostPool::run(size_t n, size_t grain, void *ctx, void (*fn)(void *, size_t, size_t), bool parallel) {
  if (n == 0) return;
  std::unique_lock<std::mutex> caller(caller_mu_, std::defer_lock);
  if (!parallel || workers_.empty() || t_in_loop || n <= grain || !caller.try_lock()) {
    fn(ctx, 0, n);
    return;
  }
  Job J;
  J.n = n;
  J.grain = grain;
  J.ctx = ctx;
  J.fn = fn;
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &J;
    gen_++;
    gen_seen_.store(gen_, std::memory_order_release);
  }
  cv_.notify_all();
  t_in_loop = true;
  work(J);
  while (J.done.load(std::memory_order_acquire) < n) _mm_pause();
  t_in_loop = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = nullptr;
  }
  // workers that joined late may still hold the job: it lives on this stack
  while (J.active.load(std::memory_order_acquire)) _mm_pause();
}

void HostPool::worker(unsigned Index) {
  t_index = Index;
  uint64_t seen = 0;
  for (;;) {
    for (int s = 0; s < kSpin && gen_seen_.load(std::memory_order_acquire) == seen; s++) _mm_pause();
    Job *j = nullptr;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      j = job_;
      if (j) j->active.fetch_add(1, std::memory_order_acq_rel);
    }
    if (!j) continue;
    t_in_loop = true;
    work(*j);
    t_in_loop = false;
    j->active.fetch_sub(1, std::memory_order_acq_rel);
  }
}

}  // namespace wtfgpu_host
