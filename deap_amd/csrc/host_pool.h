// host_pool.h — one persistent pool of host threads per library for the
// per-call passes over a population (decoding lowering metadata, launch
// plans, result copies, reading node objects).  Spawning 16 std::threads per
// pass cost ~0.1 ms a pass and several passes a call at pop 1M; the pool's
// workers sleep on a condition variable between calls.
//
// par_run(n, fn) runs fn(0) .. fn(n - 1) (the calling thread takes part) and
// returns when all have finished.  Calls are serialised.  A forked child
// gets a fresh pool (the parent's workers do not exist there).
#pragma once
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hostpool {

// threads for one pass: OMP_NUM_THREADS (the GPU box's CPU share), at most
// 16 and the hardware's count
inline int threads() {
  int t = 8;
  if (const char* env = getenv("OMP_NUM_THREADS")) t = atoi(env);
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw) t = std::min<int>(t, (int)hw);
  return std::max(1, std::min(t, 16));
}

class Pool {
 public:
  explicit Pool(int workers) : pid_(getpid()) {
    for (int i = 0; i < workers; ++i) std::thread([this] { loop(); }).detach();
  }
  pid_t pid() const { return pid_; }

  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> serial(run_mu_);
    Job j{&fn, n};
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &j;
      ++gen_;
    }
    cv_.notify_all();
    tasks(j);
    std::unique_lock<std::mutex> lk(mu_);
    job_ = nullptr;                    // no worker attaches from here on
    done_cv_.wait(lk, [&] { return j.done.load() == n && j.active == 0; });
  }

 private:
  struct Job {
    const std::function<void(int)>* fn;
    int n;
    std::atomic<int> next{0};
    std::atomic<int> done{0};
    int active = 0;                    // workers attached (under mu_)
    Job(const std::function<void(int)>* f, int k) : fn(f), n(k) {}
  };

  void tasks(Job& j) {
    for (;;) {
      const int i = j.next.fetch_add(1);
      if (i >= j.n) return;
      (*j.fn)(i);
      if (j.done.fetch_add(1) + 1 == j.n) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_all();
      }
    }
  }

  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      Job* j = job_;
      if (!j) continue;
      ++j->active;
      lk.unlock();
      tasks(*j);
      lk.lock();
      if (--j->active == 0) done_cv_.notify_all();
    }
  }

  pid_t pid_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  Job* job_ = nullptr;
  uint64_t gen_ = 0;
};

inline Pool& pool() {
  // never destroyed: its workers may still sleep in cv_ at exit
  static std::mutex mu;
  static Pool* p = nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!p || p->pid() != getpid()) p = new Pool(threads() - 1);
  return *p;
}

// fn(0) .. fn(n - 1) on the pool; n <= 1 runs inline
template <class F>
void par_run(int n, F&& fn) {
  if (n <= 1) {
    if (n == 1) fn(0);
    return;
  }
  const std::function<void(int)> f = std::forward<F>(fn);
  pool().run(n, f);
}

}  // namespace hostpool
