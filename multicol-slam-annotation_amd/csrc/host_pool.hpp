// A small persistent worker pool for the host side of a BA call (structure build and the packed
// upload of config-E-sized problems, where one thread spent ~2 ms per GlobalBA call on them).
// run(f) calls f(0) .. f(n-1) once each, f(0) on the calling thread, and returns when all are
// done.  Workers sleep on a condition variable between calls.  Host-only C++.
#pragma once
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mcs {

class HostPool {
 public:
  explicit HostPool(int n) : n_(n < 1 ? 1 : n) {
    for (int i = 1; i < n_; i++) workers_.emplace_back([this, i] { loop(i); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (std::thread& t : workers_) t.join();
  }
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;
  int size() const { return n_; }
  void run(const std::function<void(int)>& f) {
    if (n_ == 1) { f(0); return; }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      pending_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int id) {
    unsigned long long seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (quit_) return;
        job = job_;
      }
      (*job)(id);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int pending_ = 0;
  unsigned long long gen_ = 0;
  bool quit_ = false;
};

}  // namespace mcs
