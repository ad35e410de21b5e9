// Blocking jobs of the daemon (Register on kubelet.sock, health sweeps) run
// on threads of their own; their results are queued and the control loop is
// woken through a pipe it polls, so the loop never blocks on a peer.
#pragma once

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace mi355x::daemon {

template <typename Result>
class Workers {
 public:
  Workers() {
    if (::pipe2(wake_, O_CLOEXEC | O_NONBLOCK) != 0) wake_[0] = wake_[1] = -1;
  }
  ~Workers() { close(); }
  Workers(const Workers&) = delete;
  Workers& operator=(const Workers&) = delete;

  int wake_fd() const { return wake_[0]; }
  void run(std::function<Result()> job) {
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::lock_guard<std::mutex> lk(mu_);
    threads_.emplace_back(std::thread([this, done, job = std::move(job)]() mutable {
                            Result c = job();
                            job = nullptr;  // what the job holds goes before the loop sees the result
                            {
                              std::lock_guard<std::mutex> lk2(mu_);
                              done_.push_back(std::move(c));
                            }
                            done->store(true);
                            const char b = 1;
                            if (::write(wake_[1], &b, 1) < 0) {
                            }
                          }),
                          done);
  }
  std::vector<Result> take() {
    char buf[256];
    while (::read(wake_[0], buf, sizeof(buf)) > 0) {
    }
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<Result> out;
    out.swap(done_);
    return out;
  }
  // joins the threads that have finished
  void reap() {
    std::vector<std::thread> finished;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = threads_.begin(); it != threads_.end();) {
        if (it->second->load()) {
          finished.push_back(std::move(it->first));
          it = threads_.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (auto& t : finished) t.join();
  }
  void join_all() {
    std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> ts;
    {
      std::lock_guard<std::mutex> lk(mu_);
      ts.swap(threads_);
    }
    for (auto& t : ts)
      if (t.first.joinable()) t.first.join();
  }
  void close() {
    join_all();
    if (wake_[0] >= 0) ::close(wake_[0]);
    if (wake_[1] >= 0) ::close(wake_[1]);
    wake_[0] = wake_[1] = -1;
  }

 private:
  std::mutex mu_;
  std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> threads_;
  std::vector<Result> done_;
  int wake_[2] = {-1, -1};
};

}  // namespace mi355x::daemon
