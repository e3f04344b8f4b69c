// Torch-free core of the asynchronous file I/O engine (ZeRO-Infinity NVMe tier, FastFileWriter).
//
// Parity: reference csrc/aio/py_lib/deepspeed_py_aio_handle.cpp + deepspeed_aio_thread.cpp
// (`aio_handle` async_pread/async_pwrite/wait). A fixed pool of worker threads; a request (buffer
// <-> file range) is split into `block_size` pieces served with positional pread/pwrite, so one
// large swap is spread over `num_threads` concurrent NVMe queues. O_DIRECT when buffer address,
// size and offset are 4 KiB aligned and the filesystem accepts it; buffered I/O otherwise.
// Errors are kept per request: wait_request(id) throws only that request's error (a failing read
// of one client never surfaces in another client's wait); wait() throws the first outstanding one
// and clears them all. Both report std::runtime_error.
//
// Kept free of torch so the same code builds into the sanitizer stress test
// (csrc/tests/aio_stress.cpp, -fsanitize=thread / address,undefined; tests/test_sanitizers.py).
#pragma once

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace sxe_aio {

struct FileCtx {
  int fd = -1;
  int64_t id = 0;
  std::string path;
  std::atomic<int64_t> remaining{0};
  ~FileCtx() {
    if (fd >= 0) ::close(fd);
  }
};

struct Task {
  std::shared_ptr<FileCtx> file;
  char* buf = nullptr;
  int64_t nbytes = 0;
  int64_t offset = 0;
  bool write = false;
};

inline bool aligned4k(const void* p, int64_t n, int64_t off) {
  return (reinterpret_cast<uintptr_t>(p) % 4096 == 0) && (n % 4096 == 0) && (off % 4096 == 0);
}

class Engine {
 public:
  Engine(int64_t block_size, int64_t num_threads)
      : block_size_(block_size < 4096 ? 4096 : block_size), num_threads_(num_threads < 1 ? 1 : num_threads) {
    for (int64_t i = 0; i < num_threads_; ++i) workers_.emplace_back([this] { loop(); });
  }

  ~Engine() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  int64_t block_size() const { return block_size_; }
  int64_t num_threads() const { return num_threads_; }

  // Queue a whole-buffer transfer; returns its request id. Throws if the file cannot be opened.
  int64_t submit(char* base, int64_t nbytes, const std::string& path, int64_t file_offset, bool write) {
    auto file = std::make_shared<FileCtx>();
    file->path = path;
    const int flags = write ? (O_WRONLY | O_CREAT) : O_RDONLY;
    int fd = -1;
    if (aligned4k(base, nbytes, file_offset)) fd = ::open(path.c_str(), flags | O_DIRECT, 0644);
    if (fd < 0) fd = ::open(path.c_str(), flags, 0644);
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    file->fd = fd;
    std::vector<Task> tasks;
    for (int64_t o = 0; o < nbytes; o += block_size_) {
      tasks.push_back(Task{file, base + o, std::min(block_size_, nbytes - o), file_offset + o, write});
    }
    if (tasks.empty()) tasks.push_back(Task{file, base, 0, file_offset, write});
    file->remaining = static_cast<int64_t>(tasks.size());
    const int64_t id = ++request_id_;
    file->id = id;
    {
      std::lock_guard<std::mutex> g(mu_);
      live_.insert(id);
      inflight_tasks_ += static_cast<int64_t>(tasks.size());
      for (auto& t : tasks) queue_.push_back(std::move(t));
    }
    cv_.notify_all();
    return id;
  }

  // Blocks until all submitted requests completed; returns the number completed since the
  // previous wait(). Rethrows the first I/O error.
  int64_t wait() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return inflight_tasks_ == 0; });
    const int64_t n = completed_requests_;
    completed_requests_ = 0;
    if (!errors_.empty()) {
      std::string e = errors_.begin()->second;
      errors_.clear();
      throw std::runtime_error(e);
    }
    return n;
  }

  // Blocks until request `id` completed.
  void wait_request(int64_t id) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return live_.count(id) == 0; });
    auto it = errors_.find(id);
    if (it != errors_.end()) {
      std::string e = std::move(it->second);
      errors_.erase(it);
      throw std::runtime_error(e);
    }
  }

  int64_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return inflight_tasks_;
  }

 private:
  void run(Task& t) {
    int64_t done = 0;
    while (done < t.nbytes) {
      ssize_t r = t.write ? ::pwrite(t.file->fd, t.buf + done, t.nbytes - done, t.offset + done)
                          : ::pread(t.file->fd, t.buf + done, t.nbytes - done, t.offset + done);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0 && errno == EINVAL) {
        // O_DIRECT refused for this piece (filesystem without direct I/O): fall back to buffered
        const int fl = ::fcntl(t.file->fd, F_GETFL);
        if (fl & O_DIRECT) {
          ::fcntl(t.file->fd, F_SETFL, fl & ~O_DIRECT);
          continue;
        }
      }
      if (r <= 0) {
        const std::string why = (r == 0 ? std::string("unexpected end of file") : std::string(std::strerror(errno)));
        std::lock_guard<std::mutex> g(mu_);
        errors_.emplace(t.file->id, std::string(t.write ? "pwrite " : "pread ") + t.file->path + ": " + why);
        return;
      }
      done += r;
    }
  }

  void loop() {
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
        if (stop_ && queue_.empty()) return;
        t = std::move(queue_.front());
        queue_.pop_front();
      }
      run(t);
      const bool last = (--t.file->remaining == 0);
      const int64_t id = t.file->id;
      t.file.reset();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (last) {
          ++completed_requests_;
          live_.erase(id);
        }
        --inflight_tasks_;
      }
      if (last) done_cv_.notify_all();
    }
  }

  const int64_t block_size_;
  const int64_t num_threads_;
  std::vector<std::thread> workers_;
  std::deque<Task> queue_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  int64_t inflight_tasks_ = 0;
  int64_t completed_requests_ = 0;
  std::atomic<int64_t> request_id_{0};
  std::unordered_set<int64_t> live_;
  std::unordered_map<int64_t, std::string> errors_;  // request id -> its first I/O error
};

}  // namespace sxe_aio
