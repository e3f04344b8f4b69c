// Asynchronous tensor <-> file I/O engine for ZeRO-Infinity NVMe offload.
//
// Parity: reference csrc/aio/py_lib/deepspeed_py_aio_handle.cpp + deepspeed_aio_thread.cpp
// (the `aio_handle` with async_pread/async_pwrite/wait). Design here: a fixed pool of worker
// threads; a request (whole tensor <-> file range) is split into `block_size` pieces that the
// workers serve with positional pread/pwrite, so one large swap is spread over `num_threads`
// concurrent NVMe queues. O_DIRECT is used when buffer address, size and offset are all 4 KiB
// aligned (pinned allocations from the caching host allocator are page aligned) and the
// filesystem accepts it; otherwise buffered I/O. wait() blocks until every outstanding request
// finished and rethrows the first error. Exposed as torch.classes.sxe_cpu.AioHandle.
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unordered_set>
#include <unistd.h>
#include <vector>

namespace sxe_cpu {

namespace {

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
  char* buf;
  int64_t nbytes;
  int64_t offset;
  bool write;
};

bool aligned4k(const void* p, int64_t n, int64_t off) {
  return (reinterpret_cast<uintptr_t>(p) % 4096 == 0) && (n % 4096 == 0) && (off % 4096 == 0);
}

}  // namespace

class AioHandle : public torch::CustomClassHolder {
 public:
  AioHandle(int64_t block_size, int64_t queue_depth, bool single_submit, bool overlap_events, int64_t num_threads)
      : block_size_(std::max<int64_t>(block_size, 4096)),
        queue_depth_(queue_depth),
        single_submit_(single_submit),
        overlap_events_(overlap_events),
        num_threads_(std::max<int64_t>(num_threads, 1)) {
    for (int64_t i = 0; i < num_threads_; ++i) workers_.emplace_back([this] { loop(); });
  }

  ~AioHandle() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  int64_t get_block_size() const { return block_size_; }
  int64_t get_queue_depth() const { return queue_depth_; }
  bool get_single_submit() const { return single_submit_; }
  bool get_overlap_events() const { return overlap_events_; }
  int64_t get_thread_count() const { return num_threads_; }

  int64_t async_pwrite(const at::Tensor& buf, const std::string& path, int64_t file_offset) {
    return submit(buf, path, file_offset, true);
  }
  int64_t async_pread(const at::Tensor& buf, const std::string& path, int64_t file_offset) {
    return submit(buf, path, file_offset, false);
  }
  int64_t sync_pwrite(const at::Tensor& buf, const std::string& path, int64_t file_offset) {
    submit(buf, path, file_offset, true);
    return wait();
  }
  int64_t sync_pread(const at::Tensor& buf, const std::string& path, int64_t file_offset) {
    submit(buf, path, file_offset, false);
    return wait();
  }

  // Blocks until all submitted requests completed; returns the number of requests completed since
  // the previous wait(). Rethrows the first I/O error.
  int64_t wait() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return inflight_tasks_ == 0; });
    int64_t n = completed_requests_;
    completed_requests_ = 0;
    if (!error_.empty()) {
      std::string e = error_;
      error_.clear();
      TORCH_CHECK(false, "sxe aio: ", e);
    }
    return n;
  }

  // Blocks until request `id` (returned by async_*) completed.
  void wait_request(int64_t id) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return live_.count(id) == 0; });
    if (!error_.empty()) {
      std::string e = error_;
      error_.clear();
      TORCH_CHECK(false, "sxe aio: ", e);
    }
  }

  int64_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return inflight_tasks_;
  }

 private:
  int64_t submit(const at::Tensor& buf, const std::string& path, int64_t file_offset, bool write) {
    TORCH_CHECK(buf.device().is_cpu(), "sxe aio: buffer must be a host tensor");
    TORCH_CHECK(buf.is_contiguous(), "sxe aio: buffer must be contiguous");
    char* base = static_cast<char*>(buf.data_ptr());
    const int64_t nbytes = buf.numel() * buf.element_size();
    auto file = std::make_shared<FileCtx>();
    file->path = path;
    int flags = write ? (O_WRONLY | O_CREAT) : O_RDONLY;
    int fd = -1;
    if (aligned4k(base, nbytes, file_offset)) fd = ::open(path.c_str(), flags | O_DIRECT, 0644);
    if (fd < 0) fd = ::open(path.c_str(), flags, 0644);
    TORCH_CHECK(fd >= 0, "sxe aio: cannot open ", path, ": ", std::strerror(errno));
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

  void run(Task& t) {
    int64_t done = 0;
    while (done < t.nbytes) {
      ssize_t r = t.write ? ::pwrite(t.file->fd, t.buf + done, t.nbytes - done, t.offset + done)
                          : ::pread(t.file->fd, t.buf + done, t.nbytes - done, t.offset + done);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0 && errno == EINVAL) {
        // O_DIRECT refused for this piece (filesystem without direct I/O): fall back to buffered
        int fl = ::fcntl(t.file->fd, F_GETFL);
        if (fl & O_DIRECT) {
          ::fcntl(t.file->fd, F_SETFL, fl & ~O_DIRECT);
          continue;
        }
      }
      if (r <= 0) {
        std::lock_guard<std::mutex> g(mu_);
        if (error_.empty())
          error_ = std::string(t.write ? "pwrite " : "pread ") + t.file->path + ": " +
                   (r == 0 ? std::string("unexpected end of file") : std::string(std::strerror(errno)));
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
      bool last = (--t.file->remaining == 0);
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

  int64_t block_size_, queue_depth_;
  bool single_submit_, overlap_events_;
  int64_t num_threads_;
  std::vector<std::thread> workers_;
  std::deque<Task> queue_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  int64_t inflight_tasks_ = 0;
  int64_t completed_requests_ = 0;
  std::atomic<int64_t> request_id_{0};
  std::unordered_set<int64_t> live_;
  std::string error_;
};

}  // namespace sxe_cpu

TORCH_LIBRARY_FRAGMENT(sxe_cpu, m) {
  m.class_<sxe_cpu::AioHandle>("AioHandle")
      .def(torch::init<int64_t, int64_t, bool, bool, int64_t>())
      .def("async_pwrite", &sxe_cpu::AioHandle::async_pwrite)
      .def("async_pread", &sxe_cpu::AioHandle::async_pread)
      .def("sync_pwrite", &sxe_cpu::AioHandle::sync_pwrite)
      .def("sync_pread", &sxe_cpu::AioHandle::sync_pread)
      .def("wait", &sxe_cpu::AioHandle::wait)
.def("wait_request", &sxe_cpu::AioHandle::wait_request)
      .def("pending", &sxe_cpu::AioHandle::pending)
      .def("get_block_size", &sxe_cpu::AioHandle::get_block_size)
      .def("get_queue_depth", &sxe_cpu::AioHandle::get_queue_depth)
      .def("get_single_submit", &sxe_cpu::AioHandle::get_single_submit)
      .def("get_overlap_events", &sxe_cpu::AioHandle::get_overlap_events)
      .def("get_thread_count", &sxe_cpu::AioHandle::get_thread_count);
}
