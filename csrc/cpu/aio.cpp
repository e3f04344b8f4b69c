// torch.classes.sxe_cpu.AioHandle: tensor-facing binding of the async file I/O engine
// (csrc/include/sxe_aio_core.h, which carries the design notes and the reference parity:
// csrc/aio/py_lib/deepspeed_py_aio_handle.cpp `aio_handle` async_pread/async_pwrite/wait).
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>

#include "sxe_aio_core.h"

namespace sxe_cpu {

class AioHandle : public torch::CustomClassHolder {
 public:
  AioHandle(int64_t block_size, int64_t queue_depth, bool single_submit, bool overlap_events, int64_t num_threads)
      : engine_(block_size, num_threads),
        queue_depth_(queue_depth),
        single_submit_(single_submit),
        overlap_events_(overlap_events) {}

  int64_t get_block_size() const { return engine_.block_size(); }
  int64_t get_queue_depth() const { return queue_depth_; }
  bool get_single_submit() const { return single_submit_; }
  bool get_overlap_events() const { return overlap_events_; }
  int64_t get_thread_count() const { return engine_.num_threads(); }

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

  int64_t wait() {
    try {
      return engine_.wait();
    } catch (const std::exception& e) {
      TORCH_CHECK(false, "sxe aio: ", e.what());
    }
  }

  void wait_request(int64_t id) {
    try {
      engine_.wait_request(id);
    } catch (const std::exception& e) {
      TORCH_CHECK(false, "sxe aio: ", e.what());
    }
  }

  int64_t pending() { return engine_.pending(); }

 private:
  int64_t submit(const at::Tensor& buf, const std::string& path, int64_t file_offset, bool write) {
    TORCH_CHECK(buf.device().is_cpu(), "sxe aio: buffer must be a host tensor");
    TORCH_CHECK(buf.is_contiguous(), "sxe aio: buffer must be contiguous");
    try {
      return engine_.submit(static_cast<char*>(buf.data_ptr()), buf.numel() * buf.element_size(), path, file_offset,
                            write);
    } catch (const std::exception& e) {
      TORCH_CHECK(false, "sxe aio: ", e.what());
    }
  }

  sxe_aio::Engine engine_;
  int64_t queue_depth_;
  bool single_submit_, overlap_events_;
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
