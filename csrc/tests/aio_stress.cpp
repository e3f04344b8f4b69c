// Sanitizer stress test of the async I/O engine (csrc/include/sxe_aio_core.h): several client
// threads concurrently write random buffers to their own files at many offsets through one
// engine, wait on their request ids, read everything back through the engine into fresh buffers
// and compare, while another thread polls pending(); plus an error path (read past EOF) that must
// surface as an exception on the waiting client. Built by tests/test_sanitizers.py with
// -fsanitize=thread and with -fsanitize=address,undefined (host code only).
//   usage: aio_stress <scratch dir>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "sxe_aio_core.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  sxe_aio::Engine eng(64 << 10, 6);
  constexpr int kClients = 4, kChunks = 8, kIters = 3;
  constexpr int64_t kChunk = 300 * 1024 + 123;  // unaligned: buffered path; block splits mid-chunk
  std::atomic<int> failures{0};
  std::atomic<bool> stop{false};
  std::thread poller([&] {
    while (!stop.load()) {
      (void)eng.pending();
      std::this_thread::yield();
    }
  });
  std::vector<std::thread> clients;
  for (int c = 0; c < kClients; ++c) {
    clients.emplace_back([&, c] {
      std::mt19937 rng(1234 + c);
      const std::string path = dir + "/client" + std::to_string(c) + ".bin";
      for (int it = 0; it < kIters; ++it) {
        std::vector<std::vector<char>> src(kChunks, std::vector<char>(kChunk)), dst(kChunks, std::vector<char>(kChunk));
        std::vector<int64_t> ids;
        for (int k = 0; k < kChunks; ++k) {
          for (auto& b : src[k]) b = static_cast<char>(rng());
          ids.push_back(eng.submit(src[k].data(), kChunk, path, k * kChunk, true));
        }
        for (auto id : ids) eng.wait_request(id);
        ids.clear();
        for (int k = kChunks - 1; k >= 0; --k) ids.push_back(eng.submit(dst[k].data(), kChunk, path, k * kChunk, false));
        for (auto id : ids) eng.wait_request(id);
        for (int k = 0; k < kChunks; ++k)
          if (src[k] != dst[k]) failures++;
      }
      // error path: a read past the end of the file must be reported to this waiter
      std::vector<char> tail(4096);
      bool threw = false;
      try {
        eng.wait_request(eng.submit(tail.data(), 4096, path, 100LL * kChunks * kChunk, false));
      } catch (const std::runtime_error&) {
        threw = true;
      }
      if (!threw) failures++;
    });
  }
  for (auto& t : clients) t.join();
  stop = true;
  poller.join();
  (void)eng.wait();
  std::printf("aio_stress: %d mismatches/missed errors\n", failures.load());
  return failures.load() == 0 ? 0 : 1;
}
