// Host runtime: asynchronous device -> file writer with a pinned staging ring (non-blocking checkpoint saves).
//
// The mirror of h2d_engine.cpp for the other direction. A checkpoint save hands over device tensors (a snapshot the
// caller made on the device, so training may modify the live state right away) together with the file and byte
// offset each one goes to; the writer streams them out in slot-sized pieces:
//   dispatcher thread: wait for a free pinned slot, hipMemcpyAsync(D2H) of the next piece on the writer's own HIP
//                      stream (ordered after the producer's stream by an event recorded at enqueue), record the slot's
//                      event;
//   writer threads:    hipEventSynchronize on a filled slot, pwrite() it at its file offset, free the slot.
// Host memory stays at num_slots x slot_bytes whatever the checkpoint size (the round-5 synchronous save went through
// `.cpu()` of every shard: a 67 GiB RSS spike for Llama-3-8B at one rank), PCIe DMA and disk writes overlap, and the
// training step that follows the save only shares HBM bandwidth with the DMA. `finish()` blocks until every piece is
// on disk (fsync'd), closes the files and returns the number of failed writes.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#define D2H_OK(expr)                                                                                               \
  do {                                                                                                            \
    hipError_t _e = (expr);                                                                                       \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

namespace {

class D2HFileWriter {
 public:
  D2HFileWriter(int device, int64_t num_slots, int64_t slot_bytes, int64_t num_writers)
      : device_(device), slot_bytes_(slot_bytes) {
    TORCH_CHECK(num_slots >= 2 && slot_bytes >= (1 << 16), "D2HFileWriter: need >= 2 slots of >= 64 KiB");
    D2H_OK(hipSetDevice(device_));
    D2H_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, 0));
    for (int64_t i = 0; i < num_slots; ++i) {
      void* p = nullptr;
      D2H_OK(hipHostMalloc(&p, slot_bytes_, hipHostMallocDefault));
      hipEvent_t ev;
      D2H_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      slots_.push_back({p, ev});
      free_.push_back((int)i);
    }
    dispatcher_ = std::thread([this] { dispatch_loop(); });
    for (int64_t t = 0; t < std::max<int64_t>(1, num_writers); ++t) writers_.emplace_back([this] { write_loop(); });
  }

  ~D2HFileWriter() {
    try {
      finish();
    } catch (...) {
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    dispatcher_.join();
    for (auto& w : writers_) w.join();
    hipSetDevice(device_);
    hipStreamSynchronize(stream_);
    for (auto& s : slots_) {
      hipEventDestroy(s.ev);
      hipHostFree(s.ptr);
    }
    for (auto& e : order_events_) hipEventDestroy(e);
    hipStreamDestroy(stream_);
  }

  // Enqueue the bytes of `src` (contiguous; a HIP tensor, or a CPU tensor) for [offset, offset + nbytes) of `path`.
  // The DMA is ordered after everything already enqueued on the caller's current stream; `src` is kept alive until
  // its last piece has been copied out.
  void write(const std::string& path, int64_t offset, torch::Tensor src) {
    TORCH_CHECK(src.is_contiguous(), "D2HFileWriter.write: contiguous tensor expected");
    TORCH_CHECK(offset >= 0, "D2HFileWriter.write: negative offset");
    const int64_t n = src.nbytes();
    std::lock_guard<std::mutex> g(mu_);
    const int fd = open_locked(path);
    hipEvent_t after = nullptr;
    if (src.is_cuda()) {
      D2H_OK(hipSetDevice(device_));
      D2H_OK(hipEventCreateWithFlags(&after, hipEventDisableTiming));
      D2H_OK(hipEventRecord(after, at::hip::getCurrentHIPStream().stream()));
      order_events_.push_back(after);
    }
    const char* base = static_cast<const char*>(src.data_ptr());
    keep_.push_back(src);
    for (int64_t off = 0; off < n; off += slot_bytes_) {
      Piece p;
      p.src = base + off;
      p.len = std::min<int64_t>(slot_bytes_, n - off);
      p.fd = fd;
      p.file_off = offset + off;
      p.device = src.is_cuda();
      p.after = (off == 0) ? after : nullptr;
      todo_.push_back(p);
      ++pending_;
    }
    cv_.notify_all();
  }

  // Enqueue raw host bytes (a safetensors header) for [offset, offset + size) of `path`.
  void write_bytes(const std::string& path, int64_t offset, const std::string& bytes) {
    auto t = torch::empty({(int64_t)bytes.size()}, torch::TensorOptions().dtype(torch::kUInt8));
    std::memcpy(t.data_ptr(), bytes.data(), bytes.size());
    write(path, offset, t);
  }

  // Block until every enqueued piece is on disk; fsync + close the files. Returns the number of failed writes since
  // the last call (0 = all good) and resets it.
  int64_t finish() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      idle_cv_.wait(lk, [this] { return pending_ == 0; });
      for (auto& kv : fds_) {
        if (::fsync(kv.second) != 0) errors_.fetch_add(1);
        ::close(kv.second);
      }
      fds_.clear();
      keep_.clear();
      D2H_OK(hipSetDevice(device_));
      for (auto& e : order_events_) hipEventDestroy(e);
      order_events_.clear();
    }
    return errors_.exchange(0);
  }

  int64_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return pending_;
  }

  int64_t bytes_written() const { return bytes_.load(); }
  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t num_slots() const { return (int64_t)slots_.size(); }

 private:
  struct Slot {
    void* ptr;
    hipEvent_t ev;
  };
  struct Piece {
    const char* src;
    int64_t len;
    int fd;
    int64_t file_off;
    bool device;
    hipEvent_t after;
  };
  struct Filled {
    int slot;
    int64_t len;
    int fd;
    int64_t file_off;
  };

  int open_locked(const std::string& path) {
    auto it = fds_.find(path);
    if (it != fds_.end()) return it->second;
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
    TORCH_CHECK(fd >= 0, "D2HFileWriter: cannot open ", path, " for writing");
    fds_[path] = fd;
    return fd;
  }

  void dispatch_loop() {
    hipSetDevice(device_);
    for (;;) {
      Piece p;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || (!todo_.empty() && !free_.empty()); });
        if (stop_ && todo_.empty()) return;
        if (todo_.empty() || free_.empty()) continue;
        p = todo_.front();
        todo_.pop_front();
        slot = free_.front();
        free_.pop_front();
      }
      Slot& s = slots_[slot];
      if (p.device) {
        if (p.after != nullptr) D2H_OK(hipStreamWaitEvent(stream_, p.after, 0));
        D2H_OK(hipMemcpyAsync(s.ptr, p.src, p.len, hipMemcpyDeviceToHost, stream_));
        D2H_OK(hipEventRecord(s.ev, stream_));
      } else {
        std::memcpy(s.ptr, p.src, p.len);
        D2H_OK(hipEventRecord(s.ev, stream_));
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        filled_.push_back({slot, p.len, p.fd, p.file_off});
      }
      cv_.notify_all();
    }
  }

  void write_loop() {
    hipSetDevice(device_);
    for (;;) {
      Filled f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !filled_.empty(); });
        if (stop_ && filled_.empty()) return;
        f = filled_.front();
        filled_.pop_front();
      }
      Slot& s = slots_[f.slot];
      (void)hipEventSynchronize(s.ev);
      const char* q = static_cast<const char*>(s.ptr);
      int64_t done = 0;
      while (done < f.len) {
        const ssize_t put = ::pwrite(f.fd, q + done, (size_t)(f.len - done), (off_t)(f.file_off + done));
        if (put <= 0) {
          errors_.fetch_add(1);
          break;
        }
        done += put;
      }
      bytes_.fetch_add(done);
      {
        std::lock_guard<std::mutex> g(mu_);
        free_.push_back(f.slot);
        if (--pending_ == 0) idle_cv_.notify_all();
      }
      cv_.notify_all();
    }
  }

  int device_;
  int64_t slot_bytes_;
  hipStream_t stream_;
  std::vector<Slot> slots_;
  std::deque<int> free_;
  std::deque<Piece> todo_;
  std::deque<Filled> filled_;
  std::vector<torch::Tensor> keep_;
  std::vector<hipEvent_t> order_events_;
  std::map<std::string, int> fds_;
  std::thread dispatcher_;
  std::vector<std::thread> writers_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  int64_t pending_ = 0;
  bool stop_ = false;
  std::atomic<int64_t> errors_{0};
  std::atomic<int64_t> bytes_{0};
};

}  // namespace

void register_d2h_writer(pybind11::module& m) {
  pybind11::class_<D2HFileWriter>(m, "D2HFileWriter", pybind11::module_local())
      .def(pybind11::init<int, int64_t, int64_t, int64_t>(), pybind11::arg("device"), pybind11::arg("num_slots") = 8,
           pybind11::arg("slot_bytes") = 64 << 20, pybind11::arg("num_writers") = 2)
      .def("write", &D2HFileWriter::write, pybind11::arg("path"), pybind11::arg("offset"), pybind11::arg("src"),
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("write_bytes", &D2HFileWriter::write_bytes, pybind11::arg("path"), pybind11::arg("offset"), pybind11::arg("data"))
      .def("finish", &D2HFileWriter::finish, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("pending", &D2HFileWriter::pending)
      .def_property_readonly("bytes_written", &D2HFileWriter::bytes_written)
      .def_property_readonly("slot_bytes", &D2HFileWriter::slot_bytes)
      .def_property_readonly("num_slots", &D2HFileWriter::num_slots);
}
