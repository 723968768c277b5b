// Host runtime: asynchronous host->device copy engine with a pinned staging ring.
//
// Sources: a host tensor (pageable pieces are memcpy'd into the ring, pinned ones DMA'd directly), or a byte range
// of a FILE (`copy_file`: the checkpoint loader's path for safetensors shards — the workers pread() straight into the
// pinned slots, several in parallel, so the bytes are copied once on the host instead of mmap -> pageable tensor ->
// pinned, and no page-table entries are created for a 140 GB checkpoint).
//
// Used by big-model inference (offloaded weights are uploaded block by block ahead of use), checkpoint loading
// (safetensors mmap -> HBM) and FSDP CPU offload. A pageable source (e.g. an mmap'd checkpoint) cannot be
// DMA'd directly; the engine splits it into slot-sized pieces, worker threads memcpy each piece into one of
// `num_slots` pinned host slots (hipHostMalloc), and each filled slot is uploaded with hipMemcpyAsync on the
// engine's own HIP stream. A per-slot HIP event gates slot reuse, so CPU copies, PCIe DMA and GPU compute all
// overlap. Consumers order against the uploads with `wait_on_current_stream()` (hipStreamWaitEvent on the
// caller's torch stream — no host blocking).
#include "host_kernels.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <map>
#include <string>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#define HIP_OK(expr)                                                                         \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

namespace {

class H2DEngine {
 public:
  H2DEngine(int device, int64_t num_slots, int64_t slot_bytes, int64_t num_threads)
      : device_(device), slot_bytes_(slot_bytes) {
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, -1));
    HIP_OK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
    for (int64_t i = 0; i < num_slots; ++i) {
      void* p = nullptr;
      HIP_OK(hipHostMalloc(&p, slot_bytes_, hipHostMallocDefault));
      hipEvent_t ev;
      HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      slots_.push_back({p, ev, false});
    }
    for (int64_t t = 0; t < std::max<int64_t>(1, num_threads); ++t) workers_.emplace_back([this] { worker(); });
  }

  ~H2DEngine() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
    for (auto& kv : fds_) ::close(kv.second);
    hipSetDevice(device_);
    hipStreamSynchronize(stream_);
    for (auto& f : inflight_) hipEventDestroy(f.ev);
    inflight_.clear();
    for (auto& s : slots_) {
      hipEventDestroy(s.ev);
      hipHostFree(s.ptr);
    }
    hipEventDestroy(done_);
    hipStreamDestroy(stream_);
  }

  // Enqueue a copy of a CPU tensor (pageable or pinned, contiguous) into a contiguous device tensor.
  void copy(torch::Tensor src, torch::Tensor dst) {
    TORCH_CHECK(src.device().is_cpu() && dst.is_cuda(), "H2DEngine.copy: src must be CPU, dst a HIP tensor");
    TORCH_CHECK(src.is_contiguous() && dst.is_contiguous(), "H2DEngine.copy: tensors must be contiguous");
    TORCH_CHECK(src.nbytes() == dst.nbytes(), "H2DEngine.copy: size mismatch");
    const char* s = static_cast<const char*>(src.data_ptr());
    char* d = static_cast<char*>(dst.data_ptr());
    const int64_t n = src.nbytes();
    if (src.is_pinned()) {  // already DMA-able: one async copy, no staging
      std::lock_guard<std::mutex> g(mu_);
      HIP_OK(hipSetDevice(device_));
      retire_completed();
      HIP_OK(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, stream_));
      // torch's pinned allocator does not see this DMA: the source stays referenced until the copy's own event has
      // completed (not merely been enqueued), so its block cannot be recycled mid-transfer
      hipEvent_t ev;
      HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIP_OK(hipEventRecord(ev, stream_));
      inflight_.push_back({src, ev});
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int64_t off = 0; off < n; off += slot_bytes_) {
        const int64_t len = std::min<int64_t>(slot_bytes_, n - off);
        tasks_.push_back({s + off, d + off, len, -1, 0});
        ++pending_;
      }
      staged_.push_back(src);  // pageable: read by the workers' memcpy into the pinned ring, released at drain
    }
    cv_.notify_all();
  }

  // Enqueue a copy of bytes [offset, offset + dst.nbytes()) of the file at `path` into a contiguous device tensor.
  void copy_file(const std::string& path, int64_t offset, torch::Tensor dst) {
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "H2DEngine.copy_file: dst must be a contiguous HIP tensor");
    TORCH_CHECK(offset >= 0, "H2DEngine.copy_file: negative offset");
    char* d = static_cast<char*>(dst.data_ptr());
    const int64_t n = dst.nbytes();
    {
      std::lock_guard<std::mutex> g(mu_);
      int fd;
      auto it = fds_.find(path);
      if (it == fds_.end()) {
        fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        TORCH_CHECK(fd >= 0, "H2DEngine.copy_file: cannot open ", path);
        fds_[path] = fd;
      } else {
        fd = it->second;
      }
      for (int64_t off = 0; off < n; off += slot_bytes_) {
        const int64_t len = std::min<int64_t>(slot_bytes_, n - off);
        tasks_.push_back({nullptr, d + off, len, fd, offset + off});
        ++pending_;
      }
    }
    cv_.notify_all();
  }

  // Close the files opened by copy_file (after every piece has been read) and return the number of short reads
  // since the last call, resetting it: the engine is cached per device for the process lifetime, so one failed
  // load must not poison the next one.
  int64_t close_files() {
    drain_issue();
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : fds_) ::close(kv.second);
    fds_.clear();
    return read_errors_.exchange(0);
  }

  // Block the host until every enqueued piece has been staged and its DMA issued, then make the caller's
  // current torch stream wait on the engine's stream (device-side ordering, no host wait for the DMA).
  void wait_on_current_stream() {
    drain_issue();
    std::lock_guard<std::mutex> g(mu_);
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipEventRecord(done_, stream_));
    HIP_OK(hipStreamWaitEvent(at::hip::getCurrentHIPStream().stream(), done_, 0));
    staged_.clear();  // every staged piece has been memcpy'd into the ring (drain_issue)
    retire_completed();  // pinned sources: only those whose DMA has finished
  }

  void synchronize() {
    drain_issue();
    HIP_OK(hipSetDevice(device_));
    HIP_OK(hipStreamSynchronize(stream_));
    std::lock_guard<std::mutex> g(mu_);
    staged_.clear();
    retire_completed();
  }

  int64_t inflight() {
    std::lock_guard<std::mutex> g(mu_);
    retire_completed();
    return (int64_t)inflight_.size();
  }

  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t num_slots() const { return (int64_t)slots_.size(); }

 private:
  struct Slot {
    void* ptr;
    hipEvent_t ev;
    bool busy;
  };
  struct Task {
    const char* src;  // host source, or nullptr for a file range
    char* dst;
    int64_t len;
    int fd = -1;
    int64_t file_off = 0;
  };

  // caller holds mu_
  void retire_completed() {
    while (!inflight_.empty() && hipEventQuery(inflight_.front().ev) == hipSuccess) {
      hipEventDestroy(inflight_.front().ev);
      inflight_.pop_front();
    }
  }

  void drain_issue() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [this] { return pending_ == 0; });
  }

  int acquire_slot(std::unique_lock<std::mutex>& lk) {
    for (;;) {
      for (size_t i = 0; i < slots_.size(); ++i) {
        if (!slots_[i].busy) {
          slots_[i].busy = true;
          return (int)i;
        }
        // reclaim slots whose DMA has finished
        if (hipEventQuery(slots_[i].ev) == hipSuccess && slots_[i].busy && reclaimable_[i]) {
          reclaimable_[i] = false;
          return (int)i;
        }
      }
      lk.unlock();
      std::this_thread::yield();
      lk.lock();
    }
  }

  void worker() {
    HIP_OK(hipSetDevice(device_));
    for (;;) {
      Task t;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !tasks_.empty(); });
        if (stop_ && tasks_.empty()) return;
        t = tasks_.front();
        tasks_.pop_front();
        if (reclaimable_.size() != slots_.size()) reclaimable_.assign(slots_.size(), false);
        slot = acquire_slot(lk);
      }
      // a recycled slot's previous DMA must be complete before overwriting it
      HIP_OK(hipEventSynchronize(slots_[slot].ev));
      if (t.fd >= 0) {
        char* p = static_cast<char*>(slots_[slot].ptr);
        int64_t done = 0;
        while (done < t.len) {
          const ssize_t got = ::pread(t.fd, p + done, (size_t)(t.len - done), (off_t)(t.file_off + done));
          if (got <= 0) {  // short file / IO error: leave the bytes zero rather than hang; the loader validated sizes
            std::memset(p + done, 0, (size_t)(t.len - done));
            read_errors_.fetch_add(1);
            break;
          }
          done += got;
        }
      } else {
        std::memcpy(slots_[slot].ptr, t.src, t.len);
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        HIP_OK(hipMemcpyAsync(t.dst, slots_[slot].ptr, t.len, hipMemcpyHostToDevice, stream_));
        HIP_OK(hipEventRecord(slots_[slot].ev, stream_));
        reclaimable_[slot] = true;
        if (--pending_ == 0) idle_cv_.notify_all();
      }
    }
  }

  int device_;
  int64_t slot_bytes_;
  hipStream_t stream_;
  hipEvent_t done_;
  std::vector<Slot> slots_;
  std::vector<bool> reclaimable_;
  std::deque<Task> tasks_;
  struct Inflight {
    torch::Tensor src;
    hipEvent_t ev;
  };
  std::deque<Inflight> inflight_;       // pinned sources of DMAs not yet known complete (in stream order)
  std::vector<torch::Tensor> staged_;   // pageable sources still being copied into the ring
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  int64_t pending_ = 0;
  bool stop_ = false;
  std::map<std::string, int> fds_;
  std::atomic<int64_t> read_errors_{0};

 public:
  int64_t read_errors() const { return read_errors_.load(); }
};


}  // namespace

// module_local: the release (`_C`) and debug (`_C_debug`) builds register the same classes and may be loaded into one
// process (tests/test_debug_kernels_gpu.py compares them)
void register_runtime(pybind11::module& m) {
  pybind11::class_<H2DEngine>(m, "H2DEngine", pybind11::module_local())
      .def(pybind11::init<int, int64_t, int64_t, int64_t>(), pybind11::arg("device"), pybind11::arg("num_slots") = 4,
           pybind11::arg("slot_bytes") = 64 << 20, pybind11::arg("num_threads") = 4)
      .def("copy", &H2DEngine::copy, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("copy_file", &H2DEngine::copy_file, pybind11::arg("path"), pybind11::arg("offset"), pybind11::arg("dst"),
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("close_files", &H2DEngine::close_files, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("read_errors", &H2DEngine::read_errors)
      .def("wait_on_current_stream", &H2DEngine::wait_on_current_stream, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("synchronize", &H2DEngine::synchronize, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("inflight", &H2DEngine::inflight)
      .def_property_readonly("slot_bytes", &H2DEngine::slot_bytes)
      .def_property_readonly("num_slots", &H2DEngine::num_slots);
  pybind11::class_<acc_host::CollectiveSeq>(m, "CollectiveSeq", pybind11::module_local())
      .def(pybind11::init<>())
      .def("record", &acc_host::CollectiveSeq::record)
      .def("digest", &acc_host::CollectiveSeq::digest)
      .def("count", &acc_host::CollectiveSeq::count)
      .def("reset", &acc_host::CollectiveSeq::reset);
}
