// Asynchronous tensor <-> file I/O for ZeRO-Infinity (NVMe offload of params / optimizer state) and checkpoint
// swapping.
//
// Parity: reference `csrc/aio/py_lib/py_ds_aio.cpp:14-46` (aio_read, aio_write, deepspeed_memcpy, class aio_handle
// with sync_/async_ pread/pwrite, wait, new_cpu_locked_tensor) built on libaio (`deepspeed_aio_common.cpp`).
// This image has no libaio, and the GPU boxes are ordinary users, so the engine is a native thread pool issuing
// pread/pwrite in `block_size` pieces with `queue_depth` pieces in flight per thread, O_DIRECT when buffer, offset and
// length are 4 KiB aligned (falls back to buffered I/O otherwise). Pinned (page-locked) host tensors come from
// hipHostMalloc via torch's pinned allocator on the Python side; here `new_cpu_locked_tensor` uses posix_memalign +
// mlock so that O_DIRECT works and the pages stay resident.
#include <torch/extension.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr size_t kAlign = 4096;

int open_file(const std::string& fn, bool write, bool direct) {
  int flags = write ? (O_WRONLY | O_CREAT) : O_RDONLY;
  if (direct) flags |= O_DIRECT;
  int fd = ::open(fn.c_str(), flags, 0644);
  if (fd < 0 && direct) return open_file(fn, write, false);
  return fd;
}

// Transfer [buf, buf+len) at file offset `off` in pieces of `block` bytes.
int64_t do_io(int fd, char* buf, int64_t len, int64_t off, int64_t block, bool write) {
  int64_t done = 0;
  while (done < len) {
    const int64_t n = std::min(block, len - done);
    ssize_t r = write ? ::pwrite(fd, buf + done, n, off + done) : ::pread(fd, buf + done, n, off + done);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) break;
    done += r;
  }
  return done;
}

class ThreadPool {
 public:
  explicit ThreadPool(int n) : stop_(false) {
    for (int i = 0; i < std::max(1, n); ++i)
      workers_.emplace_back([this] {
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
            if (stop_ && q_.empty()) return;
            job = std::move(q_.front());
            q_.pop_front();
          }
          job();
        }
      });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  std::future<int64_t> submit(std::function<int64_t()> f) {
    auto task = std::make_shared<std::packaged_task<int64_t()>>(std::move(f));
    auto fut = task->get_future();
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_;
};

}  // namespace

class AioHandle {
 public:
  AioHandle(int64_t block_size, int64_t queue_depth, bool single_submit, bool overlap_events, int64_t thread_count)
      : block_(block_size), qd_(std::max<int64_t>(1, queue_depth)), single_submit_(single_submit),
        overlap_(overlap_events), threads_(std::max<int64_t>(1, thread_count)),
        pool_((int)(threads_ * qd_)) {}

  int64_t get_block_size() const { return block_; }
  int64_t get_queue_depth() const { return qd_; }
  bool get_single_submit() const { return single_submit_; }
  bool get_overlap_events() const { return overlap_; }
  int64_t get_thread_count() const { return threads_; }

  int64_t sync_pread(torch::Tensor buffer, const std::string& filename) { return run(buffer, filename, false, false); }
  int64_t sync_pwrite(torch::Tensor buffer, const std::string& filename) { return run(buffer, filename, true, false); }
  int64_t async_pread(torch::Tensor buffer, const std::string& filename) { return run(buffer, filename, false, true); }
  int64_t async_pwrite(torch::Tensor buffer, const std::string& filename) { return run(buffer, filename, true, true); }
  int64_t pread(torch::Tensor buffer, const std::string& filename, bool validate, bool async) {
    return run(buffer, filename, false, async);
  }
  int64_t pwrite(torch::Tensor buffer, const std::string& filename, bool validate, bool async) {
    return run(buffer, filename, true, async);
  }

  // wait for all outstanding async ops; returns the number of operations (pread / pwrite calls, not their pieces)
  // completed, as the reference's handle does
  int64_t wait() {
    std::vector<std::future<int64_t>> pend;
    std::vector<int> fds;
    int64_t n = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      pend.swap(pending_);
      fds.swap(open_fds_);
      n = pending_ops_;
      pending_ops_ = 0;
    }
    bool failed = false;
    for (auto& f : pend)
      if (f.get() < 0) failed = true;
    for (int fd : fds) ::close(fd);
    if (failed) throw std::runtime_error("aio: an asynchronous I/O operation failed");
    return n;
  }

  torch::Tensor new_cpu_locked_tensor(int64_t num_elem, torch::Tensor example) {
    const size_t bytes = ((size_t)num_elem * example.element_size() + kAlign - 1) / kAlign * kAlign;
    void* p = nullptr;
    if (posix_memalign(&p, kAlign, bytes) != 0) throw std::runtime_error("aio: posix_memalign failed");
    ::mlock(p, bytes);  // best effort (RLIMIT_MEMLOCK)
    auto deleter = [bytes](void* q) {
      ::munlock(q, bytes);
      free(q);
    };
    return torch::from_blob(p, {num_elem}, deleter, example.options().device(torch::kCPU));
  }
  bool free_cpu_locked_tensor(torch::Tensor) { return true; }  // memory freed by the tensor deleter

 private:
  int64_t run(torch::Tensor buffer, const std::string& fn, bool write, bool async) {
    TORCH_CHECK(buffer.device().is_cpu() && buffer.is_contiguous(), "aio buffers must be contiguous host tensors");
    char* base = static_cast<char*>(buffer.data_ptr());
    const int64_t len = buffer.numel() * buffer.element_size();
    const bool direct = ((uintptr_t)base % kAlign == 0) && (len % kAlign == 0) && (block_ % kAlign == 0);
    int fd = open_file(fn, write, direct);
    if (fd < 0) throw std::runtime_error("aio: cannot open " + fn + ": " + strerror(errno));
    if (!write) {
      struct stat st;
      if (fstat(fd, &st) == 0 && st.st_size < len) {
        ::close(fd);
        throw std::runtime_error("aio: file " + fn + " is smaller than the read buffer");
      }
    }
    // split across threads in aligned chunks; each worker moves its chunk in block_size pieces
    const int64_t nparts = std::max<int64_t>(1, std::min<int64_t>(threads_ * qd_, (len + block_ - 1) / block_));
    int64_t chunk = (len + nparts - 1) / nparts;
    chunk = (chunk + kAlign - 1) / kAlign * kAlign;
    std::vector<std::future<int64_t>> futs;
    for (int64_t off = 0; off < len; off += chunk) {
      const int64_t n = std::min(chunk, len - off);
      const int64_t blk = block_;
      futs.push_back(pool_.submit([=]() -> int64_t {
        int64_t r = do_io(fd, base + off, n, off, blk, write);
        if (r < 0 && direct) {
          // O_DIRECT refuses buffers the kernel cannot pin (e.g. memory mapped by the GPU driver): redo this part
          // through the page cache
          int fd2 = open_file(fn, write, false);
          if (fd2 < 0) return r;
          r = do_io(fd2, base + off, n, off, blk, write);
          if (write) ::fsync(fd2);
          ::close(fd2);
        }
        return r;
      }));
    }
    if (async) {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& f : futs) pending_.push_back(std::move(f));
      ++pending_ops_;
      open_fds_.push_back(fd);
      return 0;
    }
    int64_t total = 0;
    bool failed = false;
    for (auto& f : futs) {
      const int64_t r = f.get();
      if (r < 0) failed = true;
      else total += r;
    }
    if (write) ::fsync(fd);
    ::close(fd);
    if (failed) throw std::runtime_error("aio: I/O on " + fn + " failed");
    return total;
  }

  int64_t block_, qd_;
  bool single_submit_, overlap_;
  int64_t threads_;
  ThreadPool pool_;
  std::mutex mu_;
  std::vector<std::future<int64_t>> pending_;
  int64_t pending_ops_ = 0;
  std::vector<int> open_fds_;
};

int64_t aio_read(torch::Tensor buffer, const std::string& filename, int64_t block_size, int64_t queue_depth,
                 bool single_submit, bool overlap_events, bool validate) {
  AioHandle h(block_size, queue_depth, single_submit, overlap_events, 1);
  return h.sync_pread(buffer, filename);
}

int64_t aio_write(torch::Tensor buffer, const std::string& filename, int64_t block_size, int64_t queue_depth,
                  bool single_submit, bool overlap_events, bool validate) {
  AioHandle h(block_size, queue_depth, single_submit, overlap_events, 1);
  return h.sync_pwrite(buffer, filename);
}

int64_t deepspeed_memcpy(torch::Tensor dest, torch::Tensor src) {
  TORCH_CHECK(dest.numel() * dest.element_size() == src.numel() * src.element_size(), "memcpy size mismatch");
  std::memcpy(dest.data_ptr(), src.data_ptr(), src.numel() * src.element_size());
  return 0;
}

void register_aio(pybind11::module& m) {
  // blocking transfers and wait() run without the interpreter lock (other Python threads keep launching GPU work)
  using nogil = pybind11::call_guard<pybind11::gil_scoped_release>;
  m.def("aio_read", &aio_read);
  m.def("aio_write", &aio_write);
  m.def("deepspeed_memcpy", &deepspeed_memcpy);
  pybind11::class_<AioHandle>(m, "aio_handle")
      .def(pybind11::init<int64_t, int64_t, bool, bool, int64_t>(), pybind11::arg("block_size") = 1048576,
           pybind11::arg("queue_depth") = 128, pybind11::arg("single_submit") = false,
           pybind11::arg("overlap_events") = false, pybind11::arg("num_threads") = 1)
      .def("get_block_size", &AioHandle::get_block_size)
      .def("get_queue_depth", &AioHandle::get_queue_depth)
      .def("get_single_submit", &AioHandle::get_single_submit)
      .def("get_overlap_events", &AioHandle::get_overlap_events)
      .def("get_thread_count", &AioHandle::get_thread_count)
      .def("read", [](AioHandle& h, torch::Tensor b, const std::string& f, bool validate) { return h.sync_pread(b, f); })
      .def("write", [](AioHandle& h, torch::Tensor b, const std::string& f, bool validate) { return h.sync_pwrite(b, f); })
      .def("pread", &AioHandle::pread, nogil())
      .def("pwrite", &AioHandle::pwrite, nogil())
      .def("sync_pread", &AioHandle::sync_pread, nogil())
      .def("sync_pwrite", &AioHandle::sync_pwrite, nogil())
      .def("async_pread", &AioHandle::async_pread, nogil())
      .def("async_pwrite", &AioHandle::async_pwrite, nogil())
      .def("new_cpu_locked_tensor", &AioHandle::new_cpu_locked_tensor)
      .def("free_cpu_locked_tensor", &AioHandle::free_cpu_locked_tensor)
      .def("wait", &AioHandle::wait, nogil());
}
