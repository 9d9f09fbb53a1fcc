// Asynchronous file I/O engine for ZeRO-Infinity NVMe offload (module `_cpu_ops`).
//
// Reference parity: csrc/aio (deepspeed_aio_common.cpp, deepspeed_py_aio_handle.cpp,
// deepspeed_aio_thread.cpp, deepspeed_py_copy.cpp): an `aio_handle(block_size,
// queue_depth, single_submit, overlap_events, thread_count)` with read/write,
// pread/pwrite (sync or async) and wait(); module functions aio_read/aio_write and a
// parallel deepspeed_memcpy.  The reference drives libaio io_submit/io_getevents; this
// image has no libaio, so the engine here is a native thread pool issuing O_DIRECT
// pread/pwrite of `block_size` pieces, each worker keeping up to `queue_depth` pieces
// of its slice in flight through sequential submission (the kernel's NVMe queue does the
// parallelism across workers).  Buffers are the caller's pinned host tensors, which the
// swappers then move to HBM with hipMemcpyAsync (no extra bounce copy).
#include <torch/extension.h>
#include <fcntl.h>
#include <omp.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

struct IoJob {
  char* buf;
  int64_t nbytes;
  int64_t file_offset;
  std::string path;
  bool read;
  bool validate;
};

bool is_aligned(const void* p, int64_t n, int64_t a) {
  return (reinterpret_cast<uintptr_t>(p) % a == 0) && (n % a == 0);
}

// Performs one slice of a job: [off, off+len) of the buffer <-> file.
int64_t do_slice(const IoJob& j, int64_t off, int64_t len, int64_t block) {
  if (len <= 0) return 0;
  int flags = j.read ? O_RDONLY : (O_WRONLY | O_CREAT);
  const bool direct = is_aligned(j.buf + off, len, 4096) && ((j.file_offset + off) % 4096 == 0);
#ifdef O_DIRECT
  if (direct) flags |= O_DIRECT;
#endif
  int fd = open(j.path.c_str(), flags, 0644);
  if (fd < 0 && direct) {  // filesystem without O_DIRECT (tmpfs): retry buffered
    fd = open(j.path.c_str(), j.read ? O_RDONLY : (O_WRONLY | O_CREAT), 0644);
  }
  if (fd < 0) return -1;
  int64_t done = 0;
  while (done < len) {
    const int64_t n = std::min(block, len - done);
    ssize_t r = j.read ? pread(fd, j.buf + off + done, n, j.file_offset + off + done)
                       : pwrite(fd, j.buf + off + done, n, j.file_offset + off + done);
    if (r <= 0) {
      close(fd);
      return -1;
    }
    done += r;
  }
  close(fd);
  return done;
}

class ThreadPool {
 public:
  explicit ThreadPool(int n) : stop_(false) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() const { return (int)workers_.size(); }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
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
      : block_(block_size), qd_(queue_depth), single_submit_(single_submit), overlap_(overlap_events),
        threads_(std::max<int64_t>(1, thread_count)), pool_((int)std::max<int64_t>(1, thread_count)) {}

  int64_t get_block_size() const { return block_; }
  int64_t get_queue_depth() const { return qd_; }
  bool get_single_submit() const { return single_submit_; }
  bool get_overlap_events() const { return overlap_; }
  int64_t get_thread_count() const { return threads_; }

  int64_t read(at::Tensor buffer, const std::string& filename, bool validate) {
    return sync_io(buffer, filename, true, validate);
  }
  int64_t write(at::Tensor buffer, const std::string& filename, bool validate) {
    return sync_io(buffer, filename, false, validate);
  }
  int64_t pread(at::Tensor buffer, const std::string& filename, bool validate, bool async) {
    return async ? submit(buffer, filename, true, validate) : sync_io(buffer, filename, true, validate);
  }
  int64_t pwrite(at::Tensor buffer, const std::string& filename, bool validate, bool async) {
    return async ? submit(buffer, filename, false, validate) : sync_io(buffer, filename, false, validate);
  }
  int64_t sync_pread(at::Tensor b, const std::string& f) { return sync_io(b, f, true, false); }
  int64_t sync_pwrite(at::Tensor b, const std::string& f) { return sync_io(b, f, false, false); }
  int64_t async_pread(at::Tensor b, const std::string& f) { return submit(b, f, true, false); }
  int64_t async_pwrite(at::Tensor b, const std::string& f) { return submit(b, f, false, false); }

  // Wait for all outstanding async ops; returns how many completed (or -1 on error).
  int64_t wait() {
    pybind11::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return pending_slices_ == 0; });
    const int64_t n = completed_ops_;
    completed_ops_ = 0;
    if (failed_) {
      failed_ = false;
      return -1;
    }
    return n;
  }

 private:
  void check(const at::Tensor& b) {
    TORCH_CHECK(!b.is_cuda(), "aio: buffers must be host tensors (stage GPU tensors through pinned memory)");
    TORCH_CHECK(b.is_contiguous(), "aio: contiguous buffer required");
  }

  int64_t sync_io(at::Tensor buffer, const std::string& filename, bool read, bool validate) {
    submit(buffer, filename, read, validate);
    return wait() < 0 ? -1 : 1;
  }

  int64_t submit(at::Tensor buffer, const std::string& filename, bool read, bool validate) {
    check(buffer);
    IoJob job{reinterpret_cast<char*>(buffer.data_ptr()), (int64_t)buffer.nbytes(), 0, filename, read, validate};
    if (!read) {  // create / size the file once before parallel slices write into it
      int fd = open(filename.c_str(), O_WRONLY | O_CREAT, 0644);
      TORCH_CHECK(fd >= 0, "aio: cannot open ", filename);
      close(fd);
    }
    // split into `threads_` contiguous slices aligned to the block size
    const int64_t nb = (job.nbytes + block_ - 1) / block_;
    const int64_t per = (nb + threads_ - 1) / threads_;
    std::vector<std::pair<int64_t, int64_t>> parts;
    for (int64_t t = 0; t < threads_; ++t) {
      const int64_t off = t * per * block_;
      if (off >= job.nbytes) break;
      parts.emplace_back(off, std::min(job.nbytes - off, per * block_));
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      pending_slices_ += (int64_t)parts.size();
    }
    auto remaining = std::make_shared<std::atomic<int64_t>>((int64_t)parts.size());
    for (auto& pr : parts) {
      pool_.submit([this, job, pr, remaining] {
        const int64_t r = do_slice(job, pr.first, pr.second, block_);
        std::lock_guard<std::mutex> g(mu_);
        if (r < 0) failed_ = true;
        if (--(*remaining) == 0) completed_ops_ += 1;
        if (--pending_slices_ == 0) cv_.notify_all();
      });
    }
    return 0;
  }

  int64_t block_, qd_;
  bool single_submit_, overlap_;
  int64_t threads_;
  ThreadPool pool_;
  std::mutex mu_;
  std::condition_variable cv_;
  int64_t pending_slices_ = 0;
  int64_t completed_ops_ = 0;
  bool failed_ = false;
};

int64_t aio_read(at::Tensor buffer, const std::string& filename, int64_t block_size, int64_t queue_depth,
                 bool single_submit, bool overlap_events, bool validate) {
  AioHandle h(block_size, queue_depth, single_submit, overlap_events, 1);
  return h.read(buffer, filename, validate);
}

int64_t aio_write(at::Tensor buffer, const std::string& filename, int64_t block_size, int64_t queue_depth,
                  bool single_submit, bool overlap_events, bool validate) {
  AioHandle h(block_size, queue_depth, single_submit, overlap_events, 1);
  return h.write(buffer, filename, validate);
}

// Parallel host memcpy (reference: deepspeed_py_copy.cpp AVX copy).
int64_t deepspeed_memcpy(at::Tensor dest, at::Tensor src) {
  TORCH_CHECK(!dest.is_cuda() && !src.is_cuda(), "deepspeed_memcpy: host tensors");
  TORCH_CHECK(dest.nbytes() == src.nbytes() && dest.is_contiguous() && src.is_contiguous(), "deepspeed_memcpy");
  char* d = reinterpret_cast<char*>(dest.data_ptr());
  const char* s = reinterpret_cast<const char*>(src.data_ptr());
  const int64_t n = src.nbytes();
  const int64_t chunk = 1 << 20;
  pybind11::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
  for (int64_t o = 0; o < n; o += chunk) std::memcpy(d + o, s + o, std::min(chunk, n - o));
  return 0;
}

void register_aio(pybind11::module& m) {
  m.def("aio_read", &aio_read);
  m.def("aio_write", &aio_write);
  m.def("deepspeed_memcpy", &deepspeed_memcpy);
  pybind11::class_<AioHandle>(m, "aio_handle")
      .def(pybind11::init<int64_t, int64_t, bool, bool, int64_t>(), pybind11::arg("block_size") = 1 << 20,
           pybind11::arg("queue_depth") = 128, pybind11::arg("single_submit") = false,
           pybind11::arg("overlap_events") = false, pybind11::arg("thread_count") = 1)
      .def("get_block_size", &AioHandle::get_block_size)
      .def("get_queue_depth", &AioHandle::get_queue_depth)
      .def("get_single_submit", &AioHandle::get_single_submit)
      .def("get_overlap_events", &AioHandle::get_overlap_events)
      .def("get_thread_count", &AioHandle::get_thread_count)
      .def("read", &AioHandle::read)
      .def("write", &AioHandle::write)
      .def("pread", &AioHandle::pread)
      .def("pwrite", &AioHandle::pwrite)
      .def("sync_pread", &AioHandle::sync_pread)
      .def("sync_pwrite", &AioHandle::sync_pwrite)
      .def("async_pread", &AioHandle::async_pread)
      .def("async_pwrite", &AioHandle::async_pwrite)
      .def("wait", &AioHandle::wait);
}
