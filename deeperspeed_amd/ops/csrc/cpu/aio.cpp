// Asynchronous file I/O engine for ZeRO-Infinity NVMe offload (module `_cpu_ops`).
//
// Reference parity: csrc/aio (deepspeed_aio_common.cpp:69-160,265 io_submit/io_getevents
// with queue depth, single vs block submit, overlapped completion; deepspeed_aio_thread.cpp
// request split across worker threads; deepspeed_py_aio_handle.cpp Python handle;
// deepspeed_py_copy.cpp parallel memcpy).  API: `aio_handle(block_size, queue_depth,
// single_submit, overlap_events, thread_count)` with read/write, pread/pwrite (sync or
// async), sync_*/async_* and wait(); module functions aio_read/aio_write/deepspeed_memcpy.
//
// Engine: io_uring through raw syscalls (no liburing/libaio in the image).  Every worker
// thread owns one ring of `queue_depth` entries; a request is cut into `block_size` pieces
// and split into one contiguous slice per worker.  A worker keeps up to `queue_depth`
// pieces in flight:
//   * single_submit=true  -> one io_uring_enter per piece (reference: one iocb per
//     io_submit call); false -> the whole batch of free slots in one enter.
//   * overlap_events=true -> a freed slot is refilled as soon as its completion is reaped
//     (reference: overlapped submit/reap); false -> a batch is reaped completely before
//     the next batch is submitted (reference: lock-step submit/wait).
// O_DIRECT is used when buffer, length and file offset are 4 KiB aligned (pinned tensors
// from the swappers are page aligned) and the filesystem supports it; otherwise buffered.
// Where the kernel refuses io_uring (seccomp, old kernel) the same workers fall back to
// positional pread/pwrite ("psync" engine) -- get_engine() reports which one runs.
#include <torch/extension.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int64_t kAlign = 4096;

// ------------------------------------------------------------------------------ io_uring
class Ring {
 public:
  ~Ring() { close_ring(); }

  bool open_ring(unsigned entries) {
    io_uring_params p;
    std::memset(&p, 0, sizeof(p));
    fd_ = (int)syscall(__NR_io_uring_setup, entries, &p);
    if (fd_ < 0) return false;
    sq_sz_ = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    cq_sz_ = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    const bool single = p.features & IORING_FEAT_SINGLE_MMAP;
    if (single) sq_sz_ = cq_sz_ = std::max(sq_sz_, cq_sz_);
    sq_ptr_ = mmap(nullptr, sq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_SQ_RING);
    if (sq_ptr_ == MAP_FAILED) return fail();
    cq_ptr_ = single ? sq_ptr_
                     : mmap(nullptr, cq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_CQ_RING);
    if (cq_ptr_ == MAP_FAILED) return fail();
    sqe_sz_ = p.sq_entries * sizeof(io_uring_sqe);
    sqes_ = (io_uring_sqe*)mmap(nullptr, sqe_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_,
                                IORING_OFF_SQES);
    if (sqes_ == MAP_FAILED) return fail();
    char* sq = (char*)sq_ptr_;
    char* cq = (char*)cq_ptr_;
    sq_tail_ = (unsigned*)(sq + p.sq_off.tail);
    sq_mask_ = *(unsigned*)(sq + p.sq_off.ring_mask);
    sq_array_ = (unsigned*)(sq + p.sq_off.array);
    cq_head_ = (unsigned*)(cq + p.cq_off.head);
    cq_tail_ = (unsigned*)(cq + p.cq_off.tail);
    cq_mask_ = *(unsigned*)(cq + p.cq_off.ring_mask);
    cqes_ = (io_uring_cqe*)(cq + p.cq_off.cqes);
    entries_ = p.sq_entries;
    return true;
  }

  unsigned entries() const { return entries_; }
  unsigned unsubmitted() const { return unsubmitted_; }

  // Queue one read/write SQE (not yet visible to the kernel until enter()).
  void prep(bool read, int fd, void* buf, unsigned len, int64_t off, uint64_t tag) {
    const unsigned tail = local_tail_;
    const unsigned idx = tail & sq_mask_;
    io_uring_sqe* s = &sqes_[idx];
    std::memset(s, 0, sizeof(*s));
    s->opcode = read ? IORING_OP_READ : IORING_OP_WRITE;
    s->fd = fd;
    s->addr = (uint64_t)(uintptr_t)buf;
    s->len = len;
    s->off = (uint64_t)off;
    s->user_data = tag;
    sq_array_[idx] = idx;
    local_tail_ = tail + 1;
    ++unsubmitted_;
  }

  // Publish queued SQEs and optionally wait for `min_complete` completions.
  int enter(unsigned min_complete) {
    __atomic_store_n(sq_tail_, local_tail_, __ATOMIC_RELEASE);
    unsigned flags = min_complete ? IORING_ENTER_GETEVENTS : 0;
    int r;
    do {
      r = (int)syscall(__NR_io_uring_enter, fd_, unsubmitted_, min_complete, flags, nullptr, 0);
    } while (r < 0 && errno == EINTR);
    if (r >= 0) unsubmitted_ -= std::min<unsigned>(unsubmitted_, (unsigned)r);
    return r;
  }

  // Reap one completion if available: returns false when the CQ is empty.
  bool reap(uint64_t* tag, int* res) {
    const unsigned head = *cq_head_;
    const unsigned tail = __atomic_load_n(cq_tail_, __ATOMIC_ACQUIRE);
    if (head == tail) return false;
    const io_uring_cqe* c = &cqes_[head & cq_mask_];
    *tag = c->user_data;
    *res = c->res;
    __atomic_store_n(cq_head_, head + 1, __ATOMIC_RELEASE);
    return true;
  }

 private:
  bool fail() {
    close_ring();
    return false;
  }
  void close_ring() {
    if (sqes_ && sqes_ != MAP_FAILED) munmap(sqes_, sqe_sz_);
    if (cq_ptr_ && cq_ptr_ != MAP_FAILED && cq_ptr_ != sq_ptr_) munmap(cq_ptr_, cq_sz_);
    if (sq_ptr_ && sq_ptr_ != MAP_FAILED) munmap(sq_ptr_, sq_sz_);
    if (fd_ >= 0) close(fd_);
    sqes_ = nullptr;
    cq_ptr_ = sq_ptr_ = nullptr;
    fd_ = -1;
  }
  int fd_ = -1;
  void *sq_ptr_ = nullptr, *cq_ptr_ = nullptr;
  size_t sq_sz_ = 0, cq_sz_ = 0, sqe_sz_ = 0;
  io_uring_sqe* sqes_ = nullptr;
  io_uring_cqe* cqes_ = nullptr;
  unsigned *sq_tail_ = nullptr, *sq_array_ = nullptr, *cq_head_ = nullptr, *cq_tail_ = nullptr;
  unsigned sq_mask_ = 0, cq_mask_ = 0, entries_ = 0;
  unsigned local_tail_ = 0, unsubmitted_ = 0;
};

bool io_uring_usable() {
  static const bool ok = [] {
    if (const char* e = std::getenv("DSA_AIO_ENGINE")) {
      if (std::string(e) == "psync") return false;
    }
    Ring r;
    return r.open_ring(2);
  }();
  return ok;
}

// ------------------------------------------------------------------------------ requests
struct Request {
  char* buf;
  int64_t nbytes;
  std::string path;
  bool read;
  bool validate;
  std::atomic<int> slices_left{0};
  std::atomic<bool> failed{false};
};

struct Slice {
  std::shared_ptr<Request> req;
  int64_t off, len;  // byte range of the buffer (== file offset)
};

int open_for(const Request& r, bool direct) {
  int flags = r.read ? O_RDONLY : O_WRONLY;
  if (direct) flags |= O_DIRECT;
  return open(r.path.c_str(), flags, 0644);
}

bool slice_direct_ok(const Slice& s) {
  return (reinterpret_cast<uintptr_t>(s.req->buf + s.off) % kAlign == 0) && (s.off % kAlign == 0) &&
         (s.len % kAlign == 0);
}

// psync engine / fallback: positional I/O of `block`-sized pieces.
bool run_psync(int fd, const Slice& s, int64_t block) {
  int64_t done = 0;
  while (done < s.len) {
    const int64_t n = std::min(block, s.len - done);
    char* p = s.req->buf + s.off + done;
    const int64_t o = s.off + done;
    const ssize_t r = s.req->read ? ::pread(fd, p, n, o) : ::pwrite(fd, p, n, o);
    if (r <= 0) return false;
    done += r;
  }
  return true;
}

class Worker {
 public:
  Worker(int64_t block, int64_t qd, bool single_submit, bool overlap)
      : block_(block), qd_(std::max<int64_t>(1, qd)), single_(single_submit), overlap_(overlap) {
    uring_ = io_uring_usable() && ring_.open_ring((unsigned)qd_);
    // test hook: the N-th io_uring_enter of this worker fails as if the ring broke (EIO)
    if (const char* e = std::getenv("DSA_AIO_INJECT_ENTER_FAIL")) inject_fail_ = std::atoi(e);
    thread_ = std::thread([this] { loop(); });
  }
  ~Worker() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    thread_.join();
  }
  bool uring() const { return uring_; }

  void push(Slice s, std::function<void(const Slice&, bool)> done) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.emplace_back(std::move(s), std::move(done));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::pair<Slice, std::function<void(const Slice&, bool)>> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job.second(job.first, run(job.first));
    }
  }

  bool run(const Slice& s) {
    if (s.len <= 0) return true;
    bool direct = slice_direct_ok(s);
    int fd = open_for(*s.req, direct);
    if (fd < 0 && direct) {  // tmpfs & co. refuse O_DIRECT: buffered
      direct = false;
      fd = open_for(*s.req, false);
    }
    if (fd < 0) return false;
    bool ok = uring_ ? run_uring(fd, s) : run_psync(fd, s, block_);
    if (ok && !direct && drop_cache()) {
      // buffered fallback (overlay / tmpfs refuse O_DIRECT): keep the page cache from holding
      // the swapped bytes -- written ranges are flushed, then both kinds are dropped
      if (!s.req->read)
        sync_file_range(fd, s.off, s.len, SYNC_FILE_RANGE_WAIT_BEFORE | SYNC_FILE_RANGE_WRITE |
                                              SYNC_FILE_RANGE_WAIT_AFTER);
      posix_fadvise(fd, s.off, s.len, POSIX_FADV_DONTNEED);
    }
    close(fd);
    return ok;
  }

  // DSA_AIO_DROP_CACHE=1: buffered I/O does not leave the swapped data in the page cache (a
  // memory-capped job counts the cache; a real NVMe device is then read at its own rate)
  static bool drop_cache() {
    static const bool on = [] {
      const char* e = std::getenv("DSA_AIO_DROP_CACHE");
      return e && e[0] == '1';
    }();
    return on;
  }

  // io_uring_enter, retrying transient failures: EINTR (inside Ring::enter), EAGAIN (no kernel
  // request slots right now: back off) and EBUSY (completion queue full: return so the caller
  // reaps, then enters again).  < 0 only for a ring that is really unusable.
  int enter_retry(unsigned min_complete) {
    if (inject_fail_ > 0 && --inject_fail_ == 0) {
      errno = EIO;
      return -1;
    }
    for (int attempt = 0;; ++attempt) {
      const int r = ring_.enter(min_complete);
      if (r >= 0) return r;
      if (errno == EBUSY) return 0;
      if (errno == EAGAIN && attempt < 2000) {
        usleep(100);
        continue;
      }
      return r;
    }
  }

  // Pieces of `block_` bytes, up to qd_ in flight on this worker's ring.  Every SQE that was
  // queued is completed (or provably never reached the kernel) before this returns: the SQEs
  // point into the caller's pinned buffer, which Python may free or reuse right after.
  bool run_uring(int fd, const Slice& s) {
    const int64_t npieces = (s.len + block_ - 1) / block_;
    const int64_t depth = std::min<int64_t>(qd_, ring_.entries());
    int64_t next = 0, inflight = 0;
    bool ok = true, ring_ok = true;
    auto submit_one = [&](int64_t k, int64_t done_bytes) {
      const int64_t lo = k * block_ + done_bytes;
      const int64_t len = std::min(block_, s.len - k * block_) - done_bytes;
      ring_.prep(s.req->read, fd, s.req->buf + s.off + lo, (unsigned)len, s.off + lo,
                 ((uint64_t)k << 32) | (uint64_t)done_bytes);
    };
    auto reap_all = [&] {
      uint64_t tag;
      int res;
      while (ring_.reap(&tag, &res)) {
        --inflight;
        const int64_t k = (int64_t)(tag >> 32);
        const int64_t done0 = (int64_t)(tag & 0xffffffffu);
        const int64_t want = std::min(block_, s.len - k * block_) - done0;
        if (res <= 0) {
          ok = false;
          continue;
        }
        if (res < want && ok && ring_ok) {  // short transfer: resubmit the remainder of this piece
          submit_one(k, done0 + res);
          ++inflight;
        }
      }
    };
    while ((next < npieces || inflight > 0) && ok && ring_ok) {
      // fill free slots
      int64_t to_fill = depth - inflight;
      if (!overlap_ && inflight > 0) to_fill = 0;  // lock-step: drain the batch first
      int64_t filled = 0;
      while (filled < to_fill && next < npieces && ring_ok) {
        submit_one(next++, 0);
        ++filled;
        ++inflight;
        if (single_ && enter_retry(0) < 0) ring_ok = false;
      }
      // submit the batch (block submit) and wait for at least one completion
      if (ring_ok && enter_retry(1) < 0) ring_ok = false;
      reap_all();
    }
    // drain: an error ends the transfer, never the wait for what is already in flight
    const auto t0 = std::chrono::steady_clock::now();
    bool warned = false;
    while (inflight > 0) {
      if (ring_ok) {
        if (enter_retry(1) < 0) ring_ok = false;
      } else {
        // SQEs the kernel never consumed can never complete: the ring is abandoned with them
        inflight -= ring_.unsubmitted();
        if (inflight <= 0) break;
        usleep(1000);  // any syscall runs pending io_uring task work: completions still land
      }
      reap_all();
      const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (!ring_ok && waited > 10.0 && !warned) {
        std::fprintf(stderr, "[aio] io_uring failed with %lld request(s) in flight; waiting for them\n",
                     (long long)inflight);
        warned = true;
      }
      if (!ring_ok && waited > 300.0) {
        // returning now would let the kernel write into a buffer its owner is about to free
        std::fprintf(stderr, "[aio] %lld io_uring request(s) never completed; aborting\n", (long long)inflight);
        std::abort();
      }
    }
    if (!ring_ok) {
      std::fprintf(stderr, "[aio] io_uring unusable on this worker (errno %d); falling back to pread/pwrite\n",
                   errno);
      uring_ = false;
    }
    return ok && ring_ok;
  }

  int64_t block_, qd_;
  bool single_, overlap_;
  Ring ring_;
  std::atomic<bool> uring_{false};
  int inject_fail_ = 0;
  std::thread thread_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<Slice, std::function<void(const Slice&, bool)>>> q_;
  bool stop_ = false;
};

bool validate_request(const Request& r) {
  // re-read the file range through the page cache and compare with the buffer
  int fd = open(r.path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  std::vector<char> tmp(1 << 20);
  int64_t off = 0;
  bool same = true;
  while (off < r.nbytes && same) {
    const int64_t n = std::min<int64_t>((int64_t)tmp.size(), r.nbytes - off);
    if (::pread(fd, tmp.data(), n, off) != n) {
      same = false;
      break;
    }
    same = std::memcmp(tmp.data(), r.buf + off, n) == 0;
    off += n;
  }
  close(fd);
  return same;
}

}  // namespace

class AioHandle {
 public:
  AioHandle(int64_t block_size, int64_t queue_depth, bool single_submit, bool overlap_events, int64_t thread_count)
      : block_(std::max<int64_t>(kAlign, block_size)), qd_(std::max<int64_t>(1, queue_depth)),
        single_submit_(single_submit), overlap_(overlap_events), threads_(std::max<int64_t>(1, thread_count)) {
    for (int64_t i = 0; i < threads_; ++i)
      workers_.emplace_back(new Worker(block_, qd_, single_submit_, overlap_));
  }

  int64_t get_block_size() const { return block_; }
  int64_t get_queue_depth() const { return qd_; }
  bool get_single_submit() const { return single_submit_; }
  bool get_overlap_events() const { return overlap_; }
  int64_t get_thread_count() const { return threads_; }
  std::string get_engine() const { return workers_[0]->uring() ? "io_uring" : "psync"; }

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

  // Wait for all outstanding async requests; returns how many completed (-1 on any error).
  int64_t wait() {
    pybind11::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return pending_ == 0; });
    const int64_t n = completed_;
    completed_ = 0;
    if (failed_) {
      failed_ = false;
      return -1;
    }
    return n;
  }

 private:
  int64_t sync_io(at::Tensor buffer, const std::string& filename, bool read, bool validate) {
    submit(buffer, filename, read, validate);
    return wait() < 0 ? -1 : 1;
  }

  int64_t submit(at::Tensor buffer, const std::string& filename, bool read, bool validate) {
    TORCH_CHECK(!buffer.is_cuda(), "aio: buffers must be host tensors (stage GPU tensors through pinned memory)");
    TORCH_CHECK(buffer.is_contiguous(), "aio: contiguous buffer required");
    auto req = std::make_shared<Request>();
    req->buf = reinterpret_cast<char*>(buffer.data_ptr());
    req->nbytes = (int64_t)buffer.nbytes();
    req->path = filename;
    req->read = read;
    req->validate = validate;
    if (!read) {  // create the file before parallel slices write into it
      int fd = open(filename.c_str(), O_WRONLY | O_CREAT, 0644);
      TORCH_CHECK(fd >= 0, "aio: cannot open ", filename, " for writing");
      close(fd);
    } else {
      struct stat st;
      TORCH_CHECK(stat(filename.c_str(), &st) == 0, "aio: cannot stat ", filename);
      TORCH_CHECK(st.st_size >= req->nbytes, "aio: ", filename, " holds ", (int64_t)st.st_size,
                  " bytes, read of ", req->nbytes, " requested");
    }
    // one contiguous, block-aligned slice per worker (reference deepspeed_aio_thread.cpp)
    const int64_t nb = (req->nbytes + block_ - 1) / block_;
    const int64_t per = std::max<int64_t>(1, (nb + threads_ - 1) / threads_);
    std::vector<Slice> parts;
    for (int64_t t = 0; t < threads_; ++t) {
      const int64_t off = t * per * block_;
      if (off >= req->nbytes) break;
      parts.push_back(Slice{req, off, std::min(req->nbytes - off, per * block_)});
    }
    if (parts.empty()) parts.push_back(Slice{req, 0, 0});
    req->slices_left = (int)parts.size();
    {
      std::lock_guard<std::mutex> g(mu_);
      ++pending_;
    }
    for (size_t i = 0; i < parts.size(); ++i) {
      workers_[i % workers_.size()]->push(parts[i], [this](const Slice& s, bool ok) {
        if (!ok) s.req->failed = true;
        if (--s.req->slices_left == 0) finish(*s.req);
      });
    }
    return 0;
  }

  void finish(Request& r) {
    bool ok = !r.failed;
    if (ok && r.validate) ok = validate_request(r);
    std::lock_guard<std::mutex> g(mu_);
    if (!ok) failed_ = true;
    ++completed_;
    if (--pending_ == 0) cv_.notify_all();
  }

  int64_t block_, qd_;
  bool single_submit_, overlap_;
  int64_t threads_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  int64_t pending_ = 0;
  int64_t completed_ = 0;
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

std::string aio_engine() { return io_uring_usable() ? "io_uring" : "psync"; }

void register_aio(pybind11::module& m) {
  m.def("aio_read", &aio_read);
  m.def("aio_write", &aio_write);
  m.def("deepspeed_memcpy", &deepspeed_memcpy);
  m.def("aio_engine", &aio_engine);
  pybind11::class_<AioHandle>(m, "aio_handle")
      .def(pybind11::init<int64_t, int64_t, bool, bool, int64_t>(), pybind11::arg("block_size") = 1 << 20,
           pybind11::arg("queue_depth") = 128, pybind11::arg("single_submit") = false,
           pybind11::arg("overlap_events") = false, pybind11::arg("thread_count") = 1)
      .def("get_block_size", &AioHandle::get_block_size)
      .def("get_queue_depth", &AioHandle::get_queue_depth)
      .def("get_single_submit", &AioHandle::get_single_submit)
      .def("get_overlap_events", &AioHandle::get_overlap_events)
      .def("get_thread_count", &AioHandle::get_thread_count)
      .def("get_engine", &AioHandle::get_engine)
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
