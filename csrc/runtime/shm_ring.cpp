// ShmRing: single-producer / multi-consumer byte ring in POSIX shared memory.
//
// every engine step rank 0 of a TP group hands the step's inputs (the pinned
// InputBuffers image + the step meta, a few hundred KB) to the other ranks.  A gloo broadcast of a
// pickled object costs a TCP round per follower per step; here the driver writes each step once into
// a slot of a /dev/shm ring and the followers (processes on the same node, one per GPU) copy it out.
//
// Layout: [Header][slot 0] ... [slot n-1]; slot = [u64 length][payload <= slot_bytes].
// Protocol: the producer fills slot (seq % n) only once every reader's cursor is past seq - n, then
// publishes head = seq + 1 with a release store; reader r waits for head > its cursor (acquire), copies
// the slot, then advances its cursor (release).  Waits spin, then yield, then sleep (the GIL is
// released while waiting), bounded by a timeout so callers can check for a dead peer.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace mxs_rt {

constexpr int kMaxReaders = 64;
constexpr uint64_t kMagic = 0x6d78732d72696e67ull;  // "mxs-ring"

struct alignas(64) RingHeader {
  uint64_t magic;
  uint64_t slot_bytes;
  uint32_t nslots;
  uint32_t nreaders;
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail[kMaxReaders];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free 64-bit atomics required");

class ShmRing {
 public:
  ShmRing(const std::string& name, bool create, uint64_t slot_bytes, uint32_t nslots, uint32_t nreaders)
      : name_(name), owner_(create) {
    if (create) {
      if (nslots < 1 || nreaders < 1 || nreaders > kMaxReaders) throw std::invalid_argument("bad ring geometry");
      slot_bytes = (slot_bytes + 63) & ~uint64_t(63);
      size_ = sizeof(RingHeader) + uint64_t(nslots) * (slot_bytes + 64);
      int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
      if (ftruncate(fd, static_cast<off_t>(size_)) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("ftruncate failed (is /dev/shm large enough?)");
      }
      map(fd);
      hdr_->slot_bytes = slot_bytes;
      hdr_->nslots = nslots;
      hdr_->nreaders = nreaders;
      hdr_->head.store(0, std::memory_order_relaxed);
      for (int r = 0; r < kMaxReaders; ++r) hdr_->tail[r].store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else {
      int fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name);
      struct stat st;
      if (fstat(fd, &st) != 0) {
        close(fd);
        throw std::runtime_error("fstat failed");
      }
      size_ = static_cast<uint64_t>(st.st_size);
      map(fd);
      if (hdr_->magic != kMagic) throw std::runtime_error("not an mxs ring: " + name);
    }
  }

  ~ShmRing() {
    if (base_ != nullptr) munmap(base_, size_);
    if (owner_ && !unlinked_) shm_unlink(name_.c_str());
  }

  // Remove the name once every reader has attached: the mapping lives on, nothing is left in /dev/shm
  // if a process dies later.
  void unlink() {
    if (!unlinked_) shm_unlink(name_.c_str());
    unlinked_ = true;
  }

  uint64_t slot_bytes() const { return hdr_->slot_bytes; }
  uint32_t nslots() const { return hdr_->nslots; }
  uint64_t head() const { return hdr_->head.load(std::memory_order_acquire); }

  // Producer.  Returns false on timeout (a reader stopped consuming).
  bool push(const char* data, uint64_t n, double timeout_s) {
    if (n > hdr_->slot_bytes) throw std::length_error("payload larger than a ring slot");
    const uint64_t seq = hdr_->head.load(std::memory_order_relaxed);
    const uint64_t ns = hdr_->nslots;
    auto free_slot = [&] {
      for (uint32_t r = 0; r < hdr_->nreaders; ++r)
        if (seq - hdr_->tail[r].load(std::memory_order_acquire) >= ns) return false;
      return true;
    };
    if (!wait_until(free_slot, timeout_s)) return false;
    char* slot = slot_ptr(seq % ns);
    std::memcpy(slot, &n, sizeof(n));
    std::memcpy(slot + 64, data, n);
    hdr_->head.store(seq + 1, std::memory_order_release);
    return true;
  }

  // Reader r.  Returns false on timeout; otherwise out holds the payload.
  bool pop(uint32_t r, std::string& out, double timeout_s) {
    if (r >= hdr_->nreaders) throw std::out_of_range("reader index");
    const uint64_t seq = hdr_->tail[r].load(std::memory_order_relaxed);
    auto ready = [&] { return hdr_->head.load(std::memory_order_acquire) > seq; };
    if (!wait_until(ready, timeout_s)) return false;
    const char* slot = slot_ptr(seq % hdr_->nslots);
    uint64_t n = 0;
    std::memcpy(&n, slot, sizeof(n));
    out.assign(slot + 64, n);
    hdr_->tail[r].store(seq + 1, std::memory_order_release);
    return true;
  }

 private:
  void map(int fd) {
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed");
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<RingHeader*>(base_);
  }

  char* slot_ptr(uint64_t i) const { return base_ + sizeof(RingHeader) + i * (hdr_->slot_bytes + 64); }

  template <class F>
  static bool wait_until(F&& cond, double timeout_s) {
    if (cond()) return true;
    if (timeout_s <= 0.0) return false;  // a poll: no spinning
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
      if (cond()) return true;
      if (spin < 4096) {
        __builtin_ia32_pause();
        continue;
      }
      if (spin < 4096 + 256) {
        sched_yield();
        continue;
      }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return cond();
      struct timespec ts{0, spin < 8192 ? 20000 : 200000};  // 20 us, then 200 us once idle
      nanosleep(&ts, nullptr);
    }
  }

  std::string name_;
  bool owner_;
  bool unlinked_ = false;
  uint64_t size_ = 0;
  char* base_ = nullptr;
  RingHeader* hdr_ = nullptr;
};

void register_shm_ring(py::module_& m) {
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, bool, uint64_t, uint32_t, uint32_t>(), py::arg("name"), py::arg("create"),
           py::arg("slot_bytes") = 0, py::arg("nslots") = 0, py::arg("nreaders") = 0)
      .def("unlink", &ShmRing::unlink)
      .def_property_readonly("slot_bytes", &ShmRing::slot_bytes)
      .def_property_readonly("nslots", &ShmRing::nslots)
      .def_property_readonly("head", &ShmRing::head)
      .def(
          "push",
          [](ShmRing& r, py::buffer b, double timeout_s) {
            py::buffer_info info = b.request();
            const uint64_t n = static_cast<uint64_t>(info.size) * static_cast<uint64_t>(info.itemsize);
            const char* p = static_cast<const char*>(info.ptr);
            py::gil_scoped_release nogil;
            return r.push(p, n, timeout_s);
          },
          py::arg("data"), py::arg("timeout_s") = 60.0)
      .def(
          "pop",
          [](ShmRing& r, uint32_t reader, double timeout_s) -> py::object {
            std::string out;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = r.pop(reader, out, timeout_s);
            }
            if (!ok) return py::none();
            return py::bytes(out);
          },
          py::arg("reader"), py::arg("timeout_s") = 1.0);
}

}  // namespace mxs_rt
