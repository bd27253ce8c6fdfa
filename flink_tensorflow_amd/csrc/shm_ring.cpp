// Single-producer / single-consumer message ring in POSIX shared memory: the record
// channel between an operator's coordinator thread and its subtask running in a worker
// process ("host shared-memory ring buffers, one SPSC queue per
// producer -> GPU-worker edge"; the reference's analogue is Flink's Netty shuffle,
// records serialised through TensorValue.write/read, LIB/types/TensorValue.java:150-187).
//
// Layout: a header page (magic, capacity, producer cursor `head`, consumer cursor `tail`,
// closed flag — the cursors on separate cache lines) followed by `capacity` data bytes.
// Cursors are monotonically increasing byte counts; a message is [u32 len][payload] padded
// to 8 bytes.  A message that does not fit before the end of the data area is preceded by
// a wrap marker (len = 0xFFFFFFFF) and written at offset 0.  Payload bytes are published
// by a release store of `head` and retired by a release store of `tail`.  Waits spin
// briefly, then sleep in 20-50 us steps, with the GIL released.
#include "native.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace {

constexpr uint64_t kMagic = 0x46544d5348524e47ull;  // "FTMSHRNG"
constexpr uint32_t kWrap = 0xFFFFFFFFu;
constexpr size_t kHeader = 4096;

struct Header {
  uint64_t magic;
  uint64_t capacity;
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail;
  alignas(64) std::atomic<uint32_t> closed;
};
static_assert(sizeof(Header) <= kHeader, "header page");

uint64_t pad8(uint64_t v) { return (v + 7) & ~uint64_t(7); }

class ShmRing {
 public:
  ShmRing(const std::string& name, uint64_t capacity, bool create) : name_(name) {
    if (name.empty() || name[0] != '/') throw std::invalid_argument("ShmRing: name must start with '/'");
    if (create) {
      if (capacity < 4096 || capacity % 8) throw std::invalid_argument("ShmRing: capacity must be >= 4096, % 8 == 0");
      fd_ = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("ShmRing: shm_open(create) failed for " + name + ": " + strerror(errno));
      if (ftruncate(fd_, off_t(kHeader + capacity)) != 0) {
        ::close(fd_);
        shm_unlink(name.c_str());
        throw std::runtime_error("ShmRing: ftruncate failed: " + std::string(strerror(errno)));
      }
      size_ = kHeader + capacity;
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("ShmRing: shm_open(attach) failed for " + name + ": " + strerror(errno));
      struct stat st {};
      if (fstat(fd_, &st) != 0 || size_t(st.st_size) <= kHeader) {
        ::close(fd_);
        throw std::runtime_error("ShmRing: bad segment " + name);
      }
      size_ = size_t(st.st_size);
    }
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) {
      ::close(fd_);
      if (create) shm_unlink(name.c_str());
      throw std::runtime_error("ShmRing: mmap failed: " + std::string(strerror(errno)));
    }
    base_ = static_cast<uint8_t*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    data_ = base_ + kHeader;
    if (create) {
      new (hdr_) Header();
      hdr_->capacity = capacity;
      hdr_->head.store(0, std::memory_order_relaxed);
      hdr_->tail.store(0, std::memory_order_relaxed);
      hdr_->closed.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else if (hdr_->magic != kMagic || kHeader + hdr_->capacity != size_) {
      unmap();
      throw std::runtime_error("ShmRing: " + name + " is not a ring segment");
    }
    cap_ = hdr_->capacity;
  }

  ~ShmRing() { unmap(); }

  uint64_t capacity() const { return cap_; }
  uint64_t max_message() const { return cap_ / 2 - 8; }
  uint64_t used() const { return hdr_->head.load(std::memory_order_acquire) - hdr_->tail.load(std::memory_order_acquire); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  void close_producer() { hdr_->closed.store(1, std::memory_order_release); }
  const std::string& name() const { return name_; }

  // returns false on timeout; timeout < 0 waits forever
  bool push(const py::bytes& msg, double timeout_s) {
    std::string_view v = msg;
    if (v.size() > max_message()) throw std::invalid_argument("ShmRing.push: message larger than capacity/2");
    const uint64_t need = pad8(4 + v.size());
    py::gil_scoped_release nogil;
    return wait_until(timeout_s, [&] {
      const uint64_t head = hdr_->head.load(std::memory_order_relaxed);
      const uint64_t tail = hdr_->tail.load(std::memory_order_acquire);
      const uint64_t off = head % cap_;
      const uint64_t skip = (off + need > cap_) ? cap_ - off : 0;  // wrap to offset 0
      if (cap_ - (head - tail) < skip + need) return false;
      if (skip) {
        uint32_t w = kWrap;
        std::memcpy(data_ + off, &w, 4);
      }
      const uint64_t o = (head + skip) % cap_;
      const uint32_t len = uint32_t(v.size());
      std::memcpy(data_ + o, &len, 4);
      std::memcpy(data_ + o + 4, v.data(), v.size());
      hdr_->head.store(head + skip + need, std::memory_order_release);
      return true;
    });
  }

  // a message, or None on timeout / when the producer closed an empty ring
  py::object pop(double timeout_s) {
    std::string out;
    bool got = false;
    {
      py::gil_scoped_release nogil;
      wait_until(timeout_s, [&] {
        uint64_t tail = hdr_->tail.load(std::memory_order_relaxed);
        const uint64_t head = hdr_->head.load(std::memory_order_acquire);
        if (head == tail) return closed();  // empty: stop waiting only once closed
        uint64_t off = tail % cap_;
        uint32_t len;
        std::memcpy(&len, data_ + off, 4);
        if (len == kWrap) {
          tail += cap_ - off;
          off = 0;
          std::memcpy(&len, data_ + off, 4);
        }
        out.assign(reinterpret_cast<const char*>(data_ + off + 4), len);
        hdr_->tail.store(tail + pad8(4 + len), std::memory_order_release);
        got = true;
        return true;
      });
    }
    if (!got) return py::none();
    return py::bytes(out);
  }

  static void unlink(const std::string& name) { shm_unlink(name.c_str()); }

 private:
  template <class F>
  bool wait_until(double timeout_s, F&& attempt) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int spin = 0;; ++spin) {
      if (attempt()) return true;
      if (timeout_s >= 0 && std::chrono::duration<double>(clk::now() - t0).count() >= timeout_s) return false;
      if (spin < 256) {
        __builtin_ia32_pause();
      } else {
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 4096 ? 20 : 50));
      }
    }
  }

  void unmap() {
    if (base_) munmap(base_, size_);
    if (fd_ >= 0) ::close(fd_);
    base_ = nullptr;
    fd_ = -1;
  }

  std::string name_;
  int fd_ = -1;
  size_t size_ = 0;
  uint8_t* base_ = nullptr;
  Header* hdr_ = nullptr;
  uint8_t* data_ = nullptr;
  uint64_t cap_ = 0;
};

}  // namespace

void register_shm_ring(py::module_& m) {
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, uint64_t, bool>(), py::arg("name"), py::arg("capacity") = 0,
           py::arg("create") = false)
      .def("push", &ShmRing::push, py::arg("message"), py::arg("timeout_s") = -1.0)
      .def("pop", &ShmRing::pop, py::arg("timeout_s") = -1.0)
      .def("close_producer", &ShmRing::close_producer)
      .def_property_readonly("capacity", &ShmRing::capacity)
      .def_property_readonly("max_message", &ShmRing::max_message)
      .def_property_readonly("used", &ShmRing::used)
      .def_property_readonly("closed", &ShmRing::closed)
      .def_property_readonly("name", &ShmRing::name)
      .def_static("unlink", &ShmRing::unlink);
}
