// Single-writer / multi-reader broadcast ring over POSIX shared memory.
//
// Used by the tensor-parallel executor: the driver rank (scheduler) publishes
// each step's metadata once and every TP worker process on the node reads it,
// instead of a per-step torch.distributed broadcast (the reference relies on
// vLLM's `--distributed_executor_backend mp` shm broadcast for the same job,
// core/helm-charts/vllm/xeon-values.yaml:78-79).  The chart mounts /dev/shm
// (core/helm-charts/vllm/templates/deployment.yaml:91-92).
#include <pybind11/pybind11.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace py = pybind11;

namespace {

constexpr uint32_t kMagic = 0x45494152;  // "EIAR"

struct alignas(64) RingHeader {
  uint32_t magic;
  uint32_t n_readers;
  uint32_t n_slots;
  uint32_t pad0;
  uint64_t slot_bytes;
  std::atomic<uint64_t> write_seq;
  std::atomic<uint32_t> closed;
};

struct alignas(64) SlotHeader {
  std::atomic<uint64_t> seq;     // 1-based sequence number of the message in the slot
  std::atomic<uint32_t> acks;    // readers done with it
  uint32_t pad;
  uint64_t len;
};

class ShmRing {
 public:
  ShmRing(const std::string& name, bool create, int n_readers, int n_slots, uint64_t slot_bytes)
      : name_(name), owner_(create) {
    const size_t hdr = sizeof(RingHeader);
    if (create) {
      if (n_readers < 0 || n_slots <= 0 || slot_bytes == 0) throw std::invalid_argument("bad ring geometry");
      total_ = hdr + (size_t)n_slots * (sizeof(SlotHeader) + slot_bytes);
      shm_unlink(name.c_str());
      fd_ = shm_open(name.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(create) failed for " + name);
      if (ftruncate(fd_, (off_t)total_) != 0) throw std::runtime_error("ftruncate failed");
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("shm_open(attach) failed for " + name);
      struct stat sb;
      fstat(fd_, &sb);
      total_ = (size_t)sb.st_size;
    }
    base_ = (uint8_t*)mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = reinterpret_cast<RingHeader*>(base_);
    if (create) {
      std::memset(base_, 0, total_);
      hdr_->n_readers = (uint32_t)n_readers;
      hdr_->n_slots = (uint32_t)n_slots;
      hdr_->slot_bytes = slot_bytes;
      hdr_->write_seq.store(0);
      hdr_->closed.store(0);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else {
      for (int i = 0; i < 10000 && hdr_->magic != kMagic; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      if (hdr_->magic != kMagic) throw std::runtime_error("ring not initialised");
    }
  }

  ~ShmRing() {
    if (base_ && base_ != MAP_FAILED) munmap(base_, total_);
    if (fd_ >= 0) close(fd_);
    if (owner_) shm_unlink(name_.c_str());
  }

  uint64_t capacity() const { return hdr_->slot_bytes; }

  // Writer: returns false on timeout.
  bool put(py::bytes data, double timeout_s) {
    std::string s = data;   // copy out while holding the GIL
    if (s.size() > hdr_->slot_bytes) throw std::length_error("message larger than ring slot");
    py::gil_scoped_release nogil;
    const uint64_t seq = hdr_->write_seq.load(std::memory_order_relaxed);
    SlotHeader* sh = slot(seq % hdr_->n_slots);
    const uint64_t prev = sh->seq.load(std::memory_order_acquire);
    if (prev != 0) {
      if (!wait([&] { return sh->acks.load(std::memory_order_acquire) >= hdr_->n_readers; }, timeout_s))
        return false;
    }
    std::memcpy(reinterpret_cast<uint8_t*>(sh) + sizeof(SlotHeader), s.data(), s.size());
    sh->len = s.size();
    sh->acks.store(0, std::memory_order_relaxed);
    sh->seq.store(seq + 1, std::memory_order_release);
    hdr_->write_seq.store(seq + 1, std::memory_order_release);
    return true;
  }

  // Reader: returns None on timeout.
  py::object get(double timeout_s) {
    const uint64_t want = read_seq_ + 1;
    SlotHeader* sh = slot(read_seq_ % hdr_->n_slots);
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = wait([&] { return sh->seq.load(std::memory_order_acquire) == want || hdr_->closed.load(); }, timeout_s);
    }
    if (!ok || sh->seq.load(std::memory_order_acquire) != want) return py::none();
    py::bytes out(reinterpret_cast<const char*>(sh) + sizeof(SlotHeader), sh->len);
    sh->acks.fetch_add(1, std::memory_order_acq_rel);
    ++read_seq_;
    return out;
  }

  void close_ring() { hdr_->closed.store(1); }

 private:
  SlotHeader* slot(uint64_t i) const {
    return reinterpret_cast<SlotHeader*>(base_ + sizeof(RingHeader) + i * (sizeof(SlotHeader) + hdr_->slot_bytes));
  }

  template <class F>
  bool wait(F ready, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    int spins = 0;
    while (!ready()) {
      if (++spins < 2000) continue;
      std::this_thread::sleep_for(std::chrono::microseconds(spins < 20000 ? 5 : 100));
      if (timeout_s >= 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        return false;
    }
    return true;
  }

  std::string name_;
  bool owner_;
  int fd_ = -1;
  size_t total_ = 0;
  uint8_t* base_ = nullptr;
  RingHeader* hdr_ = nullptr;
  uint64_t read_seq_ = 0;
};

}  // namespace

void register_shm(py::module_& m) {
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, bool, int, int, uint64_t>(), py::arg("name"),
           py::arg("create"), py::arg("n_readers") = 0, py::arg("n_slots") = 8,
           py::arg("slot_bytes") = 4 << 20)
      .def_property_readonly("capacity", &ShmRing::capacity)
      .def("put", &ShmRing::put, py::arg("data"), py::arg("timeout_s") = -1.0)
      .def("get", &ShmRing::get, py::arg("timeout_s") = -1.0)
      .def("close", &ShmRing::close_ring);
}
