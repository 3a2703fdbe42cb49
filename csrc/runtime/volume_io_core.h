// Core of the native volume-store reader: pybind-free so the sanitizer stress driver
// (csrc/runtime/tests/volume_io_stress.cpp, built with -fsanitize=thread / address) links it directly.
// See volume_io.cpp for the design notes.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace nidt_io {

#pragma pack(push, 1)
struct Header {            // 128 bytes, little-endian
  char magic[8];           // "NIDTVOL1"
  uint32_t version;        // 1
  uint32_t dtype;          // 0 = uint8
  uint64_t n, d, h, w;     // subjects, volume shape
  uint64_t data_off;       // byte offset of volume 0 (page aligned)
  uint64_t labels_off;     // float32[n]
  uint64_t sites_off;      // float32[n]
  uint8_t reserved[128 - 8 - 8 - 32 - 24];
};
#pragma pack(pop)
static_assert(sizeof(Header) == 128, "header layout");

constexpr size_t kPiece = 1 << 20;  // gather work unit (bytes)

// Fixed-size worker pool; jobs are closures, completion is tracked per ticket.
class Pool {
 public:
  explicit Pool(int n) {
    n = std::max(1, n);
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size(); }
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct Ticket {
  std::atomic<int64_t> remaining{0};
  std::mutex m;
  std::condition_variable cv;
};

class VolumeReader {
 public:
  VolumeReader(const std::string& path, int threads) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("nidt_io: cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) != 0) fail("fstat failed");
    size_ = (size_t)st.st_size;
    if (size_ < sizeof(Header)) fail("file too small for a NIDTVOL1 header");
    void* p = ::mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) fail("mmap failed");
    base_ = (uint8_t*)p;
    std::memcpy(&hdr_, base_, sizeof(Header));
    if (std::memcmp(hdr_.magic, "NIDTVOL1", 8) != 0) fail("bad magic (not a NIDTVOL1 file)");
    if (hdr_.version != 1 || hdr_.dtype != 0) fail("unsupported version/dtype");
    vox_ = hdr_.d * hdr_.h * hdr_.w;
    if (hdr_.data_off + hdr_.n * vox_ > size_ || hdr_.labels_off + 4 * hdr_.n > size_ ||
        hdr_.sites_off + 4 * hdr_.n > size_)
      fail("truncated file (sections exceed its size)");
    const int hw = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    pool_ = std::make_unique<Pool>(threads > 0 ? threads : hw);
  }
  ~VolumeReader() {
    pool_.reset();  // drain workers before unmapping
    if (base_) ::munmap(base_, size_);
    if (fd_ >= 0) ::close(fd_);
  }

  uint64_t n() const { return hdr_.n; }
  std::vector<uint64_t> shape() const { return {hdr_.d, hdr_.h, hdr_.w}; }
  uint64_t voxels() const { return vox_; }
  int threads() const { return pool_->size(); }
  std::string path() const { return path_; }

  // float32[n] sections (memcpy: the sections need not be 4-byte aligned in the file)
  void copy_labels(float* out) const { std::memcpy(out, base_ + hdr_.labels_off, 4 * hdr_.n); }
  void copy_sites(float* out) const { std::memcpy(out, base_ + hdr_.sites_off, 4 * hdr_.n); }

  // Asynchronous gather of subjects `ix` into dst (ix.size() * voxels bytes); returns a ticket id.
  int64_t submit(const std::vector<int64_t>& ix, uintptr_t dst) { return start(checked(ix), dst); }
  // Synchronous gather.
  void gather(const std::vector<int64_t>& ix, uintptr_t dst) { wait(submit(ix, dst)); }
  // Block until ticket `id` completes (the ticket is retired).
  void wait(int64_t id) { wait_ticket(id); }
  bool done(int64_t id) { return find(id)->remaining.load() == 0; }

  void prefetch(const std::vector<int64_t>& idx) {
    const std::vector<int64_t> ix = checked(idx);
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    for (int64_t s : ix) {
      const size_t off = hdr_.data_off + (size_t)s * vox_;
      const size_t a = off / pg * pg;
      ::madvise(base_ + a, off + vox_ - a, MADV_WILLNEED);
    }
  }

 private:
  [[noreturn]] void fail(const std::string& msg) {
    if (base_) ::munmap(base_, size_);
    base_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    throw std::runtime_error("nidt_io: " + path_ + ": " + msg);
  }

  std::vector<int64_t> checked(const std::vector<int64_t>& v) const {
    for (int64_t s : v)
      if (s < 0 || (uint64_t)s >= hdr_.n) throw std::out_of_range("nidt_io: subject index out of range");
    return v;
  }

  // Split the copy into ~1 MiB pieces so every worker stays busy even for a handful of subjects.
  int64_t start(std::vector<int64_t> ix, uintptr_t dst) {
    if (ix.empty()) return register_ticket(0).first;
    if (dst == 0) throw std::invalid_argument("nidt_io: null destination");
    const size_t per = (vox_ + kPiece - 1) / kPiece;
    auto reg = register_ticket((int64_t)(ix.size() * per));
    auto shared_ix = std::make_shared<std::vector<int64_t>>(std::move(ix));
    uint8_t* out = reinterpret_cast<uint8_t*>(dst);
    std::shared_ptr<Ticket> t = reg.second;
    for (size_t i = 0; i < shared_ix->size(); ++i) {
      for (size_t p = 0; p < per; ++p) {
        pool_->push([this, shared_ix, i, p, out, t] {
          const size_t lo = p * kPiece, len = std::min(kPiece, (size_t)vox_ - lo);
          std::memcpy(out + i * vox_ + lo, base_ + hdr_.data_off + (size_t)(*shared_ix)[i] * vox_ + lo, len);
          if (t->remaining.fetch_sub(1) == 1) {
            std::lock_guard<std::mutex> g(t->m);
            t->cv.notify_all();
          }
        });
      }
    }
    return reg.first;
  }

  std::pair<int64_t, std::shared_ptr<Ticket>> register_ticket(int64_t njobs) {
    auto t = std::make_shared<Ticket>();
    t->remaining = njobs;
    std::lock_guard<std::mutex> g(tm_);
    const int64_t id = next_++;
    tickets_[id] = t;
    return {id, t};
  }

  std::shared_ptr<Ticket> find(int64_t id) {
    std::lock_guard<std::mutex> g(tm_);
    auto it = tickets_.find(id);
    if (it == tickets_.end()) throw std::invalid_argument("nidt_io: unknown ticket");
    return it->second;
  }

  void wait_ticket(int64_t id) {
    std::shared_ptr<Ticket> t = find(id);
    {
      std::unique_lock<std::mutex> l(t->m);
      t->cv.wait(l, [&] { return t->remaining.load() == 0; });
    }
    std::lock_guard<std::mutex> g(tm_);
    tickets_.erase(id);
  }

  std::string path_;
  int fd_ = -1;
  size_t size_ = 0;
  uint8_t* base_ = nullptr;
  Header hdr_{};
  uint64_t vox_ = 0;
  std::unique_ptr<Pool> pool_;
  std::mutex tm_;
  std::unordered_map<int64_t, std::shared_ptr<Ticket>> tickets_;
  int64_t next_ = 1;
};

}  // namespace nidt_io
