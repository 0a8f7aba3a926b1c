// Multi-threaded shuffling image loader core (no Python): the native replacement of the
// reference's input queues (string_input_producer -> 16 QueueRunner threads ->
// RandomShuffleQueue, image_input.py:77-115). loader.cpp binds it to Python; the sanitizer
// self-test (tests/native/host_selftest.cpp) drives it directly under ASan/UBSan and TSan.
//
// * reader threads pull file names from an epoch-shuffled list (infinite epochs when `loop`),
//   read TFRecords (CRC-checked), extract the `image_raw` bytes feature, and decode raw float64 /
//   float32 / uint8 pixels ONCE, straight into a reserved slot of a fixed-capacity example pool,
//   in the training dtype (fp32, bf16 or fp16; uint8 rescaled by scale/shift) -- so a bf16 run
//   ships half the bytes over H2D;
// * next_batch() waits until min_after_dequeue + batch examples are pooled (RandomShuffleQueue
//   semantics), then draws `batch` uniformly random slots and copies them into the caller's
//   buffer outside the lock.
// Deterministic mode (threads == 1): the single reader pushes records in a
// seed-determined order (epoch-shuffled files, records in file order) into an arrival FIFO, and
// every draw is taken from a window of exactly min_after_dequeue + batch examples -- the window
// is topped up from the FIFO's front before each draw -- however far the reader has run ahead.
// The batch sequence is then a function of the seed and the files alone. With threads > 1 the
// draw covers every pooled example (the readers' interleaving decides arrival order anyway).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "tfrecord.h"

namespace dcgh {

struct LoaderStats {
  uint64_t records = 0, dequeued = 0;
  int pooled = 0, capacity = 0, epochs = 0;
};

static inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// IEEE binary16, round to nearest even (images are in [-1, 1]: no overflow handling needed
// beyond saturation to inf)
static inline uint16_t f2h(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const int32_t e = (int32_t)((u >> 23) & 0xFF) - 127 + 15;
  uint32_t m = u & 0x7FFFFFu;
  if (((u >> 23) & 0xFF) == 0xFF) return (uint16_t)(sign | 0x7C00u | (m ? 0x200u : 0u));
  if (e >= 31) return (uint16_t)(sign | 0x7C00u);
  if (e <= 0) {  // subnormal half
    if (e < -10) return (uint16_t)sign;
    m |= 0x800000u;
    const int shift = 14 - e;
    uint32_t h = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}

enum SrcType { SRC_AUTO = 0, SRC_F64, SRC_F32, SRC_U8 };
enum OutType { OUT_F32 = 0, OUT_BF16, OUT_F16 };

class Loader {
 public:
  Loader(std::vector<std::string> files, std::string feature, int H, int W, int C, int batch, int capacity,
         int min_after_dequeue, int threads, uint64_t seed, std::string out_dtype, std::string src_dtype, bool loop,
         bool verify_crc, float u8_scale, float u8_shift)
      : files_(std::move(files)), feature_(std::move(feature)), elems_((size_t)H * W * C), batch_(batch),
        min_after_(std::max(0, min_after_dequeue)), loop_(loop), verify_(verify_crc), u8_scale_(u8_scale),
        u8_shift_(u8_shift), rng_(seed), file_rng_(seed ^ 0x9E3779B97F4A7C15ull) {
    if (files_.empty()) throw std::runtime_error("Loader: no input files");
    if (out_dtype == "f32") { out_bytes_ = 4; out_ = OUT_F32; }
    else if (out_dtype == "bf16") { out_bytes_ = 2; out_ = OUT_BF16; }
    else if (out_dtype == "f16") { out_bytes_ = 2; out_ = OUT_F16; }
    else throw std::runtime_error("out_dtype must be f32, bf16 or f16");
    if (src_dtype == "auto") src_ = SRC_AUTO;
    else if (src_dtype == "f64") src_ = SRC_F64;
    else if (src_dtype == "f32") src_ = SRC_F32;
    else if (src_dtype == "u8") src_ = SRC_U8;
    else throw std::runtime_error("src_dtype must be auto, f64, f32 or u8");
    capacity_ = std::max(capacity, min_after_ + batch_);
    pool_.resize((size_t)capacity_ * elems_ * out_bytes_);
    free_.reserve(capacity_);
    for (int i = capacity_ - 1; i >= 0; --i) free_.push_back(i);
    threads = std::max(1, threads);
    det_ = threads == 1;
    for (int t = 0; t < threads; ++t) workers_.emplace_back([this] { work(); });
  }

  ~Loader() { stop(); }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
    workers_.clear();
  }

  // fill `batch` examples at dst; returns number filled (< batch only at the end of a non-looping
  // dataset, 0 when exhausted)
  int next_batch(uint8_t* dst) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] {
      return stop_ || !error_.empty() || pooled() >= min_after_ + batch_ || done_workers_ == (int)workers_.size();
    });
    if (!error_.empty()) throw std::runtime_error(error_);
    if (det_) {  // the draw window: exactly min_after + batch examples, in arrival order
      while ((int)filled_.size() < min_after_ + batch_ && !arrived_.empty()) {
        filled_.push_back(arrived_.front());
        arrived_.pop_front();
      }
    }
    // draw the batch's slots under the lock (RandomShuffleQueue semantics), copy them out with
    // the lock released (the readers keep decoding meanwhile), then hand the slots back
    // the drawn slots live in a thread-local scratch vector (no allocation per batch, and two
    // consumers calling next_batch at once never share it)
    thread_local std::vector<int> taken;
    taken.clear();
    while ((int)taken.size() < batch_ && !filled_.empty()) {
      std::uniform_int_distribution<size_t> dist(0, filled_.size() - 1);
      const size_t k = dist(rng_);
      taken.push_back(filled_[k]);
      filled_[k] = filled_.back();
      filled_.pop_back();
    }
    const int n = (int)taken.size();
    dequeued_ += n;
    lk.unlock();
    const size_t ebytes = elems_ * out_bytes_;
    for (int i = 0; i < n; ++i) std::memcpy(dst + (size_t)i * ebytes, pool_.data() + (size_t)taken[i] * ebytes, ebytes);
    lk.lock();
    for (int i = 0; i < n; ++i) free_.push_back(taken[i]);
    lk.unlock();
    cv_.notify_all();
    return n;
  }

  LoaderStats stats() {
    std::lock_guard<std::mutex> g(mu_);
    LoaderStats st;
    st.records = records_.load();
    st.pooled = pooled();
    st.capacity = capacity_;
    st.dequeued = dequeued_;
    st.epochs = epochs_;
    return st;
  }

 private:
  int pooled() const { return (int)(filled_.size() + arrived_.size()); }

  bool take_file(std::string* f) {
    std::lock_guard<std::mutex> g(mu_);
    if (next_file_ >= order_.size()) {
      if (epochs_ > 0 && !loop_) return false;
      order_.resize(files_.size());
      for (size_t i = 0; i < files_.size(); ++i) order_[i] = i;
      std::shuffle(order_.begin(), order_.end(), file_rng_);
      next_file_ = 0;
      ++epochs_;
    }
    *f = files_[order_[next_file_++]];
    return true;
  }

  // raw pixels -> output dtype, one tight loop per (source, output) pair; the source type is
  // resolved per record from the payload size when "auto" (float64 is the reference's format,
  // image_input.py:48)
  template <typename Src>
  void emit(const uint8_t* raw, uint8_t* dst, Src src) const {
    const size_t n = elems_;
    if (out_ == OUT_F32) {
      float* o = reinterpret_cast<float*>(dst);
      for (size_t i = 0; i < n; ++i) o[i] = src(raw, i);
    } else if (out_ == OUT_BF16) {
      uint16_t* o = reinterpret_cast<uint16_t*>(dst);
      for (size_t i = 0; i < n; ++i) o[i] = f2bf(src(raw, i));
    } else {
      uint16_t* o = reinterpret_cast<uint16_t*>(dst);
      for (size_t i = 0; i < n; ++i) o[i] = f2h(src(raw, i));
    }
  }
  void decode_into(const uint8_t* raw, size_t len, uint8_t* dst) const {
    SrcType src = src_;
    if (src == SRC_AUTO) {
      if (len == elems_ * 8) src = SRC_F64;
      else if (len == elems_ * 4) src = SRC_F32;
      else if (len == elems_) src = SRC_U8;
      else throw std::runtime_error("image_raw has " + std::to_string(len) + " bytes, expected " +
                                    std::to_string(elems_) + " x {1,4,8}");
    } else if (len != elems_ * (src == SRC_F64 ? 8 : src == SRC_F32 ? 4 : 1)) {
      throw std::runtime_error("image_raw has " + std::to_string(len) + " bytes, not the declared dtype's size");
    }
    if (src == SRC_F64) {
      emit(raw, dst, [](const uint8_t* r, size_t i) { double d; std::memcpy(&d, r + 8 * i, 8); return (float)d; });
    } else if (src == SRC_F32) {
      emit(raw, dst, [](const uint8_t* r, size_t i) { float f; std::memcpy(&f, r + 4 * i, 4); return f; });
    } else {
      const float sc = u8_scale_, sh = u8_shift_;
      emit(raw, dst, [sc, sh](const uint8_t* r, size_t i) { return r[i] * sc + sh; });
    }
  }

  void work() {
    std::string fname, rec;
    const size_t ebytes = elems_ * out_bytes_;
    try {
      while (take_file(&fname)) {
        RecordReader rr(fname, verify_);
        while (rr.next(&rec)) {
          const uint8_t* p = nullptr;
          size_t len = 0;
          if (!example_bytes_feature(reinterpret_cast<const uint8_t*>(rec.data()), rec.size(), feature_, &p, &len))
            throw std::runtime_error("record without bytes feature '" + feature_ + "' in " + fname);
          int slot;
          {  // reserve a free slot, decode into it with the lock released
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return stop_ || !free_.empty(); });
            if (stop_) {
              lk.unlock();
              return finish();
            }
            slot = free_.back();
            free_.pop_back();
          }
          try {
            decode_into(p, len, pool_.data() + (size_t)slot * ebytes);
          } catch (...) {
            std::lock_guard<std::mutex> g(mu_);
            free_.push_back(slot);
            throw;
          }
          {
            std::lock_guard<std::mutex> g(mu_);
            if (det_) arrived_.push_back(slot);
            else filled_.push_back(slot);
            ++records_;
          }
          cv_.notify_all();
        }
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(mu_);
      if (error_.empty()) error_ = e.what();
    }
    finish();
  }

  void finish() {
    {
      std::lock_guard<std::mutex> g(mu_);
      ++done_workers_;
    }
    cv_.notify_all();
  }

  std::vector<std::string> files_;
  std::string feature_;
  SrcType src_ = SRC_AUTO;
  OutType out_ = OUT_F32;
  size_t elems_;
  int batch_, min_after_, capacity_;
  bool loop_, verify_;
  float u8_scale_, u8_shift_;
  size_t out_bytes_ = 4;
  std::vector<uint8_t> pool_;
  std::vector<int> free_, filled_;  // filled_: the draw pool (deterministic mode: the window)
  std::deque<int> arrived_;          // deterministic mode: decoded examples not yet in the window
  bool det_ = false;
  std::vector<size_t> order_;
  size_t next_file_ = 0;
  int epochs_ = 0;
  uint64_t dequeued_ = 0;
  std::atomic<uint64_t> records_{0};
  std::mt19937_64 rng_, file_rng_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  int done_workers_ = 0;
  std::string error_;
  std::vector<std::thread> workers_;
};

}  // namespace dcgh
