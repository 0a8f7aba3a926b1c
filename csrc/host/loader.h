// Multi-threaded shuffling image loader core (no Python): the native replacement of the
// reference's input queues (string_input_producer -> 16 QueueRunner threads ->
// RandomShuffleQueue, image_input.py:77-115). loader.cpp binds it to Python; the sanitizer
// self-test (tests/native/host_selftest.cpp) drives it directly under ASan/UBSan and TSan.
//
// * reader threads pull file names from an epoch-shuffled list (infinite epochs when `loop`),
//   read TFRecords (CRC-checked), extract the `image_raw` bytes feature, decode raw float64 /
//   float32 / uint8 pixels and convert them ONCE into the output dtype (fp32 or bf16, uint8
//   rescaled by scale/shift) into a slot of a fixed-capacity example pool;
// * next_batch() waits until min_after_dequeue + batch examples are pooled (RandomShuffleQueue
//   semantics), then draws `batch` uniformly random slots into the caller's buffer.
// With threads == 1 the order is a deterministic function of the seed.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
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

class Loader {
 public:
  Loader(std::vector<std::string> files, std::string feature, int H, int W, int C, int batch, int capacity,
         int min_after_dequeue, int threads, uint64_t seed, std::string out_dtype, std::string src_dtype, bool loop,
         bool verify_crc, float u8_scale, float u8_shift)
      : files_(std::move(files)), feature_(std::move(feature)), elems_((size_t)H * W * C), batch_(batch),
        min_after_(std::max(0, min_after_dequeue)), loop_(loop), verify_(verify_crc), u8_scale_(u8_scale),
        u8_shift_(u8_shift), rng_(seed), file_rng_(seed ^ 0x9E3779B97F4A7C15ull) {
    if (files_.empty()) throw std::runtime_error("Loader: no input files");
    if (out_dtype == "f32") out_bytes_ = 4;
    else if (out_dtype == "bf16") out_bytes_ = 2;
    else throw std::runtime_error("out_dtype must be f32 or bf16");
    src_ = src_dtype;
    capacity_ = std::max(capacity, min_after_ + batch_);
    pool_.resize((size_t)capacity_ * elems_ * out_bytes_);
    free_.reserve(capacity_);
    for (int i = capacity_ - 1; i >= 0; --i) free_.push_back(i);
    threads = std::max(1, threads);
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
      return stop_ || !error_.empty() || (int)filled_.size() >= min_after_ + batch_ ||
             (done_workers_ == (int)workers_.size() && !filled_.empty()) ||
             (done_workers_ == (int)workers_.size());
    });
    if (!error_.empty()) throw std::runtime_error(error_);
    int n = 0;
    const size_t ebytes = elems_ * out_bytes_;
    while (n < batch_ && !filled_.empty()) {
      std::uniform_int_distribution<size_t> dist(0, filled_.size() - 1);
      const size_t k = dist(rng_);
      const int slot = filled_[k];
      filled_[k] = filled_.back();
      filled_.pop_back();
      std::memcpy(dst + (size_t)n * ebytes, pool_.data() + (size_t)slot * ebytes, ebytes);
      free_.push_back(slot);
      ++n;
    }
    dequeued_ += n;
    lk.unlock();
    cv_.notify_all();
    return n;
  }

  LoaderStats stats() {
    std::lock_guard<std::mutex> g(mu_);
    LoaderStats st;
    st.records = records_.load();
    st.pooled = (int)filled_.size();
    st.capacity = capacity_;
    st.dequeued = dequeued_;
    st.epochs = epochs_;
    return st;
  }

 private:
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

  void decode_into(const uint8_t* raw, size_t len, uint8_t* dst) {
    std::string src = src_;
    if (src == "auto") {
      if (len == elems_ * 8) src = "f64";
      else if (len == elems_ * 4) src = "f32";
      else if (len == elems_) src = "u8";
      else throw std::runtime_error("image_raw has " + std::to_string(len) + " bytes, expected " +
                                    std::to_string(elems_) + " x {1,4,8}");
    }
    for (size_t i = 0; i < elems_; ++i) {
      float v;
      if (src == "f64") {
        double d;
        std::memcpy(&d, raw + 8 * i, 8);
        v = (float)d;
      } else if (src == "f32") {
        std::memcpy(&v, raw + 4 * i, 4);
      } else {
        v = raw[i] * u8_scale_ + u8_shift_;
      }
      if (out_bytes_ == 4) std::memcpy(dst + 4 * i, &v, 4);
      else {
        const uint16_t b = f2bf(v);
        std::memcpy(dst + 2 * i, &b, 2);
      }
    }
  }

  void work() {
    std::string fname, rec;
    std::vector<uint8_t> tmp(elems_ * out_bytes_);
    try {
      while (take_file(&fname)) {
        RecordReader rr(fname, verify_);
        while (rr.next(&rec)) {
          const uint8_t* p = nullptr;
          size_t len = 0;
          if (!example_bytes_feature(reinterpret_cast<const uint8_t*>(rec.data()), rec.size(), feature_, &p, &len))
            throw std::runtime_error("record without bytes feature '" + feature_ + "' in " + fname);
          decode_into(p, len, tmp.data());
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [this] { return stop_ || !free_.empty(); });
          if (stop_) {
            lk.unlock();
            return finish();
          }
          const int slot = free_.back();
          free_.pop_back();
          std::memcpy(pool_.data() + (size_t)slot * tmp.size(), tmp.data(), tmp.size());
          filled_.push_back(slot);
          ++records_;
          lk.unlock();
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
  std::string feature_, src_;
  size_t elems_;
  int batch_, min_after_, capacity_;
  bool loop_, verify_;
  float u8_scale_, u8_shift_;
  size_t out_bytes_ = 4;
  std::vector<uint8_t> pool_;
  std::vector<int> free_, filled_;
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
