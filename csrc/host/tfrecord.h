// Host-side I/O runtime: TFRecord framing with masked CRC32C, tf.train.Example parsing.
// Replaces TF's TFRecordReader + ParseSingleExample + DecodeRaw (reference image_input.py:40-51).
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace dcgh {

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t crc = 0);
inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

class RecordReader {
 public:
  explicit RecordReader(const std::string& path, bool verify = true);
  ~RecordReader();
  // false at EOF; throws on a truncated or corrupted record
  bool next(std::string* out);
  uint64_t records() const { return n_; }
  uint64_t crc_errors() const { return crc_err_; }

 private:
  FILE* f_ = nullptr;
  bool verify_;
  uint64_t n_ = 0, crc_err_ = 0;
  std::string path_;
};

class RecordWriter {
 public:
  explicit RecordWriter(const std::string& path);
  ~RecordWriter();
  void write(const uint8_t* data, size_t n);
  void close();

 private:
  FILE* f_ = nullptr;
};

// Find the bytes value of feature `key` in a serialized tf.train.Example (BytesList, first
// value). Returns false when absent. No allocation: (ptr, len) point into `ex`.
bool example_bytes_feature(const uint8_t* ex, size_t n, const std::string& key, const uint8_t** ptr,
                           size_t* len);

// Serialize tf.train.Example{features{feature{key: bytes_list{value: [data]}}}} (the record
// layout the reference's image_input.py:42-48 parses). Used by the native self-test.
std::string make_bytes_example(const std::string& key, const uint8_t* data, size_t n);

}  // namespace dcgh
