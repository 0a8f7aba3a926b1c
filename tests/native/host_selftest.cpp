// Native self-test of the host I/O runtime, built and run by tests/test_native_sanitizers.py
// under AddressSanitizer + UndefinedBehaviorSanitizer and, separately, ThreadSanitizer
// (race detection / sanitizers on the host code; GPU sanitizers are not
// available on the MI355X pool). Exercises: CRC32C against the RFC 3720 check value, TFRecord
// write/read round trip, corrupted-record detection, tf.train.Example parsing, and the
// multi-threaded shuffling Loader (4 reader threads) -- a non-looping run that must deliver
// every record exactly once, and a looping run stopped while readers are blocked on a full
// pool. Exit status 0 = all checks passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "loader.h"
#include "tfrecord.h"

using namespace dcgh;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static const int H = 4, W = 4, C = 3, E = H * W * C;

// image k: pixel i = k * 1000 + i (float64 payload, like the reference's records)
static std::string image_record(int k) {
  std::vector<double> px(E);
  for (int i = 0; i < E; ++i) px[i] = k * 1000.0 + i;
  return make_bytes_example("image_raw", reinterpret_cast<const uint8_t*>(px.data()), px.size() * 8);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // ---- CRC32C check value ("123456789" -> 0xE3069283)
  CHECK(crc32c(reinterpret_cast<const uint8_t*>("123456789"), 9) == 0xE3069283u);
  // unaligned start + tail paths
  std::string buf(1000, '\0');
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = (char)(i * 7 + 3);
  const uint32_t whole = crc32c(reinterpret_cast<const uint8_t*>(buf.data()), buf.size());
  const uint32_t part = crc32c(reinterpret_cast<const uint8_t*>(buf.data()) + 3, buf.size() - 3,
                               crc32c(reinterpret_cast<const uint8_t*>(buf.data()), 3));
  CHECK(whole == part);

  // ---- TFRecord files: 3 files x 50 records
  const int NF = 3, NR = 50;
  std::vector<std::string> files;
  for (int f = 0; f < NF; ++f) {
    const std::string path = dir + "/selftest-" + std::to_string(f) + ".tfrecord";
    RecordWriter w(path);
    for (int r = 0; r < NR; ++r) {
      const std::string rec = image_record(f * NR + r);
      w.write(reinterpret_cast<const uint8_t*>(rec.data()), rec.size());
    }
    w.close();
    files.push_back(path);
  }
  {  // round trip + Example parsing
    RecordReader rr(files[1]);
    std::string rec;
    int n = 0;
    while (rr.next(&rec)) {
      const uint8_t* p = nullptr;
      size_t len = 0;
      CHECK(example_bytes_feature(reinterpret_cast<const uint8_t*>(rec.data()), rec.size(), "image_raw", &p, &len));
      CHECK(len == (size_t)E * 8);
      double d0;
      std::memcpy(&d0, p, 8);
      CHECK(d0 == (NR + n) * 1000.0);
      CHECK(!example_bytes_feature(reinterpret_cast<const uint8_t*>(rec.data()), rec.size(), "label", &p, &len));
      ++n;
    }
    CHECK(n == NR);
  }
  {  // corrupted payload byte -> CRC error (throws), truncated file -> throws
    const std::string bad = dir + "/selftest-bad.tfrecord";
    {
      RecordWriter w(bad);
      const std::string rec = image_record(7);
      w.write(reinterpret_cast<const uint8_t*>(rec.data()), rec.size());
    }
    FILE* f = std::fopen(bad.c_str(), "r+b");
    std::fseek(f, 40, SEEK_SET);
    std::fputc(0x5A, f);
    std::fclose(f);
    bool threw = false;
    try {
      RecordReader rr(bad);
      std::string rec;
      rr.next(&rec);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }
  {  // non-looping loader: every record exactly once, in batches of 16 (last batch short)
    Loader L(files, "image_raw", H, W, C, 16, 64, 20, 4, 1234, "f32", "auto", false, true, 1.f, 0.f);
    std::vector<float> out(16 * E);
    std::map<int, int> seen;
    int total = 0;
    for (;;) {
      const int n = L.next_batch(reinterpret_cast<uint8_t*>(out.data()));
      if (n == 0) break;
      for (int i = 0; i < n; ++i) {
        const int k = (int)(out[(size_t)i * E] / 1000.f);
        CHECK(out[(size_t)i * E + 5] == k * 1000.f + 5);
        ++seen[k];
      }
      total += n;
    }
    CHECK(total == NF * NR);
    CHECK((int)seen.size() == NF * NR);
    for (auto& kv : seen) CHECK(kv.second == 1);
    const LoaderStats st = L.stats();
    CHECK(st.records == (uint64_t)(NF * NR) && st.dequeued == (uint64_t)(NF * NR));
  }
  {  // looping bf16 loader: a few batches, then stop() while readers block on the full pool
    Loader L(files, "image_raw", H, W, C, 8, 24, 8, 4, 99, "bf16", "f64", true, true, 1.f, 0.f);
    std::vector<uint16_t> out(8 * E);
    for (int b = 0; b < 30; ++b) CHECK(L.next_batch(reinterpret_cast<uint8_t*>(out.data())) == 8);
    L.stop();
    CHECK(L.stats().epochs >= 1);
  }
  if (g_fail) {
    std::fprintf(stderr, "host_selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_selftest: all checks passed\n");
  return 0;
}
