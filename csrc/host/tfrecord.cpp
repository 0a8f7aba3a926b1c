#include "tfrecord.h"

#include <cstring>
#include <stdexcept>

namespace dcgh {

// ---------------------------------------------------------------- CRC32C: SSE4.2, else slicing-by-8
static uint32_t g_tab[8][256];
static bool g_init = [] {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_tab[t][i] = (g_tab[t - 1][i] >> 8) ^ g_tab[0][g_tab[t - 1][i] & 0xFF];
  return true;
}();

#if defined(__x86_64__)
// SSE4.2 crc32 instruction (the same Castagnoli polynomial). It has a 3-cycle latency and issues
// every cycle, so long buffers run three independent streams over consecutive 1 KiB blocks and
// merge them with the linear "append L zero bytes" operator S_L (four 256-entry tables):
//   U(c, A|B|C) = S_L(S_L(U(c, A)) ^ U(0, B)) ^ U(0, C)    (U = raw register update, |A|=|B|=|C|=L)
namespace {
constexpr size_t kBlk = 1024;

__attribute__((target("sse4.2"))) inline uint64_t crc_u64s(uint64_t c, const uint8_t* p, size_t n8) {
  for (size_t i = 0; i < n8; ++i) {
    uint64_t v;
    std::memcpy(&v, p + 8 * i, 8);
    c = __builtin_ia32_crc32di(c, v);
  }
  return c;
}

struct ShiftTables {
  uint32_t t[4][256];
  ShiftTables() {
    uint32_t basis[32];
    static const uint8_t zeros[kBlk] = {};
    for (int b = 0; b < 32; ++b) basis[b] = (uint32_t)crc_u64s(1ull << b, zeros, kBlk / 8);
    for (int k = 0; k < 4; ++k)
      for (uint32_t x = 0; x < 256; ++x) {
        uint32_t r = 0;
        for (int b = 0; b < 8; ++b)
          if (x >> b & 1) r ^= basis[8 * k + b];
        t[k][x] = r;
      }
  }
  uint32_t shift(uint32_t c) const {
    return t[0][c & 0xFF] ^ t[1][(c >> 8) & 0xFF] ^ t[2][(c >> 16) & 0xFF] ^ t[3][c >> 24];
  }
};

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) {
  static const ShiftTables sh;
  uint64_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    --n;
  }
  while (n >= 3 * kBlk) {  // three interleaved streams
    uint64_t a = c, b = 0, d = 0;
    for (size_t i = 0; i < kBlk / 8; ++i) {
      uint64_t va, vb, vd;
      std::memcpy(&va, p + 8 * i, 8);
      std::memcpy(&vb, p + kBlk + 8 * i, 8);
      std::memcpy(&vd, p + 2 * kBlk + 8 * i, 8);
      a = __builtin_ia32_crc32di(a, va);
      b = __builtin_ia32_crc32di(b, vb);
      d = __builtin_ia32_crc32di(d, vd);
    }
    c = sh.shift(sh.shift((uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)d;
    p += 3 * kBlk;
    n -= 3 * kBlk;
  }
  c = crc_u64s(c, p, n / 8);
  p += n / 8 * 8;
  n &= 7;
  while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
  return ~(uint32_t)c;
}
const bool g_hw = __builtin_cpu_supports("sse4.2");
}  // namespace
#endif

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) {
  (void)g_init;
#if defined(__x86_64__)
  if (g_hw) return crc32c_hw(p, n, crc);
#endif
  crc = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    crc = g_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= crc;
    crc = g_tab[7][v & 0xFF] ^ g_tab[6][(v >> 8) & 0xFF] ^ g_tab[5][(v >> 16) & 0xFF] ^ g_tab[4][(v >> 24) & 0xFF] ^
          g_tab[3][(v >> 32) & 0xFF] ^ g_tab[2][(v >> 40) & 0xFF] ^ g_tab[1][(v >> 48) & 0xFF] ^
          g_tab[0][(v >> 56) & 0xFF];
    p += 8;
    n -= 8;
  }
  while (n--) crc = g_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

// ---------------------------------------------------------------- records
RecordReader::RecordReader(const std::string& path, bool verify) : verify_(verify), path_(path) {
  f_ = std::fopen(path.c_str(), "rb");
  if (!f_) throw std::runtime_error("cannot open TFRecord file: " + path);
  std::setvbuf(f_, nullptr, _IOFBF, 1 << 20);
}

RecordReader::~RecordReader() {
  if (f_) std::fclose(f_);
}

bool RecordReader::next(std::string* out) {
  uint8_t hdr[12];
  const size_t got = std::fread(hdr, 1, 12, f_);
  if (got == 0) return false;
  if (got != 12) throw std::runtime_error("truncated TFRecord header in " + path_);
  uint64_t len;
  uint32_t lcrc;
  std::memcpy(&len, hdr, 8);
  std::memcpy(&lcrc, hdr + 8, 4);
  if (verify_ && mask_crc(crc32c(hdr, 8)) != lcrc) {
    ++crc_err_;
    throw std::runtime_error("TFRecord length CRC mismatch in " + path_);
  }
  if (len > (1ull << 32)) throw std::runtime_error("implausible TFRecord length in " + path_);
  out->resize(len);
  if (len && std::fread(&(*out)[0], 1, len, f_) != len) throw std::runtime_error("truncated TFRecord in " + path_);
  uint32_t dcrc;
  if (std::fread(&dcrc, 1, 4, f_) != 4) throw std::runtime_error("truncated TFRecord footer in " + path_);
  if (verify_ && mask_crc(crc32c(reinterpret_cast<const uint8_t*>(out->data()), len)) != dcrc) {
    ++crc_err_;
    throw std::runtime_error("TFRecord data CRC mismatch in " + path_);
  }
  ++n_;
  return true;
}

RecordWriter::RecordWriter(const std::string& path) {
  f_ = std::fopen(path.c_str(), "wb");
  if (!f_) throw std::runtime_error("cannot create " + path);
}

RecordWriter::~RecordWriter() { close(); }

void RecordWriter::write(const uint8_t* data, size_t n) {
  uint8_t hdr[12];
  const uint64_t len = n;
  std::memcpy(hdr, &len, 8);
  const uint32_t lc = mask_crc(crc32c(hdr, 8));
  std::memcpy(hdr + 8, &lc, 4);
  const uint32_t dc = mask_crc(crc32c(data, n));
  std::fwrite(hdr, 1, 12, f_);
  std::fwrite(data, 1, n, f_);
  std::fwrite(&dc, 1, 4, f_);
}

void RecordWriter::close() {
  if (f_) {
    std::fclose(f_);
    f_ = nullptr;
  }
}

// ---------------------------------------------------------------- protobuf walking
static bool rd_varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  int s = 0;
  while (p < end && s < 64) {
    const uint8_t b = *p++;
    r |= (uint64_t)(b & 0x7F) << s;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
    s += 7;
  }
  return false;
}

// iterate fields; calls f(field, wiretype, ptr, len) for length-delimited and skips others
template <class F>
static bool walk(const uint8_t* p, const uint8_t* end, F&& f) {
  while (p < end) {
    uint64_t key;
    if (!rd_varint(p, end, &key)) return false;
    const int wt = key & 7;
    const uint64_t field = key >> 3;
    if (wt == 0) {
      uint64_t v;
      if (!rd_varint(p, end, &v)) return false;
    } else if (wt == 1) {
      p += 8;
    } else if (wt == 5) {
      p += 4;
    } else if (wt == 2) {
      uint64_t ln;
      if (!rd_varint(p, end, &ln) || (uint64_t)(end - p) < ln) return false;
      if (f(field, p, (size_t)ln)) return true;
      p += ln;
    } else {
      return false;
    }
  }
  return true;
}

bool example_bytes_feature(const uint8_t* ex, size_t n, const std::string& key, const uint8_t** ptr, size_t* len) {
  bool found = false;
  walk(ex, ex + n, [&](uint64_t f, const uint8_t* features, size_t fl) {
    if (f != 1) return false;  // Example.features
    walk(features, features + fl, [&](uint64_t f2, const uint8_t* entry, size_t el) {
      if (f2 != 1) return false;  // map entry
      const uint8_t* kptr = nullptr;
      size_t klen = 0;
      const uint8_t* vptr = nullptr;
      size_t vlen = 0;
      walk(entry, entry + el, [&](uint64_t f3, const uint8_t* q, size_t ql) {
        if (f3 == 1) { kptr = q; klen = ql; }
        else if (f3 == 2) { vptr = q; vlen = ql; }
        return false;
      });
      if (!kptr || klen != key.size() || std::memcmp(kptr, key.data(), klen) != 0 || !vptr) return false;
      walk(vptr, vptr + vlen, [&](uint64_t kind, const uint8_t* lst, size_t ll) {
        if (kind != 1) return false;  // BytesList
        walk(lst, lst + ll, [&](uint64_t f4, const uint8_t* v, size_t vl) {
          if (f4 != 1) return false;
          *ptr = v;
          *len = vl;
          found = true;
          return true;
        });
        return true;
      });
      return found;
    });
    return found;
  });
  return found;
}

// ---------------------------------------------------------------- Example writer
static void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back((char)(uint8_t)(v | 0x80));
    v >>= 7;
  }
  o->push_back((char)(uint8_t)v);
}

static void put_len_field(std::string* o, uint8_t tag, const std::string& payload) {
  o->push_back((char)tag);
  put_varint(o, payload.size());
  o->append(payload);
}

std::string make_bytes_example(const std::string& key, const uint8_t* data, size_t n) {
  std::string bl, feat, entry, feats, ex;
  put_len_field(&bl, 0x0A, std::string(reinterpret_cast<const char*>(data), n));  // BytesList.value
  put_len_field(&feat, 0x0A, bl);                                                   // Feature.bytes_list
  put_len_field(&entry, 0x0A, key);                                                 // map entry key
  put_len_field(&entry, 0x12, feat);                                                // map entry value
  put_len_field(&feats, 0x0A, entry);                                               // Features.feature
  put_len_field(&ex, 0x0A, feats);                                                  // Example.features
  return ex;
}

}  // namespace dcgh
