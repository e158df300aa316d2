// TFRecord framing + a minimal tf.train.Example protobuf codec (no protobuf / TensorFlow dependency).
//
//   Example  { Features features = 1; }
//   Features { map<string, Feature> feature = 1; }          map entry = { string key = 1; Feature value = 2; }
//   Feature  { oneof { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
//   *List    { repeated <T> value = 1; }                     (float/int64 packed when written by TF)
//
// Readers of the reference (src/inputs.py:254-268 decode_bytestring / decode_intstring) look up feature "text" as
// either a UTF-8 string (decoded to code points) or an int64 list; video records carry frame / concat / tokens /
// skip_frame / mask (scripts/video2tfrecord.py:133-166).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#include "rt.h"

namespace rt {

namespace {
std::mutex g_err_mu;
std::string g_err;

bool read_varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift < 64 && p < end; shift += 7) {
    uint8_t b = *p++;
    r |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}

// Skips one field of wire type `wt`; false on malformed input.
bool skip_field(const uint8_t*& p, const uint8_t* end, uint32_t wt) {
  uint64_t v;
  switch (wt) {
    case 0: return read_varint(p, end, &v);
    case 1: if (end - p < 8) return false; p += 8; return true;
    case 2: if (!read_varint(p, end, &v) || uint64_t(end - p) < v) return false; p += v; return true;
    case 5: if (end - p < 4) return false; p += 4; return true;
    default: return false;
  }
}

// Finds the first length-delimited field `field` in [p, end); returns its payload.
bool find_ld(const uint8_t* p, const uint8_t* end, uint32_t field, const uint8_t** out, size_t* n) {
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return false;
    uint32_t f = uint32_t(tag >> 3), wt = uint32_t(tag & 7);
    if (f == field && wt == 2) {
      uint64_t len;
      if (!read_varint(p, end, &len) || uint64_t(end - p) < len) return false;
      *out = p;
      *n = size_t(len);
      return true;
    }
    if (!skip_field(p, end, wt)) return false;
  }
  return false;
}

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back(char(v | 0x80));
    v >>= 7;
  }
  s.push_back(char(v));
}

void put_ld(std::string& s, uint32_t field, const std::string& payload) {
  put_varint(s, (uint64_t(field) << 3) | 2);
  put_varint(s, payload.size());
  s.append(payload);
}
}  // namespace

void set_error(const std::string& msg) {
  std::lock_guard<std::mutex> g(g_err_mu);
  g_err = msg;
}

// ---- RecordFile -----------------------------------------------------------------------------------------------------
RecordFile::~RecordFile() {
  if (base_ && len_) munmap(base_, len_);
  if (fd_ >= 0) ::close(fd_);
}

bool RecordFile::open(const std::string& path, bool verify_crc, std::string* err) {
  path_ = path;
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) {
    *err = "cannot open " + path;
    return false;
  }
  struct stat st;
  if (fstat(fd_, &st) != 0) {
    *err = "cannot stat " + path;
    return false;
  }
  len_ = size_t(st.st_size);
  if (len_ == 0) return true;
  void* m = mmap(nullptr, len_, PROT_READ, MAP_PRIVATE, fd_, 0);
  if (m == MAP_FAILED) {
    *err = "mmap failed for " + path;
    len_ = 0;
    return false;
  }
  base_ = static_cast<uint8_t*>(m);
  madvise(base_, len_, MADV_SEQUENTIAL);
  size_t off = 0;
  while (off < len_) {
    if (len_ - off < 12) {
      *err = path + ": truncated record header at offset " + std::to_string(off);
      return false;
    }
    uint64_t n;
    uint32_t hcrc;
    std::memcpy(&n, base_ + off, 8);
    std::memcpy(&hcrc, base_ + off + 8, 4);
    if (mask_crc(crc32c(base_ + off, 8)) != hcrc) {
      *err = path + ": corrupt length crc at offset " + std::to_string(off);
      return false;
    }
    if (len_ - off - 12 < n + 4) {
      *err = path + ": truncated record payload at offset " + std::to_string(off);
      return false;
    }
    if (verify_crc) {
      uint32_t dcrc;
      std::memcpy(&dcrc, base_ + off + 12 + n, 4);
      if (mask_crc(crc32c(base_ + off + 12, n)) != dcrc) {
        *err = path + ": corrupt payload crc at offset " + std::to_string(off);
        return false;
      }
    }
    index_.emplace_back(off + 12, n);
    off += 12 + n + 4;
  }
  return true;
}

// ---- RecordWriter ---------------------------------------------------------------------------------------------------
RecordWriter::~RecordWriter() { close(); }

bool RecordWriter::open(const std::string& path, std::string* err) {
  f_ = std::fopen(path.c_str(), "wb");
  if (!f_) {
    *err = "cannot create " + path;
    return false;
  }
  std::setvbuf(f_, nullptr, _IOFBF, 1 << 22);
  return true;
}

bool RecordWriter::write(const void* data, size_t n) {
  if (!f_) return false;
  uint64_t len = n;
  uint32_t hcrc = mask_crc(crc32c(&len, 8));
  uint32_t dcrc = mask_crc(crc32c(data, n));
  return std::fwrite(&len, 8, 1, f_) == 1 && std::fwrite(&hcrc, 4, 1, f_) == 1 &&
         (n == 0 || std::fwrite(data, n, 1, f_) == 1) && std::fwrite(&dcrc, 4, 1, f_) == 1;
}

bool RecordWriter::close() {
  if (!f_) return true;
  bool ok = std::fflush(f_) == 0;
  ok = (std::fclose(f_) == 0) && ok;
  f_ = nullptr;
  return ok;
}

// ---- Example decode -------------------------------------------------------------------------------------------------
bool find_feature(const uint8_t* ex, size_t n, const char* key, FeatureView* out) {
  const uint8_t *feats, *end = ex + n;
  size_t fn;
  if (!find_ld(ex, end, 1, &feats, &fn)) return false;
  const uint8_t* p = feats;
  const uint8_t* fend = feats + fn;
  size_t klen = std::strlen(key);
  while (p < fend) {  // iterate map entries (field 1 of Features)
    uint64_t tag;
    if (!read_varint(p, fend, &tag)) return false;
    if ((tag >> 3) != 1 || (tag & 7) != 2) {
      if (!skip_field(p, fend, uint32_t(tag & 7))) return false;
      continue;
    }
    uint64_t elen;
    if (!read_varint(p, fend, &elen) || uint64_t(fend - p) < elen) return false;
    const uint8_t* e = p;
    const uint8_t* eend = p + elen;
    p = eend;
    const uint8_t* k;
    size_t kn;
    if (!find_ld(e, eend, 1, &k, &kn) || kn != klen || std::memcmp(k, key, klen) != 0) continue;
    const uint8_t* fv;
    size_t fvn;
    if (!find_ld(e, eend, 2, &fv, &fvn)) {  // present but empty Feature
      out->kind = kNone;
      out->p = nullptr;
      out->n = 0;
      return true;
    }
    const uint8_t* q = fv;
    const uint8_t* qend = fv + fvn;
    while (q < qend) {
      uint64_t t;
      if (!read_varint(q, qend, &t)) return false;
      uint32_t f = uint32_t(t >> 3);
      if ((t & 7) == 2 && f >= 1 && f <= 3) {
        uint64_t ln;
        if (!read_varint(q, qend, &ln) || uint64_t(qend - q) < ln) return false;
        out->kind = int32_t(f);
        out->p = q;
        out->n = size_t(ln);
        return true;
      }
      if (!skip_field(q, qend, uint32_t(t & 7))) return false;
    }
    out->kind = kNone;
    return true;
  }
  return false;
}

bool int64_values(const FeatureView& f, std::vector<int64_t>* out) {
  if (f.kind != kInt64) return f.kind == kNone;
  const uint8_t* p = f.p;
  const uint8_t* end = f.p + f.n;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return false;
    if ((tag >> 3) != 1) {
      if (!skip_field(p, end, uint32_t(tag & 7))) return false;
      continue;
    }
    if ((tag & 7) == 2) {  // packed
      uint64_t ln;
      if (!read_varint(p, end, &ln) || uint64_t(end - p) < ln) return false;
      const uint8_t* q = p;
      const uint8_t* qe = p + ln;
      out->reserve(out->size() + ln);
      while (q < qe) {
        uint64_t v;
        if (!read_varint(q, qe, &v)) return false;
        out->push_back(int64_t(v));
      }
      p = qe;
    } else if ((tag & 7) == 0) {
      uint64_t v;
      if (!read_varint(p, end, &v)) return false;
      out->push_back(int64_t(v));
    } else {
      return false;
    }
  }
  return true;
}

bool float_values(const FeatureView& f, std::vector<float>* out) {
  if (f.kind != kFloat) return f.kind == kNone;
  const uint8_t* p = f.p;
  const uint8_t* end = f.p + f.n;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return false;
    if ((tag >> 3) != 1) {
      if (!skip_field(p, end, uint32_t(tag & 7))) return false;
      continue;
    }
    if ((tag & 7) == 2) {
      uint64_t ln;
      if (!read_varint(p, end, &ln) || uint64_t(end - p) < ln || ln % 4) return false;
      size_t k = out->size();
      out->resize(k + ln / 4);
      std::memcpy(out->data() + k, p, ln);
      p += ln;
    } else if ((tag & 7) == 5) {
      if (end - p < 4) return false;
      float v;
      std::memcpy(&v, p, 4);
      out->push_back(v);
      p += 4;
    } else {
      return false;
    }
  }
  return true;
}

size_t bytes_count(const FeatureView& f) {
  if (f.kind != kBytes) return 0;
  size_t c = 0;
  const uint8_t* p = f.p;
  const uint8_t* end = f.p + f.n;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return c;
    if ((tag >> 3) == 1 && (tag & 7) == 2) ++c;
    if (!skip_field(p, end, uint32_t(tag & 7))) return c;
  }
  return c;
}

bool bytes_value(const FeatureView& f, size_t idx, const uint8_t** out, size_t* n) {
  if (f.kind != kBytes) return false;
  const uint8_t* p = f.p;
  const uint8_t* end = f.p + f.n;
  size_t c = 0;
  while (p < end) {
    uint64_t tag;
    if (!read_varint(p, end, &tag)) return false;
    if ((tag >> 3) == 1 && (tag & 7) == 2) {
      uint64_t ln;
      if (!read_varint(p, end, &ln) || uint64_t(end - p) < ln) return false;
      if (c++ == idx) {
        *out = p;
        *n = size_t(ln);
        return true;
      }
      p += ln;
    } else if (!skip_field(p, end, uint32_t(tag & 7))) {
      return false;
    }
  }
  return false;
}

// ---- Example encode -------------------------------------------------------------------------------------------------
std::string encode_example(const FeatureIn* fs, int nf) {
  std::string features;
  for (int i = 0; i < nf; ++i) {
    const FeatureIn& f = fs[i];
    std::string list;
    if (f.kind == kBytes) {
      const char* d = static_cast<const char*>(f.data);
      if (f.offsets) {
        for (int64_t j = 0; j < f.n; ++j) put_ld(list, 1, std::string(d + f.offsets[j], d + f.offsets[j + 1]));
      } else {
        put_ld(list, 1, std::string(d, d + f.n));
      }
    } else if (f.kind == kFloat) {
      std::string packed(static_cast<const char*>(f.data), static_cast<const char*>(f.data) + 4 * f.n);
      if (f.n) put_ld(list, 1, packed);
    } else if (f.kind == kInt64) {
      std::string packed;
      const int64_t* v = static_cast<const int64_t*>(f.data);
      for (int64_t j = 0; j < f.n; ++j) put_varint(packed, uint64_t(v[j]));
      if (f.n) put_ld(list, 1, packed);
    }
    std::string feature;
    put_ld(feature, uint32_t(f.kind), list);
    std::string entry;
    put_ld(entry, 1, std::string(f.key));
    put_ld(entry, 2, feature);
    put_ld(features, 1, entry);
  }
  std::string ex;
  put_ld(ex, 1, features);
  return ex;
}

void utf8_decode(const uint8_t* p, size_t n, std::vector<int32_t>* out) {
  out->reserve(out->size() + n);
  size_t i = 0;
  while (i < n) {
    uint8_t c = p[i];
    if (c < 0x80) {
      out->push_back(c);
      ++i;
      continue;
    }
    int len = (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xe ? 3 : (c >> 3) == 0x1e ? 4 : 0;
    uint32_t cp = len == 2 ? (c & 0x1f) : len == 3 ? (c & 0x0f) : (c & 0x07);
    bool ok = len > 0 && i + len <= n;
    for (int k = 1; ok && k < len; ++k) {
      if ((p[i + k] & 0xc0) != 0x80) ok = false;
      else cp = (cp << 6) | (p[i + k] & 0x3f);
    }
    if (ok) {  // reject overlong encodings, surrogates and out-of-range values
      static const uint32_t min_cp[5] = {0, 0, 0x80, 0x800, 0x10000};
      ok = cp >= min_cp[len] && cp <= 0x10ffff && !(cp >= 0xd800 && cp <= 0xdfff);
    }
    if (ok) {
      out->push_back(int32_t(cp));
      i += len;
    } else {
      out->push_back(0xfffd);
      ++i;
    }
  }
}

}  // namespace rt

// ================================================================================================================
// C ABI
extern "C" {

const char* rt_last_error() {
  std::lock_guard<std::mutex> g(rt::g_err_mu);
  return rt::g_err.c_str();
}

void* rt_reader_open(const char* path, int verify_crc) {
  auto* f = new rt::RecordFile();
  std::string err;
  if (!f->open(path, verify_crc != 0, &err)) {
    rt::set_error(err);
    delete f;
    return nullptr;
  }
  return f;
}
int64_t rt_reader_count(void* h) { return int64_t(static_cast<rt::RecordFile*>(h)->count()); }
int64_t rt_reader_record(void* h, int64_t i, const uint8_t** data) {
  auto* f = static_cast<rt::RecordFile*>(h);
  if (i < 0 || size_t(i) >= f->count()) return -1;
  *data = f->data(size_t(i));
  return int64_t(f->size(size_t(i)));
}
void rt_reader_close(void* h) { delete static_cast<rt::RecordFile*>(h); }

void* rt_writer_open(const char* path) {
  auto* w = new rt::RecordWriter();
  std::string err;
  if (!w->open(path, &err)) {
    rt::set_error(err);
    delete w;
    return nullptr;
  }
  return w;
}
int rt_writer_write(void* h, const void* data, int64_t n) {
  return static_cast<rt::RecordWriter*>(h)->write(data, size_t(n)) ? 0 : -1;
}
int rt_writer_write_example(void* h, const rt::FeatureIn* fs, int nf) {
  std::string ex = rt::encode_example(fs, nf);
  return static_cast<rt::RecordWriter*>(h)->write(ex.data(), ex.size()) ? 0 : -1;
}
int rt_writer_close(void* h) {
  auto* w = static_cast<rt::RecordWriter*>(h);
  bool ok = w->close();
  delete w;
  return ok ? 0 : -1;
}

// Encodes into `out` (capacity `cap`); returns the encoded size (call again with a larger buffer if > cap).
int64_t rt_example_encode(const rt::FeatureIn* fs, int nf, uint8_t* out, int64_t cap) {
  std::string ex = rt::encode_example(fs, nf);
  if (int64_t(ex.size()) <= cap) std::memcpy(out, ex.data(), ex.size());
  return int64_t(ex.size());
}

// Returns the feature kind (0 none/absent, 1 bytes, 2 float, 3 int64) and its value count; -1 on malformed input.
int rt_example_feature(const uint8_t* ex, int64_t n, const char* key, int64_t* count) {
  rt::FeatureView f;
  if (!rt::find_feature(ex, size_t(n), key, &f)) {
    *count = 0;
    return 0;
  }
  if (f.kind == rt::kInt64) {
    std::vector<int64_t> v;
    if (!rt::int64_values(f, &v)) return -1;
    *count = int64_t(v.size());
  } else if (f.kind == rt::kFloat) {
    std::vector<float> v;
    if (!rt::float_values(f, &v)) return -1;
    *count = int64_t(v.size());
  } else if (f.kind == rt::kBytes) {
    *count = int64_t(rt::bytes_count(f));
  } else {
    *count = 0;
  }
  return f.kind;
}

int64_t rt_example_int64(const uint8_t* ex, int64_t n, const char* key, int64_t* out, int64_t cap) {
  rt::FeatureView f;
  if (!rt::find_feature(ex, size_t(n), key, &f)) return -1;
  std::vector<int64_t> v;
  if (!rt::int64_values(f, &v)) return -1;
  std::memcpy(out, v.data(), sizeof(int64_t) * size_t(std::min<int64_t>(cap, int64_t(v.size()))));
  return int64_t(v.size());
}

int64_t rt_example_float(const uint8_t* ex, int64_t n, const char* key, float* out, int64_t cap) {
  rt::FeatureView f;
  if (!rt::find_feature(ex, size_t(n), key, &f)) return -1;
  std::vector<float> v;
  if (!rt::float_values(f, &v)) return -1;
  std::memcpy(out, v.data(), sizeof(float) * size_t(std::min<int64_t>(cap, int64_t(v.size()))));
  return int64_t(v.size());
}

// Pointer + length of the idx-th bytes value (borrowed from `ex`); -1 if absent.
int64_t rt_example_bytes(const uint8_t* ex, int64_t n, const char* key, int64_t idx, const uint8_t** out) {
  rt::FeatureView f;
  if (!rt::find_feature(ex, size_t(n), key, &f)) return -1;
  size_t ln;
  if (!rt::bytes_value(f, size_t(idx), out, &ln)) return -1;
  return int64_t(ln);
}

int64_t rt_utf8_decode(const uint8_t* p, int64_t n, int32_t* out, int64_t cap) {
  std::vector<int32_t> v;
  rt::utf8_decode(p, size_t(n), &v);
  std::memcpy(out, v.data(), sizeof(int32_t) * size_t(std::min<int64_t>(cap, int64_t(v.size()))));
  return int64_t(v.size());
}
}
