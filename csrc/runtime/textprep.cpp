// Offline text preparation (reference native tools N1/N2: scripts/train_tokenizer.pyx:98-169 `fix_string` /
// `jsonl_to_txt`, scripts/local_text2tfrecord.pyx:45-89 `create_tfrecords`).
//
//  * rt_jsonl_to_text: streams a Pile-style .jsonl / .jsonl.gz / .jsonl.zst file, extracts one string field per
//    line, replaces four spaces by a tab (the reference's fix_string; ftfy normalisation is not available here)
//    and appends the document plus a separator byte (chr(4) in the reference) to a text file.
//  * rt_text_to_tfrecords: cuts a text file into chunks of `chunk_bytes` (on UTF-8 boundaries) and writes one
//    `Example{text: bytes}` TFRecord file per chunk, named like the reference:
//    `{prefix}bytes_{name}_{index:_>6}_{processed}_{length}.tfrecord` (the last field is what split_files /
//    simulate_data_pipeline parse as the element count).
// zstd is loaded with dlopen (the image ships libzstd.so.1 without headers), gzip through zlib.
#include <dlfcn.h>
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt.h"

namespace {

// ---- minimal zstd streaming ABI (stable since zstd 1.0) ----------------------------------------------------------
struct ZIn {
  const void* src;
  size_t size, pos;
};
struct ZOut {
  void* dst;
  size_t size, pos;
};
struct Zstd {
  void* (*create)() = nullptr;
  size_t (*free_)(void*) = nullptr;
  size_t (*init)(void*) = nullptr;
  size_t (*decompress)(void*, ZOut*, ZIn*) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
  bool load() {
    if (create) return true;
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    create = reinterpret_cast<void* (*)()>(dlsym(h, "ZSTD_createDStream"));
    free_ = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_freeDStream"));
    init = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_initDStream"));
    decompress = reinterpret_cast<size_t (*)(void*, ZOut*, ZIn*)>(dlsym(h, "ZSTD_decompressStream"));
    is_error = reinterpret_cast<unsigned (*)(size_t)>(dlsym(h, "ZSTD_isError"));
    return create && free_ && init && decompress && is_error;
  }
} g_zstd;

// Byte source over plain / gzip / zstd files.
class Source {
 public:
  bool open(const std::string& path, std::string* err) {
    auto ends = [&](const char* s) {
      size_t n = std::strlen(s);
      return path.size() >= n && path.compare(path.size() - n, n, s) == 0;
    };
    if (ends(".gz")) {
      gz_ = gzopen(path.c_str(), "rb");
      if (!gz_) *err = "cannot open " + path;
      return gz_ != nullptr;
    }
    f_ = std::fopen(path.c_str(), "rb");
    if (!f_) {
      *err = "cannot open " + path;
      return false;
    }
    if (ends(".zst")) {
      if (!g_zstd.load()) {
        *err = "libzstd.so.1 not loadable";
        return false;
      }
      zs_ = g_zstd.create();
      g_zstd.init(zs_);
      in_.resize(1 << 20);
    }
    return true;
  }
  ~Source() {
    if (gz_) gzclose(gz_);
    if (f_) std::fclose(f_);
    if (zs_) g_zstd.free_(zs_);
  }
  // reads up to n bytes; 0 at EOF, -1 on error
  long read(char* dst, size_t n) {
    if (gz_) return gzread(gz_, dst, unsigned(n));
    if (!zs_) return long(std::fread(dst, 1, n, f_));
    ZOut out{dst, n, 0};
    while (out.pos == 0) {
      if (zin_.pos == zin_.size) {
        size_t got = std::fread(in_.data(), 1, in_.size(), f_);
        if (got == 0) return 0;
        zin_ = ZIn{in_.data(), got, 0};
      }
      size_t r = g_zstd.decompress(zs_, &out, &zin_);
      if (g_zstd.is_error(r)) return -1;
    }
    return long(out.pos);
  }

 private:
  FILE* f_ = nullptr;
  gzFile gz_ = nullptr;
  void* zs_ = nullptr;
  std::vector<char> in_;
  ZIn zin_{nullptr, 0, 0};
};

void put_utf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) {
    o.push_back(char(cp));
  } else if (cp < 0x800) {
    o.push_back(char(0xc0 | (cp >> 6)));
    o.push_back(char(0x80 | (cp & 0x3f)));
  } else if (cp < 0x10000) {
    o.push_back(char(0xe0 | (cp >> 12)));
    o.push_back(char(0x80 | ((cp >> 6) & 0x3f)));
    o.push_back(char(0x80 | (cp & 0x3f)));
  } else {
    o.push_back(char(0xf0 | (cp >> 18)));
    o.push_back(char(0x80 | ((cp >> 12) & 0x3f)));
    o.push_back(char(0x80 | ((cp >> 6) & 0x3f)));
    o.push_back(char(0x80 | (cp & 0x3f)));
  }
}

struct Json {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  int hex4() {
    if (e - p < 4) return -1;
    int v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return -1;
    }
    return v;
  }
  // parses a string at p (which points at '"'); appends the unescaped text to out (if non-null)
  bool str(std::string* out) {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e) {
      char c = *p++;
      if (c == '"') return true;
      if (c != '\\') {
        if (out) out->push_back(c);
        continue;
      }
      if (p >= e) return false;
      char x = *p++;
      uint32_t cp;
      switch (x) {
        case 'n': cp = '\n'; break;
        case 't': cp = '\t'; break;
        case 'r': cp = '\r'; break;
        case 'b': cp = '\b'; break;
        case 'f': cp = '\f'; break;
        case '/': cp = '/'; break;
        case '\\': cp = '\\'; break;
        case '"': cp = '"'; break;
        case 'u': {
          int h = hex4();
          if (h < 0) return false;
          cp = uint32_t(h);
          if (cp >= 0xd800 && cp < 0xdc00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            int l = hex4();
            if (l >= 0xdc00 && l < 0xe000) cp = 0x10000 + ((cp - 0xd800) << 10) + uint32_t(l - 0xdc00);
            else p = save;
          }
          if (cp >= 0xd800 && cp < 0xe000) cp = 0xfffd;  // lone surrogate
          break;
        }
        default: return false;
      }
      if (out) put_utf8(*out, cp);
    }
    return false;
  }
  bool value() {  // skips any JSON value
    ws();
    if (p >= e) return false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      char open = *p, close = open == '{' ? '}' : ']';
      ++p;
      ws();
      if (p < e && *p == close) {
        ++p;
        return true;
      }
      for (;;) {
        if (open == '{') {
          ws();
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p++ != ':') return false;
        }
        if (!value()) return false;
        ws();
        if (p >= e) return false;
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == close) {
          ++p;
          return true;
        }
        return false;
      }
    }
    while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n') ++p;  // number / literal
    return true;
  }
  // finds top-level key `key` (string valued) of the object in [p, e)
  bool field(const std::string& key, std::string* out) {
    ws();
    if (p >= e || *p != '{') return false;
    ++p;
    for (;;) {
      ws();
      std::string k;
      if (!str(&k)) return false;
      ws();
      if (p >= e || *p++ != ':') return false;
      ws();
      if (k == key && p < e && *p == '"') return str(out);
      if (!value()) return false;
      ws();
      if (p < e && *p == ',') {
        ++p;
        continue;
      }
      return false;
    }
  }
};

void fix_string(std::string& s) {  // "    " → "\t"
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    if (s.compare(i, 4, "    ") == 0) {
      o.push_back('\t');
      i += 4;
    } else {
      o.push_back(s[i++]);
    }
  }
  s.swap(o);
}

}  // namespace

extern "C" {

// Returns the number of documents written, -1 on error. `stats[0]` = input bytes, `stats[1]` = output bytes.
int64_t rt_jsonl_to_text(const char* in_path, const char* out_path, const char* key, int separator, int fix_ws,
                         int append, int64_t* stats) {
  Source src;
  std::string err;
  if (!src.open(in_path, &err)) {
    rt::set_error(err);
    return -1;
  }
  FILE* out = std::fopen(out_path, append ? "ab" : "wb");
  if (!out) {
    rt::set_error(std::string("cannot create ") + out_path);
    return -1;
  }
  std::setvbuf(out, nullptr, _IOFBF, 1 << 22);
  std::vector<char> buf(1 << 22);
  std::string line, text;
  int64_t docs = 0, inb = 0, outb = 0, lineno = 0;
  bool eof = false;
  while (!eof) {
    long got = src.read(buf.data(), buf.size());
    if (got < 0) {
      rt::set_error(std::string("decompression failed: ") + in_path);
      std::fclose(out);
      return -1;
    }
    if (got == 0) eof = true;
    inb += got;
    size_t start = 0;
    for (long i = 0; i <= got; ++i) {
      bool at_end = i == got;
      if (!at_end && buf[size_t(i)] != '\n') continue;
      line.append(buf.data() + start, size_t(i) - start);
      start = size_t(i) + 1;
      if (at_end && !eof) break;  // partial line continues in the next read
      ++lineno;
      size_t a = line.find_first_not_of(" \t\r");
      if (a != std::string::npos) {
        Json j{line.data(), line.data() + line.size()};
        text.clear();
        if (!j.field(key, &text)) {
          rt::set_error(std::string(in_path) + ": line " + std::to_string(lineno) + " has no string field '" + key +
                        "'");
          std::fclose(out);
          return -1;
        }
        if (fix_ws) fix_string(text);
        if (separator >= 0) text.push_back(char(separator));
        std::fwrite(text.data(), 1, text.size(), out);
        outb += int64_t(text.size());
        ++docs;
      }
      line.clear();
    }
  }
  bool ok = std::fclose(out) == 0;
  if (stats) {
    stats[0] = inb;
    stats[1] = outb;
  }
  if (!ok) {
    rt::set_error(std::string("write failed: ") + out_path);
    return -1;
  }
  return docs;
}

// Returns the number of TFRecord files written (index continues from `first_index`), -1 on error.
int64_t rt_text_to_tfrecords(const char* in_path, const char* out_prefix, const char* name, int64_t chunk_bytes,
                             int64_t first_index) {
  FILE* in = std::fopen(in_path, "rb");
  if (!in) {
    rt::set_error(std::string("cannot open ") + in_path);
    return -1;
  }
  std::vector<char> buf(size_t(chunk_bytes) + 4);
  size_t carry = 0;
  int64_t processed = 0, index = first_index, files = 0;
  for (;;) {
    size_t got = std::fread(buf.data() + carry, 1, size_t(chunk_bytes) - carry, in) + carry;
    if (got == 0) break;
    // cut on a UTF-8 boundary: move an incomplete trailing sequence into the next chunk
    size_t cut = got;
    if (got == size_t(chunk_bytes)) {
      size_t k = got;
      while (k > 0 && got - k < 4 && (uint8_t(buf[k - 1]) & 0xc0) == 0x80) --k;
      if (k > 0 && (uint8_t(buf[k - 1]) & 0x80)) {
        uint8_t lead = uint8_t(buf[k - 1]);
        size_t need = (lead >> 5) == 0x6 ? 2 : (lead >> 4) == 0xe ? 3 : (lead >> 3) == 0x1e ? 4 : 1;
        if (got - (k - 1) < need) cut = k - 1;
      }
    }
    processed += int64_t(cut);
    char fname[4096];
    std::snprintf(fname, sizeof fname, "%sbytes_%s_%s%lld_%lld_%lld.tfrecord", out_prefix, name,
                  std::string(size_t(std::max(0, 6 - int(std::to_string(index).size()))), '_').c_str(),
                  (long long)index, (long long)processed, (long long)cut);
    rt::FeatureIn f{"text", rt::kBytes, buf.data(), int64_t(cut), nullptr};
    std::string ex = rt::encode_example(&f, 1);
    rt::RecordWriter w;
    std::string err;
    if (!w.open(fname, &err) || !w.write(ex.data(), ex.size()) || !w.close()) {
      rt::set_error(err.empty() ? std::string("write failed: ") + fname : err);
      std::fclose(in);
      return -1;
    }
    ++index;
    ++files;
    carry = got - cut;
    if (carry) std::memmove(buf.data(), buf.data() + cut, carry);
    if (got < size_t(chunk_bytes) && carry == 0) break;
  }
  std::fclose(in);
  return files;
}
}
