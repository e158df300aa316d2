// Native host runtime of the framework: TFRecord / tf.train.Example codec, the windowed text loader with an exact
// resume cursor and a prefetch thread, parallel checkpoint IO and the text-preparation tools.
//
// Reference equivalents (SURVEY §2.1 native table): N1 local_text2tfrecord (scripts/local_text2tfrecord.pyx:45-97),
// N2 pile preparation (scripts/train_tokenizer.pyx:45-169), N5 tf.data TFRecord reader + windowing
// (src/inputs.py:231-268,528-568), N6 TF Saver (src/run/run.py:161-175). Everything is exported through a plain C ABI
// (ctypes on the Python side), no TensorFlow, no protobuf library.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rt {

// ---- CRC32C (Castagnoli), SSE4.2 when the CPU has it --------------------------------------------------------------
uint32_t crc32c(const void* data, size_t n, uint32_t crc = 0);
inline uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

void set_error(const std::string& msg);

// ---- TFRecord file: mmapped, indexed on open ------------------------------------------------------------------------
class RecordFile {
 public:
  ~RecordFile();
  bool open(const std::string& path, bool verify_crc, std::string* err);
  size_t count() const { return index_.size(); }
  const uint8_t* data(size_t i) const { return base_ + index_[i].first; }
  size_t size(size_t i) const { return index_[i].second; }
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  size_t len_ = 0;
  std::vector<std::pair<uint64_t, uint64_t>> index_;  // payload offset, payload length
};

// Appends framed records: u64 length, masked crc(length), payload, masked crc(payload).
class RecordWriter {
 public:
  ~RecordWriter();
  bool open(const std::string& path, std::string* err);
  bool write(const void* data, size_t n);
  bool close();

 private:
  FILE* f_ = nullptr;
};

// ---- tf.train.Example (protobuf wire format, hand-rolled) -----------------------------------------------------------
enum FeatureKind : int32_t { kNone = 0, kBytes = 1, kFloat = 2, kInt64 = 3 };

struct FeatureView {  // raw payload of a BytesList / FloatList / Int64List message
  int32_t kind = kNone;
  const uint8_t* p = nullptr;
  size_t n = 0;
};

bool find_feature(const uint8_t* ex, size_t n, const char* key, FeatureView* out);
// Appends the values of an Int64List (packed or not) to `out`; false on a malformed payload.
bool int64_values(const FeatureView& f, std::vector<int64_t>* out);
bool float_values(const FeatureView& f, std::vector<float>* out);
// Iterates the entries of a BytesList: returns the `idx`-th value, false when out of range.
bool bytes_value(const FeatureView& f, size_t idx, const uint8_t** p, size_t* n);
size_t bytes_count(const FeatureView& f);

struct FeatureIn {
  const char* key;
  int32_t kind;
  const void* data;       // bytes: concatenated values; float: float[n]; int64: int64[n]
  int64_t n;              // number of values
  const int64_t* offsets; // bytes only: n+1 offsets into data (nullptr => a single value of n bytes)
};
std::string encode_example(const FeatureIn* f, int nf);

// UTF-8 → code points, invalid sequences become U+FFFD (tf.strings.unicode_decode default)
void utf8_decode(const uint8_t* p, size_t n, std::vector<int32_t>* out);

}  // namespace rt
