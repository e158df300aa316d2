// Windowed text loader with an exact resume cursor and a prefetch thread.
//
// Semantics follow the reference's tf.data graph (src/inputs.py:231-251 `_text_decoder`, :528-568 `gpt_neo_input`):
//   files (already ordered + rank-sharded by split_files in Python)
//   → interleave(cycle_length = interleaved_datasets, block_length = 1)       [tf.data round-robin state machine]
//       per file: records in order; per record: decode "text" (int64 list, or UTF-8 → code points),
//       windows of `window` = ctx + patch tokens with shift `ctx`, remainder dropped
//   → optional shuffle buffer (seeded) → batch(drop_remainder).
// Differences, on purpose:
//   * the per-file element skip is applied once to the file's token stream (the reference applies it to every
//     record of the file, src/inputs.py:245-246);
//   * resume does not replay a run log (the reference's DataLog is never written): the loader exports
//     its exact cursor (open files, record, window, shuffle-buffer contents, RNG) with every batch it hands out,
//     and `restore` continues bit-exactly from it.
// Batches are produced by a C++ thread straight into caller-owned (pinned) host buffers, so the Python side only
// issues the H2D copy on a side stream.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "rt.h"

namespace rt {

struct LoaderConfig {
  int64_t window;          // tokens per sample (sequence_length + token_patch_size * output_offset)
  int64_t shift;           // window shift (sequence_length)
  int64_t batch;           // samples per batch
  int64_t shuffle_buffer;  // 0 = no shuffle
  uint64_t seed;
  int32_t cycle;       // interleave cycle length
  int32_t repeat;      // cycle over the file list forever
  int32_t verify_crc;  // check the payload CRC of every record on open
  int32_t mode;        // 0 = by file name ("int64" → int64 tokens, else UTF-8 bytes), 1 = int64, 2 = bytes
};

namespace {

constexpr int64_t kMagic = 0x4f42535444415441LL;  // "OBSTDATA"
constexpr int64_t kVersion = 1;

uint64_t fnv1a(const std::string& s, uint64_t h) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ULL;
  return h;
}

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct Slot {
  bool open = false;
  int64_t input = 0;       // position in the (possibly repeated) input sequence; file = input % nfiles
  int64_t record = 0;
  int64_t win = 0;
  int64_t drop_front = 0;  // tokens of the current record removed by the element skip
  int64_t skip_left = 0;   // element skip still to apply to later records
  bool decoded = false;
  std::shared_ptr<RecordFile> file;
  std::vector<int32_t> toks;
};

}  // namespace

class Loader {
 public:
  Loader(const LoaderConfig& cfg, std::vector<std::string> files, std::vector<int64_t> skips)
      : cfg_(cfg), files_(std::move(files)), skips_(std::move(skips)), slots_(size_t(std::max(1, cfg.cycle))) {
    cfg_.cycle = std::max(1, cfg_.cycle);
    rng_ = cfg_.seed;
    hash_ = 1469598103934665603ULL;
    for (auto& f : files_) hash_ = fnv1a(f, hash_);
    if (cfg_.shuffle_buffer > 0) shuf_.resize(size_t(cfg_.shuffle_buffer * cfg_.window));
  }

  ~Loader() { stop(); }

  // ---- synchronous API ------------------------------------------------------------------------------------------
  // 1 = batch produced, 0 = end of data, -1 = error (see rt_last_error)
  int next(int32_t* dst) {
    int r = produce(dst);
    if (r == 1) consumed_ = state();
    return r;
  }

  // ---- prefetch API ---------------------------------------------------------------------------------------------
  void start(std::vector<int32_t*> bufs) {
    bufs_ = std::move(bufs);
    buf_state_.assign(bufs_.size(), {});
    for (size_t i = 0; i < bufs_.size(); ++i) free_.push_back(int(i));
    running_ = true;
    worker_ = std::thread([this] { run(); });
  }

  // returns buffer index, -1 end of data, -2 error, -3 timeout
  int acquire(int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [this] { return !ready_.empty() || done_; };
    if (timeout_ms < 0) cv_.wait(lk, pred);
    else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred)) return -3;
    if (!ready_.empty()) {
      int i = ready_.front();
      ready_.pop_front();
      consumed_ = buf_state_[size_t(i)];
      return i;
    }
    return failed_ ? -2 : -1;
  }

  void release(int i) {
    {
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(i);
    }
    cv_.notify_all();
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      running_ = false;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }

  // ---- cursor -----------------------------------------------------------------------------------------------------
  const std::vector<int64_t>& consumed() const { return consumed_; }

  bool restore(const int64_t* s, size_t n, std::string* err) {
    size_t k = 0;
    auto get = [&](int64_t* v) {
      if (k >= n) return false;
      *v = s[k++];
      return true;
    };
    int64_t magic, ver, nfiles, hash, cycle, window, sbuf;
    if (!get(&magic) || magic != kMagic || !get(&ver) || ver != kVersion) {
      *err = "not a loader state";
      return false;
    }
    if (!get(&nfiles) || !get(&hash) || nfiles != int64_t(files_.size()) || uint64_t(hash) != hash_) {
      *err = "loader state belongs to a different file list";
      return false;
    }
    if (!get(&cycle) || !get(&window) || !get(&sbuf) || cycle != cfg_.cycle || window != cfg_.window ||
        sbuf != cfg_.shuffle_buffer) {
      *err = "loader state was written with a different cycle / window / shuffle configuration";
      return false;
    }
    int64_t v;
    if (!get(&next_input_) || !get(&cycle_index_) || !get(&v)) return bad(err);
    rng_ = uint64_t(v);
    num_open_ = 0;
    for (auto& sl : slots_) {
      int64_t open;
      sl = Slot();
      if (!get(&open) || !get(&sl.input) || !get(&sl.record) || !get(&sl.win) || !get(&sl.drop_front) ||
          !get(&sl.skip_left))
        return bad(err);
      if (open) {
        if (!open_file(sl, sl.input, err)) return false;
        sl.open = true;
        ++num_open_;
        if (!decode(sl, err)) return false;
      }
    }
    if (!get(&shuf_count_)) return bad(err);
    if (shuf_count_ < 0 || shuf_count_ > cfg_.shuffle_buffer) return bad(err);
    size_t words = size_t(shuf_count_ * cfg_.window + 1) / 2;
    if (k + words > n) return bad(err);
    if (words) std::memcpy(shuf_.data(), s + k, size_t(shuf_count_ * cfg_.window) * 4);
    k += words;
    shuf_filled_ = shuf_count_ == cfg_.shuffle_buffer;
    if (!get(&v)) return bad(err);
    shuf_filled_ = shuf_filled_ || v != 0;
    consumed_ = state();
    return true;
  }

  std::vector<int64_t> state() const {
    std::vector<int64_t> s = {kMagic, kVersion, int64_t(files_.size()), int64_t(hash_), cfg_.cycle, cfg_.window,
                              cfg_.shuffle_buffer, next_input_, cycle_index_, int64_t(rng_)};
    for (auto& sl : slots_) {
      s.insert(s.end(), {int64_t(sl.open), sl.input, sl.record, sl.win, sl.drop_front, sl.skip_left});
    }
    s.push_back(shuf_count_);
    size_t words = size_t(shuf_count_ * cfg_.window + 1) / 2;
    size_t k = s.size();
    s.resize(k + words, 0);
    if (words) std::memcpy(s.data() + k, shuf_.data(), size_t(shuf_count_ * cfg_.window) * 4);
    s.push_back(int64_t(shuf_filled_));
    return s;
  }

  std::string error() const { return err_; }

 private:
  static bool bad(std::string* err) {
    *err = "truncated or corrupt loader state";
    return false;
  }

  bool end_of_input() const { return !cfg_.repeat && next_input_ >= int64_t(files_.size()); }

  bool open_file(Slot& s, int64_t input, std::string* err) {
    size_t fi = size_t(input % int64_t(files_.size()));
    auto f = std::make_shared<RecordFile>();
    if (!f->open(files_[fi], cfg_.verify_crc != 0, err)) return false;
    s.file = std::move(f);
    s.input = input;
    return true;
  }

  bool int64_mode(const std::string& path) const {
    if (cfg_.mode == 1) return true;
    if (cfg_.mode == 2) return false;
    std::string base = path.substr(path.find_last_of('/') == std::string::npos ? 0 : path.find_last_of('/') + 1);
    return base.find("int64") != std::string::npos;
  }

  // decodes record `s.record` into s.toks and drops `drop_front` tokens
  bool decode(Slot& s, std::string* err) {
    s.toks.clear();
    s.decoded = true;
    if (size_t(s.record) >= s.file->count()) return true;
    const uint8_t* d = s.file->data(size_t(s.record));
    size_t n = s.file->size(size_t(s.record));
    FeatureView fv;
    if (!find_feature(d, n, "text", &fv)) {
      *err = s.file->path() + ": record " + std::to_string(s.record) + " has no 'text' feature";
      return false;
    }
    if (int64_mode(s.file->path())) {
      std::vector<int64_t> v;
      if (fv.kind != kInt64 || !int64_values(fv, &v)) {
        *err = s.file->path() + ": 'text' is not an int64 list";
        return false;
      }
      s.toks.resize(v.size());
      for (size_t i = 0; i < v.size(); ++i) s.toks[i] = int32_t(v[i]);
    } else {
      const uint8_t* p;
      size_t ln;
      if (fv.kind != kBytes || !bytes_value(fv, 0, &p, &ln)) {
        *err = s.file->path() + ": 'text' is not a bytes feature";
        return false;
      }
      utf8_decode(p, ln, &s.toks);
    }
    int64_t drop = std::min<int64_t>(s.drop_front, int64_t(s.toks.size()));
    if (drop) s.toks.erase(s.toks.begin(), s.toks.begin() + drop);
    return true;
  }

  // next window of slot `s`: 1 produced, 0 exhausted, -1 error
  int slot_next(Slot& s, int32_t* dst, std::string* err) {
    for (;;) {
      if (!s.decoded) {
        if (size_t(s.record) >= s.file->count()) return 0;
        s.drop_front = 0;
        if (!decode(s, err)) return -1;
        if (s.skip_left > 0) {  // apply the element skip to the stream's first tokens
          int64_t drop = std::min<int64_t>(s.skip_left, int64_t(s.toks.size()));
          s.toks.erase(s.toks.begin(), s.toks.begin() + drop);
          s.drop_front = drop;
          s.skip_left -= drop;
        }
      }
      int64_t start = s.win * cfg_.shift;
      if (start + cfg_.window <= int64_t(s.toks.size())) {
        std::memcpy(dst, s.toks.data() + start, size_t(cfg_.window) * 4);
        ++s.win;
        return 1;
      }
      ++s.record;
      s.win = 0;
      s.decoded = false;
      s.toks.clear();
      s.toks.shrink_to_fit();
    }
  }

  // tf.data InterleaveDataset(cycle_length, block_length = 1) state machine
  int next_window(int32_t* dst, std::string* err) {
    int64_t empty_opens = 0;
    while (!end_of_input() || num_open_ > 0) {
      Slot& s = slots_[size_t(cycle_index_)];
      if (s.open) {
        int r = slot_next(s, dst, err);
        if (r < 0) return -1;
        cycle_index_ = (cycle_index_ + 1) % cfg_.cycle;
        if (r == 1) return 1;
        s = Slot();
        --num_open_;
        if (++empty_opens > 2 * int64_t(files_.size()) + cfg_.cycle && cfg_.repeat) {
          *err = "no file yields a full window (window " + std::to_string(cfg_.window) + " tokens)";
          return -1;
        }
      } else if (!end_of_input()) {
        Slot fresh;
        if (!open_file(fresh, next_input_, err)) return -1;
        fresh.skip_left = next_input_ < int64_t(files_.size()) && size_t(next_input_) < skips_.size()
                              ? skips_[size_t(next_input_)] : 0;  // skips apply to the first epoch only
        fresh.open = true;
        s = std::move(fresh);
        ++next_input_;
        ++num_open_;
      } else {
        cycle_index_ = (cycle_index_ + 1) % cfg_.cycle;
      }
    }
    return 0;
  }

  // tf.data ShuffleDataset semantics: fill, then emit a random slot and refill it
  int next_element(int32_t* dst, std::string* err) {
    if (cfg_.shuffle_buffer <= 0) return next_window(dst, err);
    const int64_t W = cfg_.window;
    while (!shuf_filled_ && shuf_count_ < cfg_.shuffle_buffer) {
      int r = next_window(shuf_.data() + shuf_count_ * W, err);
      if (r < 0) return -1;
      if (r == 0) {
        shuf_filled_ = true;
        break;
      }
      ++shuf_count_;
    }
    shuf_filled_ = true;
    if (shuf_count_ == 0) return 0;
    int64_t idx = int64_t(splitmix(rng_) % uint64_t(shuf_count_));
    int32_t* slot = shuf_.data() + idx * W;
    std::memcpy(dst, slot, size_t(W) * 4);
    int r = next_window(slot, err);
    if (r < 0) return -1;
    if (r == 0) {  // input exhausted: shrink the buffer
      --shuf_count_;
      if (idx != shuf_count_) std::memcpy(slot, shuf_.data() + shuf_count_ * W, size_t(W) * 4);
    }
    return 1;
  }

  int produce(int32_t* dst) {
    std::string err;
    for (int64_t b = 0; b < cfg_.batch; ++b) {
      int r = next_element(dst + b * cfg_.window, &err);
      if (r < 0) {
        err_ = err;
        set_error(err);
        return -1;
      }
      if (r == 0) return 0;  // drop the remainder
    }
    return 1;
  }

  void run() {
    for (;;) {
      int idx;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !free_.empty() || !running_; });
        if (!running_) break;
        idx = free_.front();
        free_.pop_front();
      }
      int r = produce(bufs_[size_t(idx)]);
      std::lock_guard<std::mutex> g(mu_);
      if (r == 1) {
        buf_state_[size_t(idx)] = state();
        ready_.push_back(idx);
      } else {
        done_ = true;
        failed_ = r < 0;
        cv_.notify_all();
        break;
      }
      cv_.notify_all();
    }
    std::lock_guard<std::mutex> g(mu_);
    done_ = true;
    cv_.notify_all();
  }

  LoaderConfig cfg_;
  std::vector<std::string> files_;
  std::vector<int64_t> skips_;
  std::vector<Slot> slots_;
  uint64_t hash_;
  uint64_t rng_;
  int64_t next_input_ = 0;
  int64_t cycle_index_ = 0;
  int64_t num_open_ = 0;
  std::vector<int32_t> shuf_;
  int64_t shuf_count_ = 0;
  bool shuf_filled_ = false;
  std::vector<int64_t> consumed_;
  std::string err_;

  // prefetch
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<int32_t*> bufs_;
  std::vector<std::vector<int64_t>> buf_state_;
  std::deque<int> free_, ready_;
  bool running_ = false, done_ = false, failed_ = false;
};

}  // namespace rt

extern "C" {

void* rt_loader_create(const rt::LoaderConfig* cfg, const char* const* files, const int64_t* skips, int nfiles) {
  if (nfiles <= 0 || cfg->window <= 0 || cfg->shift <= 0 || cfg->batch <= 0) {
    rt::set_error("loader: need files and positive window / shift / batch");
    return nullptr;
  }
  std::vector<std::string> f(files, files + nfiles);
  std::vector<int64_t> s(skips ? skips : nullptr, skips ? skips + nfiles : nullptr);
  return new rt::Loader(*cfg, std::move(f), std::move(s));
}
void rt_loader_destroy(void* h) { delete static_cast<rt::Loader*>(h); }
int rt_loader_next(void* h, int32_t* dst) { return static_cast<rt::Loader*>(h)->next(dst); }
void rt_loader_start(void* h, int32_t* const* bufs, int n) {
  static_cast<rt::Loader*>(h)->start(std::vector<int32_t*>(bufs, bufs + n));
}
int rt_loader_acquire(void* h, int64_t timeout_ms) { return static_cast<rt::Loader*>(h)->acquire(timeout_ms); }
void rt_loader_release(void* h, int idx) { static_cast<rt::Loader*>(h)->release(idx); }
void rt_loader_stop(void* h) { static_cast<rt::Loader*>(h)->stop(); }
// Writes the cursor after the last batch handed out; returns its length (call with cap 0 to size the buffer).
int64_t rt_loader_state(void* h, int64_t* out, int64_t cap) {
  const auto& s = static_cast<rt::Loader*>(h)->consumed();
  std::vector<int64_t> tmp;
  const std::vector<int64_t>* src = &s;
  if (s.empty()) {
    tmp = static_cast<rt::Loader*>(h)->state();
    src = &tmp;
  }
  if (int64_t(src->size()) <= cap) std::memcpy(out, src->data(), src->size() * 8);
  return int64_t(src->size());
}
int rt_loader_restore(void* h, const int64_t* s, int64_t n) {
  std::string err;
  if (!static_cast<rt::Loader*>(h)->restore(s, size_t(n), &err)) {
    rt::set_error(err);
    return -1;
  }
  return 0;
}
}
