// Parallel blob IO for checkpoints (the reference's sharded TF Saver, src/run/run.py:161-175).
//
// A checkpoint shard is one file holding many tensors back to back (4 KiB aligned). Large tensors are cut into
// kChunk pieces that several threads pwrite / pread concurrently; every piece carries its own CRC32C so corruption
// is detected on restore without re-reading the file. The Python side owns the index (names, shapes, dtypes,
// offsets, CRCs) and the atomic directory rename.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt.h"

namespace {

constexpr int64_t kChunk = 64LL << 20;
constexpr int64_t kAlign = 4096;

struct Piece {
  int blob;
  int64_t off_in_blob, len, file_off;
  size_t crc_slot;
};

std::vector<Piece> plan(int n, const int64_t* sizes, const int64_t* offsets) {
  std::vector<Piece> pieces;
  size_t slot = 0;
  for (int b = 0; b < n; ++b) {
    int64_t done = 0;
    do {
      int64_t len = std::min(kChunk, sizes[b] - done);
      pieces.push_back({b, done, len, offsets[b] + done, slot++});
      done += len;
    } while (done < sizes[b]);
  }
  return pieces;
}

template <typename F>
bool run_parallel(std::vector<Piece>& pieces, int threads, F fn) {
  std::atomic<size_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&] {
    for (size_t i; (i = next.fetch_add(1)) < pieces.size() && ok.load();)
      if (!fn(pieces[i])) ok = false;
  };
  threads = std::max(1, std::min<int>(threads, int(pieces.size())));
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return ok.load();
}

}  // namespace

extern "C" {

int64_t rt_blob_chunk() { return kChunk; }

// Number of CRC slots (pieces) a blob list needs.
int64_t rt_blob_pieces(int n, const int64_t* sizes) {
  int64_t c = 0;
  for (int b = 0; b < n; ++b) c += std::max<int64_t>(1, (sizes[b] + kChunk - 1) / kChunk);
  return c;
}

// Writes blobs into `path` (created/truncated); fills offsets_out[n] and crcs_out[rt_blob_pieces].
int rt_blob_write(const char* path, int n, const void* const* ptrs, const int64_t* sizes, int64_t* offsets_out,
                  uint32_t* crcs_out, int threads) {
  int64_t off = 0;
  for (int b = 0; b < n; ++b) {
    offsets_out[b] = off;
    off += (sizes[b] + kAlign - 1) / kAlign * kAlign;
  }
  int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) {
    rt::set_error(std::string("cannot create ") + path);
    return -1;
  }
  if (off > 0 && ftruncate(fd, off) != 0) {
    ::close(fd);
    rt::set_error(std::string("cannot size ") + path);
    return -1;
  }
  auto pieces = plan(n, sizes, offsets_out);
  bool ok = run_parallel(pieces, threads, [&](const Piece& p) {
    const char* src = static_cast<const char*>(ptrs[p.blob]) + p.off_in_blob;
    crcs_out[p.crc_slot] = rt::crc32c(src, size_t(p.len));
    int64_t done = 0;
    while (done < p.len) {
      ssize_t w = pwrite(fd, src + done, size_t(p.len - done), p.file_off + done);
      if (w <= 0) return false;
      done += w;
    }
    return true;
  });
  ok = ok && fsync(fd) == 0;
  ok = (::close(fd) == 0) && ok;
  if (!ok) rt::set_error(std::string("write failed: ") + path);
  return ok ? 0 : -1;
}

// Reads blobs back into `ptrs`; verifies CRCs when `crcs` is non-null. Returns 0, -1 IO error, -2 CRC mismatch.
int rt_blob_read(const char* path, int n, void* const* ptrs, const int64_t* sizes, const int64_t* offsets,
                 const uint32_t* crcs, int threads) {
  int fd = ::open(path, O_RDONLY);
  if (fd < 0) {
    rt::set_error(std::string("cannot open ") + path);
    return -1;
  }
  auto pieces = plan(n, sizes, offsets);
  std::atomic<bool> crc_bad{false};
  bool ok = run_parallel(pieces, threads, [&](const Piece& p) {
    char* dst = static_cast<char*>(ptrs[p.blob]) + p.off_in_blob;
    int64_t done = 0;
    while (done < p.len) {
      ssize_t r = pread(fd, dst + done, size_t(p.len - done), p.file_off + done);
      if (r <= 0) return false;
      done += r;
    }
    if (crcs && rt::crc32c(dst, size_t(p.len)) != crcs[p.crc_slot]) {
      crc_bad = true;
      return false;
    }
    return true;
  });
  ::close(fd);
  if (crc_bad) {
    rt::set_error(std::string("checkpoint CRC mismatch in ") + path);
    return -2;
  }
  if (!ok) rt::set_error(std::string("read failed: ") + path);
  return ok ? 0 : -1;
}
}
