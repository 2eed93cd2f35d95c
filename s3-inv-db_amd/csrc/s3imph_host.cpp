// s3imph_host.cpp — host side of the boundary: the StreamingMPHFBuilder mirror,
// the index-file writers (S3ID framing) and the synthetic prefix generator.
//
// Reference: pkg/format/mphf_streaming.go (builder, :29-232), pkg/format/writer.go
// (ArrayWriter :11-145, BlobWriter :148-246), pkg/format/format.go (header :6-45).
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "s3imph.h"
#include "s3imph_internal.h"

namespace s3imph {

// Developer knobs (s3imph_dev_knobs, include/s3imph.h section 7): off unless the caller opts in.
std::atomic<bool> g_dev_knobs{false};
const char* dev_env(const char* name) {
  return g_dev_knobs.load(std::memory_order_acquire) ? std::getenv(name) : nullptr;
}

void set_err(char* err, size_t errlen, const std::string& msg) {
  if (!err || errlen == 0) return;
  size_t k = std::min(errlen - 1, msg.size());
  std::memcpy(err, msg.data(), k);
  err[k] = '\0';
}

namespace {

void put_le64(uint8_t* p, uint64_t v) {
  for (int b = 0; b < 8; ++b) p[b] = (uint8_t)(v >> (8 * b));
}
void put_le32(uint8_t* p, uint32_t v) {
  for (int b = 0; b < 4; ++b) p[b] = (uint8_t)(v >> (8 * b));
}

bool write_all(FILE* f, const void* p, size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; }

// Large files are written by several threads, each pwrite()-ing its own byte range
// (the reference writes its two arrays in parallel goroutines, mphf_streaming.go:546-596;
// here every big file is split as well).
constexpr uint64_t kParMin = 32ull << 20;  // files from this size on are split
constexpr int kWriters = 8;

int writers_for(uint64_t bytes) { return bytes < kParMin ? 1 : (int)std::min<uint64_t>(kWriters, bytes / (16ull << 20)); }

bool pwrite_all(int fd, const void* p, uint64_t n, uint64_t off) {
  const uint8_t* q = static_cast<const uint8_t*>(p);
  while (n) {
    const ssize_t w = ::pwrite(fd, q, std::min<uint64_t>(n, 1ull << 30), (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    q += w;
    n -= (uint64_t)w;
    off += (uint64_t)w;
  }
  return true;
}

// Runs part(k, lo, hi) for k-th of T contiguous shares of [0, n) (T threads; part 0 here).
template <class F>
bool split_run(uint64_t n, int T, const F& part) {
  std::vector<char> ok(T, 1);
  std::vector<std::thread> th;
  for (int k = 1; k < T; ++k) th.emplace_back([&, k] { ok[k] = part(n * k / T, n * (k + 1) / T); });
  ok[0] = part(0, n / T);
  for (auto& t : th) t.join();
  for (char c : ok)
    if (!c) return false;
  return true;
}

// ArrayWriter of width 8 holding `n` values (+ an optional trailing sentinel), each
// value = src[i] - bias, little endian.
bool write_u64_array(const std::string& path, const uint64_t* src, uint64_t n, uint64_t bias,
                     std::string* msg) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) {
    *msg = "create array file: open " + path + ": " + std::strerror(errno);
    return false;
  }
  uint8_t hdr[kS3idHeaderSize];
  s3id_header(hdr, n, 8);
  if (!pwrite_all(fd, hdr, sizeof hdr, 0)) {
    ::close(fd);
    *msg = "write header: " + path;
    return false;
  }
  const bool ok = split_run(n, writers_for(8 * n), [&](uint64_t lo, uint64_t hi) {
    std::vector<uint8_t> buf(1 << 20);
    for (uint64_t i = lo; i < hi;) {
      const uint64_t k = std::min<uint64_t>(hi - i, buf.size() / 8);
      for (uint64_t t = 0; t < k; ++t) put_le64(buf.data() + 8 * t, src[i + t] - bias);
      if (!pwrite_all(fd, buf.data(), 8 * k, kS3idHeaderSize + 8 * i)) return false;
      i += k;
    }
    return true;
  });
  if (!ok) {
    ::close(fd);
    *msg = "write u64 batch: " + path;
    return false;
  }
  if (::close(fd) != 0) {
    *msg = "close file: " + path;
    return false;
  }
  return true;
}

// ArrayWriter of width 4 (depth.u32, max_depth_in_subtree.u32; writer.go:113-140).
bool write_u32_array(const std::string& path, const uint32_t* src, uint64_t n, std::string* msg) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) {
    *msg = "create array file: open " + path + ": " + std::strerror(errno);
    return false;
  }
  uint8_t hdr[kS3idHeaderSize];
  s3id_header(hdr, n, 4);
  bool ok = pwrite_all(fd, hdr, sizeof hdr, 0);
  if (ok)
    ok = split_run(n, writers_for(4 * n), [&](uint64_t lo, uint64_t hi) {
      std::vector<uint8_t> buf(1 << 20);
      for (uint64_t i = lo; i < hi;) {
        const uint64_t k = std::min<uint64_t>(hi - i, buf.size() / 4);
        for (uint64_t t = 0; t < k; ++t) put_le32(buf.data() + 4 * t, src[i + t]);
        if (!pwrite_all(fd, buf.data(), 4 * k, kS3idHeaderSize + 4 * i)) return false;
        i += k;
      }
      return true;
    });
  if (!ok) {
    ::close(fd);
    *msg = "write u32 batch: " + path;
    return false;
  }
  if (::close(fd) != 0) {
    *msg = "close file: " + path;
    return false;
  }
  return true;
}

bool write_raw(const std::string& path, const uint8_t* p, uint64_t n, std::string* msg) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) {
    *msg = "create " + path + ": " + std::strerror(errno);
    return false;
  }
  const bool ok = split_run(n, writers_for(n), [&](uint64_t lo, uint64_t hi) {
    return pwrite_all(fd, p + lo, hi - lo, lo);
  });
  if (!ok) {
    ::close(fd);
    *msg = "write " + path;
    return false;
  }
  if (::close(fd) != 0) {
    *msg = "close " + path;
    return false;
  }
  return true;
}

bool is_dir(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

}  // namespace

// EncodeHeader (format.go:25-32): magic, version, count, width — little endian, 20 bytes.
void s3id_header(uint8_t out[kS3idHeaderSize], uint64_t count, uint32_t width) {
  put_le32(out, kS3idMagic);
  put_le32(out + 4, kS3idVersion);
  put_le64(out + 8, count);
  put_le32(out + 16, width);
}

bool write_pieces(const std::string& path, size_t count,
                  const std::function<void(size_t, const uint8_t**, uint64_t*, uint64_t*)>& piece, std::string* msg) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) {
    *msg = "create " + path + ": " + std::strerror(errno);
    return false;
  }
  uint64_t bytes = 0;
  for (size_t i = 0; i < count; ++i) {
    const uint8_t* p;
    uint64_t n, off;
    piece(i, &p, &n, &off);
    bytes += n;
  }
  const int T = std::max(1, std::min<int>(writers_for(bytes), (int)count));
  const bool ok = split_run(count, T, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      const uint8_t* p;
      uint64_t n, off;
      piece(i, &p, &n, &off);
      if (!pwrite_all(fd, p, n, off)) return false;
    }
    return true;
  });
  if (!ok) {
    ::close(fd);
    *msg = "write " + path;
    return false;
  }
  if (::close(fd) != 0) {
    *msg = "close " + path;
    return false;
  }
  return true;
}

// mph.bin (mphf_streaming.go:152-169; 0 bytes for the empty set, :509).  On a
// marshal/write failure the reference removes the partial file (:159-168).
int write_mph_file(const std::string& dir, const uint8_t* mph_bin, uint64_t mph_len, std::string* msg) {
  const std::string mph_path = dir + "/mph.bin";
  if (!write_raw(mph_path, mph_bin, mph_len, msg)) {
    ::unlink(mph_path.c_str());
    *msg = "write MPHF: " + *msg;
    return S3IMPH_ERR_IO;
  }
  return S3IMPH_OK;
}

// prefix_blob.bin + prefix_offsets.u64 (writePrefixBlobPreorder :453-504, BlobWriter
// writer.go:148-237): N offsets plus the sentinel, counted N+1 in the header.
int write_prefix_files(const std::string& dir, const uint8_t* blob, const uint64_t* offsets, uint64_t n,
                       std::string* msg) {
  static const uint64_t kZero = 0;
  const uint64_t base = (n && offsets) ? offsets[0] : 0;
  const uint64_t nbytes = (n && offsets) ? offsets[n] - base : 0;
  if (!write_raw(dir + "/prefix_blob.bin", n ? blob + base : nullptr, nbytes, msg)) {
    *msg = "write prefix blob: " + *msg;
    return S3IMPH_ERR_IO;
  }
  if (!write_u64_array(dir + "/prefix_offsets.u64", n ? offsets : &kZero, n + 1, base, msg)) {
    *msg = "write prefix blob: " + *msg;
    return S3IMPH_ERR_IO;
  }
  return S3IMPH_OK;
}

// The finalize arrays, in the reference's order and with its messages: depth.u32 (closed
// with the streaming writers, indexbuild.go:449-457), subtree_end.u64 and
// max_depth_in_subtree.u32 (:474-503), then the depth index (depthindex.go:32-96).
int write_finalize_files(const std::string& dir, const uint32_t* depth, const uint64_t* subtree_end,
                         const uint32_t* max_depth_sub, const uint64_t* depth_offsets, uint64_t n_offsets,
                         const uint64_t* depth_positions, uint64_t n, std::string* msg) {
  if (!is_dir(dir)) {
    *msg = "create depth writer: open " + dir + "/depth.u32: no such directory";
    return S3IMPH_ERR_IO;
  }
  std::string m;
  if (!write_u32_array(dir + "/depth.u32", depth, n, &m)) {
    *msg = "write depth: " + m;
    return S3IMPH_ERR_IO;
  }
  if (!write_u64_array(dir + "/subtree_end.u64", subtree_end, n, 0, &m)) {
    *msg = "write subtree_end: " + m;
    return S3IMPH_ERR_IO;
  }
  if (!write_u32_array(dir + "/max_depth_in_subtree.u32", max_depth_sub, n, &m)) {
    *msg = "write max_depth_in_subtree: " + m;
    return S3IMPH_ERR_IO;
  }
  if (!write_u64_array(dir + "/depth_offsets.u64", depth_offsets, n_offsets, 0, &m)) {
    *msg = "build depth index: write offset: " + m;
    return S3IMPH_ERR_IO;
  }
  if (!write_u64_array(dir + "/depth_positions.u64", depth_positions, n, 0, &m)) {
    *msg = "build depth index: write position: " + m;
    return S3IMPH_ERR_IO;
  }
  return S3IMPH_OK;
}

int write_index_files(const std::string& dir, const uint8_t* mph_bin, uint64_t mph_len, const uint64_t* fp,
                      const uint64_t* pos, uint64_t n, const uint8_t* blob, const uint64_t* offsets,
                      std::string* msg) {
  int rc = write_mph_file(dir, mph_bin, mph_len, msg);
  if (rc != S3IMPH_OK) return rc;
  // mph_fp.u64 / mph_pos.u64 (writeArraysParallel :546-596), the two in parallel
  std::string pmsg;
  bool pos_ok = true;
  std::thread tp([&] { pos_ok = write_u64_array(dir + "/mph_pos.u64", pos, n, 0, &pmsg); });
  const bool fp_ok = write_u64_array(dir + "/mph_fp.u64", fp, n, 0, msg);
  tp.join();
  if (!fp_ok) {
    *msg = "write fingerprints: " + *msg;
    return S3IMPH_ERR_IO;
  }
  if (!pos_ok) {
    *msg = "write positions: " + pmsg;
    return S3IMPH_ERR_IO;
  }
  return write_prefix_files(dir, blob, offsets, n, msg);
}

namespace {

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "array files are written from memory as little endian");

// mph_fp.u64 / mph_pos.u64 written as Build's chunks arrive (feed_build): the header
// first, then each chunk straight from the pinned buffer it landed in.
struct ArrayFileSink : FeedSink {
  FILE* f[2] = {nullptr, nullptr};
  std::string path[2], err[2];
  ArrayFileSink(const std::string& dir, uint64_t n) {
    path[0] = dir + "/mph_fp.u64";
    path[1] = dir + "/mph_pos.u64";
    for (int a = 0; a < 2; ++a) {
      f[a] = std::fopen(path[a].c_str(), "wb");
      if (!f[a]) {
        err[a] = "create array file: open " + path[a] + ": " + std::strerror(errno);
        continue;
      }
      uint8_t hdr[kS3idHeaderSize];
      s3id_header(hdr, n, 8);
      if (!write_all(f[a], hdr, sizeof hdr)) err[a] = "write header: " + path[a];
    }
  }
  ~ArrayFileSink() override {
    for (int a = 0; a < 2; ++a)
      if (f[a]) std::fclose(f[a]);
  }
  bool put(int a, const uint64_t* v, uint64_t cnt) override {
    if (!err[a].empty()) return false;
    if (!write_all(f[a], v, 8 * cnt)) {
      err[a] = "write u64 batch: " + path[a];
      return false;
    }
    return true;
  }
  // close both; the first failure in the reference's order (fingerprints, positions)
  std::string finish() {
    for (int a = 0; a < 2; ++a) {
      if (f[a] && std::fclose(f[a]) != 0 && err[a].empty()) err[a] = "close file: " + path[a];
      f[a] = nullptr;
    }
    if (!err[0].empty()) return "write fingerprints: " + err[0];
    if (!err[1].empty()) return "write positions: " + err[1];
    return "";
  }
  std::string error() const override {
    return !err[0].empty() ? "write fingerprints: " + err[0] : "write positions: " + err[1];
  }
};

}  // namespace

}  // namespace s3imph

using namespace s3imph;

// --------------------------------------------------------------- builder mirror ----
// Add copies each key once into the feed's pooled pinned chunks (s3imph_feed.hip): they are
// the builder's host copy (prefix_blob.bin / prefix_offsets.u64 come straight from them) and,
// on a single GPU, DMA to HBM as they fill, so Build starts with the key set on the device.
struct s3imph_builder {
  int device = 0;
  std::vector<int> devices;  // s3imph_builder_set_gpus (empty: `device` alone)
  unsigned multi_flags = 0;
  std::string temp_dir;
  Feed* feed = nullptr;
  uint64_t count = 0;
  bool built = false;
  // the host path's contiguous copy, moved out of the feed's chunks by the first host-path
  // Build (kept for a retried Build; Adds are refused after it)
  bool host_taken = false;
  std::vector<uint8_t> h_blob;
  std::vector<uint64_t> h_offsets, h_pos;
  ~s3imph_builder() { feed_free(feed); }
  Feed* store() {
    if (!feed) feed = feed_new(device, devices.empty());
    return feed;
  }
};

extern "C" {

int s3imph_dev_knobs(int on) {
  s3imph::g_dev_knobs.store(on != 0, std::memory_order_release);
  return S3IMPH_OK;
}

int s3imph_builder_new(const char* temp_dir, int device, s3imph_builder** out, char* err, size_t errlen) {
  if (!out) return S3IMPH_ERR_INVALID;
  *out = nullptr;
  std::string td = temp_dir ? temp_dir : "";
  if (!td.empty() && !is_dir(td)) {
    set_err(err, errlen, "create temp file: open " + td + ": no such directory");
    return S3IMPH_ERR_IO;
  }
  try {
    s3imph_builder* b = new s3imph_builder();
    b->device = device;
    b->temp_dir = td;
    *out = b;
    return S3IMPH_OK;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_builder_add(s3imph_builder* b, const uint8_t* prefix, uint64_t len, uint64_t pos, char* err,
                       size_t errlen) {
  if (!b || (len && !prefix)) return S3IMPH_ERR_INVALID;
  if (b->built || b->host_taken) {
    set_err(err, errlen, b->built ? "add to MPHF builder: builder already built"
                                  : "add to MPHF builder: a failed Build already took the keys");
    return S3IMPH_ERR_STATE;
  }
  if (!feed_add(b->store(), prefix, len, pos)) {
    set_err(err, errlen, "write prefix: out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
  ++b->count;
  return S3IMPH_OK;
}

int s3imph_builder_add_batch(s3imph_builder* b, const uint8_t* blob, const uint64_t* offsets,
                             const uint64_t* pos, uint64_t n, char* err, size_t errlen) {
  if (!b) return S3IMPH_ERR_INVALID;
  if (b->built || b->host_taken) {
    set_err(err, errlen, b->built ? "add to MPHF builder: builder already built"
                                  : "add to MPHF builder: a failed Build already took the keys");
    return S3IMPH_ERR_STATE;
  }
  if (n == 0) return S3IMPH_OK;  // an empty batch may pass NULL blob / offsets
  if (!blob || !offsets) return S3IMPH_ERR_INVALID;
  if (!feed_add_batch(b->store(), blob, offsets, pos, n)) {
    set_err(err, errlen, "write prefix: out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
  b->count += n;
  return S3IMPH_OK;
}

int s3imph_builder_reserve(s3imph_builder* b, uint64_t n_keys, uint64_t n_bytes, char* err, size_t errlen) {
  if (!b) return S3IMPH_ERR_INVALID;
  if (b->built) {
    set_err(err, errlen, "reserve MPHF builder: builder already built");
    return S3IMPH_ERR_STATE;
  }
  std::string msg;
  const int rc = feed_reserve(b->store(), n_keys, n_bytes, &msg);
  if (rc != S3IMPH_OK) set_err(err, errlen, msg);  // not fatal: Build falls back to the host path
  return S3IMPH_OK;
}

uint64_t s3imph_builder_count(const s3imph_builder* b) { return b ? b->count : 0; }

int s3imph_builder_build(s3imph_builder* b, const char* out_dir, char* err, size_t errlen) {
  if (!b || !out_dir) return S3IMPH_ERR_INVALID;
  if (b->built) {
    set_err(err, errlen, "build MPHF: builder already built");
    return S3IMPH_ERR_STATE;
  }
  const std::string dir = out_dir;
  if (!is_dir(dir)) {
    set_err(err, errlen, "create mph file: open " + dir + "/mph.bin: no such directory");
    return S3IMPH_ERR_IO;
  }
  std::string msg;
  try {
    const uint64_t n = b->count;
    Feed* f = b->store();
    if (n) feed_flush(f);
    if (n && b->devices.empty() && feed_on_device(f)) {
      // the keys are on the device already.  Once the build has succeeded (a failed
      // bbhash.New writes nothing, mphf_streaming.go:141-144) the prefix files are written
      // from the host chunks on one thread while the arrays are written as their chunks
      // come back on two others
      std::string pmsg, amsg;
      int prc = S3IMPH_OK;
      std::thread tp;
      std::unique_ptr<ArrayFileSink> sink;
      std::vector<uint8_t> mph;
      int rc = feed_build(f, &mph, [&]() -> FeedSink* {
        tp = std::thread([&] { prc = feed_write_prefix_files(f, dir, &pmsg); });
        sink.reset(new ArrayFileSink(dir, n));
        return sink.get();
      }, &msg);
      if (sink) amsg = sink->finish();
      if (rc == S3IMPH_OK) {
        rc = write_mph_file(dir, mph.data(), mph.size(), &msg);
        if (rc == S3IMPH_OK && !amsg.empty()) {
          rc = S3IMPH_ERR_IO;
          msg = amsg;
        }
      }
      if (tp.joinable()) tp.join();
      if (rc == S3IMPH_OK && prc != S3IMPH_OK) {
        rc = prc;
        msg = pmsg;
      }
      if (rc != S3IMPH_OK) {
        set_err(err, errlen, msg);
        return rc;
      }
      b->built = true;
      feed_drop_device(f);  // the device copy is no longer needed
      return S3IMPH_OK;
    }
    // host path: several GPUs, or the device feed is off (it failed, or there is no GPU)
    if (!b->host_taken) {
      feed_take_host(f, &b->h_blob, &b->h_offsets, &b->h_pos);
      b->host_taken = true;
    }
    const std::vector<uint8_t>& blob = b->h_blob;
    const std::vector<uint64_t>& offsets = b->h_offsets;
    const std::vector<uint64_t>& pos = b->h_pos;
    std::vector<uint64_t> fp(n), pos_out(n);
    std::vector<uint8_t> mph;
    if (n) {
      int rc = b->devices.empty()
                   ? build_from_host(b->device, blob.data(), offsets.data(), pos.data(), n, fp.data(), pos_out.data(),
                                     &mph, &msg)
                   : build_from_host_multi(b->devices, b->multi_flags, blob.data(), offsets.data(), pos.data(), n,
                                           fp.data(), pos_out.data(), &mph, &msg);
      if (rc != S3IMPH_OK) {
        set_err(err, errlen, msg);
        return rc;
      }
    }
    int rc = write_index_files(dir, mph.data(), mph.size(), fp.data(), pos_out.data(), n, blob.data(),
                               offsets.data(), &msg);
    if (rc != S3IMPH_OK) {
      set_err(err, errlen, msg);
      return rc;
    }
    b->built = true;
    return S3IMPH_OK;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "build MPHF: out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_builder_set_gpus(s3imph_builder* b, int num_gpus, const int* devices, unsigned flags) {
  if (!b || num_gpus < 1 || num_gpus > 64) return S3IMPH_ERR_INVALID;
  if (b->built) return S3IMPH_ERR_STATE;
  b->devices.resize(num_gpus);
  for (int r = 0; r < num_gpus; ++r) b->devices[r] = devices ? devices[r] : r;
  b->multi_flags = flags;
  if (b->feed) feed_drop_device(b->feed);  // the multi-GPU build shards from the host chunks
  return S3IMPH_OK;
}

int s3imph_builder_close(s3imph_builder* b) {
  delete b;
  return S3IMPH_OK;
}

int s3imph_write_index_files(const char* out_dir, const uint8_t* mph_bin, uint64_t mph_len, const uint64_t* fp,
                             const uint64_t* pos, uint64_t n, const uint8_t* blob, const uint64_t* offsets,
                             char* err, size_t errlen) {
  if (!out_dir || (n && (!fp || !pos || !offsets || !blob)) || (mph_len && !mph_bin)) return S3IMPH_ERR_INVALID;
  std::string msg;
  try {
    int rc = write_index_files(out_dir, mph_bin, mph_len, fp, pos, n, blob, offsets, &msg);
    if (rc != S3IMPH_OK) set_err(err, errlen, msg);
    return rc;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
}

// ------------------------------------------------------------ synthetic prefixes ----
// kind 0 (C2/C3/C4): key g of the global sequence: g == 0 -> "" (the root prefix,
// aggregator.go:48); g >= 1 -> 9 lowercase hex digits of g-1, '/', then pseudo-random
// [a-z0-5] segments separated by '/' every 12 bytes, ending in '/'.  The fixed-width hex
// head makes the sequence byte-sorted and distinct by construction.
// kind 1 (C5): g == 0 -> ""; g >= 1 -> an order-preserving head of j = g-1 over the
// ASCII-sorted 64-symbol alphabet kSorted64 — 5 digits while j < 63·64^4 (1.06e9; the top
// digit stays below the last symbol), beyond that the last symbol and 6 more digits — then
// kind 0's segments up to a length L drawn log-uniform on [1, 1024] (raised to the head's
// width where it is shorter: 200M distinct keys cannot be 23 % of <= 4 bytes).  The heads are
// prefix-free and ordered like j, so the sequence is byte-sorted (types.go:160-164) and
// distinct by construction, and key g does not depend on the shard that generates it.
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

static const char kSorted64[] = "-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz";
constexpr uint64_t kShortHeads = 63ull << 24;  // j below this: 5-digit head (top digit <= 62)

static uint32_t head_len(uint64_t j) { return j < kShortHeads ? 5 : 7; }

static uint32_t gen_len(int kind, uint64_t seed, uint32_t avg, uint64_t g) {
  if (g == 0) return 0;
  const uint64_t r = splitmix64(seed * 0x9e3779b97f4a7c15ull ^ (g * 0xd1b54a32d192ed03ull));
  if (kind == 1) {
    const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
    uint32_t L = (uint32_t)std::floor(std::exp(u * std::log(1025.0)));
    L = std::min<uint32_t>(std::max<uint32_t>(L, 1), 1024);
    return std::max(L, head_len(g - 1));
  }
  uint32_t lo = std::max<uint32_t>(10, avg / 2), hi = std::max<uint32_t>(lo, avg + avg / 2);
  return lo + (uint32_t)(r % (uint64_t)(hi - lo + 1));
}

// kind 0's tail: pseudo-random [a-z0-5] segments with '/' every 12 bytes and at the end
static void gen_segments(uint64_t seed, uint64_t g, uint32_t from, uint32_t L, uint8_t* out) {
  static const char kAlpha[] = "abcdefghijklmnopqrstuvwxyz012345";
  uint64_t state = splitmix64(splitmix64(seed) ^ (g * 0xd6e8feb86659fd93ull));
  uint64_t r = 0;
  int avail = 0;
  for (uint32_t i = from; i < L; ++i) {
    if (i + 1 == L || i % 12 == 11) {
      out[i] = '/';
      continue;
    }
    if (avail == 0) {
      state += 0x9e3779b97f4a7c15ull;
      r = splitmix64(state);
      avail = 12;
    }
    out[i] = (uint8_t)kAlpha[r & 31];
    r >>= 5;
    --avail;
  }
}

static void gen_fill(int kind, uint64_t seed, uint64_t g, uint32_t L, uint8_t* out) {
  static const char kHex[] = "0123456789abcdef";
  if (L == 0) return;
  const uint64_t j = g - 1;
  if (kind == 1) {
    const uint32_t h = head_len(j);
    const uint64_t v = j < kShortHeads ? j : j - kShortHeads;
    if (h == 7) out[0] = (uint8_t)kSorted64[63];
    for (uint32_t i = 0; i < 5 + (h == 7); ++i) {  // the digits, most significant first
      const uint32_t sh = 6 * (4 + (h == 7) - i);
      out[h - 5 - (h == 7) + i] = (uint8_t)kSorted64[(v >> sh) & 63];
    }
    if (L > h) gen_segments(seed, g, h, L, out);
    return;
  }
  for (int d = 0; d < 9; ++d) out[d] = (uint8_t)kHex[(j >> (4 * (8 - d))) & 0xf];
  out[9] = '/';
  gen_segments(seed, g, 10, L, out);
}

int s3imph_gen_keys(int kind, uint64_t seed, uint32_t avg_len, uint64_t lo, uint64_t n, uint8_t* blob,
                    uint64_t* offsets, uint64_t* total_bytes) {
  if ((kind != 0 && kind != 1) || (kind == 0 && avg_len == 0)) return S3IMPH_ERR_INVALID;
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 100000) nt = 1;
  // pass 1: lengths (threaded) and the exclusive prefix sum.
  std::vector<uint64_t> part(nt + 1, 0);
  auto len_range = [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t s = 0;
    for (uint64_t i = a; i < b; ++i) {
      const uint32_t L = gen_len(kind, seed, avg_len, lo + i);
      if (offsets) offsets[i + 1] = L;
      s += L;
    }
    part[t + 1] = s;
  };
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(len_range, t, n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
  th.clear();
  for (unsigned t = 0; t < nt; ++t) part[t + 1] += part[t];
  if (total_bytes) *total_bytes = part[nt];
  if (!offsets) return S3IMPH_OK;
  offsets[0] = 0;
  auto scan_fill = [&](unsigned t, uint64_t a, uint64_t b) {
    uint64_t acc = part[t];
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t L = offsets[i + 1];
      if (blob) gen_fill(kind, seed, lo + i, (uint32_t)L, blob + acc);
      acc += L;
      offsets[i + 1] = acc;
    }
  };
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(scan_fill, t, n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
  return S3IMPH_OK;
}

}  // extern "C"
