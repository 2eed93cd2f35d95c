// s3imph_feed.hip — the builder mirror's key store, its upstream feed to the GPU and the
// output emission on one GPU.
//
// The reference's StreamingMPHFBuilder.Add (mphf_streaming.go:68-97) keeps hashes,
// fingerprints and positions in growing slices and appends every prefix to a temp file
// that Build reads back for prefix_blob.bin (writePrefixBlobPreorder, :453-504).  Here Add
// copies each key ONCE, into a list of pinned host chunks (a process-wide pool, so a
// second builder pays no pinning and no page faults).  The chunks are the builder's host
// copy — prefix_blob.bin / prefix_offsets.u64 are written straight from them — and, as a
// chunk fills, it is DMA'd to the device arrays (blob, offsets, positions) on the feed's
// stream.  A chunk is never rewritten, so no DMA is ever waited for during Add.  With a
// capacity hint (s3imph_builder_reserve) the device arrays are allocated once; without
// one they double (device-to-device copy on the same stream, old buffers freed at Build).
// Build then runs the single-GPU pipeline on the device arrays and streams mph_fp /
// mph_pos back through pooled pinned chunks, two threads (one per array, as
// writeArraysParallel, :546-596) each handing chunk k to the caller's sink while the DMA
// of chunk k+1 runs.  The sink (the output files) is opened only once the build has
// succeeded: like the reference's Build, a failed bbhash.New leaves out_dir untouched.
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <thread>

#include "s3imph_ctx.h"

namespace s3imph {

s3imph_ctx* default_ctx(int device, std::string* msg);

namespace {

constexpr uint64_t kMinChunk = 256ull << 10;  // first chunk of an arena; each next one doubles
constexpr uint64_t kMaxChunk = 64ull << 20;   // ... up to this
constexpr uint64_t kPoolKeep = 16ull << 30;   // pinned bytes the pool keeps cached between builders (at most)

// The pool's cap: 16 GiB, or an eighth of physical memory if that is less, or
// S3IMPH_PINNED_KEEP bytes.  Page-locked memory a long-lived host process (the cgo caller)
// keeps between builds is memory the rest of the box cannot page.
uint64_t pool_keep() {
  static const uint64_t keep = [] {
    if (const char* e = std::getenv("S3IMPH_PINNED_KEEP")) return (uint64_t)std::strtoull(e, nullptr, 10);
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
    const uint64_t phys = pages > 0 && psz > 0 ? (uint64_t)pages * (uint64_t)psz : 0;
    return phys ? std::min<uint64_t>(kPoolKeep, phys / 8) : kPoolKeep;
  }();
  return keep;
}

// Process-wide cache of pinned host chunks by size.  hipHostMalloc pins (and zeroes) every
// page: ~5 GB/s, the cost that dominated round 2's Add.  Chunks come back at Build / close.
struct PinnedPool {
  std::mutex mu;
  std::map<uint64_t, std::vector<void*>> idle;
  uint64_t cached = 0;
  void* get(uint64_t sz) {
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = idle.find(sz);
      if (it != idle.end() && !it->second.empty()) {
        void* p = it->second.back();
        it->second.pop_back();
        cached -= sz;
        return p;
      }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
  }
  void put(void* p, uint64_t sz) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (cached + sz <= pool_keep()) {
        idle[sz].push_back(p);
        cached += sz;
        return;
      }
    }
    (void)hipHostFree(p);
  }
  // Unpin idle chunks, largest first, until at most `keep` bytes stay cached.
  void trim(uint64_t keep) {
    std::vector<std::pair<void*, uint64_t>> drop;
    {
      std::lock_guard<std::mutex> lk(mu);
      for (auto it = idle.rbegin(); it != idle.rend() && cached > keep; ++it)
        while (!it->second.empty() && cached > keep) {
          drop.emplace_back(it->second.back(), it->first);
          it->second.pop_back();
          cached -= it->first;
        }
    }
    for (auto& d : drop) (void)hipHostFree(d.first);
  }
};
// Builders alive (feed_new .. feed_free): when the last one closes, the pool keeps only the
// chunks of one typical builder (1 GiB) pinned, not the largest build's working set.
std::atomic<int> g_live_feeds{0};
constexpr uint64_t kPoolKeepIdle = 1ull << 30;

PinnedPool& pool() {
  static PinnedPool* p = new PinnedPool();  // never destroyed: chunks may return during exit
  return *p;
}

// One append-only byte array: host chunks (pinned, or plain heap memory when no GPU is
// usable) and, while the device path is on, its device copy at byte offset dev_base.
struct Arena {
  struct Chunk {
    uint8_t* p;
    uint64_t size, start;  // capacity, arena offset of its first byte
    bool pinned;
  };
  std::vector<Chunk> ch;
  uint64_t total = 0;  // bytes appended
  uint64_t fill = 0;   // bytes in ch.back()
  uint64_t dev_base = 0, sent = 0;  // device offset of arena byte 0; arena bytes enqueued to DMA
  uint8_t* d = nullptr;
  uint64_t cap = 0;  // device capacity (bytes, dev_base included)
  std::vector<uint8_t*> retired;  // outgrown device buffers, freed once the stream has passed them

  ~Arena() {
    for (auto& c : ch) {
      if (c.pinned)
        pool().put(c.p, c.size);
      else
        std::free(c.p);
    }
  }
  bool new_chunk(bool want_pinned) {
    const uint64_t sz = std::min(kMaxChunk, kMinChunk << std::min<size_t>(ch.size(), 16));
    void* p = want_pinned ? pool().get(sz) : nullptr;
    const bool pinned = p != nullptr;
    if (!p) p = std::malloc(sz);
    if (!p) return false;
    ch.push_back(Chunk{static_cast<uint8_t*>(p), sz, total, pinned});
    fill = 0;
    return true;
  }
  // copies the whole arena to dst chunk by chunk, giving each chunk back (pool or heap) as
  // soon as it is copied: the host copy moves instead of doubling
  void drain(uint8_t* dst) {
    for (size_t k = 0; k < ch.size(); ++k) {
      const uint64_t m = k + 1 < ch.size() ? ch[k].size : fill;
      std::memcpy(dst + ch[k].start, ch[k].p, m);
      if (ch[k].pinned)
        pool().put(ch[k].p, ch[k].size);
      else
        std::free(ch[k].p);
    }
    ch.clear();
    fill = 0;
  }
  // reads [a, a+n) of the arena into dst
  void read(uint64_t a, uint8_t* dst, uint64_t n) const {
    size_t k = 0;
    while (k + 1 < ch.size() && ch[k + 1].start <= a) ++k;
    while (n) {
      const uint64_t o = a - ch[k].start, m = std::min(n, ch[k].size - o);
      std::memcpy(dst, ch[k].p + o, m);
      dst += m;
      a += m;
      n -= m;
      ++k;
    }
  }
};

}  // namespace

struct Feed {
  int device = 0;
  bool dev_on = false;  // the device copy is being fed (single GPU, no failure so far)
  bool pinned_ok = true;
  hipStream_t s = nullptr;
  hipStream_t out_s[2] = {nullptr, nullptr};
  Arena blob, ends, pos;  // ends: each key's end offset in the builder's blob (offsets[1..n])
  uint64_t n = 0;
  uint64_t reserve_keys = 0, reserve_bytes = 0;
  uint64_t* d_out[2] = {nullptr, nullptr};  // fp_out, pos_out
  bool host_taken = false;  // feed_take_host moved the host chunks out: no more Adds
  uint64_t out_cap = 0;

  void drop_device() {
    if (s) (void)hipStreamSynchronize(s);
    for (Arena* a : {&blob, &ends, &pos}) {
      for (uint8_t* r : a->retired) (void)hipFree(r);
      a->retired.clear();
      if (a->d) (void)hipFree(a->d);
      a->d = nullptr;
      a->cap = 0;
      a->sent = 0;
    }
    for (int k = 0; k < 2; ++k) {
      if (d_out[k]) (void)hipFree(d_out[k]);
      d_out[k] = nullptr;
    }
    out_cap = 0;
    dev_on = false;
  }
  ~Feed() {
    if (s || dev_on) {
      (void)hipSetDevice(device);
      drop_device();
    }
    for (int a = 0; a < 2; ++a)
      if (out_s[a]) (void)hipStreamDestroy(out_s[a]);
    if (s) (void)hipStreamDestroy(s);
  }

  // device capacity of `a` for `need` bytes (dev_base included)
  void dev_reserve(Arena& a, uint64_t need) {
    if (need <= a.cap) return;
    uint64_t nc = std::max<uint64_t>(a.cap ? 2 * a.cap : (16ull << 20), need);
    nc = (nc + 4095) & ~4095ull;
    uint8_t* nd = nullptr;
    HIPCHECK(hipMalloc(&nd, nc));
    if (a.d) {
      if (a.dev_base + a.sent) HIPCHECK(hipMemcpyAsync(nd, a.d, a.dev_base + a.sent, hipMemcpyDeviceToDevice, s));
      a.retired.push_back(a.d);
    } else if (a.dev_base) {
      HIPCHECK(hipMemsetAsync(nd, 0, a.dev_base, s));  // offsets[0] = 0
    }
    a.d = nd;
    a.cap = nc;
  }
  // enqueue arena bytes [a.sent, upto) — whole chunks during Add, the tail at Build
  void dev_send(Arena& a, uint64_t upto) {
    if (!dev_on || upto <= a.sent) return;
    try {
      HIPCHECK(hipSetDevice(device));
      dev_reserve(a, a.dev_base + upto);
      size_t k = 0;
      while (k + 1 < a.ch.size() && a.ch[k + 1].start <= a.sent) ++k;
      while (a.sent < upto) {
        const Arena::Chunk& c = a.ch[k];
        const uint64_t o = a.sent - c.start, m = std::min(upto - a.sent, c.size - o);
        HIPCHECK(hipMemcpyAsync(a.d + a.dev_base + a.sent, c.p + o, m, hipMemcpyHostToDevice, s));
        a.sent += m;
        ++k;
      }
    } catch (const Fail&) {
      drop_device();  // Build falls back to the host copy (build_from_host)
    }
  }
  bool append(Arena& a, const void* src, uint64_t bytes) {
    const uint8_t* p = static_cast<const uint8_t*>(src);
    while (bytes) {
      if (a.ch.empty() || a.fill == a.ch.back().size) {
        if (!a.ch.empty()) dev_send(a, a.total);  // the full chunk goes to the device
        if (!a.new_chunk(pinned_ok)) return false;
      }
      Arena::Chunk& c = a.ch.back();
      const uint64_t k = std::min(bytes, c.size - a.fill);
      std::memcpy(c.p + a.fill, p, k);
      a.fill += k;
      a.total += k;
      p += k;
      bytes -= k;
    }
    return true;
  }
  // room for `bytes` more in the current chunk of `a` (a new chunk when it is full)
  uint8_t* span(Arena& a, uint64_t* room) {
    if (a.ch.empty() || a.fill == a.ch.back().size) {
      if (!a.ch.empty()) dev_send(a, a.total);
      if (!a.new_chunk(pinned_ok)) return nullptr;
    }
    *room = a.ch.back().size - a.fill;
    return a.ch.back().p + a.fill;
  }
  void advance(Arena& a, uint64_t bytes) {
    a.fill += bytes;
    a.total += bytes;
  }
};

Feed* feed_new(int device, bool use_gpu) {
  Feed* f = new Feed();
  g_live_feeds.fetch_add(1);
  f->device = device;
  f->ends.dev_base = 8;  // device offsets array = [0, ends...]
  if (use_gpu) {
    try {
      HIPCHECK(hipSetDevice(device));
      HIPCHECK(hipStreamCreateWithFlags(&f->s, hipStreamNonBlocking));
      for (int a = 0; a < 2; ++a) HIPCHECK(hipStreamCreateWithFlags(&f->out_s[a], hipStreamNonBlocking));
      f->dev_on = true;
    } catch (const Fail&) {
      f->dev_on = false;
    }
  }
  f->pinned_ok = f->dev_on;  // no GPU: plain heap chunks (the keys still reach the files)
  return f;
}

void feed_free(Feed* f) {
  if (!f) return;  // only feeds feed_new made are counted (a builder that never stored a key has none)
  delete f;  // its chunks go back to the pool
  if (g_live_feeds.fetch_sub(1) == 1) pool().trim(std::min(pool_keep(), kPoolKeepIdle));
}

void feed_drop_device(Feed* f) {
  if (!f->dev_on) return;
  (void)hipSetDevice(f->device);
  f->drop_device();
}

int feed_reserve(Feed* f, uint64_t n_keys, uint64_t n_bytes, std::string* msg) {
  f->reserve_keys = std::max(f->reserve_keys, n_keys);
  f->reserve_bytes = std::max(f->reserve_bytes, n_bytes);
  if (!f->dev_on) return S3IMPH_OK;
  try {
    HIPCHECK(hipSetDevice(f->device));
    // the blob stays readable 16 bytes past its 8-byte-rounded end (the kernels' wide loads)
    f->dev_reserve(f->blob, ((n_bytes + 7) & ~7ull) + 16);
    f->dev_reserve(f->ends, 8 * (n_keys + 1));
    f->dev_reserve(f->pos, 8 * std::max<uint64_t>(n_keys, 1));
    return S3IMPH_OK;
  } catch (const Fail& e) {
    *msg = "reserve MPHF builder: " + e.msg;
    f->drop_device();
    return e.code;
  }
}

bool feed_add(Feed* f, const uint8_t* key, uint64_t len, uint64_t pos) {
  if (!f->append(f->blob, key, len)) return false;
  const uint64_t end = f->blob.total;
  if (!f->append(f->ends, &end, 8) || !f->append(f->pos, &pos, 8)) return false;
  ++f->n;
  return true;
}

bool feed_add_batch(Feed* f, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n) {
  const uint64_t base = offsets[0];
  const uint64_t shift = f->blob.total;
  if (!f->append(f->blob, blob + base, offsets[n] - base)) return false;
  // end offsets rebased to the builder's blob, written straight into the chunks
  for (uint64_t i = 0; i < n;) {
    uint64_t room = 0;
    uint8_t* dst = f->span(f->ends, &room);
    if (!dst) return false;
    const uint64_t k = std::min(n - i, room / 8);
    if (k == 0) return false;  // chunks hold whole u64 words (sizes are multiples of 8)
    uint64_t* o = reinterpret_cast<uint64_t*>(dst);
    for (uint64_t t = 0; t < k; ++t) o[t] = offsets[i + t + 1] - base + shift;
    f->advance(f->ends, 8 * k);
    i += k;
  }
  if (pos) {
    if (!f->append(f->pos, pos, 8 * n)) return false;
  } else {
    const uint64_t c0 = f->n;
    for (uint64_t i = 0; i < n;) {
      uint64_t room = 0;
      uint8_t* dst = f->span(f->pos, &room);
      if (!dst) return false;
      const uint64_t k = std::min(n - i, room / 8);
      uint64_t* o = reinterpret_cast<uint64_t*>(dst);
      for (uint64_t t = 0; t < k; ++t) o[t] = c0 + i + t;
      f->advance(f->pos, 8 * k);
      i += k;
    }
  }
  f->n += n;
  return true;
}

uint64_t feed_count(const Feed* f) { return f ? f->n : 0; }

void feed_flush(Feed* f) {
  f->dev_send(f->blob, f->blob.total);
  f->dev_send(f->ends, f->ends.total);
  f->dev_send(f->pos, f->pos.total);
}

bool feed_on_device(const Feed* f) { return f && f->dev_on; }

void feed_take_host(Feed* f, std::vector<uint8_t>* blob, std::vector<uint64_t>* offsets, std::vector<uint64_t>* pos) {
  blob->assign(((f->blob.total + 7) & ~7ull) + 16, 0);  // the host build's staging reads whole words
  f->blob.drain(blob->data());
  offsets->assign(f->n + 1, 0);
  f->ends.drain(reinterpret_cast<uint8_t*>(offsets->data() + 1));
  pos->resize(f->n);
  f->pos.drain(reinterpret_cast<uint8_t*>(pos->data()));
  f->host_taken = true;
}

// prefix_blob.bin / prefix_offsets.u64 straight from the chunks (writePrefixBlobPreorder,
// mphf_streaming.go:453-504; BlobWriter, writer.go:148-237): every chunk is one pwrite at
// its file offset, spread over up to 8 threads.
int feed_write_prefix_files(const Feed* f, const std::string& dir, std::string* msg) {
  struct Piece {
    const uint8_t* p;
    uint64_t n, off;
  };
  auto pieces = [](const Arena& a, uint64_t file_off) {
    std::vector<Piece> v;
    for (size_t k = 0; k < a.ch.size(); ++k) {
      const uint64_t n = k + 1 < a.ch.size() ? a.ch[k].size : a.fill;
      if (n) v.push_back(Piece{a.ch[k].p, n, file_off + a.ch[k].start});
    }
    return v;
  };
  uint8_t hdr[kS3idHeaderSize + 8];
  s3id_header(hdr, f->n + 1, 8);
  std::memset(hdr + kS3idHeaderSize, 0, 8);  // offsets[0]
  std::vector<Piece> off_pieces = pieces(f->ends, kS3idHeaderSize + 8);
  off_pieces.insert(off_pieces.begin(), Piece{hdr, sizeof hdr, 0});
  const std::pair<std::string, std::vector<Piece>> files[2] = {
      {dir + "/prefix_blob.bin", pieces(f->blob, 0)}, {dir + "/prefix_offsets.u64", off_pieces}};
  for (const auto& fl : files) {
    std::string m;
    if (!write_pieces(fl.first, fl.second.size(), [&](size_t i, const uint8_t** p, uint64_t* n, uint64_t* off) {
          *p = fl.second[i].p;
          *n = fl.second[i].n;
          *off = fl.second[i].off;
        }, &m)) {
      *msg = "write prefix blob: " + m;
      return S3IMPH_ERR_IO;
    }
  }
  return S3IMPH_OK;
}

int feed_build(Feed* f, std::vector<uint8_t>* mph, const std::function<FeedSink*()>& open_sink, std::string* msg) {
  const uint64_t n = f->n;
  mph->clear();
  if (n == 0) return S3IMPH_OK;
  s3imph_ctx* c = default_ctx(f->device, msg);
  if (!c) return S3IMPH_ERR_HIP;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(f->device));
    feed_flush(f);  // the last partial chunks
    if (!f->dev_on) {
      *msg = "feed prefixes to the GPU: device copy unavailable";
      return S3IMPH_ERR_HIP;
    }
    f->dev_reserve(f->blob, ((f->blob.total + 7) & ~7ull) + 16);  // readable 16 B past the rounded end
    if (n > f->out_cap) {
      for (int a = 0; a < 2; ++a) {
        if (f->d_out[a]) HIPCHECK(hipFree(f->d_out[a]));
        f->d_out[a] = nullptr;
        HIPCHECK(hipMalloc(&f->d_out[a], n * 8));
      }
      f->out_cap = n;
    }
    hipEvent_t fed, built;
    HIPCHECK(hipEventCreateWithFlags(&fed, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&built, hipEventDisableTiming));
    struct EvGuard {
      hipEvent_t a, b;
      ~EvGuard() {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
      }
    } evg{fed, built};
    HIPCHECK(hipEventRecord(fed, f->s));
    hipStream_t s = c->own_stream;
    HIPCHECK(hipStreamWaitEvent(s, fed, 0));
    s3imph_build_info info;
    int rc = retry_on_nomem(c, s, msg, [&] {
      return build_single(c, f->blob.d, reinterpret_cast<const uint64_t*>(f->ends.d),
                          reinterpret_cast<const uint64_t*>(f->pos.d), n, f->d_out[0], f->d_out[1], s, &info, msg);
    });
    if (rc != S3IMPH_OK) return rc;  // nothing was written
    HIPCHECK(hipEventRecord(built, s));
    // the outgrown device buffers: the feed stream is past them (the build waited for it)
    HIPCHECK(hipStreamSynchronize(f->s));
    for (Arena* a : {&f->blob, &f->ends, &f->pos}) {
      for (uint8_t* r : a->retired) HIPCHECK(hipFree(r));
      a->retired.clear();
    }
    FeedSink* sink = open_sink();
    // fp (array 0) and pos (array 1) back through pooled pinned chunks, one thread each:
    // DMA chunk k+1 while the sink takes chunk k
    std::string errs[2];
    bool sink_ok[2] = {true, true};
    auto drain = [&](int a) {
      void* pin[2] = {nullptr, nullptr};
      hipEvent_t ev[2] = {nullptr, nullptr};
      try {
        HIPCHECK(hipSetDevice(f->device));
        for (int b = 0; b < 2; ++b) {
          pin[b] = pool().get(kMaxChunk);
          if (!pin[b]) throw Fail{S3IMPH_ERR_NOMEM, "pinned staging for the output arrays"};
          HIPCHECK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
        }
        hipStream_t os = f->out_s[a];
        HIPCHECK(hipStreamWaitEvent(os, built, 0));
        const uint64_t per = kMaxChunk / 8, nch = (n + per - 1) / per;
        auto issue = [&](uint64_t chn, int b) {
          const uint64_t cnt = std::min(per, n - chn * per);
          HIPCHECK(hipMemcpyAsync(pin[b], f->d_out[a] + chn * per, cnt * 8, hipMemcpyDeviceToHost, os));
          HIPCHECK(hipEventRecord(ev[b], os));
        };
        issue(0, 0);
        for (uint64_t chn = 0; chn < nch; ++chn) {
          const int b = (int)(chn & 1);
          if (chn + 1 < nch) issue(chn + 1, b ^ 1);  // pin[b^1]'s last chunk went to the sink already
          HIPCHECK(hipEventSynchronize(ev[b]));
          if (sink_ok[a] && !sink->put(a, static_cast<const uint64_t*>(pin[b]), std::min(per, n - chn * per)))
            sink_ok[a] = false;  // keep draining the DMA; report the sink's failure after
        }
        HIPCHECK(hipStreamSynchronize(os));
      } catch (const Fail& e) {
        errs[a] = e.msg;
      }
      for (int b = 0; b < 2; ++b) {
        if (ev[b]) (void)hipEventDestroy(ev[b]);
        if (pin[b]) pool().put(pin[b], kMaxChunk);
      }
    };
    std::thread t1(drain, 1);
    drain(0);
    t1.join();
    for (int a = 0; a < 2; ++a)
      if (!errs[a].empty()) throw Fail{S3IMPH_ERR_HIP, errs[a]};
    mph->resize(info.mph_bin_len);
    uint64_t len = 0;
    rc = marshal_locked(c, mph->data(), mph->size(), &len, msg);
    if (rc != S3IMPH_OK) return rc;
    if (!sink_ok[0] || !sink_ok[1]) {
      *msg = sink->error();
      return S3IMPH_ERR_IO;
    }
    return S3IMPH_OK;
  } catch (const Fail& e) {
    *msg = e.msg;
    return e.code;
  }
}

}  // namespace s3imph
