// s3imph_feed.hip — the builder mirror's upstream feed and output emission on one GPU
// (SURVEY §8 rows f3 and f2).
//
// The reference's StreamingMPHFBuilder.Add (mphf_streaming.go:68-97) appends each
// prefix to a temp file and Build reads it back; the keys reach the MPHF only at Build.
// Here Add copies each key into pinned host chunks and, as a chunk fills, DMAs it to
// growing device arrays (blob, offsets, positions) on the feed's stream, so by the time
// the caller calls Build the key set is already in HBM: Build pays for the last partial
// chunk only.  Build then runs the single-GPU pipeline on those arrays and streams
// mph_fp / mph_pos back through pinned chunks, two threads (one per array, as
// writeArraysParallel, mphf_streaming.go:546-596) each handing chunk k to the caller's
// sink (the file writer) while the DMA of chunk k+1 runs.
#include <cstring>
#include <thread>

#include "s3imph_ctx.h"

namespace s3imph {

s3imph_ctx* default_ctx(int device, std::string* msg);

namespace {

constexpr uint64_t kFeedChunk = 8ull << 20;  // pinned chunk (bytes)

// One device array fed through two pinned chunks: bytes are copied into the current
// chunk; a full chunk goes to the device asynchronously and the other chunk is filled
// meanwhile (its previous DMA is waited for first).
struct FedArray {
  uint8_t* d = nullptr;  // device buffer
  uint64_t cap = 0;      // its capacity
  uint64_t sent = 0;     // bytes already handed to the DMA
  uint8_t* pin[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  int cur = 0;
  uint64_t fill = 0;  // bytes in pin[cur]

  void init(uint64_t cap0) {
    for (int b = 0; b < 2; ++b) {
      HIPCHECK(hipHostMalloc(&pin[b], kFeedChunk, hipHostMallocDefault));
      HIPCHECK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
    }
    HIPCHECK(hipMalloc(&d, cap0));
    cap = cap0;
  }
  void release() {
    for (int b = 0; b < 2; ++b) {
      if (ev[b]) (void)hipEventSynchronize(ev[b]);
      if (pin[b]) (void)hipHostFree(pin[b]);
      if (ev[b]) (void)hipEventDestroy(ev[b]);
      pin[b] = nullptr;
      ev[b] = nullptr;
    }
    if (d) (void)hipFree(d);
    d = nullptr;
  }
  // device capacity for `need` bytes: double, copy what was sent, free the old buffer
  void reserve(uint64_t need, hipStream_t s) {
    if (need <= cap) return;
    uint64_t nc = std::max<uint64_t>(2 * cap, need);
    nc = (nc + 4095) & ~4095ull;
    uint8_t* nd = nullptr;
    HIPCHECK(hipMalloc(&nd, nc));
    if (sent) HIPCHECK(hipMemcpyAsync(nd, d, sent, hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    HIPCHECK(hipFree(d));
    d = nd;
    cap = nc;
  }
  void flush(hipStream_t s) {
    if (!fill) return;
    reserve(sent + fill, s);
    HIPCHECK(hipMemcpyAsync(d + sent, pin[cur], fill, hipMemcpyHostToDevice, s));
    HIPCHECK(hipEventRecord(ev[cur], s));
    sent += fill;
    fill = 0;
    cur ^= 1;
    HIPCHECK(hipEventSynchronize(ev[cur]));  // the other chunk's DMA has landed: refill it
  }
  void append(const void* src, uint64_t bytes, hipStream_t s) {
    const uint8_t* p = static_cast<const uint8_t*>(src);
    while (bytes) {
      const uint64_t k = std::min(bytes, kFeedChunk - fill);
      std::memcpy(pin[cur] + fill, p, k);
      fill += k;
      p += k;
      bytes -= k;
      if (fill == kFeedChunk) flush(s);
    }
  }
  uint64_t total() const { return sent + fill; }
};

}  // namespace

struct Feed {
  int device = 0;
  hipStream_t s = nullptr;
  hipStream_t out_s[2] = {nullptr, nullptr};
  FedArray blob, offs, pos;
  uint64_t n = 0;
  uint64_t* d_out[2] = {nullptr, nullptr};  // fp_out, pos_out
  uint64_t out_cap = 0;

  ~Feed() {
    blob.release();
    offs.release();
    pos.release();
    for (int a = 0; a < 2; ++a) {
      if (d_out[a]) (void)hipFree(d_out[a]);
      if (out_s[a]) (void)hipStreamDestroy(out_s[a]);
    }
    if (s) (void)hipStreamDestroy(s);
  }
};

Feed* feed_new(int device, std::string* msg) {
  Feed* f = new Feed();
  try {
    f->device = device;
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(hipStreamCreateWithFlags(&f->s, hipStreamNonBlocking));
    for (int a = 0; a < 2; ++a) HIPCHECK(hipStreamCreateWithFlags(&f->out_s[a], hipStreamNonBlocking));
    f->blob.init(64ull << 20);
    f->offs.init(16ull << 20);
    f->pos.init(16ull << 20);
    const uint64_t zero = 0;  // offsets[0]: the builder's blob starts at 0
    f->offs.append(&zero, 8, f->s);
    return f;
  } catch (const Fail& e) {
    *msg = e.msg;
    delete f;
    return nullptr;
  }
}

void feed_free(Feed* f) {
  if (!f) return;
  (void)hipSetDevice(f->device);
  delete f;
}

int feed_append(Feed* f, const uint8_t* bytes, uint64_t nbytes, const uint64_t* ends, const uint64_t* pos, uint64_t n,
                std::string* msg) {
  try {
    HIPCHECK(hipSetDevice(f->device));
    f->blob.append(bytes, nbytes, f->s);
    f->offs.append(ends, 8 * n, f->s);
    f->pos.append(pos, 8 * n, f->s);
    f->n += n;
    return S3IMPH_OK;
  } catch (const Fail& e) {
    *msg = "feed prefixes to the GPU: " + e.msg;
    return e.code;
  }
}

uint64_t feed_count(const Feed* f) { return f ? f->n : 0; }

int feed_build(Feed* f, std::vector<uint8_t>* mph, FeedSink* sink, std::string* msg) {
  const uint64_t n = f->n;
  mph->clear();
  if (n == 0) return S3IMPH_OK;
  s3imph_ctx* c = default_ctx(f->device, msg);
  if (!c) return S3IMPH_ERR_HIP;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(f->device));
    // the last partial chunks; the blob stays readable 16 bytes past its rounded end
    f->blob.flush(f->s);
    f->offs.flush(f->s);
    f->pos.flush(f->s);
    f->blob.reserve(((f->blob.sent + 7) & ~7ull) + 16, f->s);
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
    int rc = build_single(c, f->blob.d, reinterpret_cast<const uint64_t*>(f->offs.d),
                          reinterpret_cast<const uint64_t*>(f->pos.d), n, f->d_out[0], f->d_out[1], s, &info, msg);
    if (rc != S3IMPH_OK) return rc;
    HIPCHECK(hipEventRecord(built, s));
    // fp (array 0) and pos (array 1) back through the idle pinned chunks of the blob and
    // offsets feeds, one thread each: DMA chunk k+1 while the sink takes chunk k
    std::string errs[2];
    bool sink_ok[2] = {true, true};
    auto drain = [&](int a) {
      try {
        HIPCHECK(hipSetDevice(f->device));
        FedArray& fa = a == 0 ? f->blob : f->offs;
        hipStream_t os = f->out_s[a];
        HIPCHECK(hipStreamWaitEvent(os, built, 0));
        const uint64_t per = kFeedChunk / 8, nch = (n + per - 1) / per;
        auto issue = [&](uint64_t ch, int b) {
          const uint64_t cnt = std::min(per, n - ch * per);
          HIPCHECK(hipMemcpyAsync(fa.pin[b], f->d_out[a] + ch * per, cnt * 8, hipMemcpyDeviceToHost, os));
          HIPCHECK(hipEventRecord(fa.ev[b], os));
        };
        issue(0, 0);
        for (uint64_t ch = 0; ch < nch; ++ch) {
          const int b = (int)(ch & 1);
          if (ch + 1 < nch) issue(ch + 1, b ^ 1);
          HIPCHECK(hipEventSynchronize(fa.ev[b]));
          if (sink_ok[a] && !sink->put(a, reinterpret_cast<const uint64_t*>(fa.pin[b]), std::min(per, n - ch * per)))
            sink_ok[a] = false;  // keep draining the DMA; report the sink's failure after
        }
        HIPCHECK(hipStreamSynchronize(os));
      } catch (const Fail& e) {
        errs[a] = e.msg;
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
