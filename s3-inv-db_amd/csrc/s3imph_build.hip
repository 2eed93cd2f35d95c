// s3imph_build.hip — build orchestration and the device-side C ABI.
//
// Single GPU (s3imph_build_device): one stream, no host synchronisation until the
// very end.  Level sizes live on the device (LevelState); big levels run as
// full-grid kernels gated on the device-resident key count, the geometric tail of
// small levels runs inside one workgroup with LDS bit vectors.
//
// Multi-GPU (s3imph_build_device_dist): one process per GPU, RCCL over xGMI.  Keys
// shard by contiguous index range.  Per level every rank marks its keys into a
// full-size local A/C pair, expands it to one saturating count byte per position,
// RCCL reduce-scatters the bytes (sum), decides "exactly one key here" on its slice,
// and all-gathers the packed final bit vector.  Keys then settle or move to the next
// level locally.  At the end (p, fp, pos) triples go to the rank owning p's range.
//
// Reference: pkg/format/mphf_streaming.go:122-232 (Build), :141 (bbhash.New),
// :176-204 + :237-261 (positions and scatter).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "s3imph.h"
#include "s3imph_internal.h"

using namespace s3imph;

namespace {

struct DistState {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  uint64_t cap_local = 0, cap_global_words = 0, cap_out = 0;
  uint32_t* A = nullptr;          // local seen bits, full level size (u32 words)
  uint32_t* C = nullptr;          // local collided bits
  uint8_t* cnt = nullptr;         // count bytes, full (padded) level size
  uint8_t* sum = nullptr;         // this rank's reduce-scatter slice
  uint64_t* packed = nullptr;     // this rank's packed final bits
  unsigned long long* counters = nullptr;  // [0] local redo count, [1] global, [2..] scratch
  unsigned long long* owner_counts = nullptr;  // nranks
  unsigned long long* count_matrix = nullptr;  // nranks * nranks
  unsigned long long* bucket_fill = nullptr;   // nranks
  unsigned long long* bucket_off = nullptr;    // nranks
  uint64_t* send = nullptr;       // 3 * cap_local
  uint64_t* recv = nullptr;       // 3 * cap_out
  unsigned* status = nullptr;
  unsigned long long* h_pinned = nullptr;      // host staging
};

}  // namespace

struct s3imph_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  std::mutex mu;

  uint64_t cap_keys = 0, cap_words = 0, cap_blocks = 0;
  uint64_t *kh = nullptr, *fp = nullptr, *settle = nullptr, *bits = nullptr, *rank_base = nullptr;
  uint64_t* rkeys[2] = {nullptr, nullptr};   // multi-GPU redo lists
  uint32_t* ridx[2] = {nullptr, nullptr};
  unsigned long long* block_sums = nullptr;
  LevelState* d_st = nullptr;
  LevelState* h_st = nullptr;
  bool rank_valid = false;                   // rank_base matches the last build

  // single-GPU binned pipeline (s3imph_binned.hip)
  Rec* bucket = nullptr;
  Rec* list[2] = {nullptr, nullptr};
  unsigned *hist = nullptr, *hoff = nullptr, *tile_start = nullptr, *scan_sums = nullptr;
  unsigned long long* flags = nullptr;
  unsigned long long* sflags = nullptr;
  unsigned* tcnt = nullptr;  // reservation-path shard fills, kResLevels x kMaxTiles x kResShards
  int tile_mode = 0;
  int tile_block = 1024;
  uint64_t target_tiles = kTargetTiles, target_tiles0 = kTargetTiles0, target_chunks = kTargetChunks;
  uint64_t res_max_keys = kResMaxKeys;
  uint64_t target_tiles_res = kTargetTilesRes;
  bool debug = false;
  unsigned long long* tile_prof = nullptr;  // debug: tile phase timestamps
  bool lds_attr_set = false;

  // staging for host-memory builds
  uint8_t* s_blob = nullptr;
  uint64_t s_blob_cap = 0;
  uint64_t *s_offsets = nullptr, *s_pos = nullptr, *s_fp = nullptr, *s_posout = nullptr;
  uint64_t s_cap = 0;

  bool have_build = false;
  uint64_t last_n = 0;
  s3imph_build_info info{};

  bool profiling = false;
  std::vector<hipEvent_t> events;
  std::vector<std::string> ev_names;
  int ev_used = 0;
  std::vector<float> stage_ms;
  std::vector<std::string> stage_names;

  bool dist = false;
  DistState d;
};

namespace {

constexpr uint64_t kU32Limit = 0xffffffffull;

const char* status_name(int s) {
  switch (s) {
    case S3IMPH_OK: return "ok";
    case S3IMPH_ERR_INVALID: return "invalid argument";
    case S3IMPH_ERR_DUP_KEY_HASH: return "duplicate key hashes: bbhash cannot place them";
    case S3IMPH_ERR_TOO_MANY_LEVELS: return "can't find minimal perfect hash within the level budget";
    case S3IMPH_ERR_KEY_HASH_ZERO: return "a key hash is 0 (ambiguous with the reverse-map sentinel)";
    case S3IMPH_ERR_HIP: return "HIP error";
    case S3IMPH_ERR_RCCL: return "RCCL error";
    case S3IMPH_ERR_IO: return "I/O error";
    case S3IMPH_ERR_NOMEM: return "out of memory";
    case S3IMPH_ERR_FORMAT: return "bad format";
    case S3IMPH_ERR_INTERNAL: return "internal error";
    case S3IMPH_ERR_STATE: return "invalid state";
    default: return "unknown status";
  }
}

struct Fail {
  int code;
  std::string msg;
};

#define HIPCHECK(x)                                                                           \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
      throw Fail{e_ == hipErrorOutOfMemory ? S3IMPH_ERR_NOMEM : S3IMPH_ERR_HIP,               \
                 std::string(#x) + ": " + hipGetErrorString(e_)};                             \
  } while (0)

#define NCCLCHECK(x)                                                                          \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess)                                                                    \
      throw Fail{S3IMPH_ERR_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_)};           \
  } while (0)

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <typename T>
void dalloc(T*& p, uint64_t count) {
  dfree(p);
  void* v = nullptr;
  HIPCHECK(hipMalloc(&v, std::max<uint64_t>(count, 1) * sizeof(T)));
  p = static_cast<T*>(v);
}

uint64_t cap_words_for(uint64_t n) {
  // Sum over levels of ceil(n_L/32): n_L ~ n*0.3935^L so sum ~ 1.65n/32; allow 2.5n/32.
  return (n * 5) / 64 + 4 * (uint64_t)kMaxLevels + 64;
}

void alloc_common(s3imph_ctx* c, uint64_t n_global) {
  c->cap_words = cap_words_for(std::max<uint64_t>(n_global, 1024));
  if (!c->d_st) dalloc(c->d_st, 1);
  if (!c->h_st) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, sizeof(LevelState), hipHostMallocDefault));
    c->h_st = static_cast<LevelState*>(h);
  }
}

// Single-GPU workspace: ~88 B per key (level-0 list, tile buckets, two next-level lists).
void ensure_workspace(s3imph_ctx* c, uint64_t n) {
  if (n <= c->cap_keys && c->hist) return;
  const uint64_t cap = std::max<uint64_t>(n, 1024);
  dalloc(c->kh, cap);
  dalloc(c->fp, cap);
  dalloc(c->bucket, cap);
  dalloc(c->list[0], cap);
  dalloc(c->list[1], cap);
  dalloc(c->hist, kHistCap);
  dalloc(c->hoff, kHistCap);
  dalloc(c->tile_start, kMaxTiles + 2);
  dalloc(c->scan_sums, kHistCap / 2048 + 2);
  dalloc(c->flags, kMaxTiles + 2);
  dalloc(c->sflags, kHistCap / kScanSeg + 2);
  dalloc(c->tcnt, (uint64_t)kResLevels * kMaxTiles * kResShards);
  alloc_common(c, cap);
  dalloc(c->bits, c->cap_words);
  dalloc(c->rank_base, c->cap_words);
  c->cap_blocks = (c->cap_words + 2047) / 2048 + 1;
  dalloc(c->block_sums, c->cap_blocks);
  c->cap_keys = cap;
}

void free_workspace(s3imph_ctx* c) {
  dfree(c->kh); dfree(c->fp); dfree(c->settle); dfree(c->bits); dfree(c->rank_base);
  dfree(c->rkeys[0]); dfree(c->rkeys[1]); dfree(c->ridx[0]); dfree(c->ridx[1]);
  dfree(c->block_sums); dfree(c->d_st);
  dfree(c->bucket); dfree(c->list[0]); dfree(c->list[1]);
  dfree(c->tcnt);
  dfree(c->tile_prof);
  dfree(c->hist); dfree(c->hoff); dfree(c->tile_start); dfree(c->scan_sums); dfree(c->flags); dfree(c->sflags);
  if (c->h_st) (void)hipHostFree(c->h_st);
  c->h_st = nullptr;
  dfree(c->s_blob); dfree(c->s_offsets); dfree(c->s_pos); dfree(c->s_fp); dfree(c->s_posout);
  DistState& d = c->d;
  dfree(d.A); dfree(d.C); dfree(d.cnt); dfree(d.sum); dfree(d.packed); dfree(d.counters);
  dfree(d.owner_counts); dfree(d.count_matrix); dfree(d.bucket_fill); dfree(d.bucket_off);
  dfree(d.send); dfree(d.recv); dfree(d.status);
  if (d.h_pinned) (void)hipHostFree(d.h_pinned);
  d.h_pinned = nullptr;
  for (auto e : c->events) (void)hipEventDestroy(e);
  c->events.clear();
  c->cap_keys = 0;
}

// ---- stage timing (HIP events on the build stream) -------------------------------
void ev_begin(s3imph_ctx* c) {
  c->ev_used = 0;
  c->ev_names.clear();
}
void ev_mark(s3imph_ctx* c, hipStream_t s, const char* name) {
  if (!c->profiling) return;
  if (c->ev_used >= (int)c->events.size()) {
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    c->events.push_back(e);
  }
  HIPCHECK(hipEventRecord(c->events[c->ev_used++], s));
  c->ev_names.push_back(name);
}
void ev_collect(s3imph_ctx* c) {
  c->stage_ms.clear();
  c->stage_names.clear();
  if (!c->profiling) return;
  for (int i = 1; i < c->ev_used; ++i) {
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, c->events[i - 1], c->events[i]));
    c->stage_ms.push_back(ms);
    c->stage_names.push_back(c->ev_names[i]);
  }
}

int predict_big_levels(uint64_t n) {
  // Expected keys entering level L: n * (1 - e^{-1/2})^L for gamma = 2.
  const double q = 1.0 - std::exp(-0.5);
  double m = (double)n * q;
  int big = 0;
  while (m > 0.9 * (double)kTailKeys && big < kMaxLevels - 2) {
    ++big;
    m *= q;
  }
  return std::min(big + 1, kMaxLevels - 2);
}

bool has_duplicates(const uint64_t* d_keys, uint64_t n) {
  std::vector<uint64_t> h(n);
  if (n) HIPCHECK(hipMemcpy(h.data(), d_keys, n * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  return std::adjacent_find(h.begin(), h.end()) != h.end();
}

int map_status(s3imph_ctx* c, unsigned flags, uint64_t n, std::string* msg) {
  if (flags & (kStTooManyLevels | kStOverflow)) {
    if (has_duplicates(c->kh, n)) {
      *msg = "build MPHF: duplicate FNV-1a key hashes: bbhash cannot place them";
      return S3IMPH_ERR_DUP_KEY_HASH;
    }
    *msg = (flags & kStTooManyLevels) ? "build MPHF: can't find minimal perfect hash after " +
                                            std::to_string(kMaxLevels) + " levels"
                                      : "build MPHF: workspace overflow";
    return (flags & kStTooManyLevels) ? S3IMPH_ERR_TOO_MANY_LEVELS : S3IMPH_ERR_INTERNAL;
  }
  if (flags & kStKeyZero) {
    *msg = "MPHF Key(...) returned 0, possible hash collision with sentinel";
    return S3IMPH_ERR_KEY_HASH_ZERO;
  }
  if (flags) {
    *msg = "build MPHF: internal error (device flags " + std::to_string(flags) + ")";
    return S3IMPH_ERR_INTERNAL;
  }
  return S3IMPH_OK;
}

// Enqueue one attempt of the binned pipeline.  `conservative` sizes every level with
// the level-0 geometry (always inside the workspace bounds) and runs every level that
// is still big as a full-grid level; the default predicts each level's size.
void enqueue_binned(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                    uint64_t n, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s, bool conservative) {
  BinBuffers b{};
  b.kh = c->kh;
  b.fp = c->fp;
  b.pos = pos;
  b.pos_base = 0;
  b.bucket = c->bucket;
  b.list[0] = c->list[0];
  b.list[1] = c->list[1];
  b.hist = c->hist;
  b.off = c->hoff;
  b.tile_start = c->tile_start;
  b.scan_sums = c->scan_sums;
  b.flags = c->flags;
  b.sflags = c->sflags;
  b.tcnt = c->tcnt;
  b.bucket_cap = c->cap_keys;
  b.tile_mode = c->tile_mode;
  b.tile_block = c->tile_block;
  b.tile_prof = nullptr;
  if (c->debug) {
    const size_t nprof = (size_t)kMaxLevels * kMaxTiles * 8;
    if (!c->tile_prof) HIPCHECK(hipMalloc(&c->tile_prof, nprof * sizeof(unsigned long long)));
    HIPCHECK(hipMemsetAsync(c->tile_prof, 0, nprof * sizeof(unsigned long long), s));
    b.tile_prof = c->tile_prof;
  }
  b.bits = c->bits;
  b.cap_words = c->cap_words;
  b.fp_out = fp_out;
  b.pos_out = pos_out;
  b.st = c->d_st;

  const double q = 1.0 - std::exp(-0.5);  // fraction of keys that collide at load 1/2
  const LevelGeom g0 = choose_geom(n, c->target_tiles0, c->target_chunks, kRegTileMaxBits);
  int gc, gt, gs;
  // Grids from a (predicted) key count; kernels loop over whatever the device finds.
  auto grids = [&](uint64_t nk, LevelGeom g) {
    const uint64_t T = (64 * level_words(nk ? nk : 1) + (1ull << g.tb) - 1) >> g.tb;
    const uint64_t B = std::max<uint64_t>((nk + g.chunk - 1) / g.chunk, 1);
    gc = (int)std::min<uint64_t>(B, 2048);
    gt = (int)std::min<uint64_t>(std::max<uint64_t>(T, 1), 2048);
    gs = (int)std::min<uint64_t>((T * B + kScanSeg - 1) / kScanSeg + 2, 256);
  };
  launch_init_state(c->d_st, n, 0, s);
  ev_mark(c, s, "init");
  grids(n, g0);
  launch_binned_count(0, blob, offsets, n, b, g0, gc, s);
  ev_mark(c, s, "hash_count0");
  launch_binned_scan(0, b, gs, s);
  ev_mark(c, s, "hscan0");
  launch_binned_scatter(0, b, g0, s);
  ev_mark(c, s, "scatter0");
  launch_binned_tile(0, b, g0, gt, s);
  ev_mark(c, s, "tile0");
  const int big = conservative ? kMaxLevels - 2 : predict_big_levels(n);
  int launched = 0;
  for (int L = 1; L <= big; ++L) {
    // Level sizes concentrate tightly around n q^L; a level predicted within 1/kTailMargin
    // of the tail's capacity is left to the tail (an unexpectedly large one is caught by
    // kStTailOverflow and rerun conservatively).
    const double pred = (double)n * std::pow(q, L);
    if (!conservative && pred * kTailMargin < (double)kTailKeys) break;
    launched = L;
    const uint64_t nb = conservative ? n : (uint64_t)(pred * 1.1) + 4096;
    const bool res = !conservative && nb <= c->res_max_keys && L < kResLevels && c->tile_mode == 0;
    const LevelGeom g = conservative ? g0
                        : res        ? choose_geom(nb, c->target_tiles_res, c->target_chunks, kRegTileMaxBits)
                                     : choose_geom(nb, c->target_tiles, c->target_chunks, kRegTileMaxBits);
    grids(nb, g);
    if (res && g.tb <= kRegTileMaxBits) {
      const int gr = (int)std::min<uint64_t>((nb + kSubRound - 1) / kSubRound, 256);
      launch_binned_scatter_res(L, b, g, gr, s);
      launch_binned_tile(L, b, g, gt, s, true);
    } else {
      launch_binned_count(L, nullptr, nullptr, 0, b, g, gc, s);
      launch_binned_scan(L, b, gs, s);
      launch_binned_scatter(L, b, g, s);
      launch_binned_tile(L, b, g, gt, s);
    }
  }
  ev_mark(c, s, "levels");
  launch_binned_tail(launched, b, s);
  ev_mark(c, s, "tail");
}

void set_lds_attrs(s3imph_ctx* c) {
  if (c->lds_attr_set) return;
  // The tile kernels take up to 2 x 64 KiB of dynamic LDS (tiles of 2^19 positions).
  binned_set_lds_limits();
  c->lds_attr_set = true;
}

// Debug: per-level averages of the tile kernel's phase durations (wall clock, 100 MHz).
void print_tile_profile(s3imph_ctx* c) {
  if (!c->tile_prof) return;
  std::vector<unsigned long long> h((size_t)kMaxLevels * kMaxTiles * 8);
  HIPCHECK(hipMemcpy(h.data(), c->tile_prof, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  static const char* names[7] = {"mark", "final", "lookbk", "rank", "output", "redoN", "redoW"};
  {
    const unsigned long long* tl = &h[(size_t)(kMaxLevels - 1) * kMaxTiles * 8];
    std::fprintf(stderr, "  tail level starts (us from first):");
    unsigned long long t0 = 0;
    for (int L = 0; L < kMaxLevels; ++L) {
      if (!tl[L]) continue;
      if (!t0) t0 = tl[L];
      std::fprintf(stderr, " L%d@%.1f", L, (tl[L] - t0) / 100.0);
    }
    std::fprintf(stderr, "\n");
  }
  for (int L = 0; L < kMaxLevels - 1; ++L) {
    double sum[7] = {0};
    unsigned long long lo = ~0ull, hi = 0;
    int cnt = 0;
    for (int t = 0; t < kMaxTiles; ++t) {
      const unsigned long long* p = &h[((size_t)L * kMaxTiles + t) * 8];
      if (!p[0] || !p[7]) continue;
      ++cnt;
      lo = std::min(lo, p[0]);
      hi = std::max(hi, p[7]);
      unsigned long long prev = p[0];
      for (int i = 1; i < 8; ++i) {
        const unsigned long long v = p[i] ? p[i] : prev;
        sum[i - 1] += (double)(v - prev);
        prev = v;
      }
    }
    if (!cnt) continue;
    static const char* snames[7] = {"count", "resv", "stage", "write", "-", "-", "-"};
    const bool sc = L >= 32;
    std::fprintf(stderr, "  %s L%d: %d %s, span %.1f us, avg us:", sc ? "scatter_res" : "tile", sc ? L - 32 : L, cnt,
                 sc ? "blocks (round 0)" : "tiles", (hi - lo) / 100.0);
    for (int i = 0; i < (sc ? 4 : 7); ++i) std::fprintf(stderr, " %s %.2f", (sc ? snames : names)[i], sum[i] / cnt / 100.0);
    std::fprintf(stderr, "\n");
  }
}

int build_single(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                 uint64_t n, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s,
                 s3imph_build_info* info, std::string* msg) {
  c->have_build = false;
  c->rank_valid = false;
  *info = s3imph_build_info{};
  info->n_keys = n;
  if (n == 0) {
    c->have_build = true;
    c->last_n = 0;
    c->info = *info;
    return S3IMPH_OK;
  }
  if (n > kU32Limit) {
    *msg = "build MPHF: more than 2^32-1 keys on one GPU";
    return S3IMPH_ERR_INVALID;
  }
  ensure_workspace(c, n);
  set_lds_attrs(c);
  for (int attempt = 0; attempt < 2; ++attempt) {
    ev_begin(c);
    ev_mark(c, s, "start");
    enqueue_binned(c, blob, offsets, pos, n, fp_out, pos_out, s, attempt > 0);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(c->h_st, c->d_st, sizeof(LevelState), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    ev_collect(c);
    if (c->debug) {
      const LevelState& d = *c->h_st;
      std::fprintf(stderr, "[s3imph] attempt %d: status 0x%x nlevels %u tail_first %u rank_total %llu\n  n:", attempt,
                   d.status, d.nlevels, d.tail_first, (unsigned long long)d.rank_total);
      for (int L = 0; L <= (int)d.nlevels + 1 && L < kMaxLevels; ++L)
        std::fprintf(stderr, " %llu", (unsigned long long)d.n[L]);
      std::fprintf(stderr, "\n  T:");
      for (int L = 0; L <= (int)d.nlevels + 1 && L < kMaxLevels; ++L)
        std::fprintf(stderr, " %llu", (unsigned long long)d.ntiles[L]);
      std::fprintf(stderr, "\n");
      print_tile_profile(c);
    }
    // Geometry/tail-capacity misses only mean the level-size prediction was off:
    // rerun with workspace-safe geometry (same bytes, slower schedule).
    if (c->h_st->status & (kStGeometry | kStTailOverflow | kStResOverflow)) continue;
    break;
  }
  const LevelState& st = *c->h_st;
  int rc = map_status(c, st.status, n, msg);
  if (rc != S3IMPH_OK) return rc;
  if (st.rank_total != n || st.nlevels == 0) {
    *msg = "build MPHF: internal error: ranked " + std::to_string(st.rank_total) + " of " +
           std::to_string(n) + " keys";
    return S3IMPH_ERR_INTERNAL;
  }
  info->status = S3IMPH_OK;
  info->num_levels = st.nlevels;
  info->total_words = st.woff[st.nlevels];
  info->mph_bin_len = 8 * kPartitions + 8 + 8ull * st.nlevels + 8ull * info->total_words;
  info->big_levels = st.tail_first ? st.tail_first : st.nlevels;
  c->have_build = true;
  c->last_n = n;
  c->info = *info;
  return S3IMPH_OK;
}

// -------------------------------------------------------------------- distributed ----
void ensure_dist_workspace(s3imph_ctx* c, uint64_t n_local, uint64_t n_global) {
  DistState& d = c->d;
  const int P = d.nranks;
  const uint64_t per_rank = (n_global + P - 1) / P;
  if (n_local <= d.cap_local && level_words(n_global) <= d.cap_global_words && per_rank <= d.cap_out &&
      c->d_st)
    return;
  const uint64_t capl = std::max<uint64_t>(n_local, 1024);
  const uint64_t w0 = level_words(std::max<uint64_t>(n_global, 1024));
  const uint64_t pos_pad = ((64 * w0 + 64ull * P - 1) / (64ull * P)) * (64ull * P);
  dalloc(c->kh, capl);
  dalloc(c->fp, capl);
  dalloc(c->settle, capl);
  dalloc(c->rkeys[0], capl);
  dalloc(c->rkeys[1], capl);
  dalloc(c->ridx[0], capl);
  dalloc(c->ridx[1], capl);
  c->cap_keys = capl;
  c->cap_words = cap_words_for(std::max<uint64_t>(n_global, 1024)) + (pos_pad / 64);
  dalloc(c->bits, c->cap_words);
  dalloc(c->rank_base, c->cap_words);
  c->cap_blocks = (c->cap_words + 2047) / 2048 + 1;
  dalloc(c->block_sums, c->cap_blocks);
  if (!c->d_st) dalloc(c->d_st, 1);
  if (!c->h_st) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, sizeof(LevelState), hipHostMallocDefault));
    c->h_st = static_cast<LevelState*>(h);
  }
  dalloc(d.A, pos_pad / 32);
  dalloc(d.C, pos_pad / 32);
  dalloc(d.cnt, pos_pad);
  dalloc(d.sum, pos_pad / P);
  dalloc(d.packed, pos_pad / P / 64 + 1);
  dalloc(d.counters, 8);
  dalloc(d.owner_counts, P);
  dalloc(d.count_matrix, (uint64_t)P * P);
  dalloc(d.bucket_fill, P);
  dalloc(d.bucket_off, P);
  const uint64_t per = std::max<uint64_t>(per_rank, 1024);
  dalloc(d.send, 3 * capl);
  dalloc(d.recv, 3 * per);
  dalloc(d.status, 1);
  if (!d.h_pinned) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, sizeof(unsigned long long) * (4 + 2 * 64 * 64), hipHostMallocDefault));
    d.h_pinned = static_cast<unsigned long long*>(h);
  }
  HIPCHECK(hipMemset(d.A, 0, pos_pad / 32 * 4));
  HIPCHECK(hipMemset(d.C, 0, pos_pad / 32 * 4));
  d.cap_local = capl;
  d.cap_global_words = w0;
  d.cap_out = per;
}

uint64_t allreduce_sum_u64(s3imph_ctx* c, unsigned long long* dbuf, uint64_t v, hipStream_t s) {
  DistState& d = c->d;
  d.h_pinned[0] = v;
  HIPCHECK(hipMemcpyAsync(dbuf, d.h_pinned, 8, hipMemcpyHostToDevice, s));
  NCCLCHECK(ncclAllReduce(dbuf, dbuf, 1, ncclUint64, ncclSum, d.comm, s));
  HIPCHECK(hipMemcpyAsync(d.h_pinned, dbuf, 8, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  return d.h_pinned[0];
}

int build_dist(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
               uint64_t n_local, uint64_t key_base, uint64_t* fp_out, uint64_t* pos_out,
               uint64_t out_cap, uint64_t* out_lo, uint64_t* out_n, hipStream_t s,
               s3imph_build_info* info, std::string* msg) {
  DistState& d = c->d;
  const int P = d.nranks, R = d.rank;
  c->have_build = false;
  c->rank_valid = false;
  *info = s3imph_build_info{};
  if (n_local > kU32Limit) {
    *msg = "build MPHF: more than 2^32-1 keys on one rank";
    return S3IMPH_ERR_INVALID;
  }
  ev_begin(c);
  ev_mark(c, s, "start");
  // Global key count (also a rendezvous: every rank must reach the same build).
  if (!d.counters) dalloc(d.counters, 8);
  if (!d.h_pinned) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, sizeof(unsigned long long) * (4 + 2 * 64 * 64), hipHostMallocDefault));
    d.h_pinned = static_cast<unsigned long long*>(h);
  }
  const uint64_t N = allreduce_sum_u64(c, d.counters + 2, n_local, s);
  info->n_keys = N;
  const uint64_t per_rank = (N + P - 1) / P;
  *out_lo = std::min<uint64_t>((uint64_t)R * per_rank, N);
  *out_n = std::min<uint64_t>(per_rank, N - *out_lo);
  if (N == 0) {
    c->have_build = true;
    c->last_n = 0;
    c->info = *info;
    return S3IMPH_OK;
  }
  if (*out_n > out_cap) {
    *msg = "build MPHF: output slice capacity too small";
    return S3IMPH_ERR_INVALID;
  }
  ensure_dist_workspace(c, n_local, N);
  HIPCHECK(hipMemsetAsync(d.status, 0, 4, s));
  HIPCHECK(hipMemsetAsync(c->bits, 0, c->cap_words * 8, s));
  LevelState& hs = *c->h_st;
  std::memset(&hs, 0, sizeof(LevelState));
  const int grid = default_grid(std::max<uint64_t>(n_local, 1), 256);

  uint64_t nL = N, nloc = n_local, woff = 0;
  int L = 0;
  ev_mark(c, s, "init");
  for (;;) {
    if (L >= kMaxLevels) {
      *msg = "build MPHF: can't find minimal perfect hash after " + std::to_string(kMaxLevels) + " levels";
      return S3IMPH_ERR_TOO_MANY_LEVELS;
    }
    const uint64_t words = level_words(nL);
    const uint64_t positions = 64 * words;
    const uint64_t pos_pad = ((positions + 64ull * P - 1) / (64ull * P)) * (64ull * P);
    const uint64_t S = pos_pad / P;
    if (woff + pos_pad / 64 > c->cap_words) {
      *msg = "build MPHF: workspace overflow";
      return S3IMPH_ERR_INTERNAL;
    }
    hs.n[L] = nL;
    hs.words[L] = words;
    hs.woff[L] = woff;
    hs.magic[L] = level_magic(words);
    const uint64_t* kin = (L == 0) ? c->kh : c->rkeys[(L - 1) & 1];
    const uint32_t* iin = (L == 0) ? nullptr : c->ridx[(L - 1) & 1];
    if (L == 0)
      launch_dist_hash_mark0(blob, offsets, nloc, c->kh, c->fp, words, d.A, d.C, d.status, grid, s);
    else if (nloc)
      launch_dist_mark(L, kin, nloc, words, d.A, d.C, default_grid(nloc, 256), s);
    launch_dist_counts(d.A, d.C, pos_pad, d.cnt, default_grid(pos_pad / 32, 256), s);
    NCCLCHECK(ncclReduceScatter(d.cnt, d.sum, S, ncclUint8, ncclSum, d.comm, s));
    launch_dist_pack(d.sum, S, d.packed, default_grid(S / 64, 256), s);
    NCCLCHECK(ncclAllGather(d.packed, c->bits + woff, S / 64, ncclUint64, d.comm, s));
    HIPCHECK(hipMemsetAsync(d.counters, 0, 8, s));
    if (nloc)
      launch_dist_resolve(L, kin, iin, nloc, words, woff, c->bits, c->rkeys[L & 1], c->ridx[L & 1],
                          d.counters, c->settle, default_grid(nloc, 256), s);
    NCCLCHECK(ncclAllReduce(d.counters, d.counters + 1, 1, ncclUint64, ncclSum, d.comm, s));
    HIPCHECK(hipMemcpyAsync(d.h_pinned, d.counters, 16, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    nloc = d.h_pinned[0];
    const uint64_t next = d.h_pinned[1];
    woff += words;
    ++L;
    if (L == 1) ev_mark(c, s, "level0");
    if (next == 0) break;
    if (next >= nL && nL <= 64) {
      // no progress on a tiny remainder: keep going until the level budget says stop
    }
    nL = next;
  }
  ev_mark(c, s, "levels");
  hs.nlevels = L;
  hs.woff[L] = woff;
  // Ranks over all level words (identical on every rank).
  d.h_pinned[2] = woff;
  HIPCHECK(hipMemcpyAsync(d.counters + 4, d.h_pinned + 2, 8, hipMemcpyHostToDevice, s));
  launch_words_scan(c->bits, woff, c->rank_base, c->block_sums, d.counters + 4, s);
  c->rank_valid = true;
  ev_mark(c, s, "rank_scan");

  // Output exchange: (p, fp, pos) to the owner of p's range.
  HIPCHECK(hipMemsetAsync(d.owner_counts, 0, 8 * P, s));
  HIPCHECK(hipMemsetAsync(d.bucket_fill, 0, 8 * P, s));
  if (n_local)
    launch_dist_count_owners(n_local, c->settle, c->bits, c->rank_base, per_rank, P, d.owner_counts,
                             grid, s);
  NCCLCHECK(ncclAllGather(d.owner_counts, d.count_matrix, P, ncclUint64, d.comm, s));
  HIPCHECK(hipMemcpyAsync(d.h_pinned + 8, d.count_matrix, 8ull * P * P, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(d.h_pinned + 3, d.counters + 5, 8, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  const unsigned long long* M = d.h_pinned + 8;  // M[src * P + dst]
  if (d.h_pinned[3] != N) {
    *msg = "build MPHF: internal error: ranked " + std::to_string(d.h_pinned[3]) + " of " + std::to_string(N);
    return S3IMPH_ERR_INTERNAL;
  }
  std::vector<unsigned long long> soff(P), roff(P);
  uint64_t acc = 0, racc = 0;
  for (int q = 0; q < P; ++q) {
    soff[q] = acc;
    acc += M[(uint64_t)R * P + q];
    roff[q] = racc;
    racc += M[(uint64_t)q * P + R];
  }
  if (racc != *out_n) {
    *msg = "build MPHF: internal error: received " + std::to_string(racc) + " of " + std::to_string(*out_n);
    return S3IMPH_ERR_INTERNAL;
  }
  std::memcpy(d.h_pinned + 8 + (uint64_t)P * P, soff.data(), 8 * P);
  HIPCHECK(hipMemcpyAsync(d.bucket_off, d.h_pinned + 8 + (uint64_t)P * P, 8 * P, hipMemcpyHostToDevice, s));
  if (n_local)
    launch_dist_place(n_local, c->settle, c->fp, pos, key_base, c->bits, c->rank_base, per_rank, P,
                      d.bucket_fill, d.bucket_off, d.send, d.status, grid, s);
  NCCLCHECK(ncclGroupStart());
  for (int q = 0; q < P; ++q) {
    const uint64_t sc = M[(uint64_t)R * P + q], rc = M[(uint64_t)q * P + R];
    if (sc) NCCLCHECK(ncclSend(d.send + 3 * soff[q], 3 * sc, ncclUint64, q, d.comm, s));
    if (rc) NCCLCHECK(ncclRecv(d.recv + 3 * roff[q], 3 * rc, ncclUint64, q, d.comm, s));
  }
  NCCLCHECK(ncclGroupEnd());
  if (racc)
    launch_dist_unpack(d.recv, racc, *out_lo, *out_n, fp_out, pos_out, d.status,
                       default_grid(racc, 256), s);
  ev_mark(c, s, "exchange");
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpyAsync(d.h_pinned + 4, d.status, 4, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(c->d_st, c->h_st, sizeof(LevelState), hipMemcpyHostToDevice, s));
  HIPCHECK(hipStreamSynchronize(s));
  ev_collect(c);
  const unsigned flags = (unsigned)(d.h_pinned[4] & 0xffffffffu);
  if (flags & kStKeyZero) {
    *msg = "MPHF Key(...) returned 0, possible hash collision with sentinel";
    return S3IMPH_ERR_KEY_HASH_ZERO;
  }
  if (flags) {
    *msg = "build MPHF: internal error flags " + std::to_string(flags);
    return S3IMPH_ERR_INTERNAL;
  }
  info->status = S3IMPH_OK;
  info->num_levels = L;
  info->total_words = woff;
  info->mph_bin_len = 8 * kPartitions + 8 + 8ull * L + 8ull * woff;
  info->big_levels = L;
  c->have_build = true;
  c->last_n = N;
  c->info = *info;
  return S3IMPH_OK;
}

s3imph_ctx* g_default[64] = {nullptr};
std::mutex g_default_mu;

}  // namespace

namespace s3imph {
int marshal_locked(s3imph_ctx* c, uint8_t* out, uint64_t cap, uint64_t* len, std::string* msg);

s3imph_ctx* default_ctx(int device, std::string* msg) {
  if (device < 0 || device >= 64) {
    *msg = "invalid device";
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (!g_default[device]) {
    s3imph_ctx* c = nullptr;
    char err[256] = {0};
    if (s3imph_ctx_create(device, &c, err, sizeof err) != S3IMPH_OK) {
      *msg = err;
      return nullptr;
    }
    g_default[device] = c;
  }
  return g_default[device];
}

// Host-memory build through the device path (used by s3imph_build_host and the builder).
int build_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                    uint64_t n, uint64_t* fp_out, uint64_t* pos_out, std::vector<uint8_t>* mph,
                    std::string* msg) {
  s3imph_ctx* c = default_ctx(device, msg);
  if (!c) return S3IMPH_ERR_HIP;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(c->device));
    mph->clear();
    if (n == 0) return S3IMPH_OK;
    const uint64_t b0 = offsets[0], nbytes = offsets[n] - offsets[0];
    const uint64_t bcap = ((nbytes + 7) & ~7ull) + 8;
    if (bcap > c->s_blob_cap) {
      dalloc(c->s_blob, bcap);
      c->s_blob_cap = bcap;
    }
    if (n > c->s_cap) {
      dalloc(c->s_offsets, n + 1);
      dalloc(c->s_pos, n);
      dalloc(c->s_fp, n);
      dalloc(c->s_posout, n);
      c->s_cap = n;
    }
    hipStream_t s = c->own_stream;
    std::vector<uint64_t> rel;
    const uint64_t* offs = offsets;
    if (b0 != 0) {
      rel.resize(n + 1);
      for (uint64_t i = 0; i <= n; ++i) rel[i] = offsets[i] - b0;
      offs = rel.data();
    }
    if (nbytes) HIPCHECK(hipMemcpyAsync(c->s_blob, blob + b0, nbytes, hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemcpyAsync(c->s_offsets, offs, (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (pos) HIPCHECK(hipMemcpyAsync(c->s_pos, pos, n * 8, hipMemcpyHostToDevice, s));
    s3imph_build_info info;
    int rc = build_single(c, c->s_blob, c->s_offsets, pos ? c->s_pos : nullptr, n, c->s_fp, c->s_posout, s,
                          &info, msg);
    if (rc != S3IMPH_OK) return rc;
    HIPCHECK(hipMemcpyAsync(fp_out, c->s_fp, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(pos_out, c->s_posout, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    mph->resize(info.mph_bin_len);
    uint64_t len = 0;
    // ctx mutex already held: marshal inline.
    return marshal_locked(c, mph->data(), mph->size(), &len, msg);
  } catch (const Fail& f) {
    *msg = f.msg;
    return f.code;
  } catch (const std::bad_alloc&) {
    *msg = "out of host memory";
    return S3IMPH_ERR_NOMEM;
  }
}

int marshal_locked(s3imph_ctx* c, uint8_t* out, uint64_t cap, uint64_t* len, std::string* msg) {
  if (!c->have_build) {
    *msg = "no completed build";
    return S3IMPH_ERR_STATE;
  }
  if (c->last_n == 0) {
    *len = 0;
    return S3IMPH_OK;
  }
  const LevelState& st = *c->h_st;
  const uint64_t need = c->info.mph_bin_len;
  *len = need;
  if (cap < need) {
    *msg = "buffer too small";
    return S3IMPH_ERR_INVALID;
  }
  std::vector<uint64_t> words(c->info.total_words);
  HIPCHECK(hipMemcpy(words.data(), c->bits, words.size() * 8, hipMemcpyDeviceToHost));
  uint8_t* p = out;
  auto put = [&](uint64_t v) {
    for (int b = 0; b < 8; ++b) *p++ = (uint8_t)(v >> (8 * b));
  };
  put(kPartitions);
  put(st.nlevels);
  for (unsigned L = 0; L < st.nlevels; ++L) {
    put(st.words[L]);
    const uint64_t* w = words.data() + st.woff[L];
    for (uint64_t k = 0; k < st.words[L]; ++k) put(w[k]);
  }
  return S3IMPH_OK;
}
}  // namespace s3imph

// ===================================================================== C ABI ====
extern "C" {

int s3imph_abi_version(void) { return S3IMPH_ABI_VERSION; }

const char* s3imph_status_string(int status) { return status_name(status); }

int s3imph_ctx_create(int device, s3imph_ctx** out, char* err, size_t errlen) {
  if (!out) return S3IMPH_ERR_INVALID;
  *out = nullptr;
  s3imph_ctx* c = nullptr;
  try {
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw Fail{S3IMPH_ERR_INVALID, "no such HIP device " + std::to_string(device)};
    HIPCHECK(hipSetDevice(device));
    c = new s3imph_ctx();
    c->device = device;
    if (const char* m = std::getenv("S3IMPH_TILE_MODE")) c->tile_mode = std::atoi(m);  // A/B knobs
    if (const char* m = std::getenv("S3IMPH_TARGET_TILES")) c->target_tiles = std::strtoull(m, nullptr, 10);
    if (const char* m = std::getenv("S3IMPH_TARGET_TILES0")) c->target_tiles0 = std::strtoull(m, nullptr, 10);
    if (const char* m = std::getenv("S3IMPH_CHUNKS")) c->target_chunks = std::strtoull(m, nullptr, 10);
    if (const char* m = std::getenv("S3IMPH_RES_MAX")) c->res_max_keys = std::strtoull(m, nullptr, 10);
    if (const char* m = std::getenv("S3IMPH_TARGET_TILES_RES")) c->target_tiles_res = std::strtoull(m, nullptr, 10);
    c->debug = std::getenv("S3IMPH_DEBUG") != nullptr;
    if (const char* m = std::getenv("S3IMPH_TILE_BLOCK")) c->tile_block = std::atoi(m);
    // A blocking stream: implicitly ordered with the legacy NULL stream, so work a
    // caller queued there (e.g. torch's default stream) completes before ours starts.
    HIPCHECK(hipStreamCreate(&c->own_stream));
    *out = c;
    return S3IMPH_OK;
  } catch (const Fail& f) {
    delete c;
    set_err(err, errlen, f.msg);
    return f.code;
  } catch (const std::bad_alloc&) {
    delete c;
    set_err(err, errlen, "out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_ctx_destroy(s3imph_ctx* c) {
  if (!c) return S3IMPH_OK;
  {
    std::lock_guard<std::mutex> lk(g_default_mu);
    for (auto& g : g_default)
      if (g == c) g = nullptr;
  }
  (void)hipSetDevice(c->device);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  free_workspace(c);
  if (c->d.comm) (void)ncclCommDestroy(c->d.comm);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return S3IMPH_OK;
}

int s3imph_ctx_reserve(s3imph_ctx* c, uint64_t max_keys, uint64_t max_global_keys) {
  if (!c) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(c->device));
    if (c->dist)
      ensure_dist_workspace(c, max_keys, std::max(max_keys, max_global_keys));
    else
      ensure_workspace(c, max_keys);
    HIPCHECK(hipDeviceSynchronize());
    return S3IMPH_OK;
  } catch (const Fail& f) {
    return f.code;
  }
}

int s3imph_build_device(s3imph_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets,
                        const uint64_t* d_pos, uint64_t n, uint64_t* d_fp_out, uint64_t* d_pos_out,
                        void* stream, s3imph_build_info* info) {
  if (!c || !info || (n && (!d_blob || !d_offsets || !d_fp_out || !d_pos_out))) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  std::string msg;
  try {
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    int rc = c->dist ? S3IMPH_ERR_STATE
                     : build_single(c, d_blob, d_offsets, d_pos, n, d_fp_out, d_pos_out, s, info, &msg);
    info->status = rc;
    return rc;
  } catch (const Fail& f) {
    info->status = f.code;
    return f.code;
  } catch (const std::bad_alloc&) {
    info->status = S3IMPH_ERR_NOMEM;
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_ctx_mph_bin(s3imph_ctx* c, uint8_t* out, uint64_t cap, uint64_t* len) {
  if (!c || !len) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  std::string msg;
  try {
    HIPCHECK(hipSetDevice(c->device));
    return marshal_locked(c, out, cap, len, &msg);
  } catch (const Fail& f) {
    return f.code;
  }
}

int s3imph_ctx_set_profiling(s3imph_ctx* c, int on) {
  if (!c) return S3IMPH_ERR_INVALID;
  c->profiling = on != 0;
  return S3IMPH_OK;
}

int s3imph_ctx_stage_times(s3imph_ctx* c, float* ms, int cap, int* count, char* names, size_t names_len) {
  if (!c || !count) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  const int n = (int)c->stage_ms.size();
  *count = n;
  std::string joined;
  for (int i = 0; i < n; ++i) {
    if (ms && i < cap) ms[i] = c->stage_ms[i];
    if (i) joined += ",";
    joined += c->stage_names[i];
  }
  if (names && names_len) set_err(names, names_len, joined);
  return S3IMPH_OK;
}

int s3imph_dist_unique_id(uint8_t id_out[128]) {
  if (!id_out) return S3IMPH_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return S3IMPH_ERR_RCCL;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(id_out, &id, 128);
  return S3IMPH_OK;
}

int s3imph_ctx_create_dist(int device, const uint8_t id[128], int rank, int nranks, s3imph_ctx** out,
                           char* err, size_t errlen) {
  if (!id || !out || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) return S3IMPH_ERR_INVALID;
  int rc = s3imph_ctx_create(device, out, err, errlen);
  if (rc != S3IMPH_OK) return rc;
  s3imph_ctx* c = *out;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  ncclResult_t r = ncclCommInitRank(&c->d.comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    set_err(err, errlen, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    s3imph_ctx_destroy(c);
    *out = nullptr;
    return S3IMPH_ERR_RCCL;
  }
  c->dist = true;
  c->d.rank = rank;
  c->d.nranks = nranks;
  return S3IMPH_OK;
}

int s3imph_build_device_dist(s3imph_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets,
                             const uint64_t* d_pos, uint64_t n_local, uint64_t key_base,
                             uint64_t* d_fp_out, uint64_t* d_pos_out, uint64_t out_cap, uint64_t* out_lo,
                             uint64_t* out_n, void* stream, s3imph_build_info* info) {
  if (!c || !c->dist || !info || !out_lo || !out_n) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  std::string msg;
  try {
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    int rc = build_dist(c, d_blob, d_offsets, d_pos, n_local, key_base, d_fp_out, d_pos_out, out_cap, out_lo,
                        out_n, s, info, &msg);
    info->status = rc;
    return rc;
  } catch (const Fail& f) {
    info->status = f.code;
    return f.code;
  } catch (const std::bad_alloc&) {
    info->status = S3IMPH_ERR_NOMEM;
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_lookup_device(s3imph_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets, uint64_t n,
                         const uint64_t* d_fp, const uint64_t* d_pos, uint64_t count, uint64_t* d_result,
                         void* stream) {
  if (!c || (n && (!d_blob || !d_offsets || !d_result))) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(c->device));
    if (!c->have_build) return S3IMPH_ERR_STATE;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    if (n == 0) return S3IMPH_OK;
    if (c->last_n == 0) {
      HIPCHECK(hipMemsetAsync(d_result, 0xff, n * 8, s));
    } else {
      if (!c->rank_valid) {  // word-level rank prefix, built on first lookup after a build
        launch_rank_scan(c->bits, c->cap_words, c->rank_base, c->block_sums, c->cap_blocks, c->d_st, s);
        c->rank_valid = true;
      }
      launch_lookup(d_blob, d_offsets, n, c->bits, c->rank_base, c->d_st, d_fp, d_pos, count, d_result,
                    default_grid(n, 256), s);
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return S3IMPH_OK;
  } catch (const Fail& f) {
    return f.code;
  }
}

int s3imph_build_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                      uint64_t n, uint64_t* fp_out, uint64_t* pos_out, uint8_t** mph_bin, uint64_t* mph_len,
                      char* err, size_t errlen) {
  if (!mph_bin || !mph_len || (n && (!blob || !offsets || !fp_out || !pos_out))) {
    set_err(err, errlen, "invalid argument");
    return S3IMPH_ERR_INVALID;
  }
  *mph_bin = nullptr;
  *mph_len = 0;
  std::vector<uint8_t> mph;
  std::string msg;
  int rc = build_from_host(device, blob, offsets, pos, n, fp_out, pos_out, &mph, &msg);
  if (rc != S3IMPH_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  if (!mph.empty()) {
    *mph_bin = static_cast<uint8_t*>(std::malloc(mph.size()));
    if (!*mph_bin) return S3IMPH_ERR_NOMEM;
    std::memcpy(*mph_bin, mph.data(), mph.size());
    *mph_len = mph.size();
  }
  return S3IMPH_OK;
}

void s3imph_free(void* p) { std::free(p); }

}  // extern "C"
