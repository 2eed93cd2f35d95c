// s3imph_build.hip — build orchestration and the device-side C ABI.
//
// Single GPU (s3imph_build_device): one stream, no host synchronisation until the
// very end.  Level sizes live on the device (LevelState); big levels run as
// full-grid kernels gated on the device-resident key count, the geometric tail of
// small levels runs inside one workgroup with LDS bit vectors.
//
// Multi-GPU (s3imph_build_device_dist): one process per GPU.  Position-range
// ownership (s3imph_dist.hip): per level every rank routes its records to the owner of
// their position with one all-to-all, each owner runs the single-GPU tile pipeline on
// its range, and once the active set is small every rank finishes it identically.
// Collectives go through a Comm: RCCL over xGMI in production, or host callbacks
// (the test transport that runs several ranks on one GPU).
//
// Reference: pkg/format/mphf_streaming.go:122-232 (Build), :141 (bbhash.New),
// :176-204 + :237-261 (positions and scatter).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "s3imph_ctx.h"

using namespace s3imph;

namespace s3imph {

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
  c->cap_keys = 0;  // set again only once every buffer is in place (a NOMEM midway reallocates next time)
  const uint64_t cap = std::max<uint64_t>(n, 1024);
  dalloc(c->kh, cap);
  dalloc(c->fp, cap);
  const uint64_t bcap = cap + cap / 4 + 4096;  // level-0 reservation slots: >= 1.25x the mean fill
  dalloc(c->bucket, bcap);
  dalloc(c->list[0], cap);
  dalloc(c->list[1], cap);
  dalloc(c->hist, kHistCap);
  dalloc(c->hoff, kHistCap);
  dalloc(c->tile_start, kMaxTiles + 2);
  dalloc(c->scan_sums, kHistCap / 2048 + 2);
  dalloc(c->flags, kMaxTiles + 2);
  dalloc(c->sflags, kHistCap / kScanSeg + 2);
  dalloc(c->tcnt, (uint64_t)kResLevels * kTcntStride);
  alloc_common(c, cap);
  dalloc(c->bits, c->cap_words);
  dfree(c->rank_base);  // the Lookup rank directory: made on the first lookup (ensure_rank_dir)
  c->rank_base_cap = 0;
  c->cap_blocks = (c->cap_words + 2047) / 2048 + 1;
  dalloc(c->block_sums, c->cap_blocks);
  c->cap_keys = cap;
  c->bucket_cap = bcap;
}

void free_bm_workspace(DistState& d);

void free_workspace(s3imph_ctx* c) {
  dfree(c->mid);
  c->mid_cap = 0;
  dfree(c->split);
  dfree(c->kh); dfree(c->fp); dfree(c->bits); dfree(c->rank_base);
  c->rank_base_cap = 0;
  c->bucket_cap = 0;
  dfree(c->block_sums); dfree(c->d_st);
  dfree(c->bucket); dfree(c->list[0]); dfree(c->list[1]);
  dfree(c->tcnt);
  dfree(c->p0_tcnt); dfree(c->p0_flags); dfree(c->p0_scnt); dfree(c->p0_pcnt); dfree(c->p0_sup); dfree(c->p0_x);
  dfree(c->p0_ov);
  c->p0_x_cap = 0;
  c->p0_tiles = 0;
  c->p0_sup_cap = 0;
  dfree(c->tile_prof);
  dfree(c->hist); dfree(c->hoff); dfree(c->tile_start); dfree(c->scan_sums); dfree(c->flags); dfree(c->sflags);
  if (c->h_st) (void)hipHostFree(c->h_st);
  c->h_st = nullptr;
  dfree(c->s_blob); dfree(c->s_offsets); dfree(c->s_pos); dfree(c->s_fp); dfree(c->s_posout);
  c->s_blob_cap = c->s_cap = c->s_pos_cap = 0;
  for (int w = 0; w < kStageWorkers; ++w) {
    for (int b = 0; b < 2; ++b) {
      if (c->stager.pin[w][b]) (void)hipHostFree(c->stager.pin[w][b]);
      if (c->stager.ev[w][b]) (void)hipEventDestroy(c->stager.ev[w][b]);
      c->stager.pin[w][b] = nullptr;
      c->stager.ev[w][b] = nullptr;
    }
    if (c->stager.st[w]) (void)hipStreamDestroy(c->stager.st[w]);
    c->stager.st[w] = nullptr;
  }
  c->stager.ready = false;
  DistState& d = c->d;
  free_bm_workspace(d);
  dfree(d.send); dfree(d.stage_bits); dfree(d.scnt); dfree(d.mat); dfree(d.gslot); dfree(d.small);
  if (d.h_pinned) (void)hipHostFree(d.h_pinned);
  d.h_pinned = nullptr;
  d.cap_list = d.cap_send = d.cap_stage_words = 0;
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
  if (c->profiling == 2 && std::strcmp(name, "init") != 0 && std::strcmp(name, "hash_count0") != 0 &&
      std::strcmp(name, "hash_part0") != 0 &&
      std::strcmp(name, "hash_route0") != 0 && std::strcmp(name, "route0") != 0)
    return;  // light mode: two events per build, around the dominant kernel
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
    // a stage marked more than once (a bitmap build's "levels", once per level) sums
    const auto at = std::find(c->stage_names.begin(), c->stage_names.end(), c->ev_names[i]);
    if (at != c->stage_names.end()) {
      c->stage_ms[at - c->stage_names.begin()] += ms;
      continue;
    }
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

// Values that occur more than once among n device records' key hashes (sorted, distinct,
// at most `cap` of them): the keys a stopped build could not place.
std::vector<uint64_t> record_dup_values(const Rec* d_list, uint64_t n, size_t cap, bool r20 = false) {
  std::vector<uint64_t> k(n);
  if (r20) {  // an R20 list (BinBuffers::l20): k is dwords 0-1
    std::vector<R20> h(n);
    if (n) HIPCHECK(hipMemcpy(h.data(), d_list, n * sizeof(R20), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; ++i) k[i] = (uint64_t)h[i].w[0] | ((uint64_t)h[i].w[1] << 32);
  } else {
    std::vector<Rec> h(n);
    if (n) HIPCHECK(hipMemcpy(h.data(), d_list, n * sizeof(Rec), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; ++i) k[i] = h[i].k;
  }
  std::sort(k.begin(), k.end());
  std::vector<uint64_t> out;
  for (uint64_t i = 1; i < n && out.size() < cap; ++i)
    if (k[i] == k[i - 1] && (out.empty() || out.back() != k[i])) out.push_back(k[i]);
  return out;
}

// The ORIGINAL key hashes, recomputed from the key bytes (c->kh is scratch here: the
// level-0 pipeline may keep them only in its record layouts), sorted, on the host.
std::vector<uint64_t> original_key_hashes(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, uint64_t n,
                                          hipStream_t s) {
  std::vector<uint64_t> h(n);
  if (n) {
    launch_key_hashes(blob, offsets, n, c->kh, s);
    HIPCHECK(hipMemcpyAsync(h.data(), c->kh, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
  }
  std::sort(h.begin(), h.end());
  return h;
}

// A build that stopped (kStTooManyLevels: a level placed no key) or overflowed blames the
// caller's keys (DUP_KEY_HASH, the reference's bbhash failure on equal hashes) only when
// equal FNV-1a hashes exist among the ORIGINAL keys.  Leftover records with equal hashes
// while every key hash is distinct mean a record was duplicated inside the build: an
// internal fault, reported as one (with the level), never as the user's duplicates.
int classify_stop(s3imph_ctx* c, unsigned flags, const uint8_t* blob, const uint64_t* offsets, uint64_t n,
                  hipStream_t s, std::string* msg) {
  const LevelState& h = *c->h_st;
  const unsigned S = h.stop_level;
  std::vector<uint64_t> left;
  if ((flags & kStTooManyLevels) && S >= 1 && S < (unsigned)kMaxLevels + 2 && h.n[S])
    left = record_dup_values(c->list[(S - 1) & 1], h.n[S], 1, S < 32 && ((c->l20_mask >> S) & 1u));
  const std::vector<uint64_t> orig = original_key_hashes(c, blob, offsets, n, s);
  if (std::adjacent_find(orig.begin(), orig.end()) != orig.end()) {
    *msg = "build MPHF: duplicate FNV-1a key hashes: bbhash cannot place them";
    return S3IMPH_ERR_DUP_KEY_HASH;
  }
  if (!left.empty()) {
    *msg = "build MPHF: internal error: level " + std::to_string(S) +
           " holds records with equal key hashes although every key hash is distinct (a record was duplicated)";
    return S3IMPH_ERR_INTERNAL;
  }
  *msg = (flags & kStTooManyLevels) ? "build MPHF: can't find minimal perfect hash after " +
                                          std::to_string(kMaxLevels) + " levels"
                                    : "build MPHF: workspace overflow";
  return (flags & kStTooManyLevels) ? S3IMPH_ERR_TOO_MANY_LEVELS : S3IMPH_ERR_INTERNAL;
}

int map_status(s3imph_ctx* c, unsigned flags, const uint8_t* blob, const uint64_t* offsets, uint64_t n,
               hipStream_t s, std::string* msg) {
  if (flags & (kStTooManyLevels | kStOverflow)) return classify_stop(c, flags, blob, offsets, n, s, msg);
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

// Test hook (S3IMPH_FAULT_DUP_REC, read at context creation): copy record 0 of a list over
// record 1, as a kernel race that duplicated a record would, so the tests can check that the
// stop it causes is reported as an internal fault and not as the caller's duplicate keys.
void fault_dup_record(s3imph_ctx* c, Rec* list, hipStream_t s, bool r20 = false) {
  const size_t sz = r20 ? sizeof(R20) : sizeof(Rec);
  if (c->fault_dup)
    HIPCHECK(hipMemcpyAsync(reinterpret_cast<uint8_t*>(list) + sz, list, sz, hipMemcpyDeviceToDevice, s));
}

int mid_big_mode();
BinBuffers make_bufs(s3imph_ctx* c, const uint64_t* pos, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s) {
  BinBuffers b{};
  b.feed = c->feed;
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
  b.bucket_cap = c->bucket_cap;
  b.tile_prof = nullptr;
  if (c->debug) {
    const size_t nprof = (size_t)kMaxLevels * kMaxTiles * 8;
    if (!c->tile_prof) HIPCHECK(hipMalloc(&c->tile_prof, nprof * sizeof(unsigned long long)));
    HIPCHECK(hipMemsetAsync(c->tile_prof, 0, nprof * sizeof(unsigned long long), s));
    b.tile_prof = c->tile_prof;
  }
  {  // the 256-workgroup mid levels' scratch (201 MB) for sets that may have a level of 440k-1.75M keys
    const uint64_t need = c->cap_keys >= kMidBigMinKeys && mid_big_mode() != 0
                              ? std::max<uint64_t>(kMidScratchU32, MidCfg<kMidGBig>::kScratchU32)
                              : kMidScratchU32;
    if (!c->mid || c->mid_cap < need) {
      c->mid_cap = 0;
      dfree(c->mid);
      dalloc(c->mid, need);
      c->mid_cap = need;
    }
  }
  b.mid = c->mid;
  // 2^15 / 2^16-position tiles appear once a level has more than 2^14 x 4096 positions
  if (!c->split && c->cap_keys > (kMaxTiles << kRegTileMaxBits) / 2) dalloc(c->split, split_scratch_records());
  b.split = c->split;
  b.scat_cfg = c->scat_cfg;
  b.pipe_tiles = c->p0 != 0;
  b.skew_cfg = c->skew_cfg;
  b.bits = c->bits;
  b.cap_words = c->cap_words;
  b.fp_out = fp_out;
  b.pos_out = pos_out;
  b.st = c->d_st;
  b.dist = c->dist;
  return b;
}

// Launch grids for a level of about nk records over `size` positions; the kernels loop
// over whatever the device finds.
struct Grids {
  int gc, gt, gs;
};
Grids level_grids(uint64_t nk, uint64_t size, LevelGeom g) {
  const uint64_t T = (size + (1ull << g.tb) - 1) >> g.tb;
  const uint64_t B = std::max<uint64_t>((nk + g.chunk - 1) / g.chunk, 1);
  Grids r;
  r.gc = (int)std::min<uint64_t>(B, 2048);
  r.gt = (int)std::min<uint64_t>(std::max<uint64_t>(T, 1), 2048);
  r.gs = (int)std::min<uint64_t>((T * B + kScanSeg - 1) / kScanSeg + 2, 256);
  return r;
}

// Do reservation slots (bucket_cap / T records per tile, cut into kResShards shards)
// hold a level of about nb records over `size` positions (T tiles; 0: the list-level
// geometry)?  Small levels keep 4x the mean fill; larger ones res_fill x; and tiles so
// large that a shard's mean fill m is >= 768 need only 1 + 7/sqrt(m) (7 sigma of a
// Poisson fill) plus 2 % for the size estimate (1.24x at m = 1024: level 0 of 10M keys).
// Shards follow the XCDs (blockIdx % 8): 16 shards measured far slower (C3 level-0
// scatter 1.60 -> 2.87 ms), the runs of an XCD's blocks no longer meet in its L2.  An overflow is caught on the device and
// the build reruns on the counted path.
// Mid levels over every CU (k_mid_levels<kMidGBig>) for levels of 440k-1.75M keys (A/B knob
// S3IMPH_MID_BIG: 0 off (default), 1 those levels only, 2 every level down to the tail).
// Bit-exact, and slower than the binned kernels it replaces (C2 levels 0.280 -> 0.320 / 0.354
// ms, C5 0.54 -> 0.58 / 0.61): a level's barrier and all-gather over 256
// workgroups cost more than a level's two launches.
int mid_big_mode() {
  static const int v = [] {
    const char* e = dev_env("S3IMPH_MID_BIG");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

bool res_fits(const s3imph_ctx* c, uint64_t nb, uint64_t size, uint64_t T = 0) {
  if (nb * (nb > kResSmallKeys ? c->res_fill : 4) <= c->bucket_cap) return true;
  if (T == 0) {
    const LevelGeom g = choose_geom_sz(nb, size, kTargetTilesRes, kTargetChunks, kRegTileMaxBits);
    T = (size + (1ull << g.tb) - 1) >> g.tb;
  }
  const double m = (double)nb / ((double)T * kResShards);
  return m >= 768.0 && (double)c->bucket_cap >= (double)nb * (1.02 + 7.0 / std::sqrt(m));
}

// Split-kernel tile size for a reservation-path level of `size` positions (predicted,
// ~10 % high, unless `exact`: the sharded build's levels): the split kernel runs one persistent workgroup per CU taking tiles by ticket,
// so a level of T tiles takes ceil(T / 256) rounds of a tile's time, and a tile's time is
// proportional to its ts sub-tiles.  Pick ts (2..16) minimising ceil(T / 256) x ts with a
// 5 % margin under each round boundary, the larger ts on ties (fewer tiles: longer
// scatter runs).  C3 level 1: 601 tiles of 8 sub-tiles (3 rounds) -> 481 of 10 (2 rounds).
unsigned choose_split_ts(uint64_t size, bool exact) {
  const double est = exact ? (double)size : (double)size / 1.1;
  unsigned best = 0;
  double best_cost = 0;
  // A/B knob S3IMPH_TS_MAX: the largest ts tried (smaller sub-tile scratch per workgroup)
  static const unsigned ts_max = [] {
    const char* e = dev_env("S3IMPH_TS_MAX");
    return e ? std::max(2u, std::min((unsigned)std::atoi(e), 1u << (kSplitMaxBits - 14))) : 1u << (kSplitMaxBits - 14);
  }();
  for (unsigned ts = 2; ts <= ts_max; ++ts) {
    const double T = est / (double)((uint64_t)ts << 14);
    if (T > (double)kSplitTargetTiles) continue;
    const double rounds = std::ceil(T / ((exact ? 1.0 : 0.95) * kSplitGridHost));
    const double cost = rounds * ts;
    if (best == 0 || cost <= best_cost) {
      best = ts;
      best_cost = cost;
    }
  }
  return best;
}

// One list-input level L (records in list[(L-1)&1]): about nb records over `size`
// positions.  Small levels take the reservation scatter (no count / histogram scan).
struct ListPlan {
  bool res;
  LevelGeom g;
};
ListPlan plan_list_level(s3imph_ctx* c, const BinBuffers& b, int L, uint64_t nb, uint64_t size, bool conservative,
                         const LevelGeom* force, bool exact_size) {
  // reservation slots are bucket_cap / T records per tile: keep them >= 4x the mean fill
  const bool res = !conservative && nb <= c->res_max_keys && res_fits(c, nb, size) && L < kResLevels;
  LevelGeom g = force ? *force
                : res ? choose_geom_sz(nb, size, kTargetTilesRes, kTargetChunks, kRegTileMaxBits)
                      : choose_geom_sz(nb, size, kTargetTiles, kTargetChunks, kRegTileMaxBits);
  if (res && !force && b.split && g.tb > kRegTileMaxBits && g.tb <= kSplitMaxBits) g.ts = choose_split_ts(size, exact_size);
  return ListPlan{res, g};
}

void enqueue_list_level(s3imph_ctx* c, const BinBuffers& b, int L, uint64_t nb, uint64_t size, bool conservative,
                        const LevelGeom* force, hipStream_t s, bool exact_size = false) {
  const ListPlan pl = plan_list_level(c, b, L, nb, size, conservative, force, exact_size);
  const LevelGeom g = pl.g;
  const Grids gr = level_grids(nb, size, g);
  if (pl.res) {
    const int gsr = (int)std::min<uint64_t>((nb + kSubRound - 1) / kSubRound, 256);
    launch_binned_scatter_res(L, b, g, std::max(gsr, 1), s, 0, 0, tiles_of((size + 63) / 64, g.tb, b.split ? g.ts : 0));
    launch_binned_tile(L, b, g, gr.gt, s, true);
  } else {
    launch_binned_count(L, nullptr, nullptr, 0, b, g, gr.gc, s);
    launch_binned_scan(L, b, gr.gs, s);
    launch_binned_scatter(L, b, g, s);
    launch_binned_tile(L, b, g, gr.gt, s);
  }
}

// Does a reservation level of geometry g run a tile kernel that reads and writes R20 records
// (k_tile_p0 on 2^14-position tiles, k_tile_split on 2^15-2^18)?  launch_binned_tile's choice.
bool r20_tiles(const BinBuffers& b, const LevelGeom& g) {
  return (g.tb == kRegTileMaxBits && b.pipe_tiles) || (b.split && g.tb > kRegTileMaxBits && g.tb <= kSplitMaxBits);
}

// The levels enqueue_levels_from runs from L0 (n0 records in list[(L0-1)&1]): predicted-big
// levels as full-grid kernels (lv, consecutive from L0), then at most one k_mid_levels range.
struct LevelsPlan {
  struct Lv {
    int L;
    uint64_t nb, size;
    bool tight;
    ListPlan pl;
  };
  std::vector<Lv> lv;
  int midB0 = -1, midB1 = -1;  // levels over kMidGBig workgroups (k_mid_levels<kMidGBig>), before mid0..mid1
  int mid0 = -1, mid1 = -1;
  int launched;  // the last big level launched (L0 - 1 if none)
};
LevelsPlan plan_levels_from(s3imph_ctx* c, const BinBuffers& b, int L0, uint64_t n0, const LevelGeom& gcons,
                            bool conservative) {
  const double q = 1.0 - std::exp(-0.5);  // fraction of keys that collide at load 1/2
  const int big = conservative ? kMaxLevels - 2 : L0 - 1 + predict_big_levels(n0 / q);
  LevelsPlan P;
  P.launched = L0 - 1;
  for (int L = L0; L <= big && L < kMaxLevels - 1; ++L) {
    // Level sizes concentrate tightly around n q^L; a level predicted within 1/kTailMargin
    // of the tail's capacity is left to the tail (an unexpectedly large one is caught by
    // kStTailOverflow and rerun conservatively).
    const double pred = (double)n0 * std::pow(q, L - L0);
    if (!conservative && pred * kTailMargin < (double)kTailKeys) break;
    // a level of 440k-1.75M keys (bound: 2 % + 6 sigma, as the binned geometry's): the
    // 256-workgroup mid kernel, with the levels after it that the small one would not take
    // (mode 2: every level down to the tail)
    // (its grid barrier needs all 256 CUs at once: not while other ranks share the GPU)
    const int mb = !c->dist || (c->d.comm && c->d.comm->owns_gpu()) ? mid_big_mode() : 0;
    if (!conservative && mb != 0 && P.midB0 < 0 && pred * kMidMargin > (double)kMidMaxKeys &&
        c->mid_cap >= MidCfg<kMidGBig>::kScratchU32 &&
        pred * 1.02 + 6.0 * std::sqrt(pred) + 1024.0 <= (double)kMidMaxKeysBig) {
      int L1 = L;
      while (L1 + 1 <= big && L1 + 1 < kMaxLevels - 1) {
        const double pn = pred * std::pow(q, L1 + 1 - L);
        if (pn * kTailMargin < (double)kTailKeys) break;
        if (mb == 1 && pn * kMidMargin <= (double)kMidMaxKeys) break;
        ++L1;
      }
      P.midB0 = L;
      P.midB1 = L1;
      P.launched = L1;
      L = L1;
      continue;
    }
    if (!conservative && pred * kMidMargin <= (double)kMidMaxKeys) {
      // this level and the rest above the tail: one persistent launch
      int L1 = L;
      while (L1 + 1 <= big && L1 + 1 < kMaxLevels - 1 && pred * std::pow(q, L1 + 1 - L) * kTailMargin >= (double)kTailKeys)
        ++L1;
      P.mid0 = L;
      P.mid1 = L1;
      P.launched = L1;
      break;
    }
    P.launched = L;
    const uint64_t nb = conservative ? n0 : (uint64_t)(pred * 1.1) + 4096;
    // geometry from a tight bound on the level's size (level sizes concentrate: sigma ~ sqrt(n));
    // a level past it flags kStGeometry and the build reruns conservatively
    const bool tight = !conservative && !c->loose_geom;
    const uint64_t nsz = tight ? (uint64_t)(pred * 1.02 + 6.0 * std::sqrt(pred)) + 1024 : nb;
    const uint64_t size = 64 * level_words(nsz);
    P.lv.push_back({L, nb, size, tight,
                    plan_list_level(c, b, L, nb, size, conservative, conservative ? &gcons : nullptr, tight)});
  }
  return P;
}

// BinBuffers::l20 for a single-GPU build with identity positions: level L's list is R20 when
// level L - 1's tile kernel writes R20 (prev_r20 for L0 - 1) and level L is a reservation
// level on an R20 tile kernel.  Mid and tail levels read Rec lists.
unsigned plan_l20(const s3imph_ctx* c, const BinBuffers& b, const LevelsPlan& P, bool prev_r20, uint64_t n) {
  if (!c->l20 || b.pos || b.dist || n >= (1ull << 32)) return 0;
  unsigned m = 0;
  bool prev = prev_r20;
  for (const auto& v : P.lv) {
    const bool cap = v.pl.res && r20_tiles(b, v.pl.g);
    if (prev && cap && v.L < 32) m |= 1u << v.L;
    prev = cap;
  }
  return m;
}

// Levels L0, L0+1, ... of a whole-level build (every position on this GPU), starting
// from n0 records in list[(L0-1)&1]: predicted-big levels as full-grid kernels, then
// the single-workgroup tail.  Returns the last big level launched (L0-1 if none).
int run_levels(s3imph_ctx* c, const BinBuffers& b, const LevelsPlan& P, int L0, hipStream_t s) {
  for (const auto& v : P.lv) {
    const LevelGeom g = v.pl.g;
    enqueue_list_level(c, b, v.L, v.nb, v.size, false, &g, s, v.tight);
  }
  if (P.midB0 >= 0) launch_binned_mid(P.midB0, P.midB1, b, s, true);
  if (P.mid0 >= 0) launch_binned_mid(P.mid0, P.mid1, b, s);
  ev_mark(c, s, "levels");
  launch_binned_tail(L0, P.launched, b, s);
  ev_mark(c, s, "tail");
  return P.launched;
}
int enqueue_levels_from(s3imph_ctx* c, const BinBuffers& b, int L0, uint64_t n0, const LevelGeom& gcons,
                        bool conservative, hipStream_t s) {
  const LevelsPlan P = plan_levels_from(c, b, L0, n0, gcons, conservative);
  if (!conservative) return run_levels(c, b, P, L0, s);
  for (const auto& v : P.lv) enqueue_list_level(c, b, v.L, v.nb, v.size, true, &gcons, s, v.tight);
  if (P.mid0 >= 0) launch_binned_mid(P.mid0, P.mid1, b, s);
  ev_mark(c, s, "levels");
  launch_binned_tail(L0, P.launched, b, s);
  ev_mark(c, s, "tail");
  return P.launched;
}

// Chunks (hash blocks) of the level-0 hash over n keys.  Blocks are scheduled as they
// free up, so more, smaller chunks even out long-key chunks on big sets; on small ones
// each block's fixed cost wins (S3IMPH_CHUNKS sweep, hash_count0 ms at 768 / 1536
// chunks: C2 0.229 / 0.243, C3 3.89 / 3.75, C5 4.28 / 4.05).
uint64_t chunks0(uint64_t n) {
  return n >= kBigChunksKeys ? 2 * kTargetChunks : kTargetChunks;
}

// Enqueue one attempt of the binned pipeline.  `conservative` sizes every level with
// the level-0 geometry (always inside the workspace bounds) and runs every level that
// is still big as a full-grid level; the default predicts each level's size.
// Profiling aid (tools/hash_only.py): with S3IMPH_HASH_ONLY set the build stops after the
// level-0 hash so that kernel can be timed alone, and FAILS with S3IMPH_ERR_INTERNAL — the
// outputs are not an index, and no caller may mistake the run for a build.
bool hash_only_knob() {
  static const bool on = dev_env("S3IMPH_HASH_ONLY") != nullptr;
  return on;
}

// Level 0 takes P0 above this many 2^14-position tiles (A/B knob S3IMPH_P0_MIN_TILES)
uint64_t p0_min_tiles() {
  static const uint64_t v = [] {
    const char* e = dev_env("S3IMPH_P0_MIN_TILES");
    return e ? std::strtoull(e, nullptr, 10) : kP0MinTiles;
  }();
  return v;
}

// The most super-tiles P0 cuts level 0 into (A/B knob S3IMPH_P0_MAXS, at most kP0MaxS = 64, the
// default).  How many a level takes follows kP0TargetTps (C3: 24); the cap matters for levels of
// more than 64 x 512 tiles, and for S3IMPH_P0_TPS sweeps.
uint64_t p0_max_s() {
  static const uint64_t v = [] {
    const char* e = dev_env("S3IMPH_P0_MAXS");
    return e ? std::max<uint64_t>(1, std::min<uint64_t>(std::strtoull(e, nullptr, 10), kP0MaxS)) : kP0MaxS;
  }();
  return v;
}
uint64_t p0_super_tiles(uint64_t T, uint64_t target) {
  const uint64_t S = std::min<uint64_t>((T + target - 1) / target, p0_max_s());
  return std::max<uint64_t>(S, (T + kP0MaxTps - 1) / kP0MaxTps);  // <= kP0MaxS under the callers' gate
}

// P0 geometry and buffers for level 0 of n keys over the positions of n_geom keys (the whole
// level: n_geom = n, or the global key count of the bitmap decomposition), identity
// positions: T 2^14-position tiles
// in S super-tiles of tps (about kP0TargetTps; S <= kP0MaxS), the super-tiles' records in
// c->p0_sup (sized for the hash's per-block regions and for the slot layout of the pass that
// stands in for it), the tiles' slots in the bucket, both as R20.
// The geometry alone (no allocation, no memset): what p0_bufs takes for the same arguments,
// and the R20 records c->p0_sup must hold for it
P0Bufs p0_geom(const s3imph_ctx* c, uint64_t n, uint64_t n_geom, unsigned tb, uint64_t* need) {
  const uint64_t T = tiles_of(level_words(n_geom), tb, 0);
  P0Bufs p;
  p.tb = tb;
  static const uint64_t target = [] {  // A/B knob S3IMPH_P0_TPS: tiles per super-tile aimed at
    const char* e = dev_env("S3IMPH_P0_TPS");
    return e ? std::max<uint64_t>(16, std::strtoull(e, nullptr, 10)) : kP0TargetTps;
  }();
  p.S = (unsigned)p0_super_tiles(T, target);
  p.tps = (unsigned)((T + p.S - 1) / p.S);
  p.reg_cap = p0_region_cap(n, p.S, kH0GridHost);
  const unsigned nbs = p0_skew_blocks(c->skew_cfg);
  p.reg_cap_skew = p0_region_cap(n, p.S, nbs);
  *need = std::max<uint64_t>(std::max<uint64_t>((uint64_t)kH0GridHost * p.S * p.reg_cap,
                                                (uint64_t)nbs * p.S * p.reg_cap_skew),
                             n + n / 4 + (uint64_t)4096 * p.S * kResShards);
  return p;
}

P0Bufs p0_bufs(s3imph_ctx* c, uint64_t n, uint64_t n_geom, hipStream_t s, unsigned tb = kRegTileMaxBits,
               bool want_x = false) {
  const uint64_t T = tiles_of(level_words(n_geom), tb, 0);
  uint64_t need = 0;
  P0Bufs p = p0_geom(c, n, n_geom, tb, &need);
  // (a capacity is zeroed before its buffer is replaced and set only once the allocation
  // succeeded: a NOMEM leaves a null buffer that the next build reallocates, never one that a
  // smaller build would take as big enough)
  if (need > c->p0_sup_cap) {
    c->p0_sup_cap = 0;
    dfree(c->p0_sup);
    if (dev_env("S3IMPH_FAULT_P0_NOMEM"))  // test hook: this allocation fails (the callers fall back)
      throw Fail{S3IMPH_ERR_NOMEM, "p0_bufs: injected allocation failure (S3IMPH_FAULT_P0_NOMEM)"};
    dalloc(c->p0_sup, need);
    c->p0_sup_cap = need;
  }
  if (T > c->p0_tiles) {
    c->p0_tiles = 0;
    dalloc(c->p0_tcnt, T * kResShards);
    dalloc(c->p0_flags, T);
    c->p0_tiles = T;
  }
  if (!c->p0_scnt) dalloc(c->p0_scnt, (uint64_t)kMaxRanks * kResShards);
  if (!c->p0_pcnt) dalloc(c->p0_pcnt, (uint64_t)kH0GridHost * kMaxRanks);
  p.sup = c->p0_sup;
  p.sup_cap = c->p0_sup_cap;
  p.pcnt = c->p0_pcnt;
  p.scnt = c->p0_scnt;
  p.bucket = reinterpret_cast<R20*>(c->bucket);
  p.bucket_cap = c->bucket_cap * sizeof(Rec) / sizeof(R20);
  if (want_x) {  // the bitmap decomposition's level 0: each slot's position beside its record
    if (p.bucket_cap > c->p0_x_cap) {
      c->p0_x_cap = 0;
      dalloc(c->p0_x, p.bucket_cap);
      c->p0_x_cap = p.bucket_cap;
    }
    p.x = c->p0_x;
  }
  p.tcnt = c->p0_tcnt;
  p.flags = c->p0_flags;
  HIPCHECK(hipMemsetAsync(p.tcnt, 0, T * kResShards * sizeof(unsigned), s));
  HIPCHECK(hipMemsetAsync(p.scnt, 0, (uint64_t)p.S * kResShards * sizeof(unsigned), s));
  return p;
}

// p0_bufs, or false when its allocation fails (NOMEM): the caller takes the non-P0 path
bool p0_try_bufs(s3imph_ctx* c, uint64_t n, uint64_t n_geom, hipStream_t s, P0Bufs* out,
                 unsigned tb = kRegTileMaxBits, bool want_x = false) {
  try {
    *out = p0_bufs(c, n, n_geom, s, tb, want_x);
    return true;
  } catch (const Fail& f) {
    if (f.code != S3IMPH_ERR_NOMEM) throw;
    (void)hipGetLastError();  // an out-of-memory hipMalloc is not sticky; clear it
    if (c->debug) std::fprintf(stderr, "[s3imph] P0 buffers: %s; level 0 without P0\n", f.msg.c_str());
    return false;
  }
}

// P0F (developer knob S3IMPH_P0F=1; off by default): level 1 of a P0 build fed by level 0's
// tile kernel.  Bit-exact, but measured slower on C3 (level 1 -0.32 ms, the
// count pass +0.15, the in-tile positions' partial-line writes +0.17, the fed tile +0.08)
// The super-tile scatter overlapped on the level-0 hash (bit-exact, measured slower:
// the hash loses more beside it than the scatter's time): S3IMPH_P0_OV=1 turns it on (developer
// switch); S3IMPH_P0_DIRECT=1 runs the direct form alone after the hash (A/B knob)
bool p0_ov_on() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_P0_OV");
    return e && std::atoi(e) != 0;
  }();
  return v;
}
bool p0_direct_on() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_P0_DIRECT");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// Overlap set-up, on s after the build's state init: every region fill open, no part done;
// the overlapped scatter then starts on c->ov_stream (it spins on the fills the hash publishes)
void p0_ov_launch(s3imph_ctx* c, const BinBuffers& b, P0Bufs& p, hipStream_t s) {
  if (!c->ov_stream) {
    HIPCHECK(hipStreamCreateWithFlags(&c->ov_stream, hipStreamNonBlocking));
    for (auto& e : c->ov_ev) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  if (!c->p0_ov) dalloc(c->p0_ov, (uint64_t)kH0GridHost + 8ull * kP0OvChunks * kMaxRanks);
  p.hxcc = c->p0_ov;
  p.ov_done = c->p0_ov + kH0GridHost;
  HIPCHECK(hipMemsetAsync(p.pcnt, 0xff, (uint64_t)kH0GridHost * p.S * sizeof(unsigned), s));
  HIPCHECK(hipMemsetAsync(p.hxcc, 0xff, (uint64_t)kH0GridHost * sizeof(unsigned), s));
  HIPCHECK(hipMemsetAsync(p.ov_done, 0, 8ull * kP0OvChunks * p.S * sizeof(unsigned), s));
  HIPCHECK(hipEventRecord(c->ov_ev[0], s));
  HIPCHECK(hipStreamWaitEvent(c->ov_stream, c->ov_ev[0], 0));
  launch_p0_scatter_direct(b, p, true, c->ov_stream);
  HIPCHECK(hipEventRecord(c->ov_ev[1], c->ov_stream));
}

bool p0f_on() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_P0F");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// P0F region capacity: level 0's tile kernel takes its tiles by ticket, so one block's share of
// level 1's records follows its share of the tiles, not a Poisson fill: regions hold twice the
// mean (a block would have to run twice its share of the tiles to overflow; then the build reruns)
uint64_t p0f_region_cap(uint64_t n1, unsigned S) {
  const double mean = (double)n1 / ((double)kP0FedGrid * S);
  return (uint64_t)(2.0 * mean + 10.0 * std::sqrt(mean) + 256.0);
}

void enqueue_binned(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                    uint64_t n, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s, bool conservative) {
  BinBuffers b = make_bufs(c, pos, fp_out, pos_out, s);
  b.dist = false;  // the whole set on this GPU (also a one-rank sharded build, build_dist's routed fallback)
  c->l20_mask = 0;
  const double q = 1.0 - std::exp(-0.5);
  const uint64_t T14 = tiles_of(level_words(n), kRegTileMaxBits, 0);
  if (!conservative && c->p0 && !pos && n <= kP0MaxKeys && !hash_only_knob() && T14 > p0_min_tiles() &&
      T14 <= kP0MaxS * kP0MaxTps) {
    // level 0 in 2^14-position register tiles through super-tiles (s3imph_internal.h, P0); its
    // buffers (~1.2 n x 20 B) may not fit next to the workspace: then the split-kernel path.
    // P0F: a level 1 past the reservation scatter's 4096 tiles (C3: 4.8k) is fed by level 0's
    // tile kernel when its regions fit the super-tile buffer; level 0's scatter then also writes
    // each slot's in-tile position for the count pass (k_p0_count).
    const double n1m = (double)n * q;
    const uint64_t ng1 = (uint64_t)(n1m * 1.02 + 6.0 * std::sqrt(n1m)) + 1024;  // level 1's size bound
    const uint64_t T1 = tiles_of(level_words(ng1), kRegTileMaxBits, 0);
    bool fed = p0f_on() && T1 > kScatterTiles && T1 <= kP0MaxS * kP0MaxTps;
    P0Bufs p;
    if (p0_try_bufs(c, n, n, s, &p, kRegTileMaxBits, fed)) {
      P0Bufs p1{};
      if (fed) {  // level 1's super-tiles, its regions in c->p0_sup (free once level 0's scatter ran)
        uint64_t need1 = 0;
        p1 = p0_geom(c, ng1, ng1, kRegTileMaxBits, &need1);
        p1.reg_cap = p0f_region_cap(ng1, p1.S);
        fed = p1.S <= (unsigned)kMaxRanks && (uint64_t)kP0FedGrid * p1.S * p1.reg_cap <= c->p0_sup_cap &&
              T1 <= c->p0_tiles && p0_fused(blob, p);
        p1.sup = c->p0_sup;
        p1.sup_cap = c->p0_sup_cap;
        p1.nb = kP0FedGrid;
        p1.pcnt = c->p0_pcnt;
        p1.scnt = c->p0_scnt;
        p1.bucket = p.bucket;  // (level 0's slots: read by its tile kernel before level 1's scatter)
        p1.bucket_cap = p.bucket_cap;
        p1.tcnt = p.tcnt;
        p1.flags = p.flags;
      }
      if (!fed) p.x = nullptr;
      const LevelGeom g0 = choose_geom(n, kTargetTiles0, chunks0(n), kRegTileMaxBits);
      if (fed) {
        const LevelsPlan P = plan_levels_from(c, b, 2, (uint64_t)(n1m * q), g0, false);
        b.l20 = c->l20_mask = plan_l20(c, b, P, true, n);
        launch_init_state(c->d_st, n, n, s, offsets);
        ev_mark(c, s, "init");
        launch_p0_hash(blob, offsets, n, b, g0, p, s);
        ev_mark(c, s, "hash_part0");
        launch_p0_scatter(b, p, true, s);
        launch_p0_count(b, p, s);
        ev_mark(c, s, "scatter0_p0");
        const NextPart np{p1.sup, p1.reg_cap, p1.pcnt, p1.tps_sub(), p1.S, nullptr};
        launch_p0_tile_fed(b, p, np, s);
        ev_mark(c, s, "tile0_p0");
        HIPCHECK(hipMemsetAsync(p1.tcnt, 0, c->p0_tiles * kResShards * sizeof(unsigned), s));
        launch_p0_scatter(b, p1, true, s, 1);
        launch_p0_tile_level(1, b, p1, s);
        ev_mark(c, s, "level1_p0");
        fault_dup_record(c, c->list[1], s, b.list20(2));
        run_levels(c, b, P, 2, s);
        return;
      }
      // the list levels' plan first: level 0's tile kernel writes level 1's list as R20 or Rec
      const LevelsPlan P = plan_levels_from(c, b, 1, (uint64_t)((double)n * q), g0, false);
      b.l20 = c->l20_mask = plan_l20(c, b, P, true, n);
      launch_init_state(c->d_st, n, n, s, offsets);
      ev_mark(c, s, "init");
      // the super-tile scatter overlapped on the hash (fused regions of a device-resident set)
      const bool ov = p0_ov_on() && p0_fused(blob, p) && !b.feed && p.tps <= 1024;
      if (ov) p0_ov_launch(c, b, p, s);
      launch_p0_hash(blob, offsets, n, b, g0, p, s);
      ev_mark(c, s, "hash_part0");
      if (ov) {
        HIPCHECK(hipStreamWaitEvent(s, c->ov_ev[1], 0));
        launch_p0_scatter_direct(b, p, false, s);
      } else if (p0_direct_on() && p0_fused(blob, p) && p.tps <= 1024) {
        launch_p0_scatter_direct(b, p, false, s);
      } else {
        launch_p0_scatter(b, p, p0_fused(blob, p), s);
      }
      ev_mark(c, s, "scatter0_p0");
      launch_p0_tile(b, p, s);
      ev_mark(c, s, "tile0_p0");
      fault_dup_record(c, c->list[0], s, b.list20(1));
      run_levels(c, b, P, 1, s);
      return;
    }
  }
  const LevelGeom g0 = choose_geom(n, kTargetTiles0, chunks0(n), kRegTileMaxBits);
  launch_init_state(c->d_st, n, n, s, offsets);
  ev_mark(c, s, "init");
  const Grids gr = level_grids(n, 64 * level_words(n), g0);
  // Level 0 through the reservation scatter when its tiles are big enough that every
  // (tile, shard) slot's headroom (bucket_cap = 1.25 n) covers 7 sigma of its fill
  const uint64_t T0 = (64 * level_words(n) + (1ull << g0.tb) - 1) >> g0.tb;
  const bool res0 = !conservative && c->res0 && T0 <= kScatterTiles && (res_fits(c, n, 64 * level_words(n), T0) || c->res0 == 2);
  launch_binned_count(0, blob, offsets, n, b, g0, gr.gc, s, !res0);  // no histogram for the reservation path
  ev_mark(c, s, "hash_count0");
  if (hash_only_knob()) return;
  if (res0) {
    LevelGeom gr0 = g0;  // split-kernel level 0: tiles in whole rounds over the CUs (exact size)
    if (b.split && g0.tb > kRegTileMaxBits && g0.tb <= kSplitMaxBits) gr0.ts = choose_split_ts(64 * level_words(n), true);
    const LevelsPlan P = plan_levels_from(c, b, 1, (uint64_t)((double)n * q), g0, false);
    b.l20 = c->l20_mask = plan_l20(c, b, P, r20_tiles(b, gr0), n);
    launch_binned_scatter_res(0, b, gr0, 256, s, 0, 0, tiles_of(level_words(n), gr0.tb, b.split ? gr0.ts : 0));
    ev_mark(c, s, "scatter0");
    launch_binned_tile(0, b, gr0, gr.gt, s, true);
    ev_mark(c, s, "tile0");
    fault_dup_record(c, c->list[0], s, b.list20(1));
    run_levels(c, b, P, 1, s);
    return;
  }
  launch_binned_scan(0, b, gr.gs, s);
  ev_mark(c, s, "hscan0");
  launch_binned_scatter(0, b, g0, s);
  ev_mark(c, s, "scatter0");
  launch_binned_tile(0, b, g0, gr.gt, s);
  ev_mark(c, s, "tile0");
  fault_dup_record(c, c->list[0], s);
  enqueue_levels_from(c, b, 1, conservative ? n : (uint64_t)((double)n * q), g0, conservative, s);
}

void set_lds_attrs(s3imph_ctx* c) {
  if (c->lds_attr_set) return;
  // The tile kernels take up to 2 x 64 KiB of dynamic LDS (tiles of 2^19 positions).
  binned_set_lds_limits();
  bm_set_lds_limits();
  c->lds_attr_set = true;
}

// Debug: per-level averages of the tile kernel's phase durations (wall clock, 100 MHz).
void print_tile_profile(s3imph_ctx* c) {
  if (!c->tile_prof) return;
  std::vector<unsigned long long> h((size_t)kMaxLevels * kMaxTiles * 8);
  HIPCHECK(hipMemcpy(h.data(), c->tile_prof, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  {  // level-0 hash waves (k_hash0_pair debug clock, first 8192 waves): total / hash / barrier wait after hash / rest
    const unsigned long long* q = &h[(size_t)(kMaxLevels - 3) * kMaxTiles * 8];  // two rows: 8 words per wave
    double a[5] = {0, 0, 0, 0, 0};
    int cnt = 0;
    for (int w = 0; w < (int)(2 * kMaxTiles * 8 / 8); ++w) {
      if (!q[8 * w]) continue;
      ++cnt;
      for (int k = 0; k < 5; ++k) a[k] += (double)q[8 * w + k];
    }
    if (cnt) {  // wave start / end spread (100 MHz real-time counter)
      std::vector<double> st, en;
      for (int w = 0; w < (int)(2 * kMaxTiles * 8 / 8); ++w)
        if (q[8 * w]) {
          st.push_back((double)q[8 * w + 5]);
          en.push_back((double)q[8 * w + 6]);
        }
      std::sort(st.begin(), st.end());
      std::sort(en.begin(), en.end());
      const double t0 = st[0];
      auto pc = [&](const std::vector<double>& v, double f) { return (v[(size_t)(f * (v.size() - 1))] - t0) / 100.0; };
      {  // by XCD (block % 8) and by block-index decile: mean end (us) and shader clock (MHz)
        const int nw = (int)st.size(), wpb = 4, nb = nw / wpb;  // k_hash0_pair: 4 waves per block
        double xe[8] = {0}, xc[8] = {0}, xn[8] = {0}, de[10] = {0}, dn[10] = {0};
        for (int w = 0; w < (int)(2 * kMaxTiles * 8 / 8); ++w) {
          if (!q[8 * w]) continue;
          const int blk = w / wpb, x = blk % 8, d = std::min(9, blk * 10 / std::max(1, nb));
          const double e = ((double)q[8 * w + 6] - t0) / 100.0;
          xe[x] += e;
          xc[x] += 100.0 * (double)q[8 * w] / (double)q[8 * w + 4];
          xn[x] += 1;
          de[d] += e;
          dn[d] += 1;
        }
        std::fprintf(stderr, "  hash0 by xcd (end us / MHz):");
        for (int x = 0; x < 8; ++x) std::fprintf(stderr, " %.0f/%.0f", xe[x] / std::max(1.0, xn[x]), xc[x] / std::max(1.0, xn[x]));
        std::fprintf(stderr, "\n  hash0 by block decile (end us):");
        for (int d = 0; d < 10; ++d) std::fprintf(stderr, " %.0f", de[d] / std::max(1.0, dn[d]));
        std::fprintf(stderr, "\n");
      }
      std::fprintf(stderr, "  hash0 wave starts (us) p50 %.1f p90 %.1f max %.1f; ends min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n",
                   pc(st, 0.5), pc(st, 0.9), pc(st, 1.0), pc(en, 0.0), pc(en, 0.1), pc(en, 0.5), pc(en, 0.9), pc(en, 1.0));
    }
    if (cnt)
      std::fprintf(stderr,
                   "  hash0 waves %d: avg cycles %.0f (%.1f us, shader clock %.0f MHz), hash %.1f%%, barrier wait "
                   "%.1f%%, rest %.1f%%\n",
                   cnt, a[0] / cnt, a[4] / cnt / 100.0, a[4] ? 100.0 * a[0] / a[4] : 0.0, 100 * a[1] / a[0],
                   100 * a[2] / a[0], 100 * a[3] / a[0]);
    if (cnt) {  // k_hash_skew: q[7] = group sort cycles << 32 | group-end (barrier + write-back) cycles
      double gs = 0, ge = 0;
      for (int w = 0; w < (int)(2 * kMaxTiles * 8 / 8); ++w)
        if (q[8 * w]) {
          gs += (double)(q[8 * w + 7] >> 32);
          ge += (double)(q[8 * w + 7] & 0xffffffffull);
        }
      if (gs + ge > 0)
        std::fprintf(stderr, "  hash_skew groups: sort %.1f%%, end barrier + write-back %.1f%% (wait = chunk loads)\n",
                     100 * gs / a[0], 100 * ge / a[0]);
    }
  }
  {  // k_mid_levels phase stamps: workgroup 0 and the last one, 8 per level
    const unsigned long long* m = &h[(size_t)(kMaxLevels - 4) * kMaxTiles * 8];
    static const char* mn[5] = {"route", "bar1", "own", "bar2", "settle"};
    for (int wg = 0; wg < 2; ++wg)
      for (int li = 0; li < 64; ++li) {
        const unsigned long long* q = m + wg * 512 + li * 8;
        if (!q[0]) break;
        std::fprintf(stderr, "  mid wg%s level+%d:", wg ? "last" : "0", li);
        for (int k = 0; k < 5; ++k) std::fprintf(stderr, " %s %.2f", mn[k], q[k + 1] ? (q[k + 1] - q[k]) / 100.0 : -1.0);
        std::fprintf(stderr, " us\n");
      }
  }
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
                 sc ? "blocks (all rounds)" : "tiles", (hi - lo) / 100.0);
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
  if (64 * level_words(n) > ((uint64_t)kMaxTiles << kTileMaxBits)) {  // level 0 past 4096 tiles of 2^19
    *msg = "build MPHF: more than 2^30 keys on one GPU (level 0 past 2^31 positions): shard them over several GPUs";
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
    if (hash_only_knob()) {
      *msg = "build MPHF: S3IMPH_HASH_ONLY is set (profiling run: level-0 hash only, no index built)";
      return S3IMPH_ERR_INTERNAL;
    }
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
  int rc = map_status(c, st.status, blob, offsets, n, s, msg);
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
// Host-callback transport (s3imph_host_comm): the test harness's collectives (e.g.
// torch.distributed/gloo) on host copies.  Lets several ranks share one GPU.
struct HostComm final : Comm {
  s3imph_host_comm cb{};
  std::vector<uint8_t> hs, hr;
  void d2h(void* h, const void* d, uint64_t bytes, hipStream_t s) {
    if (bytes) HIPCHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
  }
  void h2d(void* d, const void* h, uint64_t bytes, hipStream_t s) {
    if (bytes) HIPCHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
  }
  void allgather(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    hs.resize(bytes + 1);
    hr.resize(bytes * nranks + 1);
    d2h(hs.data(), d_send, bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    if (cb.allgather(cb.user, hs.data(), hr.data(), bytes) != 0) throw Fail{S3IMPH_ERR_RCCL, "host allgather failed"};
    h2d(d_recv, hr.data(), bytes * nranks, s);
    HIPCHECK(hipStreamSynchronize(s));
  }
  void reduce_scatter_u8(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    // block q of this rank's lanes to rank q (the harness's all-to-all), summed here
    std::vector<uint64_t> off(nranks), cnt(nranks, bytes);
    for (int q = 0; q < nranks; ++q) off[q] = (uint64_t)q * bytes;
    hs.resize(bytes * nranks + 1);
    hr.resize(bytes * nranks + 1);
    d2h(hs.data(), d_send, bytes * nranks, s);
    HIPCHECK(hipStreamSynchronize(s));
    if (cb.alltoallv(cb.user, hs.data(), off.data(), cnt.data(), hr.data(), off.data(), cnt.data()) != 0)
      throw Fail{S3IMPH_ERR_RCCL, "host alltoallv failed"};
    std::vector<uint8_t> sum(bytes + 1, 0);
    for (int r = 0; r < nranks; ++r)
      for (uint64_t i = 0; i < bytes; ++i) sum[i] = (uint8_t)(sum[i] + hr[(uint64_t)r * bytes + i]);
    h2d(d_recv, sum.data(), bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
  }
  void allreduce_u64(const unsigned long long* d_in, unsigned long long* d_out, uint64_t count,
                     hipStream_t s) override {
    const uint64_t bytes = 8 * count;
    hs.resize(bytes + 1);
    hr.resize(bytes * nranks + 1);
    d2h(hs.data(), d_in, bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    if (cb.allgather(cb.user, hs.data(), hr.data(), bytes) != 0) throw Fail{S3IMPH_ERR_RCCL, "host allgather failed"};
    std::vector<unsigned long long> sum(count, 0);
    for (int r = 0; r < nranks; ++r)
      for (uint64_t i = 0; i < count; ++i) {
        unsigned long long v;
        std::memcpy(&v, hr.data() + r * bytes + 8 * i, 8);
        sum[i] += v;
      }
    h2d(d_out, sum.data(), bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
  }
  void alltoallv(const void* d_send, const uint64_t* soff, const uint64_t* sbytes, void* d_recv,
                 const uint64_t* roff, const uint64_t* rbytes, hipStream_t s) override {
    std::vector<uint64_t> ps(nranks), pr(nranks);
    uint64_t st = 0, rt = 0;
    for (int q = 0; q < nranks; ++q) {
      ps[q] = st;
      st += sbytes[q];
      pr[q] = rt;
      rt += rbytes[q];
    }
    hs.resize(st + 1);
    hr.resize(rt + 1);
    for (int q = 0; q < nranks; ++q) d2h(hs.data() + ps[q], static_cast<const char*>(d_send) + soff[q], sbytes[q], s);
    HIPCHECK(hipStreamSynchronize(s));
    if (cb.alltoallv(cb.user, hs.data(), ps.data(), sbytes, hr.data(), pr.data(), rbytes) != 0)
      throw Fail{S3IMPH_ERR_RCCL, "host alltoallv failed"};
    for (int q = 0; q < nranks; ++q) h2d(static_cast<char*>(d_recv) + roff[q], hr.data() + pr[q], rbytes[q], s);
    HIPCHECK(hipStreamSynchronize(s));
  }
};

constexpr int kMaxDistLevels = 16;
constexpr uint64_t kSmallWords = 2 * 64 * 64;

void ensure_dist_small(s3imph_ctx* c) {
  DistState& d = c->d;
  if (d.small) return;
  dalloc(d.scnt, kMaxRanks + 1);
  dalloc(d.mat, (uint64_t)(kMaxRanks + 1) * kMaxRanks);
  dalloc(d.gslot, kMaxLevels + 2);
  dalloc(d.small, kSmallWords);
  void* h = nullptr;
  HIPCHECK(hipHostMalloc(&h, sizeof(unsigned long long) * (kSmallWords + 256), hipHostMallocDefault));
  d.h_pinned = static_cast<unsigned long long*>(h);
  if (!c->d_st) dalloc(c->d_st, 1);
  if (!c->h_st) {
    void* hs = nullptr;
    HIPCHECK(hipHostMalloc(&hs, sizeof(LevelState), hipHostMallocDefault));
    c->h_st = static_cast<LevelState*>(hs);
  }
}

// Rank-local checks in front of a collective: every rank learns whether ANY rank failed
// (an all-reduce of per-status flags on stream s), so all of them return at the same point
// instead of the healthy ones blocking in the next collective.  A rank that did not fail
// itself returns the failing ranks' lowest status, saying so.  Scratch: the last 32 words
// of d.small and the 256 spare words of the pinned stage.
int dist_agree(s3imph_ctx* c, int rc, hipStream_t s, std::string* msg) {
  DistState& d = c->d;
  if (d.nranks == 1) return rc;  // nothing to agree on (and no stream drain)
  constexpr int kCodes = 16;
  unsigned long long* h = d.h_pinned + kSmallWords;
  unsigned long long* dv = d.small + kSmallWords - 2 * kCodes;
  std::fill(h, h + kCodes, 0ull);
  if (rc > 0 && rc < kCodes) h[rc] = 1;
  HIPCHECK(hipMemcpyAsync(dv, h, 8 * kCodes, hipMemcpyHostToDevice, s));
  d.comm->allreduce_u64(dv, dv + kCodes, kCodes, s);
  HIPCHECK(hipMemcpyAsync(h, dv + kCodes, 8 * kCodes, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  if (rc > 0) return rc;
  for (int k = 1; k < kCodes; ++k)
    if (h[k]) {
      *msg = "build MPHF: another rank failed (" + std::string(status_name(k)) + ")";
      return k;
    }
  return S3IMPH_OK;
}

// Output entries one rank may need: its share of the positions settles about N/P keys
// (binomial spread), and rank 0 also writes the replicated tail levels.
uint64_t dist_out_cap(const s3imph_ctx* c, uint64_t n_global) {
  const uint64_t P = (uint64_t)c->d.nranks;
  const uint64_t share = (n_global + P - 1) / P;
  return share + share / 16 + 65536 + std::min<uint64_t>(n_global, c->dist_switch + c->dist_switch / 4);
}

// Multi-GPU workspace: records this rank may hold at a distributed level (its received
// share, about N/P, or its own keys), or all records of the first replicated level.
void ensure_dist_workspace(s3imph_ctx* c, uint64_t n_local, uint64_t n_global) {
  DistState& d = c->d;
  const int P = d.nranks;
  ensure_dist_small(c);
  const uint64_t share = std::max<uint64_t>(n_local, (n_global + P - 1) / P);
  const uint64_t capl = std::max<uint64_t>(share + share / 10 + 65536, c->dist_switch + c->dist_switch / 4 + 65536);
  const uint64_t caps = capl + 4096ull * P;
  const uint64_t stagew = level_words(std::max<uint64_t>(n_global, 1)) + 2ull * P + 64;
  const uint64_t capw = cap_words_for(std::max<uint64_t>(n_global, 1024)) + stagew;
  (void)caps;
  if (capl <= d.cap_list && stagew <= d.cap_stage_words && capw <= c->cap_words && c->hist) return;
  // the bucket gets 1.3x the list capacity: reservation slots need headroom over the mean fill
  const uint64_t capb = capl + capl * 3 / 10;
  d.cap_list = d.cap_stage_words = 0;  // set again once every buffer is in place
  c->cap_keys = 0;
  dalloc(c->bucket, capb);
  dalloc(c->list[0], capl);
  dalloc(c->list[1], capl);
  dalloc(c->kh, capl);  // level-0 hashes of this rank's keys (capl >= n_local)
  dalloc(c->fp, capl);
  c->bucket_cap = capb;
  c->cap_keys = capl;
  dalloc(c->hist, kHistCap);
  dalloc(c->hoff, kHistCap);
  dalloc(c->tile_start, kMaxTiles + 2);
  dalloc(c->scan_sums, kHistCap / 2048 + 2);
  dalloc(c->flags, kMaxTiles + 2);
  dalloc(c->sflags, kHistCap / kScanSeg + 2);
  dalloc(c->tcnt, (uint64_t)kResLevels * kTcntStride);
  c->cap_words = capw;
  dalloc(c->bits, capw);
  dfree(c->rank_base);  // the Lookup rank directory: made on the first lookup (ensure_rank_dir)
  c->rank_base_cap = 0;
  c->cap_blocks = (capw + 2047) / 2048 + 1;
  dalloc(c->block_sums, c->cap_blocks);
  // d.send (the routed build's send regions, the replicated gather's staging) is made by
  // the paths that use it (ensure_send): the bitmap decomposition needs only the gather's
  dalloc(d.stage_bits, stagew);
  d.cap_list = capl;
  d.cap_stage_words = stagew;
}


constexpr int kDistRetry = -1;
// the bitmap decomposition missed a capacity, not a size bound (a reservation slot overflow,
// a fed level whose P0 buffers could not be had, a tail geometry miss): rerun it once in its
// conservative form (no settle-fed levels, no list levels through P0) before routing
constexpr int kDistRetryBm = -2;
constexpr uint64_t kChunkedRoute0Keys = 8ull << 20;  // sharded level 0 of this many keys per rank (N / P): 4 chunks
constexpr int kRoute0Chunks = 4;

// Level 0 of the sharded build in K key chunks: chunk c is hashed and routed on the build
// stream s while chunk c-1's records cross xGMI on the exchange stream d.xs, so the
// level-0 all-to-all hides behind the hash instead of following it.  Records for a peer
// go to its send region in chunk order (scnt keeps counting across chunks); this rank's
// own records of chunk c land in list[1] right after everything received for chunks < c
// (self_dst = lin + received so far), and chunk c's received records follow them.  On
// return, M holds the cumulative gathered counts, the exchanges are complete on s, and
// *recv_total is the level's record count on this rank.  Per-chunk counts need one host
// round trip each, taken while the next chunk is hashed.  Returns kDistRetry when a send
// region overflowed (the caller reruns on the conservative, unchunked path).
int route0_chunked(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                   uint64_t n_local, uint64_t key_base, uint64_t N, const BinBuffers& b, uint64_t C, Rec* lin,
                   hipStream_t s, unsigned long long* M, uint64_t* recv_total) {
  DistState& d = c->d;
  Comm& cm = *d.comm;
  const int P = d.nranks, R = d.rank;
  LevelState* st = c->d_st;
  if (!d.xs) {
    HIPCHECK(hipStreamCreateWithFlags(&d.xs, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&d.ev_route, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&d.ev_counts, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&d.ev_x, hipEventDisableTiming));
  }
  const int K = kRoute0Chunks;
  d.agree_msg.clear();
  const uint64_t per = (n_local + K - 1) / K;
  const LevelGeom gh = choose_geom_sz(n_local, 64 * level_words(N), kTargetTiles0, chunks0(n_local), kTileMaxBits);
  HIPCHECK(hipMemsetAsync(d.scnt, 0, 8ull * (P + 1), s));
  std::vector<unsigned long long> prev((size_t)(P + 1) * P, 0);
  std::vector<uint64_t> sbytes(P), soff(P), rbytes(P), roff(P);
  uint64_t received = 0;  // records received from peers in chunks < k
  // Build stream: chunk k hashed and routed in one pass; its own records land past
  // everything received for chunks < k, which the kernel reads from the previous gather
  // (d.mat), so it waits for that gather (a few us), not for the exchange it feeds, and is
  // enqueued before the host blocks on the previous chunk's counts.
  auto enqueue_build = [&](int k) {
    const uint64_t k0 = std::min(n_local, (uint64_t)k * per), k1 = std::min(n_local, k0 + per);
    if (k) HIPCHECK(hipStreamWaitEvent(s, d.ev_x, 0));  // chunk k-1's counts gathered: d.mat, scnt free
    if (k1 > k0) {
      BinBuffers bc = b;
      bc.kh = c->kh + k0;
      bc.fp = c->fp + k0;
      const Route0 rt{pos ? pos + k0 : nullptr, key_base + k0, d.send, C, d.scnt, lin, d.cap_list,
                      k ? d.mat : nullptr, P, R};
      launch_hash0_route(blob, offsets + k0, k1 - k0, bc, gh, level_grids(k1 - k0, 64 * level_words(N), gh).gc, rt, s);
    }
    launch_route_flag(st, d.scnt, P, s);
    HIPCHECK(hipEventRecord(d.ev_route, s));
  };
  // Exchange stream: gather chunk k's cumulative counts, then to the host.
  auto enqueue_gather = [&]() {
    HIPCHECK(hipStreamWaitEvent(d.xs, d.ev_route, 0));
    cm.allgather(d.scnt, d.mat, 8ull * (P + 1), d.xs);
    HIPCHECK(hipEventRecord(d.ev_x, d.xs));
    HIPCHECK(hipMemcpyAsync(M, d.mat, 8ull * (P + 1) * P, hipMemcpyDeviceToHost, d.xs));
    HIPCHECK(hipEventRecord(d.ev_counts, d.xs));
  };
  enqueue_build(0);
  enqueue_gather();
  for (int k = 0; k < K; ++k) {
    if (k + 1 < K) enqueue_build(k + 1);  // the build stream keeps hashing while the counts travel
    HIPCHECK(hipEventSynchronize(d.ev_counts));
    bool over = false;
    for (int r = 0; r < P; ++r) over |= M[(uint64_t)r * (P + 1) + P] != 0;
    if (over) {  // every rank sees the same flags: all return, after draining the exchange stream
      HIPCHECK(hipStreamSynchronize(d.xs));
      HIPCHECK(hipStreamSynchronize(s));
      return kDistRetry;
    }
    // chunk k: this rank's own records sit at [self_before + received, self_now + received);
    // the peers' records of chunk k follow them
    auto at = [&](const unsigned long long* m, int r, int t) { return m[(uint64_t)r * (P + 1) + t]; };
    uint64_t acc = (at(M, R, R) + received) * sizeof(Rec);
    uint64_t got = 0;
    for (int t = 0; t < P; ++t) {
      const uint64_t sn = at(M, R, t) - at(prev.data(), R, t), rn = at(M, t, R) - at(prev.data(), t, R);
      soff[t] = ((uint64_t)t * C + at(prev.data(), R, t)) * sizeof(Rec);
      sbytes[t] = t == R ? 0 : sn * sizeof(Rec);
      roff[t] = t == R ? 0 : acc;
      rbytes[t] = t == R ? 0 : rn * sizeof(Rec);
      if (t != R) {
        acc += rbytes[t];
        got += rn;
      }
    }
    {  // a local capacity check: agreed on the exchange stream before its all-to-all
      const int rc = dist_agree(c, at(M, R, R) + received + got > d.cap_list ? S3IMPH_ERR_NOMEM : S3IMPH_OK, d.xs,
                                &d.agree_msg);
      if (rc != S3IMPH_OK) {
        HIPCHECK(hipStreamSynchronize(s));
        return rc;
      }
    }
    cm.alltoallv(d.send, soff.data(), sbytes.data(), lin, roff.data(), rbytes.data(), d.xs);
    received += got;
    std::copy(M, M + (size_t)(P + 1) * P, prev.begin());
    if (k + 1 < K) enqueue_gather();
  }
  ev_mark(c, s, "hash_route0");
  HIPCHECK(hipEventRecord(d.ev_x, d.xs));
  HIPCHECK(hipStreamWaitEvent(s, d.ev_x, 0));  // level 0's pipeline reads the received records
  *recv_total = M[(uint64_t)R * (P + 1) + R] + received;
  if (c->debug)
    std::fprintf(stderr, "[s3imph] rank %d: level 0 exchanged in %d chunks (%llu records)\n", R, K,
                 (unsigned long long)*recv_total);
  return S3IMPH_OK;
}

// kStTooManyLevels on a sharded build, decided on every rank together (the flags are
// gathered, so every rank calls this): each rank's leftover duplicate hash values (at most
// 32) are all-gathered, every rank counts them among its ORIGINAL key hashes (recomputed),
// and the counts are summed over ranks.  DUP_KEY_HASH only if some value occurs twice among
// the original keys; leftovers with equal hashes otherwise are an internal fault.
int dist_classify_stop(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, uint64_t n_local, hipStream_t s,
                       std::string* msg) {
  DistState& d = c->d;
  Comm& cm = *d.comm;
  const int P = d.nranks;
  constexpr int kCand = 32;
  const LevelState& hs = *c->h_st;
  const unsigned nl = hs.stop_level ? hs.stop_level : hs.nlevels;
  const uint64_t rem = nl >= 1 && nl < (unsigned)kMaxLevels + 2 ? hs.n[nl] : 0;
  // (a bitmap level's list may be R20: c->l20_mask is the attempt's mask, as for one GPU)
  const bool r20 = nl < 32 && ((c->l20_mask >> nl) & 1u);
  const std::vector<uint64_t> mine =
      rem ? record_dup_values(c->list[(nl - 1) & 1], rem, kCand, r20) : std::vector<uint64_t>{};
  unsigned long long* M = d.h_pinned;
  std::fill(M, M + kCand + 1, 0ull);
  M[0] = mine.size();
  std::copy(mine.begin(), mine.end(), M + 1);
  HIPCHECK(hipMemcpyAsync(d.small, M, 8ull * (kCand + 1), hipMemcpyHostToDevice, s));
  cm.allgather(d.small, d.small + 64, 8ull * (kCand + 1), s);
  HIPCHECK(hipMemcpyAsync(M, d.small + 64, 8ull * (kCand + 1) * P, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  std::vector<uint64_t> u;
  for (int r = 0; r < P; ++r) {
    const unsigned long long* row = M + (uint64_t)r * (kCand + 1);
    for (uint64_t i = 0; i < std::min<uint64_t>(row[0], kCand); ++i) u.push_back(row[1 + i]);
  }
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  if (u.empty()) {
    *msg = "build MPHF: can't find minimal perfect hash after " + std::to_string(kMaxLevels) + " levels";
    return S3IMPH_ERR_TOO_MANY_LEVELS;
  }
  // the leftover records hold the key hash itself, or (left by the single-workgroup tail)
  // mix64 of it — a bijection, so both forms are counted, each summed over the ranks
  const std::vector<uint64_t> orig = original_key_hashes(c, blob, offsets, n_local, s);
  std::vector<uint64_t> mixed(orig.size());
  for (size_t i = 0; i < orig.size(); ++i) mixed[i] = mix64(orig[i]);
  std::sort(mixed.begin(), mixed.end());
  const size_t U = u.size();
  std::vector<unsigned long long> cnt(2 * U, 0);
  for (size_t i = 0; i < U; ++i) {
    const auto r = std::equal_range(orig.begin(), orig.end(), u[i]);
    const auto m = std::equal_range(mixed.begin(), mixed.end(), u[i]);
    cnt[i] = (unsigned long long)(r.second - r.first);
    cnt[U + i] = (unsigned long long)(m.second - m.first);
  }
  unsigned long long* ds = nullptr;  // error path only: a scratch of its own (2 |u| <= 4096 entries each way)
  dalloc(ds, 4 * U);
  struct Free {
    unsigned long long*& p;
    ~Free() { dfree(p); }
  } free_ds{ds};
  HIPCHECK(hipMemcpyAsync(ds, cnt.data(), 8 * cnt.size(), hipMemcpyHostToDevice, s));
  cm.allreduce_u64(ds, ds + 2 * U, cnt.size(), s);
  if (c->debug)
    for (size_t i = 0; i < U; ++i)
      std::fprintf(stderr, "[s3imph] rank %d stop level %u: leftover hash %016llx occurs %llu (raw) / %llu (mixed) "
                   "times in %llu local keys\n", d.rank, nl, (unsigned long long)u[i], cnt[i], cnt[U + i],
                   (unsigned long long)n_local);
  HIPCHECK(hipMemcpyAsync(cnt.data(), ds + 2 * U, 8 * cnt.size(), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  for (unsigned long long v : cnt)
    if (v >= 2) {
      *msg = "build MPHF: duplicate FNV-1a key hashes: bbhash cannot place them";
      return S3IMPH_ERR_DUP_KEY_HASH;
    }
  *msg = "build MPHF: internal error: level " + std::to_string(nl) +
         " holds records with equal key hashes although every key hash is distinct (a record was duplicated)";
  return S3IMPH_ERR_INTERNAL;
}

// One attempt of the multi-GPU build (see s3imph_dist.hip for the decomposition).
// `conservative` runs every level on the counted path and the replicated levels with
// one geometry; every rank takes the same branches (all decisions use global counts).
int dist_attempt(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                 uint64_t n_local, uint64_t key_base, uint64_t N, uint64_t* fp_out, uint64_t* pos_out,
                 uint64_t out_cap, hipStream_t s, bool conservative, s3imph_build_info* info, std::string* msg) {
  DistState& d = c->d;
  Comm& cm = *d.comm;
  const int P = d.nranks, R = d.rank;
  {  // the send regions (ensure_dist_workspace leaves them to the routed build)
    const uint64_t caps = d.cap_list + 4096ull * P;
    if (caps > d.cap_send) {
      d.cap_send = 0;
      dalloc(d.send, caps);
      d.cap_send = caps;
    }
  }
  LevelState* st = c->d_st;
  const BinBuffers b = make_bufs(c, nullptr, fp_out, pos_out, s);
  // Distributed levels keep their input in list[1] and their collided records in list[0]:
  // the route of level L reads list[0] and writes this rank's own records straight into
  // list[1] (no exchange copy), the received ones after them.  The tile pipeline reads
  // level L from list[(L-1)&1] and writes redo to list[L&1], so odd levels see the two
  // buffers swapped.
  BinBuffers bsw = b;
  std::swap(bsw.list[0], bsw.list[1]);
  Rec* const lin = c->list[1];
  Rec* const lredo = c->list[0];
  Rec* redo = lredo;  // where the last level's collided records are (one rank: ping-pong)
  // one rank routes nothing (S3IMPH_DIST_ROUTE_SELF: route anyway, so tests drive the routed
  // kernels and the RCCL exchange with nranks = 1)
  const bool one = P == 1 && !c->route_self;
  const double q = 1.0 - std::exp(-0.5);
  launch_init_state(st, n_local, out_cap, s, n_local ? offsets : nullptr);  // samples key lengths (st->skew)
  HIPCHECK(hipMemsetAsync(c->tcnt, 0, (size_t)kResLevels * kTcntStride * sizeof(unsigned), s));
  launch_dist_setup(st, 0, nullptr, N, R, P, s);
  ev_mark(c, s, "init");
  // level 0's key hashes and fingerprints, once (the routing below may be retried); a big
  // sharded level 0 hashes chunk by chunk inside route0_chunked instead
  // (decided from global values only: every rank must issue the same collectives)
  const bool chunked = !conservative && P > 1 && N / (uint64_t)P >= kChunkedRoute0Keys;
  const LevelGeom gh0 = choose_geom_sz(std::max<uint64_t>(n_local, 1), 64 * level_words(N), kTargetTiles0,
                                       chunks0(std::max<uint64_t>(n_local, 1)), kTileMaxBits);
  const int gc0 = level_grids(std::max<uint64_t>(n_local, 1), 64 * level_words(N), gh0).gc;
  bool have_kh = false;  // kh / fp written (a retried level-0 route reads them)
  std::vector<uint64_t> sbytes(P), soff(P), rbytes(P), roff(P);
  double src_pred = (double)n_local;  // records this rank routes at the current level
  unsigned long long* M = d.h_pinned;  // (P + 1) x P gathered counts, row r = rank r's [scnt, overflow]
  int L = 0;
  for (;;) {
    // ---- routed levels >= 1 with device-side counts: every (sender, owner) region has a
    // fixed size C derived from N alone (identical on every rank), the route pads each
    // region's unused tail with k = 0 records that the reservation scatter skips, and the
    // regions are exchanged whole, so no count crosses to the host until the build ends.
    // A region that overflows sets kStRouteOverflow and the attempt reruns on the
    // host-counted path (conservative).
    if (L >= 1 && !conservative) {
      const double mean_l = (double)N * std::pow(q, L);           // level L's global keys
      const double pair = mean_l / ((double)P * P);                // records per (sender, owner)
      const uint64_t Cf = (uint64_t)std::ceil(pair * 1.03 + 8.0 * std::sqrt(pair)) + 1024;
      const uint64_t list_n = (uint64_t)P * Cf;
      const uint64_t wpred = level_words((uint64_t)(mean_l * 1.02 + 6.0 * std::sqrt(mean_l)) + 1024);
      const uint64_t Spred = (wpred + P - 1) / P;
      const bool dev = list_n <= d.cap_list && list_n <= c->res_max_keys && L < kResLevels &&
                       res_fits(c, list_n, 64 * Spred);
      if (dev && one) {
        // one rank: every record is its own, so nothing is routed — the level reads the
        // previous level's collided records where they lie and writes its own to the other
        // list (the single-GPU ping-pong)
        Rec* const other = redo == c->list[0] ? c->list[1] : c->list[0];
        BinBuffers bp = b;
        bp.list[(L - 1) & 1] = redo;
        bp.list[L & 1] = other;
        ev_mark(c, s, "route");
        enqueue_list_level(c, bp, L, (uint64_t)(mean_l * 1.02 + 6.0 * std::sqrt(mean_l)) + 1024, 64 * Spred, false,
                           nullptr, s, false);
        ev_mark(c, s, "levels");
        redo = other;
        cm.allreduce_u64(&st->n[L + 1], d.gslot + L + 1, 1, s);
        if (L + 1 >= kMaxDistLevels || mean_l * q <= (double)c->dist_switch) break;
        ++L;
        launch_dist_setup(st, L, d.gslot + L, 0, R, P, s);
        continue;
      }
      if (dev) {
        if (list_n > d.cap_send) {
          HIPCHECK(hipStreamSynchronize(s));
          dalloc(d.send, list_n);
          d.cap_send = list_n;
        }
        HIPCHECK(hipMemsetAsync(d.scnt, 0, 8ull * (P + 1), s));
        Rec* const own = lin + (uint64_t)R * Cf;
        launch_route(L, lredo, (uint64_t)(mean_l / P * 1.05) + 4096, d.send, Cf, d.scnt, st, P, R, own, Cf, s);
        launch_route_pad(d.send, Cf, d.scnt, P, R, own, s);
        for (int t = 0; t < P; ++t) {
          soff[t] = roff[t] = (uint64_t)t * Cf * sizeof(Rec);
          sbytes[t] = rbytes[t] = t == R ? 0 : Cf * sizeof(Rec);
        }
        if (P > 1) cm.alltoallv(d.send, soff.data(), sbytes.data(), lin, roff.data(), rbytes.data(), s);
        launch_set_u64(&st->n[L], list_n, s);  // the list's length, padding included
        ev_mark(c, s, "route");
        BinBuffers bp = (L & 1) ? bsw : b;
        bp.padded = true;
        enqueue_list_level(c, bp, L, list_n, 64 * Spred, false, nullptr, s, false);
        ev_mark(c, s, "levels");
        cm.allreduce_u64(&st->n[L + 1], d.gslot + L + 1, 1, s);
        if (L + 1 >= kMaxDistLevels || mean_l * q <= (double)c->dist_switch) break;
        ++L;
        launch_dist_setup(st, L, d.gslot + L, 0, R, P, s);
        continue;
      }
    }
    if (L == 0 && one && !conservative && n_local) {
      // one rank: level 0 is the single-GPU level 0 (nothing to route) — the pair-round hash
      // into kh / fp, the reservation scatter from them (20-byte records when positions are
      // identities), the tile kernels writing outputs and collided records (into lredo)
      const LevelGeom g0 = choose_geom(n_local, kTargetTiles0, chunks0(n_local), kRegTileMaxBits);
      const uint64_t T0 = tiles_of(level_words(N), g0.tb, 0);
      if (N == n_local && T0 <= kScatterTiles && c->res0 && res_fits(c, n_local, 64 * level_words(N), T0)) {
        BinBuffers b0 = b;
        b0.dist = false;
        b0.pos = pos;
        b0.pos_base = key_base;
        launch_hash0_only(blob, offsets, n_local, b0, gh0, gc0, s);
        ev_mark(c, s, "hash_count0");
        LevelGeom gr0 = g0;
        if (b0.split && g0.tb > kRegTileMaxBits && g0.tb <= kSplitMaxBits) gr0.ts = choose_split_ts(64 * level_words(N), true);
        launch_binned_scatter_res(0, b0, gr0, 256, s, 0, 0, tiles_of(level_words(N), gr0.tb, b0.split ? gr0.ts : 0));
        launch_binned_tile(0, b0, gr0, level_grids(n_local, 64 * level_words(N), g0).gt, s, true);
        ev_mark(c, s, "level0");
        cm.allreduce_u64(&st->n[1], d.gslot + 1, 1, s);
        src_pred = (double)n_local * q * 1.05 + 1024;
        if (1 >= kMaxDistLevels || (double)N * q <= (double)c->dist_switch) break;
        ++L;
        launch_dist_setup(st, L, d.gslot + L, 0, R, P, s);
        continue;
      }
    }
    if (redo != lredo) {  // a one-rank level ping-ponged before this host-counted one: the route reads lredo
      HIPCHECK(hipStreamSynchronize(s));
      unsigned long long nr = 0;
      HIPCHECK(hipMemcpy(&nr, &st->n[L], 8, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpyAsync(lredo, redo, nr * sizeof(Rec), hipMemcpyDeviceToDevice, s));
      redo = lredo;
    }
    // ---- route level L's records to their owners
    uint64_t C = (uint64_t)(src_pred / P * 1.15) + 4096;
    uint64_t m_chunked = 0;
    if (L == 0 && chunked) {
      if ((uint64_t)P * C > d.cap_send) {
        HIPCHECK(hipStreamSynchronize(s));
        dalloc(d.send, (uint64_t)P * C);
        d.cap_send = (uint64_t)P * C;
      }
      const int rc = route0_chunked(c, blob, offsets, pos, n_local, key_base, N, b, C, lin, s, M, &m_chunked);
      if (rc != S3IMPH_OK) {
        if (rc == S3IMPH_ERR_NOMEM) *msg = "build MPHF: rank " + std::to_string(R) + " received too many records";
        if (rc > 0 && !d.agree_msg.empty()) *msg = d.agree_msg;
        return rc;
      }
    }
    for (int tries = 0; !(L == 0 && chunked); ++tries) {
      if ((uint64_t)P * C > d.cap_send) {
        HIPCHECK(hipStreamSynchronize(s));
        dalloc(d.send, (uint64_t)P * C);
        d.cap_send = (uint64_t)P * C;
      }
      HIPCHECK(hipMemsetAsync(d.scnt, 0, 8ull * (P + 1), s));
      if (L == 0 && tries == 0) {  // hash + route in one pass
        if (n_local) {
          const Route0 rt{pos, key_base, d.send, C, d.scnt, lin, d.cap_list, nullptr, P, R};
          launch_hash0_route(blob, offsets, n_local, b, gh0, gc0, rt, s);
        }
        ev_mark(c, s, "hash_route0");
      } else if (L == 0) {  // a retry routes from kh / fp (hashed once)
        if (n_local && !have_kh) launch_hash0_only(blob, offsets, n_local, b, gh0, gc0, s);
        have_kh = true;
        launch_route0_arrays(c->kh, c->fp, pos, key_base, n_local, d.send, C, d.scnt, st, P, R, lin, d.cap_list, s);
      } else
        launch_route(L, lredo, (uint64_t)src_pred, d.send, C, d.scnt, st, P, R, lin, d.cap_list, s);
      launch_route_flag(st, d.scnt, P, s);
      cm.allgather(d.scnt, d.mat, 8ull * (P + 1), s);
      HIPCHECK(hipMemcpyAsync(M, d.mat, 8ull * (P + 1) * P, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      bool over = false;
      uint64_t need = 0;
      for (int r = 0; r < P; ++r) over |= M[(uint64_t)r * (P + 1) + P] != 0;
      for (int t = 0; t < P; ++t) need = std::max<uint64_t>(need, M[(uint64_t)R * (P + 1) + t]);
      if (!over) break;
      if (tries >= 3) {
        *msg = "build MPHF: route regions keep overflowing";
        return S3IMPH_ERR_INTERNAL;
      }
      C = need + need / 8 + 4096;
    }
    uint64_t nL = 0, m = 0;
    for (int r = 0; r < P; ++r)
      for (int t = 0; t < P; ++t) nL += M[(uint64_t)r * (P + 1) + t];
    for (int r = 0; r < P; ++r) m += M[(uint64_t)r * (P + 1) + R];
    const uint64_t w = level_words(nL), S = (w + P - 1) / P;
    const uint64_t lo = std::min<uint64_t>((uint64_t)R * S, w), rw = std::min<uint64_t>(S, w - lo);
    {  // rank-local checks, agreed before the exchange
      int lrc = S3IMPH_OK;
      if (m > d.cap_list) {
        *msg = "build MPHF: rank " + std::to_string(R) + " received " + std::to_string(m) + " records (capacity " +
               std::to_string(d.cap_list) + ")";
        lrc = S3IMPH_ERR_NOMEM;
      } else if (L == 0 && chunked && m_chunked != m) {
        *msg = "build MPHF: internal error: chunked level-0 exchange received " + std::to_string(m_chunked) +
               " of " + std::to_string(m) + " records";
        lrc = S3IMPH_ERR_INTERNAL;
      }
      const int rc = dist_agree(c, lrc, s, msg);
      if (rc != S3IMPH_OK) return rc;
    }
    // ---- exchange: the received records follow this rank's own ones in list[1]
    if (!(L == 0 && chunked)) {
      uint64_t acc = M[(uint64_t)R * (P + 1) + R] * sizeof(Rec);
      for (int t = 0; t < P; ++t) {
        soff[t] = (uint64_t)t * C * sizeof(Rec);
        sbytes[t] = t == R ? 0 : M[(uint64_t)R * (P + 1) + t] * sizeof(Rec);
        roff[t] = t == R ? 0 : acc;
        rbytes[t] = t == R ? 0 : M[(uint64_t)t * (P + 1) + R] * sizeof(Rec);
        acc += rbytes[t];
      }
      cm.alltoallv(d.send, soff.data(), sbytes.data(), lin, roff.data(), rbytes.data(), s);
    }
    launch_set_u64(&st->n[L], m, s);
    ev_mark(c, s, L == 0 ? "route0" : "route");
    // ---- the owner's tile pipeline over positions [64 lo, 64 (lo + rw))
    enqueue_list_level(c, (L & 1) ? bsw : b, L, m, 64 * rw, conservative, nullptr, s, true);
    ev_mark(c, s, L == 0 ? "level0" : "levels");
    // ---- size the next level from the global redo count (device side, no host sync)
    cm.allreduce_u64(&st->n[L + 1], d.gslot + L + 1, 1, s);
    src_pred = (double)m * q * 1.05 + 1024;
    if (L + 1 >= kMaxDistLevels || (double)nL * q <= (double)c->dist_switch) break;
    ++L;
    launch_dist_setup(st, L, d.gslot + L, 0, R, P, s);
  }
  const int Ls = L + 1;  // first replicated level
  // ---- gather every rank's remaining records; all ranks finish the build identically
  HIPCHECK(hipMemcpyAsync(d.small, &st->n[Ls], 8, hipMemcpyDeviceToDevice, s));
  cm.allgather(d.small, d.small + 64, 8, s);
  HIPCHECK(hipMemcpyAsync(M, d.small + 64, 8ull * P, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  uint64_t total = 0, maxc = 0;
  std::vector<uint64_t> cnt(M, M + P);
  for (int r = 0; r < P; ++r) {
    total += cnt[r];
    maxc = std::max(maxc, cnt[r]);
  }
  {  // the list capacity is per rank (it follows n_local): agreed before the gather
    int lrc = S3IMPH_OK;
    if (total > d.cap_list) {
      *msg = "build MPHF: replicated level of " + std::to_string(total) + " records exceeds the workspace";
      lrc = S3IMPH_ERR_NOMEM;
    }
    const int rc = dist_agree(c, lrc, s, msg);
    if (rc != S3IMPH_OK) return rc;
  }
  Rec* rl = c->list[(Ls - 1) & 1];
  if (total) {
    if ((uint64_t)P * maxc > d.cap_send) {
      dalloc(d.send, (uint64_t)P * maxc);
      d.cap_send = (uint64_t)P * maxc;
    }
    cm.allgather(redo, d.send, maxc * sizeof(Rec), s);
    uint64_t o = 0;
    for (int r = 0; r < P; ++r) {
      if (cnt[r])
        HIPCHECK(hipMemcpyAsync(rl + o, d.send + (uint64_t)r * maxc, cnt[r] * sizeof(Rec), hipMemcpyDeviceToDevice, s));
      o += cnt[r];
    }
  }
  if (total >= 2) fault_dup_record(c, rl, s);
  launch_dist_replicate(st, Ls, total, R == 0 ? 0 : (uint64_t)Ls, s);
  ev_mark(c, s, "gather");
  const LevelGeom gcons = choose_geom(std::max<uint64_t>(total, 1), kTargetTiles, kTargetChunks, kRegTileMaxBits);
  enqueue_levels_from(c, b, Ls, total, gcons, conservative, s);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpyAsync(c->h_st, st, sizeof(LevelState), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  // ---- level bit vectors of the distributed levels: all-gather each rank's word range
  // (level sizes from the device state: the routed levels >= 1 never sent them to the host)
  {
    uint64_t woff = 0;
    for (int l = 0; l < Ls; ++l) {
      const uint64_t w = c->h_st->words[l], S = (w + P - 1) / P;
      if (w > d.cap_stage_words || (uint64_t)P * S > d.cap_stage_words) {
        *msg = "build MPHF: internal error: level " + std::to_string(l) + " of " + std::to_string(w) +
               " words exceeds the bit-vector stage";
        return S3IMPH_ERR_INTERNAL;
      }
      cm.allgather(c->bits + woff + (uint64_t)R * S, d.stage_bits, S * 8, s);
      HIPCHECK(hipMemcpyAsync(c->bits + woff, d.stage_bits, w * 8, hipMemcpyDeviceToDevice, s));
      woff += w;
    }
  }
  ev_mark(c, s, "bits");
  // ---- per-rank level bases, totals and flags -> this rank's output segments
  const LevelState& hs = *c->h_st;
  const int K = Ls + 3;
  for (int l = 0; l <= Ls; ++l) M[l] = hs.lvl_base[l];
  M[Ls + 1] = hs.rank_total;
  M[Ls + 2] = hs.status;
  HIPCHECK(hipMemcpyAsync(d.small, M, 8ull * K, hipMemcpyHostToDevice, s));
  cm.allgather(d.small, d.small + 64, 8ull * K, s);
  HIPCHECK(hipMemcpyAsync(M, d.small + 64, 8ull * K * P, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  ev_collect(c);
  auto lb = [&](int r, int l) { return M[(uint64_t)r * K + l]; };
  unsigned flags = 0;
  for (int r = 0; r < P; ++r) flags |= (unsigned)lb(r, Ls + 2);
  if (flags & (kStGeometry | kStTailOverflow | kStResOverflow | kStRouteOverflow)) return conservative ? S3IMPH_ERR_INTERNAL : kDistRetry;
  if (flags & kStTooManyLevels) return dist_classify_stop(c, blob, offsets, n_local, s, msg);
  if (flags & kStKeyZero) {
    *msg = "MPHF Key(...) returned 0, possible hash collision with sentinel";
    return S3IMPH_ERR_KEY_HASH_ZERO;
  }
  if (flags) {
    *msg = "build MPHF: internal error (device flags " + std::to_string(flags) + ")";
    return S3IMPH_ERR_INTERNAL;
  }
  d.seg.clear();
  uint64_t G = 0;
  for (int l = 0; l < Ls; ++l) {
    uint64_t before = 0, tot = 0;
    for (int r = 0; r < P; ++r) {
      const uint64_t cl = lb(r, l + 1) - lb(r, l);
      if (r < R) before += cl;
      tot += cl;
    }
    const uint64_t mine = lb(R, l + 1) - lb(R, l);
    if (mine) d.seg.insert(d.seg.end(), {G + before, mine, lb(R, l)});
    G += tot;
  }
  const uint64_t rep = lb(0, Ls + 1) - lb(0, Ls);  // replicated levels, written by rank 0
  if (R == 0 && rep) d.seg.insert(d.seg.end(), {G, rep, lb(0, Ls)});
  G += rep;
  if (G != N) {
    *msg = "build MPHF: internal error: ranked " + std::to_string(G) + " of " + std::to_string(N) + " keys";
    return S3IMPH_ERR_INTERNAL;
  }
  d.out_n = R == 0 ? lb(0, Ls + 1) : lb(R, Ls);
  info->status = S3IMPH_OK;
  info->num_levels = hs.nlevels;
  info->total_words = hs.woff[hs.nlevels];
  info->mph_bin_len = 8 * kPartitions + 8 + 8ull * hs.nlevels + 8ull * info->total_words;
  info->big_levels = (uint64_t)Ls;
  return S3IMPH_OK;
}

// ------------------------------------------------------- bitmap decomposition ----
// The north_star's multi-GPU build (s3imph_bitmap.hip): per distributed level, local
// count lanes -> reduce-scatter -> final bits of this rank's slice -> all-gather -> every
// rank settles its own records; then the replicated tail as in the routed build, and one
// all-to-all of the settled (p, fp, pos) triples to the owners of the output slices.

void ensure_bm_workspace(s3imph_ctx* c, uint64_t N) {
  DistState& d = c->d;
  const uint64_t P = (uint64_t)d.nranks;
  const uint64_t w0 = level_words(N), S = (w0 + P - 1) / P, wpad = S * P;
  if (d.bm_cap_out < d.cap_list) {  // a rank settles at most the records it holds (<= its list capacity)
    d.bm_cap_out = 0;
    dalloc(d.bm_out, d.cap_list);
    d.bm_cap_out = d.cap_list;
  }
  if (wpad <= d.bm_cap_words && d.bm_a) return;
  d.bm_cap_words = 0;  // set again once every buffer is in place
  dalloc(d.bm_a, wpad);
  dalloc(d.bm_g, wpad);
  dalloc(d.bm_dec, S);
  dalloc(d.bm_lanes, (c->bm_counts ? 64 : 16) * wpad);  // count bytes (64 per word), or the (A, C) planes (16)
  dalloc(d.bm_slice, 64 * S);
  dalloc(d.bm_recv, 16 * wpad);   // the planes' all-to-all: P slices of 2 S words
  if (!d.bm_tsum) dalloc(d.bm_tsum, kBmMaxTiles);
  if (!d.bm_tbase) dalloc(d.bm_tbase, 2 * kBmMaxTiles);
  d.bm_cap_words = wpad;
}

void free_bm_workspace(DistState& d) {
  if (d.xo) (void)hipStreamSynchronize(d.xo);  // (a level group's exchange reads these buffers)
  dfree(d.xrecv);
  dfree(d.xch);
  d.cap_xrecv = 0;
  dfree(d.bm_a); dfree(d.bm_g); dfree(d.bm_dec);
  dfree(d.bm_lanes); dfree(d.bm_slice); dfree(d.bm_recv); dfree(d.bm_tsum); dfree(d.bm_tbase);
  dfree(d.bm_out);
  dfree(d.bm_bnd);
  d.bm_bnd_cap = 0;
  d.bm_cap_words = 0;
  d.bm_cap_out = 0;
}

// Tile count a bitmap level aims at (A/B knob S3IMPH_BM_TILES).  Fewer, larger tiles suit
// the reservation scatter (C3 level 0: 3052 tiles of 2^16 take its 4096-tile form, 1.66 ms;
// 763 of 2^18 the 1024-tile form, 0.99 ms) but not the settle, whose random writes by rank
// spread over a 4x larger window per tile (1.88 -> 3.64 ms).
// Tile bits at which a rank holds ~8k records of a bitmap level's tile (2^14 at one rank, as a
// single GPU's register tile): 14 + floor(lg P), at most kBmP0MaxTb
// The bitmap settle partitioning the next level's records into its super-tile regions
// (NextPart; A/B knob S3IMPH_BM_FEED=0: the partition pass over the list instead)
bool bm_feed_next() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_BM_FEED");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}

unsigned bm_dense_tb(int P) {
  static const unsigned base = [] {  // A/B knob S3IMPH_BM_DENSE: the tile bits at one rank (14)
    const char* e = dev_env("S3IMPH_BM_DENSE");
    return e ? (unsigned)std::max(13, std::min(16, std::atoi(e))) : kBmMinTb;
  }();
  unsigned tb = base;
  for (int q = 2; q <= P && tb < kBmP0MaxTb; q *= 2) ++tb;
  return std::max(tb, kBmMinTb);
}

uint64_t bm_target_tiles() {
  static const uint64_t v = [] {
    const char* e = dev_env("S3IMPH_BM_TILES");
    return e ? std::max<uint64_t>(64, std::strtoull(e, nullptr, 10)) : kScatterTiles;
  }();
  return v;
}

// The bitmap decomposition's output exchange by level group: levels 0 and 1 each
// leave once settled, beside the next levels (S3IMPH_XCH_LEVELS=0: one exchange at the end, as
// before round 6; A/B knob).  S3IMPH_XCH_STREAM=1 (test knob) puts the host-side transports'
// exchanges on the exchange stream too (RCCL with a split communicator always does).
bool xch_levels_on() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_XCH_LEVELS");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}
bool xch_stream_knob() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_XCH_STREAM");
    return e && std::atoi(e) != 0;
  }();
  return v;
}
constexpr int kXchGroups = 3;  // level 0, level 1, the rest
constexpr uint64_t kXchStride = (uint64_t)(kMaxRanks + 3) * (kMaxRanks + 1);  // a group's snapshot + gathered words

// the exchange's buffers: per group the snapshot, gathered (device) and its pinned mirror, then
// the merge's run descriptors; the received entries (this rank's slice at most); the merge's
// window bounds over the slice; the exchange stream and its events
void ensure_xch(s3imph_ctx* c, uint64_t mine, uint64_t es, int P) {
  DistState& d = c->d;
  const uint64_t words = kXchGroups * kXchStride + (uint64_t)kXchGroups * 3 * kMaxRanks;
  if (!d.xch) dalloc(d.xch, words);
  if (!d.h_xch) {
    void* h = nullptr;
    HIPCHECK(hipHostMalloc(&h, 8 * words, hipHostMallocDefault));
    d.h_xch = static_cast<unsigned long long*>(h);
  }
  const uint64_t need = mine * es + 16;
  if (need > d.cap_xrecv) {
    d.cap_xrecv = 0;
    dalloc(d.xrecv, need);
    d.cap_xrecv = need;
  }
  const uint64_t bw = bm_place_bound_words(P, mine);
  if (bw > d.bm_bnd_cap) {
    d.bm_bnd_cap = 0;
    dalloc(d.bm_bnd, bw);
    d.bm_bnd_cap = bw;
  }
  if (!d.xo) {
    HIPCHECK(hipStreamCreateWithFlags(&d.xo, hipStreamNonBlocking));
    for (auto& e : d.ev_xg) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&d.ev_xdone, hipEventDisableTiming));
  }
}

int dist_attempt_bitmap(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                        uint64_t n_local, uint64_t key_base, uint64_t N, uint64_t* fp_out, uint64_t* pos_out,
                        uint64_t out_cap, hipStream_t s, bool conservative, s3imph_build_info* info,
                        std::string* msg) {
  DistState& d = c->d;
  Comm& cm = *d.comm;
  const int P = d.nranks, R = d.rank;
  LevelState* st = c->d_st;
  // level 0 beyond kScatterTiles tiles of 2^kBmMaxTb positions (N > ~2^30): the routed build
  if (tiles_of(level_words(N), kBmMaxTb, 0) > kScatterTiles) return kDistRetry;
  ensure_bm_workspace(c, N);
  c->l20_mask = 0;
  const BinBuffers b = make_bufs(c, nullptr, fp_out, pos_out, s);
  const double q = 1.0 - std::exp(-0.5);
  launch_init_state(st, n_local, out_cap, s, n_local ? offsets : nullptr);
  launch_dist_setup(st, 0, nullptr, N, R, P, s);
  launch_bm_range(st, 0, s);  // the whole level before the hash: P0's partition pass reads the range
  ev_mark(c, s, "init");
  // Level 0 through the P0 super-tiles when the whole level's tile count is
  // in P0's range and positions are the identity: the fused hash partition, the super-tile
  // scatter (which also writes each slot's position), then the bitmap tile kernels over R20
  // slots.  Tiles hold 2^tbd positions, tbd = 14 + floor(lg P) (at most kBmP0MaxTb): a rank's
  // share of a tile stays ~8k records, as one GPU's 2^14 tile, so the settle stages them.
  // (Tiles are rank-local geometry — only whole words of planes and bits cross ranks — so a
  // rank may take P0 or not on its own, e.g. one without keys or out of memory.)
  const unsigned tbd = bm_dense_tb(P);
  unsigned tb0 = tbd;
  while (tb0 < kBmP0MaxTb && tiles_of(level_words(N), tb0, 0) > kBmMaxTiles) ++tb0;
  const uint64_t T0 = tiles_of(level_words(N), tb0, 0);
  // (the single-GPU threshold, p0_min_tiles, weighs P0 against the split kernel; here the
  // alternative is a Rec level 0 without staged settles, so P0 takes any level of a tile per CU)
  bool p0 = c->p0 && !pos && n_local && n_local <= kP0MaxKeys && !hash_only_knob() && T0 >= kBmP0MinTiles &&
            T0 <= kP0MaxS * kP0MaxTps && T0 <= kBmMaxTiles;
  P0Bufs pb{};
  if (p0) p0 = p0_try_bufs(c, n_local, N, s, &pb, tb0, true);
  if (n_local) {
    const LevelGeom gh0 = choose_geom_sz(n_local, 64 * level_words(N), kTargetTiles0, chunks0(n_local), kTileMaxBits);
    if (p0) {
      launch_p0_hash(blob, offsets, n_local, b, gh0, pb, s);
    } else {
      launch_hash0_only(blob, offsets, n_local, b, gh0, level_grids(n_local, 64 * level_words(N), gh0).gc, s);
    }
  }
  ev_mark(c, s, p0 ? "hash_part0" : "hash_count0");
  if (c->debug && p0)
    std::fprintf(stderr, "[s3imph] rank %d bitmap: level 0 through P0 super-tiles (%llu tiles of 2^%u)\n", R,
                 (unsigned long long)T0, tb0);
  Rec* const out = d.bm_out;                   // this rank's settled (p, fp, pos) triples
  unsigned long long* const out_cnt = d.small + 4096;
  HIPCHECK(hipMemsetAsync(out_cnt, 0, 8, s));
  // this rank's output slice: its settled keys land in fp_out / pos_out during the settle;
  // d.scnt counts every settled key per slice (the output all-to-all's send counts)
  const uint64_t slice = (N + P - 1) / P;
  const uint64_t lo = std::min<uint64_t>((uint64_t)R * slice, N), mine = std::min<uint64_t>(N, lo + slice) - lo;
  {  // out_cap is the caller's, per rank: agreed before the first level
    int lrc = S3IMPH_OK;
    if (mine > out_cap) {
      *msg = "build MPHF: output capacity " + std::to_string(out_cap) + " < " + std::to_string(mine);
      lrc = S3IMPH_ERR_INVALID;
    }
    const int rc = dist_agree(c, lrc, s, msg);
    if (rc != S3IMPH_OK) return rc;
  }
  // (one rank writes its settled keys straight to fp_out / pos_out; at P > 1 they join the settled
  // list, and the slices are assembled by the P-way merge below)
  const OwnSlice own_slice{lo, mine, slice, level_magic(slice), P == 1 ? R : -1, P, fp_out, pos_out, d.scnt};
  // with identity positions the settled keys bound for other slices cross as 16-B entries
  // (offset in the slice, this rank's key index, fp) instead of 24-B (p, fp, pos) records
  const bool out16 = !pos;
  const uint64_t es = out16 ? sizeof(BmT16) : sizeof(Rec);
  HIPCHECK(hipMemsetAsync(d.scnt, 0, 8ull * (P + 1), s));
  // ---- the output exchange by level group ---------------------------------
  // Settled keys bound for other slices leave in groups — level 0, level 1, then the rest —
  // each once its levels are settled: a snapshot of the settle's cumulative per-slice counts
  // (with this rank's list length, its key base and the group's end rank) is gathered on the
  // build's stream; a level later the host reads it (an event) and puts the group's all-to-all
  // and its slice merge on the exchange stream (RCCL: its own communicator), beside the next
  // levels' work.  The checks read the gathered counts only: every rank takes the same branch.
  const uint64_t XW = (uint64_t)P + 4;  // snapshot words per rank
  const uint64_t out_cap_e = out16 ? d.bm_cap_out * sizeof(Rec) / sizeof(BmT16) : d.bm_cap_out;  // list entries
  const bool xin = P > 1 && xch_levels_on();
  const bool xasync = P > 1 && (d.xcomm != nullptr || xch_stream_knob());
  Comm& xcm = d.xcomm && xasync ? *d.xcomm : cm;
  hipStream_t xst = s;
  int xsnaps = 0, xsent = 0;
  uint64_t xracc = 0, xp_end = 0;
  bool xbad = false;
  if (P > 1) {
    ensure_xch(c, mine, es, P);
    if (xasync) xst = d.xo;
  }
  struct XJoin {  // every exit waits for the exchanges in flight (they read this build's buffers)
    hipStream_t x;
    ~XJoin() {
      if (x) (void)hipStreamSynchronize(x);
    }
  } xjoin{xasync ? d.xo : nullptr};
  // group xsnaps's snapshot, after the settle of level Lnext - 1
  auto xsnap = [&](int Lnext) {
    unsigned long long* dv = d.xch + (uint64_t)xsnaps * kXchStride;
    HIPCHECK(hipMemcpyAsync(dv, d.scnt, 8ull * P, hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipMemcpyAsync(dv + P, out_cnt, 8, hipMemcpyDeviceToDevice, s));
    launch_set_u64(dv + P + 1, key_base, s);
    HIPCHECK(hipMemcpyAsync(dv + P + 2, &st->lvl_base[Lnext], 8, hipMemcpyDeviceToDevice, s));
    launch_set_u64(dv + P + 3, out_cap_e, s);
    cm.allgather(dv, dv + XW, 8 * XW, s);
    HIPCHECK(hipMemcpyAsync(d.h_xch + (uint64_t)xsnaps * kXchStride + XW, dv + XW, 8 * XW * P, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipEventRecord(d.ev_xg[xsnaps], s));
    ++xsnaps;
  };
  // group xsent's all-to-all and merge (its snapshot taken)
  auto xsend = [&]() {
    const int gi = xsent++;
    HIPCHECK(hipEventSynchronize(d.ev_xg[gi]));
    const unsigned long long* G = d.h_xch + (uint64_t)gi * kXchStride + XW;
    const unsigned long long* Gp = gi ? d.h_xch + (uint64_t)(gi - 1) * kXchStride + XW : nullptr;
    auto at = [&](const unsigned long long* M, int r, uint64_t j) -> uint64_t { return M ? M[(uint64_t)r * XW + j] : 0; };
    auto cnt = [&](int r, int t) -> uint64_t { return at(G, r, t) - at(Gp, r, t); };
    const uint64_t p_lo = at(Gp, 0, P + 2), p_hi = at(G, 0, P + 2);
    // every rank's receipts against its slice's share of the group's ranks, its sends against
    // its list's growth, one end rank everywhere
    bool ok = p_lo <= p_hi && p_lo == xp_end;
    for (int r = 0; r < P && ok; ++r) {
      const uint64_t rlo = std::min<uint64_t>((uint64_t)r * slice, N), rhi = std::min<uint64_t>(N, rlo + slice);
      uint64_t in = 0, lst = 0;
      for (int q = 0; q < P; ++q) {
        in += cnt(q, r);
        lst += cnt(r, q);
      }
      const uint64_t a = std::min(std::max(p_lo, rlo), rhi), b = std::min(std::max(p_hi, rlo), rhi);
      if (in != b - a || lst != at(G, r, P) - at(Gp, r, P) || at(G, r, P + 2) != p_hi || at(G, r, P) > at(G, r, P + 3))
        ok = false;
    }
    xp_end = p_hi;
    if (!ok) {
      xbad = true;
      return;
    }
    std::vector<uint64_t> soff(P), sbytes(P), roff(P), rbytes(P);
    const uint64_t olo = at(Gp, R, P);  // this rank's list entries before the group
    uint64_t sent = 0, got = 0;
    for (int t = 0; t < P; ++t) {
      soff[t] = (olo + sent) * es;
      sbytes[t] = t == R ? 0 : cnt(R, t) * es;
      sent += cnt(R, t);
      roff[t] = (xracc + got) * es;
      rbytes[t] = t == R ? 0 : cnt(t, R) * es;
      if (t != R) got += cnt(t, R);
    }
    if (xasync) HIPCHECK(hipStreamWaitEvent(xst, d.ev_xg[gi], 0));
    xcm.alltoallv(out, soff.data(), sbytes.data(), d.xrecv, roff.data(), rbytes.data(), xst);
    // the merge's runs: sender q's entries of this slice and group (this rank's own in place)
    unsigned long long* run_h = d.h_xch + kXchGroups * kXchStride + (uint64_t)gi * 3 * kMaxRanks;
    unsigned long long* run_d = d.xch + kXchGroups * kXchStride + (uint64_t)gi * 3 * kMaxRanks;
    for (int q = 0; q < P; ++q) {
      const uint8_t* rb = q == R ? reinterpret_cast<const uint8_t*>(out) + soff[R] : d.xrecv + roff[q];
      run_h[3 * q] = (unsigned long long)(uintptr_t)rb;
      run_h[3 * q + 1] = cnt(q, R);
      run_h[3 * q + 2] = at(G, q, P + 1);
    }
    HIPCHECK(hipMemcpyAsync(run_d, run_h, 24ull * P, hipMemcpyHostToDevice, xst));
    const uint64_t a = std::min(std::max(p_lo, lo), lo + mine) - lo, b = std::min(std::max(p_hi, lo), lo + mine) - lo;
    launch_bm_place_merge(run_d, out16, P, lo, a, b, d.bm_bnd, fp_out, pos_out, st, xst);
    xracc += got;
  };
  HIPCHECK(hipMemsetAsync(c->tcnt, 0, (size_t)kMaxDistLevels * kTcntStride * sizeof(unsigned), s));
  // The level's records go through the reservation scatter into tiles over the level's
  // whole position range (this rank's records only); the tile kernels then mark and
  // settle a tile at a time in LDS.  Level 0 reads the hash kernel's key-order arrays.
  BinBuffers bs = b;
  bs.dist = false;
  bs.split = nullptr;
  bs.pipe_tiles = false;  // the bitmap kernels read Rec buckets (R20 ones on R20 list levels, BinBuffers::l20)
  bs.pos = pos;
  bs.pos_base = key_base;
  // Level sizes: the host bounds n_L from above (mean q n + 6 sigma), so every collective's
  // size is known without a host round trip; a level outgrowing its bound sets
  // kStBitmapBound and the build reruns on the routed decomposition.
  double nb = (double)N, npred = (double)n_local;
  // what crosses xGMI per position: the 2-bit (A, C) planes (default), or count lanes summed
  // by RCCL — a nibble while the rank sums cannot carry out of it (2P <= 14), else a byte
  const int lanes = c->bm_counts ? (P <= kBmNibRanks ? kBmNibbles : kBmBytes) : kBmPlanes;
  std::vector<uint64_t> xoff(P), xbytes(P);
  int L = 0;
  // this level's records were partitioned into its super-tiles' regions by the previous level's
  // settle (NextPart): fed_nb settle blocks' regions of fed_rc records
  bool fed = false;
  uint64_t fed_rc = 0;
  unsigned fed_nb = 0;
  for (;;) {
    const uint64_t wmax = level_words((uint64_t)std::ceil(nb)), S = (wmax + P - 1) / P, wpad = S * (uint64_t)P;
    // tiles of 2^tb positions: from the dense size (a rank's ~8k records), the smallest
    // leaving at most bm_target_tiles() tiles (level 0 under P0: tb0)
    const uint64_t np = (uint64_t)(npred * 1.1) + 4096;
    // an R20 list level with more dense tiles than the reservation scatter takes goes through
    // the P0 super-tiles too: its list into the super-tiles' slots, then into the dense tiles
    // (C3 level 1 at one rank: 4.8k tiles of 2^14)
    P0Bufs pl{};
    const uint64_t Td = tiles_of(wmax, tbd, 0);
    const bool lp = L > 0 && !conservative && c->p0 && bs.list20(L) && Td > bm_target_tiles() && Td <= kBmMaxTiles &&
                    p0_try_bufs(c, np, (uint64_t)std::ceil(nb), s, &pl, tbd, true);
    const bool l0p = L == 0 && p0;
    unsigned tb = l0p ? tb0 : tbd;
    while (!l0p && !lp && tb < kBmMaxTb && tiles_of(wmax, tb, 0) > bm_target_tiles()) ++tb;
    const uint64_t tiles = tiles_of(wmax, tb, 0);
    // > 2^30 positions: the routed build (same on every rank); P0's levels take up to kBmMaxTiles
    if (tiles > (l0p || lp ? kBmMaxTiles : kScatterTiles)) return kDistRetry;
    launch_bm_level_begin(st, L, L > 0, d.gslot + L, R, P, wmax, s);
    LevelGeom g{};
    g.tb = tb;
    g.chunk = kTargetChunks;
    g.ts = 0;
    const int gsr = (int)std::max<uint64_t>(1, std::min<uint64_t>((np + kSubRound - 1) / kSubRound, 256));
    const void* bk = c->bucket;
    uint64_t bcap = c->bucket_cap;
    const unsigned* tc = c->tcnt + (uint64_t)L * kTcntStride;
    const uint16_t* xs = nullptr;
    if (l0p) {
      if (n_local) launch_p0_scatter(b, pb, p0_fused(blob, pb), s);
      bk = pb.bucket;
      bcap = pb.bucket_cap;
      tc = pb.tcnt;
      xs = pb.x;
    } else if (lp) {
      if (c->debug)
        std::fprintf(stderr, "[s3imph] rank %d bitmap: level %d through P0 super-tiles (%llu tiles of 2^%u%s)\n", R, L,
                     (unsigned long long)tiles, tb, fed ? ", partitioned by the previous settle" : "");
      if (fed) {  // the regions are in place: straight to the tiles
        pl.reg_cap = fed_rc;
        pl.nb = fed_nb;
        launch_p0_scatter(bs, pl, true, s, L);
      } else {
        launch_p0_partition_list(L, bs, pl, s);
        launch_p0_scatter(bs, pl, false, s, L);
      }
      bk = pl.bucket;
      bcap = pl.bucket_cap;
      tc = pl.tcnt;
      xs = pl.x;
    } else {
      // (a level fed by regions always takes P0 with the geometry its feeder used; a failed
      // allocation here leaves its records in those regions: the build reruns)
      if (fed) launch_bm_flag(st, kStResOverflow, s);
      launch_binned_scatter_res(L, bs, g, gsr, s, 0, 0, tiles);
    }
    const bool in20 = l0p || bs.list20(L);  // R20 slots: P0's level 0, or a level whose list is R20
    launch_bm_tile_mark(L, bk, in20, tc, bcap, tb, tiles, st, wpad, d.bm_lanes, d.bm_a, lanes, S, s, xs);
    const bool solo = lanes == kBmPlanes && P == 1;
    if (solo) {
      // one rank: its planes are the level's, merged straight into the final bits (no
      // self-copies through the collectives)
      launch_bm_merge(reinterpret_cast<const uint64_t*>(d.bm_lanes), S, 1, d.bm_g, st, s);
    } else if (lanes == kBmPlanes) {
      // slice t's planes (2 S words) to rank t; rank q's planes of this rank's slice land at 2 S q
      for (int t = 0; t < P; ++t) {
        xoff[t] = 16 * S * (uint64_t)t;
        xbytes[t] = 16 * S;
      }
      cm.alltoallv(d.bm_lanes, xoff.data(), xbytes.data(), d.bm_recv, xoff.data(), xbytes.data(), s);
      launch_bm_merge(reinterpret_cast<const uint64_t*>(d.bm_recv), S, P, d.bm_dec, st, s);
    } else {
      cm.reduce_scatter_u8(d.bm_lanes, d.bm_slice, (lanes == kBmNibbles ? 32 : 64) * S, s);
      launch_bm_decide(d.bm_slice, S, d.bm_dec, st, lanes == kBmNibbles, s);
    }
    if (!solo) cm.allgather(d.bm_dec, d.bm_g, 8 * S, s);
    launch_bm_level_end(L, d.bm_g, d.bm_a, tb, tiles, c->bits, d.bm_tsum, d.bm_tbase, st, d.gslot, out_cnt, s);
    // the next level is a bitmap level too (else the replicated tail, which reads Rec): its
    // list goes out as R20 with identity positions (BinBuffers::l20)
    const double nbn = nb * q + 6.0 * std::sqrt(nb) + 64.0;
    const bool more = !(L + 1 >= kMaxDistLevels || nbn <= (double)c->dist_switch);
    const bool next20 = more && c->l20 && !pos && L + 1 < 32;
    if (next20) bs.l20 |= 1u << (L + 1);
    c->l20_mask = bs.l20;  // dist_classify_stop reads a stop level's list in this format
    // R20 tiles at the dense size stage their settled keys (each rank's ~8k records a tile)
    const bool staged = tb <= tbd || l0p;
    // the next level through the P0 super-tiles: its records go from this settle straight into
    // its super-tiles' regions (level L + 1's exact size is known now: the tile scan wrote it),
    // when its geometry is known to fit the buffers it will take (no reallocation under them)
    NextPart npart{};
    bool feed = false;
    uint64_t rc1 = 0;
    unsigned nb1 = 0;
    if (more && next20 && staged && in20 && c->p0 && !conservative && bm_feed_next()) {
      const uint64_t ng1 = (uint64_t)std::ceil(nbn), Td1 = tiles_of(level_words(ng1), tbd, 0);
      if (Td1 > bm_target_tiles() && Td1 <= kBmMaxTiles) {
        const uint64_t np1 = (uint64_t)(npred * q * 1.1) + 4096;
        uint64_t need1 = 0;
        const P0Bufs g1 = p0_geom(c, np1, ng1, tbd, &need1);
        nb1 = bm_settle_grid(tiles, bm_settle_threads(tb, P, true));
        rc1 = p0_region_cap(np1, g1.S, nb1);
        if (g1.S <= (unsigned)kMaxRanks && c->p0_sup && c->p0_pcnt &&
            std::max<uint64_t>(need1, (uint64_t)nb1 * g1.S * rc1) <= c->p0_sup_cap) {
          npart = NextPart{c->p0_sup, rc1, c->p0_pcnt, g1.tps_sub(), g1.S, d.gslot + L + 1};
          feed = true;
        }
      }
    }
    launch_bm_tile_settle(L, bk, in20, key_base, tc, bcap, tb, tiles, st, d.bm_g, d.bm_a, d.bm_tbase, out,
                          out16 ? d.bm_cap_out * sizeof(Rec) / sizeof(BmT16) : d.bm_cap_out, c->list[L & 1], d.cap_list,
                          next20, own_slice, s, staged, xs, out16, feed ? &npart : nullptr);
    if (!conservative && L == 0 && dev_env("S3IMPH_FAULT_BM_OVERFLOW"))
      launch_bm_flag(st, kStResOverflow, s);  // test hook: a capacity miss (the conservative rerun)
    {  // levels 0 and 1: their group's snapshot now, the previous group's exchange out
      const bool snap = xin && more && L <= 1;
      if (snap) xsnap(L + 1);
      while (xsent < xsnaps - (snap ? 1 : 0)) xsend();
    }
    fed = feed;
    fed_rc = rc1;
    fed_nb = nb1;
    ev_mark(c, s, L == 0 ? "level0" : "levels");
    if (c->debug) {  // the level's device status as it ends (a flag's level, for the report)
      unsigned long long* M = d.h_pinned;
      HIPCHECK(hipMemcpyAsync(M, &st->status, 4, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipMemcpyAsync(M + 1, &st->pad0_, 4, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
      std::fprintf(stderr, "[s3imph] rank %d bitmap: level %d (tiles 2^%u x %llu%s) status 0x%x site %u\n", R, L, tb,
                   (unsigned long long)tiles, l0p || lp ? ", P0" : "", (unsigned)(M[0] & 0xffffffffu),
                   (unsigned)(M[1] & 0xffffffffu));
    }
    npred *= q;
    if (!more) break;
    nb = nbn;
    ++L;
  }
  const int Ls = L + 1;  // first replicated level
  if (P > 1) {  // the level groups still pending, then the last group's snapshot (sent beside the tail)
    while (xsent < xsnaps) xsend();
    xsnap(Ls);
  }
  // ---- gather every rank's remaining records; all ranks finish the build identically,
  // the tail's outputs (global p in [N - total, N)) into scratch (kh / fp are free now)
  unsigned long long* M = d.h_pinned;
  if (P > 1) {
    HIPCHECK(hipMemcpyAsync(d.small, &st->n[Ls], 8, hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipMemcpyAsync(d.small + 1, &st->status, 4, hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipMemsetAsync(reinterpret_cast<uint8_t*>(d.small + 1) + 4, 0, 4, s));
    cm.allgather(d.small, d.small + 64, 16, s);
    HIPCHECK(hipMemcpyAsync(M, d.small + 64, 16ull * P, hipMemcpyDeviceToHost, s));
  } else {  // one rank: its own count and flags (no self-gather)
    M[1] = 0;
    HIPCHECK(hipMemcpyAsync(M, &st->n[Ls], 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(M + 1, &st->status, 4, hipMemcpyDeviceToHost, s));
  }
  HIPCHECK(hipStreamSynchronize(s));
  uint64_t total = 0, maxc = 0;
  unsigned flags = 0;
  std::vector<uint64_t> cnt(P);
  for (int r = 0; r < P; ++r) {
    cnt[r] = M[2 * r];
    flags |= (unsigned)M[2 * r + 1];
    total += cnt[r];
    maxc = std::max(maxc, cnt[r]);
  }
  if (c->debug)
    std::fprintf(stderr, "[s3imph] rank %d bitmap: %d sharded levels, replicated %llu records, flags 0x%x\n", R, Ls,
                 (unsigned long long)total, flags);
  // global facts (the flags are gathered): every rank returns here.  A level beyond its
  // bound reruns on the routed build; a reservation slot overflow (a skewed tile, or a fed
  // level without its P0 buffers) reruns this decomposition conservatively first.
  if (flags & kStBitmapBound) return kDistRetry;
  if (flags & (kStResOverflow | kStGeometry)) return conservative ? kDistRetry : kDistRetryBm;
  if (flags & kStOverflow) {
    *msg = "build MPHF: bitmap decomposition: list capacity exceeded";
    return S3IMPH_ERR_INTERNAL;
  }
  {  // per-rank capacities: agreed before the gather
    int lrc = S3IMPH_OK;
    if (total > d.cap_list || total > c->cap_keys) {
      *msg = "build MPHF: replicated level of " + std::to_string(total) + " records exceeds the workspace";
      lrc = S3IMPH_ERR_NOMEM;
    }
    const int rc = dist_agree(c, lrc, s, msg);
    if (rc != S3IMPH_OK) return rc;
  }
  Rec* rl = c->list[(Ls - 1) & 1];  // (the last bitmap level's collided records: one rank's are all)
  if (total && P > 1) {
    if ((uint64_t)P * maxc > d.cap_send) {
      dalloc(d.send, (uint64_t)P * maxc);
      d.cap_send = (uint64_t)P * maxc;
    }
    cm.allgather(rl, d.send, maxc * sizeof(Rec), s);
    uint64_t o = 0;
    for (int r = 0; r < P; ++r) {
      if (cnt[r])
        HIPCHECK(hipMemcpyAsync(rl + o, d.send + (uint64_t)r * maxc, cnt[r] * sizeof(Rec), hipMemcpyDeviceToDevice, s));
      o += cnt[r];
    }
  }
  if (total >= 2) fault_dup_record(c, rl, s);
  launch_dist_replicate(st, Ls, total, 0, s);
  launch_set_u64(&st->lvl_base[Ls], 0, s);  // tail ranks count from 0: scratch index = p - (N - total)
  ev_mark(c, s, "gather");
  BinBuffers bt = b;
  bt.fp_out = c->kh;
  bt.pos_out = c->fp;
  const LevelGeom gcons = choose_geom(std::max<uint64_t>(total, 1), kTargetTiles, kTargetChunks, kRegTileMaxBits);
  enqueue_levels_from(c, bt, Ls, total, gcons, false, s);
  HIPCHECK(hipGetLastError());
  if (P > 1)
    while (xsent < xsnaps) xsend();  // the last level group's exchange, beside the tail's levels
  HIPCHECK(hipMemcpyAsync(c->h_st, st, sizeof(LevelState), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipMemcpyAsync(M, out_cnt, 8, hipMemcpyDeviceToHost, s));
  if (P == 1) HIPCHECK(hipMemcpyAsync(M + 8, d.scnt, 8, hipMemcpyDeviceToHost, s));  // the exchange's counts
  HIPCHECK(hipStreamSynchronize(s));
  const uint64_t n_out = M[0], own1 = P == 1 ? M[8] : 0;
  // ---- every rank's flags, tail result and settled count
  {
    const LevelState& hs = *c->h_st;
    M[0] = hs.status;
    M[1] = hs.rank_total;
    M[2] = n_out;
    if (P > 1) {
      HIPCHECK(hipMemcpyAsync(d.small, M, 24, hipMemcpyHostToDevice, s));
      cm.allgather(d.small, d.small + 64, 24, s);
      HIPCHECK(hipMemcpyAsync(M, d.small + 64, 24ull * P, hipMemcpyDeviceToHost, s));
      HIPCHECK(hipStreamSynchronize(s));
    }
  }
  uint64_t settled = 0;
  flags = 0;
  for (int r = 0; r < P; ++r) {
    flags |= (unsigned)M[3 * r];
    settled += M[3 * r + 2];
  }
  const LevelState& hs = *c->h_st;
  if (c->debug) {
    std::fprintf(stderr, "[s3imph] rank %d bitmap: after tail flags 0x%x settled %llu tail ranked %llu nlevels %u\n  n:",
                 R, flags, (unsigned long long)settled, (unsigned long long)hs.rank_total, hs.nlevels);
    for (int l = 0; l <= (int)hs.nlevels + 1 && l < kMaxLevels; ++l)
      std::fprintf(stderr, " %llu/%llu", (unsigned long long)hs.n[l], (unsigned long long)hs.lvl_base[l]);
    std::fprintf(stderr, "\n");
  }
  if (flags & (kStGeometry | kStTailOverflow | kStResOverflow)) return conservative ? kDistRetry : kDistRetryBm;
  if (flags & kStTooManyLevels) return dist_classify_stop(c, blob, offsets, n_local, s, msg);
  if (flags & kStKeyZero) {
    *msg = "MPHF Key(...) returned 0, possible hash collision with sentinel";
    return S3IMPH_ERR_KEY_HASH_ZERO;
  }
  if (flags) {
    *msg = "build MPHF: internal error (device flags " + std::to_string(flags) + ")";
    return S3IMPH_ERR_INTERNAL;
  }
  if (hs.rank_total != total || settled + total != N) {
    *msg = "build MPHF: internal error: placed " + std::to_string(settled) + " + " + std::to_string(hs.rank_total) +
           " of " + std::to_string(N) + " keys";
    return S3IMPH_ERR_INTERNAL;
  }
  // ---- the settled keys reached their slices' owners by level group (the last group beside
  // the tail, above); every rank checked every group against the gathered counts
  const uint64_t g0 = N - total;
  if (P > 1) {
    if (xbad || xp_end != g0) {
      *msg = "build MPHF: internal error: the output exchange's counts do not cover the slices";
      return S3IMPH_ERR_INTERNAL;
    }
    if (xasync) {  // the build's stream resumes once every group is placed
      HIPCHECK(hipEventRecord(d.ev_xdone, xst));
      HIPCHECK(hipStreamWaitEvent(s, d.ev_xdone, 0));
    }
  } else {  // one rank placed its settled keys during the settles: they and the tail's cover the slice
    const uint64_t tail_mine = std::min<uint64_t>(N, lo + mine) > std::max(g0, lo)
                                   ? std::min<uint64_t>(N, lo + mine) - std::max(g0, lo) : 0;
    if (own1 != n_out || own1 + tail_mine != mine) {
      *msg = "build MPHF: internal error: output slice of rank " + std::to_string(R) + " holds " +
             std::to_string(own1) + " + " + std::to_string(tail_mine) + " of " + std::to_string(mine) + " entries";
      return S3IMPH_ERR_INTERNAL;
    }
  }
  launch_bm_tail_copy(c->kh, c->fp, g0, total, lo, mine, fp_out, pos_out, s);
  ev_mark(c, s, "exchange_out");
  HIPCHECK(hipMemcpyAsync(M, &st->status, 4, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  ev_collect(c);
  if (c->debug) {  // the level-0 hash's waves: duration and shader clock of this rank's hash
    std::fprintf(stderr, "[s3imph] rank %d bitmap: level-0 hash profile\n", R);
    print_tile_profile(c);
  }
  {  // this rank's placement flag: agreed, so every rank returns the same way
    int lrc = S3IMPH_OK;
    if ((unsigned)M[0] & kStRank) {
      *msg = "build MPHF: internal error: a settled position fell outside its owner's slice";
      lrc = S3IMPH_ERR_INTERNAL;
    }
    const int rc = dist_agree(c, lrc, s, msg);
    if (rc != S3IMPH_OK) return rc;
  }
  d.seg.clear();
  if (mine) d.seg.insert(d.seg.end(), {lo, mine, 0});
  d.out_n = mine;
  info->status = S3IMPH_OK;
  info->num_levels = hs.nlevels;
  info->total_words = hs.woff[hs.nlevels];
  info->mph_bin_len = 8 * kPartitions + 8 + 8ull * hs.nlevels + 8ull * info->total_words;
  info->big_levels = (uint64_t)Ls;
  return S3IMPH_OK;
}

int build_dist(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
               uint64_t n_local, uint64_t key_base, uint64_t* fp_out, uint64_t* pos_out, uint64_t out_cap,
               uint64_t* out_n, hipStream_t s, s3imph_build_info* info, std::string* msg) {
  DistState& d = c->d;
  c->have_build = false;
  c->rank_valid = false;
  *info = s3imph_build_info{};
  *out_n = 0;
  d.seg.clear();
  d.out_n = 0;
  if (n_local > kU32Limit) {
    *msg = "build MPHF: more than 2^32-1 keys on one rank";
    return S3IMPH_ERR_INVALID;
  }
  ensure_dist_small(c);
  ev_begin(c);
  ev_mark(c, s, "start");
  // global key count (also a rendezvous: every rank must reach the same build)
  d.h_pinned[0] = n_local;
  HIPCHECK(hipMemcpyAsync(d.small, d.h_pinned, 8, hipMemcpyHostToDevice, s));
  d.comm->allreduce_u64(d.small, d.small + 1, 1, s);
  HIPCHECK(hipMemcpyAsync(d.h_pinned + 1, d.small + 1, 8, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  const uint64_t N = d.h_pinned[1];
  info->n_keys = N;
  if (N == 0) {
    c->have_build = true;
    c->last_n = 0;
    c->info = *info;
    ev_collect(c);
    return S3IMPH_OK;
  }
  ensure_dist_workspace(c, n_local, N);
  set_lds_attrs(c);
  int rc = kDistRetry;
  // bitmap decomposition first when selected (a capacity miss reruns it once conservatively);
  // its bound miss, and the routed build's geometry misses, fall back to the routed build and
  // then to its conservative form.  Strict mode fails instead of routing.
  if (d.mode == kDistBitmap) {
    for (int bm = 0; bm < 2; ++bm) {
      ev_begin(c);
      ev_mark(c, s, "start");
      rc = dist_attempt_bitmap(c, blob, offsets, pos, n_local, key_base, N, fp_out, pos_out, out_cap, s, bm == 1,
                               info, msg);
      if (rc != kDistRetryBm) break;
      if (c->debug)
        std::fprintf(stderr, "[s3imph] rank %d bitmap: a capacity miss, rerunning conservatively\n", d.rank);
    }
    if (rc == kDistRetryBm) rc = kDistRetry;
    if (rc == kDistRetry && (d.strict || dev_env("S3IMPH_DIST_STRICT"))) {
      *msg = "build MPHF: the bitmap decomposition missed its size bounds (S3IMPH_DIST_STRICT: no fallback)";
      return S3IMPH_ERR_INTERNAL;  // tests use this to prove the bitmap path built the index
    }
  }
  // one rank has nothing to route: its routed build is the single-GPU build (P0 level 0 up to
  // 2^31 keys, where the routed level 0 stops at 2^30 positions), outputs at their global p
  // (S3IMPH_DIST_ROUTE_SELF keeps the routed kernels for the tests that drive them)
  if (rc == kDistRetry && d.nranks == 1 && !c->route_self && (pos || key_base == 0)) {
    if (n_local > out_cap) {
      *msg = "build MPHF: output capacity " + std::to_string(out_cap) + " < " + std::to_string(n_local);
      return S3IMPH_ERR_INVALID;
    }
    rc = build_single(c, blob, offsets, pos, n_local, fp_out, pos_out, s, info, msg);
    if (rc != S3IMPH_OK) return rc;
    d.seg.assign({0, n_local, 0});
    d.out_n = n_local;
  }
  for (int attempt = 1; rc == kDistRetry && attempt < 3; ++attempt) {
    ev_begin(c);
    ev_mark(c, s, "start");
    rc = dist_attempt(c, blob, offsets, pos, n_local, key_base, N, fp_out, pos_out, out_cap, s, attempt > 1, info,
                      msg);
  }
  if (rc != S3IMPH_OK) return rc;
  if (d.out_n > out_cap) {
    *msg = "build MPHF: output capacity " + std::to_string(out_cap) + " < " + std::to_string(d.out_n) +
           " (see s3imph_dist_out_cap)";
    return S3IMPH_ERR_INVALID;
  }
  *out_n = d.out_n;
  info->n_keys = N;
  c->have_build = true;
  c->last_n = N;
  c->info = *info;
  return S3IMPH_OK;
}

s3imph_ctx* g_default[64] = {nullptr};
std::mutex g_default_mu;

bool reclaim_cached(s3imph_ctx* keep, const void* keep_set) {
  bool any = release_idle_multi_sets(keep_set) > 0;
  {
    std::lock_guard<std::mutex> glk(g_default_mu);
    for (s3imph_ctx* c : g_default) {
      if (!c || c == keep) continue;
      std::unique_lock<std::mutex> lk(c->mu, std::try_to_lock);
      if (!lk.owns_lock()) continue;  // building right now
      if (!c->hist && !c->s_blob && !c->fin) continue;  // nothing cached
      (void)hipSetDevice(c->device);
      if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
      free_workspace(c);
      fin_scratch_free(c);
      c->have_build = false;
      c->rank_valid = false;
      any = true;
    }
  }
  if (keep && keep->fin) {
    fin_scratch_free(keep);
    any = true;
  }
  if (keep) (void)hipSetDevice(keep->device);
  if (any && (dev_env("S3IMPH_DEBUG") || (keep && keep->debug)))
    std::fprintf(stderr, "[s3imph] out of device memory: released cached workspaces, retrying once\n");
  return any;
}

}  // namespace s3imph

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

void stager_init(s3imph_ctx* c) {
  Stager& g = c->stager;
  if (g.ready) return;
  for (int w = 0; w < kStageWorkers; ++w) {
    for (int b = 0; b < 2; ++b) {
      HIPCHECK(hipHostMalloc(&g.pin[w][b], kStageChunk, hipHostMallocDefault));
      HIPCHECK(hipEventCreateWithFlags(&g.ev[w][b], hipEventDisableTiming));
    }
    HIPCHECK(hipStreamCreateWithFlags(&g.st[w], hipStreamNonBlocking));
  }
  g.ready = true;
}

// Chunked copy between pageable host memory and the device through the pinned
// buffers.  h2d: device dst <- host src; with `bias`, src holds u64 words and each is
// stored minus bias (offsets rebased to a blob that starts at offsets[0]).
// conv 1 (h2d): host u64 words, minus bias, stored as device u32 (`bytes` = device
// bytes); conv 2 (d2h): device u32 words widened to host u64.  Both halve the PCIe bytes
// of an array whose values fit 32 bits.
// Device -> pageable host copies of one or more arrays through the pinned buffers, all
// their chunks dealt over one worker pool: each worker issues its next chunk's DMA, then
// copies out (conv 2: widens u32 -> u64) the chunk that landed, so the CPU copies of one
// worker overlap the DMA of the others and the arrays' transfers share the link.
struct D2HJob {
  void* dst;
  const void* src;
  uint64_t bytes;  // device bytes
  int conv;        // 0 copy, 2 widen u32 -> u64
};
// D2H chunk bytes (<= kStageChunk; A/B knob S3IMPH_D2H_CHUNK in MiB)
uint64_t d2h_chunk() {
  static const uint64_t v = [] {
    const char* e = dev_env("S3IMPH_D2H_CHUNK");
    const uint64_t m = e ? std::strtoull(e, nullptr, 10) : 0;
    return m ? std::min<uint64_t>(m << 20, kStageChunk) : kStageChunk;
  }();
  return v;
}

// The copy-out of a landed chunk into the caller's (pageable) array with non-temporal stores:
// the destination is written once and not read back here, so its lines need not be read for
// ownership first (regular stores read every destination line in: half the copy's memory
// traffic).  A/B knob S3IMPH_D2H_NT=0: memcpy and a plain widening loop.
bool d2h_nt() {
  static const bool v = [] {
    const char* e = dev_env("S3IMPH_D2H_NT");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}
void copy_out_nt(uint8_t* dst, const uint8_t* src, uint64_t len) {
  uint64_t h = (8 - ((uintptr_t)dst & 7)) & 7;  // bytes up to an 8-aligned destination
  if (h > len) h = len;
  std::memcpy(dst, src, h);
  uint64_t* d = reinterpret_cast<uint64_t*>(dst + h);
  const uint8_t* s8 = src + h;
  const uint64_t nw = (len - h) / 8;
  for (uint64_t i = 0; i < nw; ++i) {
    uint64_t v;
    std::memcpy(&v, s8 + 8 * i, 8);
    __builtin_nontemporal_store(v, d + i);
  }
  std::memcpy(dst + h + 8 * nw, s8 + 8 * nw, len - h - 8 * nw);
}
void widen_out_nt(uint64_t* d64, const uint32_t* s32, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) __builtin_nontemporal_store((uint64_t)s32[i], d64 + i);
}

void staged_d2h(s3imph_ctx* c, const std::vector<D2HJob>& jobs) {
  stager_init(c);
  Stager& g = c->stager;
  const uint64_t chunk = d2h_chunk();
  std::vector<uint64_t> first(jobs.size() + 1, 0);  // first global chunk of each job
  for (size_t j = 0; j < jobs.size(); ++j) first[j + 1] = first[j] + (jobs[j].bytes + chunk - 1) / chunk;
  const uint64_t nch = first.back();
  if (!nch) return;
  const int nw = (int)std::min<uint64_t>(kStageWorkers, nch);
  std::vector<std::string> errs(nw);
  auto work = [&](int w) {
    try {
      HIPCHECK(hipSetDevice(c->device));
      auto job = [&](uint64_t ch) { return (size_t)(std::upper_bound(first.begin(), first.end(), ch) - first.begin() - 1); };
      auto issue = [&](uint64_t ch, int buf) {
        const D2HJob& J = jobs[job(ch)];
        const uint64_t off = (ch - first[job(ch)]) * chunk, len = std::min(chunk, J.bytes - off);
        HIPCHECK(hipMemcpyAsync(g.pin[w][buf], static_cast<const uint8_t*>(J.src) + off, len, hipMemcpyDeviceToHost,
                                g.st[w]));
        HIPCHECK(hipEventRecord(g.ev[w][buf], g.st[w]));
      };
      int b = 0;
      if ((uint64_t)w < nch) issue(w, 0);
      for (uint64_t ch = w; ch < nch; ch += nw, b ^= 1) {
        if (ch + nw < nch) issue(ch + nw, b ^ 1);
        HIPCHECK(hipEventSynchronize(g.ev[w][b]));
        const D2HJob& J = jobs[job(ch)];
        const uint64_t off = (ch - first[job(ch)]) * chunk, len = std::min(chunk, J.bytes - off);
        const bool nt = d2h_nt();
        if (J.conv == 2) {
          const uint32_t* s32 = static_cast<const uint32_t*>(g.pin[w][b]);
          uint64_t* d64 = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(J.dst) + 2 * off);
          if (nt) widen_out_nt(d64, s32, len / 4);
          else
            for (uint64_t i = 0; i < len / 4; ++i) d64[i] = s32[i];
        } else if (nt) {
          copy_out_nt(static_cast<uint8_t*>(J.dst) + off, static_cast<const uint8_t*>(g.pin[w][b]), len);
        } else {
          std::memcpy(static_cast<uint8_t*>(J.dst) + off, g.pin[w][b], len);
        }
      }
      __atomic_thread_fence(__ATOMIC_SEQ_CST);  // the non-temporal stores drained before the join
      HIPCHECK(hipStreamSynchronize(g.st[w]));
    } catch (const Fail& f) {
      errs[w] = f.msg.empty() ? "staged copy failed" : f.msg;
    }
  };
  std::vector<std::thread> th;
  for (int w = 1; w < nw; ++w) th.emplace_back(work, w);
  work(0);
  for (auto& t : th) t.join();
  for (const auto& e : errs)
    if (!e.empty()) throw Fail{S3IMPH_ERR_HIP, e};
}

void staged_copy(s3imph_ctx* c, bool h2d, void* dst, const void* src, uint64_t bytes, uint64_t bias, int conv,
                 std::atomic<bool>* wide) {
  if (!bytes) return;
  if (!h2d) return staged_d2h(c, {D2HJob{dst, src, bytes, conv}});
  // Pageable H2D through the runtime already runs at the PCIe rate (C2: 400 MB in
  // 7.4 ms, 54 GB/s); pageable D2H does not (17 GB/s), and neither does rebasing.
  if (!bias && !conv && h2d) {
    HIPCHECK(hipMemcpy(dst, src, bytes, h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost));
    return;
  }
  stager_init(c);
  Stager& g = c->stager;
  const uint64_t nch = (bytes + kStageChunk - 1) / kStageChunk;
  const int nw = (int)std::min<uint64_t>(kStageWorkers, nch);
  std::vector<std::string> errs(nw);
  auto work = [&](int w) {
    try {
      HIPCHECK(hipSetDevice(c->device));
      auto clen = [&](uint64_t ch) { return std::min(kStageChunk, bytes - ch * kStageChunk); };
      int b = 0;
      if (h2d) {
        for (uint64_t ch = w; ch < nch; ch += nw, b ^= 1) {
          const uint64_t off = ch * kStageChunk, len = clen(ch);
          HIPCHECK(hipEventSynchronize(g.ev[w][b]));  // this buffer's previous DMA is done
          if (conv == 1) {
            const uint64_t* s64 = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(src) + 2 * off);
            uint32_t* d32 = static_cast<uint32_t*>(g.pin[w][b]);
            for (uint64_t i = 0; i < len / 4; ++i) d32[i] = (uint32_t)(s64[i] - bias);
          } else if (conv == 3) {  // u64 offsets -> u16 key lengths (src holds one more word)
            const uint64_t* s64 = reinterpret_cast<const uint64_t*>(src) + off / 2;
            uint16_t* d16 = static_cast<uint16_t*>(g.pin[w][b]);
            uint64_t over = 0;
            for (uint64_t i = 0; i < len / 2; ++i) {
              const uint64_t l = s64[i + 1] - s64[i];
              over |= l >> 16;
              d16[i] = (uint16_t)l;
            }
            if (over) {
              wide->store(true);
              break;
            }
            if (wide->load(std::memory_order_relaxed)) break;
          } else if (bias) {
            const uint64_t* s64 = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(src) + off);
            uint64_t* d64 = static_cast<uint64_t*>(g.pin[w][b]);
            for (uint64_t i = 0; i < len / 8; ++i) d64[i] = s64[i] - bias;
          } else {
            std::memcpy(g.pin[w][b], static_cast<const uint8_t*>(src) + off, len);
          }
          HIPCHECK(hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, g.pin[w][b], len, hipMemcpyHostToDevice,
                                  g.st[w]));
          HIPCHECK(hipEventRecord(g.ev[w][b], g.st[w]));
        }
      }
      HIPCHECK(hipStreamSynchronize(g.st[w]));
    } catch (const Fail& f) {
      errs[w] = f.msg.empty() ? "staged copy failed" : f.msg;
    }
  };
  std::vector<std::thread> th;
  for (int w = 1; w < nw; ++w) th.emplace_back(work, w);
  work(0);
  for (auto& t : th) t.join();
  for (const auto& e : errs)
    if (!e.empty()) throw Fail{S3IMPH_ERR_HIP, e};
}

// S3IMPH_OFF16=0: offsets cross PCIe as before (u32 / u64), the A/B reference
bool off16_disabled() {
  static const bool off = [] {
    const char* e = dev_env("S3IMPH_OFF16");
    return e && std::atoi(e) == 0;
  }();
  return off;
}

// Host-memory build through the device path (used by s3imph_build_host and the builder).
// the caller positions' staging (host builds with pos != NULL only)
void ensure_s_pos(s3imph_ctx* c, uint64_t n) {
  if (n <= c->s_pos_cap && c->s_pos) return;
  c->s_pos_cap = 0;
  dalloc(c->s_pos, n);
  c->s_pos_cap = n;
}

uint64_t mph_bin_bound(uint64_t n) { return 8 * kPartitions + 8 + 8ull * kMaxLevels + 8 * cap_words_for(n); }

// One-shot host build (s3imph_build_host): offsets (as u16 key lengths where they fit) and
// then the blob cross PCIe, the blob in pieces that the level-0 hash launches wait for one by
// one (HashFeed), so the hash of arrived keys runs beside the rest of the copy; the build;
// mph.bin marshalled on a second thread while fp / positions stream back through the pinned
// workers.  With S3IMPH_DEBUG every phase is timed from entry to return (they sum to it).
int build_from_host_once(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                         uint64_t n, uint64_t* fp_out, uint64_t* pos_out, MphOut* mph, std::string* msg) {
  using clk = std::chrono::steady_clock;
  const auto te = clk::now();
  s3imph_ctx* c = default_ctx(device, msg);
  if (!c) return S3IMPH_ERR_HIP;
  std::lock_guard<std::mutex> lk(c->mu);
  struct FeedReset {  // the feed lives on this frame
    s3imph_ctx* c;
    ~FeedReset() { c->feed = nullptr; }
  } feed_reset{c};
  try {
    HIPCHECK(hipSetDevice(c->device));
    mph->len = 0;
    if (mph->vec) mph->vec->clear();
    if (n == 0) return S3IMPH_OK;
    const uint64_t b0 = offsets[0], nbytes = offsets[n] - offsets[0];
    const uint64_t bcap = ((nbytes + 7) & ~7ull) + 8;
    if (bcap > c->s_blob_cap) {
      c->s_blob_cap = 0;
      dalloc(c->s_blob, bcap);
      c->s_blob_cap = bcap;
    }
    if (n > c->s_cap) {
      c->s_cap = 0;
      dalloc(c->s_offsets, n + 1);
      dalloc(c->s_fp, n);
      dalloc(c->s_posout, n);
      c->s_cap = n;
    }
    if (pos) ensure_s_pos(c, n);
    if (!c->copy_stream) HIPCHECK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (auto& e : c->copy_evs)
      if (!e) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipStream_t s = c->own_stream;
    HIPCHECK(hipStreamSynchronize(s));  // staging buffers may be in use by the last build
    const auto t0 = clk::now();
    // The blob crosses in pieces (one for a blob under 256 MiB; at most kCopyPieces) on the copy
    // stream, from a thread of its own that starts at once, beside the offsets' conversion and
    // copy below; the level-0 hash launches wait for the piece holding their keys (HashFeed).
    static const unsigned piece_bits = [] {  // A/B knob S3IMPH_PIECE_BITS: log2 of the smallest piece
      const char* e = dev_env("S3IMPH_PIECE_BITS");
      const unsigned v = e ? (unsigned)std::atoi(e) : 28u;
      return std::min(34u, std::max(20u, v));
    }();
    const int pieces = (int)std::min<uint64_t>(kCopyPieces, std::max<uint64_t>(1, nbytes >> piece_bits));
    std::vector<uint64_t> piece_hi(pieces);
    for (int j = 0; j < pieces; ++j) piece_hi[j] = j + 1 == pieces ? nbytes : (nbytes * (j + 1) / pieces + 15) & ~15ull;
    std::mutex pmu;
    std::condition_variable pcv;
    int pdone = 0;
    Fail copy_err{S3IMPH_OK, ""};
    clk::time_point t_copied{};
    std::thread tcopy([&]() {
      try {
        HIPCHECK(hipSetDevice(c->device));
        uint64_t lo = 0;
        for (int j = 0; j < pieces; ++j) {
          HIPCHECK(hipMemcpyAsync(c->s_blob + lo, blob + b0 + lo, piece_hi[j] - lo, hipMemcpyHostToDevice,
                                  c->copy_stream));
          HIPCHECK(hipEventRecord(c->copy_evs[j], c->copy_stream));
          lo = piece_hi[j];
          std::lock_guard<std::mutex> g(pmu);
          pdone = j + 1;
          pcv.notify_all();
        }
        HIPCHECK(hipStreamSynchronize(c->copy_stream));
      } catch (const Fail& f) {
        std::lock_guard<std::mutex> g(pmu);
        copy_err = f;
        pdone = pieces;
        pcv.notify_all();
      }
      t_copied = clk::now();
    });
    struct Join {
      std::thread& t;
      ~Join() {
        if (t.joinable()) t.join();
      }
    } join_copy{tcopy};
    // Offsets cross PCIe first, as u16 key lengths (2 B per key: C3's 800 MB of u64 offsets
    // become 200 MB) rebuilt on the device by a scan; a key longer than 65535 B sends them as
    // u32 (blob under 4 GiB, widened on the device) or u64 instead.  Staged in s_fp's space
    // (the build writes s_fp only later on the same stream).
    const bool off32 = nbytes < (1ull << 32);
    uint32_t* tmp32 = reinterpret_cast<uint32_t*>(c->s_fp);
    uint16_t* tmp16 = reinterpret_cast<uint16_t*>(c->s_fp);
    uint64_t* sums16 = c->s_fp + (2 * n + 255) / 256 * 32;  // after the lengths, 256-B aligned
    std::atomic<bool> wide{off16_disabled()};
    if (!wide.load()) staged_copy(c, true, tmp16, offsets, n * 2, 0, 3, &wide);
    if (wide.load()) {
      if (off32) staged_copy(c, true, tmp32, offsets, (n + 1) * 4, b0, 1);
      else staged_copy(c, true, c->s_offsets, offsets, (n + 1) * 8, b0);
    }
    if (!wide.load()) launch_len16_offsets(tmp16, n, sums16, c->s_offsets, s);
    else if (off32) launch_widen32(tmp32, c->s_offsets, n + 1, s);
    if (pos) staged_copy(c, true, c->s_pos, pos, n * 8);
    const auto t1 = clk::now();
    // ensure(k): the build stream waits for the piece that holds keys [0, k) and the 16 bytes
    // after them (a piece the copy thread has enqueued; its event marks it landed)
    int waited = 0;
    clk::duration t_wait{};
    HashFeed feed;
    feed.pieces = pieces;  // one hash launch per blob piece
    feed.ensure = [&](uint64_t k) {
      const uint64_t want = k >= n ? nbytes : std::min<uint64_t>(nbytes, offsets[k] - b0 + 16);
      int j = 0;  // the piece whose end covers want
      while (j < pieces - 1 && piece_hi[j] < want) ++j;
      if (j < waited) return;  // waited for already (the hash of a rerun asks again)
      const auto tw = clk::now();
      {
        std::unique_lock<std::mutex> g(pmu);
        pcv.wait(g, [&] { return pdone > j; });
        if (copy_err.code != S3IMPH_OK) throw copy_err;
      }
      HIPCHECK(hipStreamWaitEvent(s, c->copy_evs[j], 0));
      waited = j + 1;
      t_wait += clk::now() - tw;
    };
    if (pieces == 1) {  // a blob of one piece: the build starts once it has landed (no event wait)
      const auto tw = clk::now();
      tcopy.join();
      if (copy_err.code != S3IMPH_OK) throw copy_err;
      t_wait += clk::now() - tw;
    } else {
      c->feed = &feed;
    }
    s3imph_build_info info;
    int rc = build_single(c, c->s_blob, c->s_offsets, pos ? c->s_pos : nullptr, n, c->s_fp, c->s_posout, s,
                          &info, msg);
    c->feed = nullptr;
    if (tcopy.joinable()) tcopy.join();  // (a path that never hashed: nothing may still be in flight into s_blob)
    if (copy_err.code != S3IMPH_OK) throw copy_err;
    if (rc != S3IMPH_OK) return rc;
    const auto t2 = clk::now();
    // mph.bin (level words D2H, ~40 MB at C3) is marshalled on a second thread, straight into
    // its destination, while the output arrays stream back (ctx mutex held by this call)
    std::string mmsg;
    int mrc = S3IMPH_OK;
    clk::time_point t3m;
    std::thread tm([&]() {
      try {
        HIPCHECK(hipSetDevice(c->device));
        const uint64_t need = info.mph_bin_len;
        uint8_t* dst = nullptr;
        if (mph->vec) {
          mph->vec->resize(need);
          dst = mph->vec->data();
        } else if (mph->alloc) {
          dst = static_cast<uint8_t*>(std::malloc(need ? need : 1));
          if (!dst) throw std::bad_alloc();
          mph->buf = dst;
        } else {
          if (mph->cap < need) throw Fail{S3IMPH_ERR_INVALID, "build MPHF: mph.bin buffer of " +
                                                                   std::to_string(mph->cap) + " B < " +
                                                                   std::to_string(need) + " B"};
          dst = mph->buf;
        }
        uint64_t len = 0;
        mrc = marshal_locked(c, dst, need, &len, &mmsg);
        mph->len = len;
      } catch (const Fail& f) {
        mrc = f.code;
        mmsg = f.msg;
      } catch (const std::bad_alloc&) {
        mrc = S3IMPH_ERR_NOMEM;
        mmsg = "out of host memory";
      }
      t3m = clk::now();
    });
    try {
      // both output arrays in one pass over the pinned workers (identity positions are < n <
      // 2^32: u32 over PCIe, narrowed into the offsets' space, which is free now)
      if (!pos) {
        uint32_t* pos32 = reinterpret_cast<uint32_t*>(c->s_offsets);
        launch_narrow32(c->s_posout, pos32, n, s);
        HIPCHECK(hipStreamSynchronize(s));
        staged_d2h(c, {D2HJob{fp_out, c->s_fp, n * 8, 0}, D2HJob{pos_out, pos32, n * 4, 2}});
      } else {
        staged_d2h(c, {D2HJob{fp_out, c->s_fp, n * 8, 0}, D2HJob{pos_out, c->s_posout, n * 8, 0}});
      }
    } catch (...) {
      tm.join();
      throw;
    }
    const auto t3 = clk::now();
    tm.join();
    if (mrc != S3IMPH_OK) {
      *msg = mmsg;
      if (mph->alloc && mph->buf) {
        std::free(mph->buf);
        mph->buf = nullptr;
      }
    }
    static const bool phases = dev_env("S3IMPH_HOST_PHASES") != nullptr;  // the phase line without debug builds
    if (c->debug || phases) {
      auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
      const auto tx = clk::now();
      std::fprintf(stderr,
                   "[s3imph] host build: entry %.2f + offsets h2d %.2f (as %s; the blob copy beside it) + build %.2f "
                   "(hash launches waited %.2f for blob pieces; blob copied %.2f ms after the start, %d pieces) + "
                   "d2h %.2f + marshal wait %.2f = %.2f ms (marshal ended %.2f ms after the build)\n",
                   ms(t0 - te), ms(t1 - t0), wide.load() ? (off32 ? "u32" : "u64") : "u16 lengths", ms(t2 - t1),
                   ms(t_wait), ms(t_copied - t0), pieces, ms(t3 - t2), ms(tx - t3), ms(tx - te), ms(t3m - t2));
    }
    return mrc;
  } catch (const Fail& f) {
    *msg = f.msg;
    return f.code;
  } catch (const std::bad_alloc&) {
    *msg = "out of host memory";
    return S3IMPH_ERR_NOMEM;
  }
}

// ... and once more when it ran out of HBM, after the other builds' cached workspaces are freed
int build_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                    uint64_t n, uint64_t* fp_out, uint64_t* pos_out, MphOut* mph, std::string* msg) {
  const int rc = build_from_host_once(device, blob, offsets, pos, n, fp_out, pos_out, mph, msg);
  if (rc != S3IMPH_ERR_NOMEM) return rc;
  std::string m2;
  s3imph_ctx* c = default_ctx(device, &m2);
  if (!c) return rc;
  bool freed;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    freed = reclaim_cached(c);
  }
  if (!freed) return rc;
  msg->clear();
  return build_from_host_once(device, blob, offsets, pos, n, fp_out, pos_out, mph, msg);
}

int build_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n,
                    uint64_t* fp_out, uint64_t* pos_out, std::vector<uint8_t>* mph, std::string* msg) {
  MphOut o;
  o.vec = mph;
  return build_from_host(device, blob, offsets, pos, n, fp_out, pos_out, &o, msg);
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
  // Little-endian host: each level's words are copied straight behind its header.
  static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "mph.bin words are little-endian");
  uint8_t* p = out;
  auto put = [&](uint64_t v) {
    std::memcpy(p, &v, 8);
    p += 8;
  };
  put(kPartitions);
  put(st.nlevels);
  for (unsigned L = 0; L < st.nlevels; ++L) {
    put(st.words[L]);
    if (st.words[L]) HIPCHECK(hipMemcpy(p, c->bits + st.woff[L], 8 * st.words[L], hipMemcpyDeviceToHost));
    p += 8 * st.words[L];
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
    if (const char* m = dev_env("S3IMPH_RES_MAX")) c->res_max_keys = std::strtoull(m, nullptr, 10);
    if (const char* m = dev_env("S3IMPH_RES_FILL")) c->res_fill = std::strtoull(m, nullptr, 10);
    if (const char* m = dev_env("S3IMPH_RES0")) c->res0 = std::atoi(m);
    c->loose_geom = dev_env("S3IMPH_LOOSE_GEOM") != nullptr;
    c->route_self = dev_env("S3IMPH_DIST_ROUTE_SELF") != nullptr;  // A/B knob: list-level geometry from 1.1x bounds
    c->debug = std::getenv("S3IMPH_DEBUG") != nullptr;
    c->fault_dup = dev_env("S3IMPH_FAULT_DUP_REC") != nullptr;
    if (const char* m = dev_env("S3IMPH_P0")) c->p0 = std::atoi(m);
    if (const char* m = dev_env("S3IMPH_L20")) c->l20 = std::atoi(m) != 0;
    if (const char* m = dev_env("S3IMPH_BM_LANES")) c->bm_counts = std::strcmp(m, "counts") == 0;
    if (const char* m = dev_env("S3IMPH_SCAT_CFG")) c->scat_cfg = std::atoi(m);
    if (const char* m = dev_env("S3IMPH_SKEW_CFG")) c->skew_cfg = std::atoi(m);
    if (const char* m = dev_env("S3IMPH_DIST_SWITCH")) c->dist_switch = std::strtoull(m, nullptr, 10);
    if (const char* m = std::getenv("S3IMPH_DIST_MODE")) c->d.mode = std::strcmp(m, "bitmap") == 0 ? kDistBitmap : kDistRoute;
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
  fin_scratch_free(c);
  if (c->d.xo) (void)hipStreamSynchronize(c->d.xo);
  delete c->d.xcomm;
  c->d.xcomm = nullptr;
  delete c->d.comm;
  c->d.comm = nullptr;
  if (c->d.xs) (void)hipStreamDestroy(c->d.xs);
  if (c->d.xo) (void)hipStreamDestroy(c->d.xo);
  for (hipEvent_t e : c->d.ev_xg)
    if (e) (void)hipEventDestroy(e);
  if (c->d.ev_xdone) (void)hipEventDestroy(c->d.ev_xdone);
  if (c->d.h_xch) (void)hipHostFree(c->d.h_xch);
  for (hipEvent_t e : {c->d.ev_route, c->d.ev_counts, c->d.ev_x})
    if (e) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  for (hipEvent_t e : c->copy_evs)
    if (e) (void)hipEventDestroy(e);
  if (c->ov_stream) (void)hipStreamDestroy(c->ov_stream);
  for (hipEvent_t e : c->ov_ev)
    if (e) (void)hipEventDestroy(e);
  delete c;
  return S3IMPH_OK;
}

int s3imph_ctx_reserve(s3imph_ctx* c, uint64_t max_keys, uint64_t max_global_keys) {
  if (!c) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(c->device));
    std::string msg;
    return retry_on_nomem(c, nullptr, &msg, [&] {
      if (c->dist)
        ensure_dist_workspace(c, max_keys, std::max(max_keys, max_global_keys));
      else
        ensure_workspace(c, max_keys);
      HIPCHECK(hipDeviceSynchronize());
      return (int)S3IMPH_OK;
    });
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
    c->last_msg.clear();
    int rc = c->dist ? S3IMPH_ERR_STATE : retry_on_nomem(c, s, &msg, [&] {
      return build_single(c, d_blob, d_offsets, d_pos, n, d_fp_out, d_pos_out, s, info, &msg);
    });
    c->last_msg = msg;
    info->status = rc;
    return rc;
  } catch (const Fail& f) {
    c->last_msg = f.msg;
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
  c->profiling = on < 0 ? 0 : on > 2 ? 1 : on;
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
  if (!id || !out || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return S3IMPH_ERR_INVALID;
  int rc = s3imph_ctx_create(device, out, err, errlen);
  if (rc != S3IMPH_OK) return rc;
  s3imph_ctx* c = *out;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  RcclComm* rc_comm = new RcclComm();
  ncclResult_t r = ncclCommInitRank(&rc_comm->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    set_err(err, errlen, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    delete rc_comm;
    s3imph_ctx_destroy(c);
    *out = nullptr;
    return S3IMPH_ERR_RCCL;
  }
  rc_comm->rank = rank;
  rc_comm->nranks = nranks;
  c->dist = true;
  c->d.comm = rc_comm;
  if (nranks > 1) {
    // the output exchange's own communicator (split from this one: the same ranks), so that a
    // level group's exchange on its stream never waits behind, or holds up, the next levels'
    // collectives; every rank keeps it only if every rank got it
    ncclComm_t xc = nullptr;
    const bool got = ncclCommSplit(rc_comm->comm, 0, rank, &xc, nullptr) == ncclSuccess && xc;
    int ok = got ? 1 : 0;
    int* d_ok = nullptr;
    bool agreed = hipMalloc(&d_ok, sizeof(int)) == hipSuccess &&
                  hipMemcpy(d_ok, &ok, sizeof(int), hipMemcpyHostToDevice) == hipSuccess &&
                  ncclAllReduce(d_ok, d_ok, 1, ncclInt32, ncclMin, rc_comm->comm, nullptr) == ncclSuccess &&
                  hipMemcpy(&ok, d_ok, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
    if (d_ok) (void)hipFree(d_ok);
    if (agreed && ok == 1) {
      RcclComm* x = new RcclComm();
      x->comm = xc;
      x->rank = rank;
      x->nranks = nranks;
      c->d.xcomm = x;
    } else if (got) {
      (void)ncclCommDestroy(xc);
    }
  }
  c->d.rank = rank;
  c->d.nranks = nranks;
  return S3IMPH_OK;
}

int s3imph_ctx_create_dist_host(int device, const s3imph_host_comm* comm, int rank, int nranks, s3imph_ctx** out,
                                char* err, size_t errlen) {
  if (!comm || !comm->allgather || !comm->alltoallv || !out || nranks < 1 || nranks > kMaxRanks || rank < 0 ||
      rank >= nranks)
    return S3IMPH_ERR_INVALID;
  int rc = s3imph_ctx_create(device, out, err, errlen);
  if (rc != S3IMPH_OK) return rc;
  s3imph_ctx* c = *out;
  HostComm* hc = new HostComm();
  hc->cb = *comm;
  hc->rank = rank;
  hc->nranks = nranks;
  c->dist = true;
  c->d.comm = hc;
  c->d.rank = rank;
  c->d.nranks = nranks;
  return S3IMPH_OK;
}

int s3imph_build_device_dist(s3imph_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets,
                             const uint64_t* d_pos, uint64_t n_local, uint64_t key_base,
                             uint64_t* d_fp_out, uint64_t* d_pos_out, uint64_t out_cap, uint64_t* out_n,
                             void* stream, s3imph_build_info* info) {
  if (!c || !c->dist || !info || !out_n || (n_local && (!d_blob || !d_offsets))) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  std::string msg;
  try {
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    c->last_msg.clear();
    int rc = build_dist(c, d_blob, d_offsets, d_pos, n_local, key_base, d_fp_out, d_pos_out, out_cap, out_n, s,
                        info, &msg);
    c->last_msg = msg;
    info->status = rc;
    return rc;
  } catch (const Fail& f) {
    c->last_msg = f.msg;
    info->status = f.code;
    return f.code;
  } catch (const std::bad_alloc&) {
    info->status = S3IMPH_ERR_NOMEM;
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_dist_segments(s3imph_ctx* c, uint64_t* seg, uint64_t cap, uint64_t* count) {
  if (!c || !c->dist || !count) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  const uint64_t n = c->d.seg.size() / 3;
  *count = n;
  if (!c->have_build) return S3IMPH_ERR_STATE;
  if (seg && cap) std::memcpy(seg, c->d.seg.data(), 8 * 3 * std::min(n, cap));
  return cap >= n || !seg ? S3IMPH_OK : S3IMPH_ERR_INVALID;
}

int s3imph_ctx_set_dist_mode(s3imph_ctx* c, int mode) {
  const int m = mode & ~S3IMPH_DIST_STRICT;
  if (!c || !c->dist || (m != S3IMPH_DIST_ROUTE && m != S3IMPH_DIST_BITMAP)) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->d.mode = m == S3IMPH_DIST_BITMAP ? kDistBitmap : kDistRoute;
  c->d.strict = (mode & S3IMPH_DIST_STRICT) != 0;
  return S3IMPH_OK;
}

uint64_t s3imph_dist_out_cap(s3imph_ctx* c, uint64_t n_global) {
  if (!c || !c->dist) return n_global;
  return dist_out_cap(c, n_global);
}

const char* s3imph_ctx_last_error(s3imph_ctx* c) { return c ? c->last_msg.c_str() : ""; }

int s3imph_ctx_load_mph_bin(s3imph_ctx* c, const uint8_t* mph_bin, uint64_t len) {
  if (!c || (len && !mph_bin)) return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    HIPCHECK(hipSetDevice(c->device));
    c->have_build = false;
    c->rank_valid = false;
    c->last_msg.clear();
    LevelState h{};
    std::vector<uint64_t> words;  // concatenated level words
    uint64_t keys = 0;
    if (len) {
      // MarshalBinary framing (restated): [u64 partitions][u64 levels]
      // then per level [u64 words][words x u64], little endian; nothing may follow
      static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "mph.bin words are little-endian");
      uint64_t at = 0;
      auto get = [&](uint64_t* v) {
        if (len - at < 8) return false;
        std::memcpy(v, mph_bin + at, 8);
        at += 8;
        return true;
      };
      uint64_t parts = 0, nl = 0;
      if (!get(&parts) || parts != kPartitions || !get(&nl) || nl == 0 || nl > (uint64_t)kMaxLevels) {
        c->last_msg = "open MPHF: unmarshal: bad header";
        return S3IMPH_ERR_FORMAT;
      }
      for (uint64_t L = 0; L < nl; ++L) {
        uint64_t w = 0;
        if (!get(&w) || w > (len - at) / 8) {
          c->last_msg = "open MPHF: unmarshal: truncated level " + std::to_string(L);
          return S3IMPH_ERR_FORMAT;
        }
        if (w == 0) {  // a level holds >= 1 key, so >= 1 word; 0 would make every probe index garbage
          c->last_msg = "open MPHF: unmarshal: empty level " + std::to_string(L);
          return S3IMPH_ERR_FORMAT;
        }
        h.words[L] = w;
        h.woff[L] = words.size();
        h.magic[L] = level_magic(w);
        const size_t o = words.size();
        words.resize(o + w);
        std::memcpy(words.data() + o, mph_bin + at, 8 * w);
        at += 8 * w;
        for (uint64_t q = 0; q < w; ++q) keys += (uint64_t)__builtin_popcountll(words[o + q]);
      }
      if (at != len) {
        c->last_msg = "open MPHF: unmarshal: trailing bytes";
        return S3IMPH_ERR_FORMAT;
      }
      h.nlevels = (unsigned)nl;
      h.woff[nl] = words.size();
      h.rank_total = keys;
      h.out_cap = keys;
    }
    const uint64_t need = std::max<uint64_t>(words.size(), 1);
    if (need > c->cap_words || !c->bits) {
      dalloc(c->bits, need);
      dfree(c->rank_base);
      c->rank_base_cap = 0;
      c->cap_blocks = (need + 2047) / 2048 + 1;
      dalloc(c->block_sums, c->cap_blocks);
      c->cap_words = need;
    }
    if (!c->d_st) dalloc(c->d_st, 1);
    if (!c->h_st) {
      void* hp = nullptr;
      HIPCHECK(hipHostMalloc(&hp, sizeof(LevelState), hipHostMallocDefault));
      c->h_st = static_cast<LevelState*>(hp);
    }
    *c->h_st = h;
    HIPCHECK(hipMemcpy(c->d_st, c->h_st, sizeof(LevelState), hipMemcpyHostToDevice));
    if (!words.empty()) HIPCHECK(hipMemcpy(c->bits, words.data(), 8 * words.size(), hipMemcpyHostToDevice));
    c->info = s3imph_build_info{};
    c->info.num_levels = h.nlevels;
    c->info.total_words = words.size();
    c->info.mph_bin_len = len;
    c->info.n_keys = keys;
    c->last_n = keys;
    c->have_build = true;
    return S3IMPH_OK;
  } catch (const Fail& f) {
    c->last_msg = f.msg;
    return f.code;
  } catch (const std::bad_alloc&) {
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
        if (c->rank_base_cap < 2 * c->cap_words) {  // (word, rank) pairs
          c->rank_base_cap = 0;
          dalloc(c->rank_base, 2 * c->cap_words);
          c->rank_base_cap = 2 * c->cap_words;
        }
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
  MphOut o;
  o.alloc = true;  // marshalled straight into the returned buffer (no second host copy)
  std::string msg;
  int rc = build_from_host(device, blob, offsets, pos, n, fp_out, pos_out, &o, &msg);
  if (rc != S3IMPH_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  *mph_bin = o.len ? o.buf : nullptr;
  if (!o.len) std::free(o.buf);
  *mph_len = o.len;
  return S3IMPH_OK;
}

int s3imph_build_host_into(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos,
                           uint64_t n, uint64_t* fp_out, uint64_t* pos_out, uint8_t* mph_out, uint64_t mph_cap,
                           uint64_t* mph_len, char* err, size_t errlen) {
  if (!mph_len || (n && (!blob || !offsets || !fp_out || !pos_out || !mph_out))) {
    set_err(err, errlen, "invalid argument");
    return S3IMPH_ERR_INVALID;
  }
  *mph_len = 0;
  MphOut o;
  o.buf = mph_out;
  o.cap = mph_cap;
  std::string msg;
  int rc = build_from_host(device, blob, offsets, pos, n, fp_out, pos_out, &o, &msg);
  if (rc != S3IMPH_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  *mph_len = o.len;
  return S3IMPH_OK;
}

uint64_t s3imph_mph_bin_bound(uint64_t n) { return n ? mph_bin_bound(n) : 0; }

int s3imph_release_workspaces(void) {
  release_multi_sets();
  std::lock_guard<std::mutex> glk(g_default_mu);
  for (s3imph_ctx* c : g_default) {
    if (!c) continue;
    std::lock_guard<std::mutex> lk(c->mu);
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    free_workspace(c);
    fin_scratch_free(c);
    c->have_build = false;
    c->rank_valid = false;
  }
  return S3IMPH_OK;
}

void s3imph_free(void* p) { std::free(p); }

}  // extern "C"
