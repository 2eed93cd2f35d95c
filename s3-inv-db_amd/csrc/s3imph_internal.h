// s3imph_internal.h — shared declarations between the kernels, the build
// orchestration and the host-side mirror of StreamingMPHFBuilder.  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "bbhash_spec.h"

namespace s3imph {

// A developer knob's value from the environment, or null unless the caller opted in with
// s3imph_dev_knobs(1) (include/s3imph.h section 7; s3imph_host.cpp).  Every A/B geometry
// knob, test-only fallback and fault hook goes through this; user settings use getenv.
const char* dev_env(const char* name);

// Device-resident per-build level bookkeeping.  Written only by kernels (and the
// init kernel); the host copies it back once, after the build.
struct LevelState {
  unsigned long long n[kMaxLevels + 2];      // active keys entering level L
  unsigned long long words[kMaxLevels + 2];  // u64 words of level L's bit vector
  unsigned long long woff[kMaxLevels + 2];   // first word of level L in the concatenated bits
  unsigned long long magic[kMaxLevels + 2];  // Barrett reciprocal of words[L]
  unsigned long long rank_total;             // popcount over all levels (== N on success)
  unsigned int nlevels;
  unsigned int status;                       // kSt* flags
  unsigned int tail_first;                   // first level run by the single-workgroup tail
  unsigned int skew;                         // sampled key lengths are skewed: hash length-sorted
  unsigned int stop_level;  // kStTooManyLevels: the level whose n[stop_level] keys could not be
                            // placed; they are left in list[(stop_level - 1) & 1]
  unsigned int mid_bar;     // k_mid_levels' grid-barrier counter (zeroed with the rest by k_init_state)
  unsigned int pad0_;
  // Binned pipeline (s3imph_binned.hip).
  unsigned long long lvl_base[kMaxLevels + 2];  // set bits in all levels < L (= ranks[L] - 1)
  unsigned long long ntiles[kMaxLevels + 2];    // position tiles of level L
  unsigned long long nchunks[kMaxLevels + 2];   // key chunks of level L (count/scatter blocks)
  unsigned long long ticket[kMaxLevels + 2];    // tile tickets (look-back order)
  unsigned long long sticket[kMaxLevels + 2];   // histogram-scan segment tickets
  // Output bound and gating.  out_cap: fp_out/pos_out entries (= n on one GPU);
  // out_skip_from != 0 disables output writes of levels >= out_skip_from (the
  // replicated tail levels of a multi-GPU build run on every rank, written by rank 0).
  unsigned long long out_cap;
  unsigned long long out_skip_from;
  // Multi-GPU position-range ownership (s3imph_dist.hip).  A level with preset[L] != 0
  // was sized by the host/collectives: words[L] is the GLOBAL level size, n[L] the
  // records this rank received, and this rank owns words [wlo[L], wlo[L] + rw[L]).
  // Levels with preset[L] == 0 cover the whole level (plo = 0, rw = words).
  unsigned long long preset[kMaxLevels + 2];
  unsigned long long wlo[kMaxLevels + 2];
  unsigned long long rw[kMaxLevels + 2];
  unsigned long long dS[kMaxLevels + 2];       // words per rank range (owner = word / dS)
  unsigned long long dmagic[kMaxLevels + 2];   // Barrett reciprocal of dS
  unsigned long long gn[kMaxLevels + 2];       // global key count of level L
  // P0F (single GPU): level 0's settled keys, counted before its tile kernel (k_p0_count)
  unsigned long long settled0;
  // P0 overlap (single GPU): level-0 hash blocks done, the overlapped scatter's per-XCD tickets
  unsigned int h0_done;
  unsigned int mid_bar2;  // k_mid_levels<kMidGBig>'s grid-barrier counter (zeroed by k_init_state)
  unsigned long long ov_ticket[8];
};

#if defined(__HIPCC__)
// Position range [plo, plo + 64 rw) of level L handled by this GPU.
struct LevelRange {
  uint64_t plo, rw;
};
__device__ __forceinline__ LevelRange level_range(const LevelState* st, int L, uint64_t words) {
  if (st->preset[L]) return {64 * st->wlo[L], st->rw[L]};
  return {0, words};
}
__device__ __forceinline__ bool level_out_on(const LevelState* st, int L) {
  return !(st->out_skip_from && (unsigned long long)L >= st->out_skip_from);
}
#endif

// Binned pipeline geometry.  A level of `size` positions is cut into tiles of 2^tb
// positions (one workgroup each, A/C in LDS); keys are counted and scattered into
// per-tile buckets in chunks of `chunk` keys.
constexpr unsigned kTileMaxBits = 19;                 // 2 x 64 KiB LDS bit vectors
constexpr unsigned kTileMinBits = 10;
constexpr uint64_t kMaxTiles = 4096;                  // tiles per level (LDS histogram / scatter cursors)
constexpr uint64_t kScatterTiles = kMaxTiles;         // LDS-staged scatters (count/start/cursor per tile)
constexpr uint64_t kTargetTiles0 = 2048;              // level 0: 2^14-position tiles at 10M keys
constexpr uint64_t kTargetTiles = 1024;               // levels >= 1 on the counted path
constexpr uint64_t kTargetTilesRes = 256;             // reservation-path levels: ~1 tile per CU
constexpr unsigned kRegTileMaxBits = 14;              // largest tile of the register-resident kernel
// Levels too big for 2^14-position tiles (C3/C4's first levels) take the split kernel's
// 2^15..2^18 tiles, the smallest with at most kSplitTargetTiles tiles: fewer, bigger tiles give
// the reservation scatter longer runs and fewer slot atomics per round (C3 level 0:
// 2^16 / 2^17 / 2^18 tiles, scatter 1.73 / 1.45 / 1.19 ms).
constexpr unsigned kSplitMaxBits = 18;
constexpr int kSplitGridHost = 256;                   // k_tile_split's persistent workgroups (one per CU)
constexpr uint64_t kSplitTargetTiles = 1024;
constexpr uint64_t kHistCap = 8ull << 20;             // tiles x chunks entries
constexpr unsigned kStTailOverflow = 16u;             // tail reached with a level too big for LDS
constexpr unsigned kStGeometry = 32u;                 // tiles/chunks outside the workspace
constexpr unsigned kStLookback = 64u;                 // a look-back wait timed out
constexpr unsigned kStResOverflow = 128u;  // a reservation-path tile slot overflowed (rerun counted)
constexpr uint64_t kSubRound = 4096;                  // keys per LDS-sorted scatter round
constexpr uint64_t kScanSeg = 8192;                   // histogram entries per scan segment

struct LevelGeom {
  unsigned tb;        // tile bits
  uint64_t chunk;     // keys per count/scatter chunk
  unsigned ts = 0;    // split tiles of ts x 2^14 positions (2..16; 0: 2^tb)
};
// Tiles of a level of 64 * rw positions: 2^tb positions each, or ts 2^14-position
// sub-tiles each (split-kernel levels sized for a whole number of rounds over the CUs).
__host__ __device__ inline uint64_t tiles_of(uint64_t rw, unsigned tb, unsigned ts) {
  const uint64_t tp = ts ? (uint64_t)ts << 14 : 1ull << tb;
  return (64 * rw + tp - 1) / tp;
}

// Host-side choice for a level of about n keys: the smallest tile (>= 2^kTileMinBits
// positions) that leaves at most target_tiles tiles, and about target_chunks chunks of
// a multiple of kChunkGran keys (a chunk is one count block's unit of work, so the
// chunk count is sized to fill the resident blocks in one round), few enough that
// tiles x chunks stays under kHistCap.
constexpr uint64_t kChunkGran = 1024;
// Levels take the reservation scatter whenever its slots fit (res_fits), whatever their
// size: a sharded level 0 of 100M records per rank on the counted path (histogram + scan)
// took 4.11 ms against 2.85 ms reserved (C3, N = 1).  S3IMPH_RES_MAX lowers it for tests.
constexpr uint64_t kResMaxKeys = 1ull << 32;
constexpr uint64_t kResSmallKeys = 2ull << 20;  // ... with 4x slot headroom up to this size, 2x above
constexpr int kResShards = 8;                 // per-tile reservation counters (one per XCD)
constexpr int kResLevels = 32;                // levels that may use the reservation path
constexpr uint64_t kTcntStride = kScatterTiles * kResShards;  // tcnt words per level
constexpr double kTailMargin = 1.1;
constexpr uint64_t kTargetChunks = 768;  // 3 resident 1024-thread count blocks x 256 CUs
constexpr uint64_t kBigChunksKeys = 20ull << 20;  // level-0 hash of this many keys or more: 2x the chunks
// n records over `size` positions (64 * level_words(n) for a whole level).
inline LevelGeom choose_geom_sz(uint64_t n, uint64_t size, uint64_t target_tiles = kTargetTiles,
                                uint64_t target_chunks = kTargetChunks, unsigned max_tb = kTileMaxBits) {
  if (size == 0) size = 64;
  unsigned tb = kTileMinBits;
  while (tb < max_tb && (size >> tb) > target_tiles) ++tb;
  while (tb < kTileMaxBits && ((size + (1ull << tb) - 1) >> tb) > kMaxTiles) ++tb;  // workspace bound
  if (tb > kRegTileMaxBits)
    while (tb < kSplitMaxBits && ((size + (1ull << tb) - 1) >> tb) > kSplitTargetTiles) ++tb;
  const uint64_t T = (size + (1ull << tb) - 1) >> tb;
  uint64_t chunk = ((n + target_chunks - 1) / target_chunks + kChunkGran - 1) / kChunkGran * kChunkGran;
  if (chunk < kSubRound) chunk = kSubRound;
  while (((n + chunk - 1) / chunk) * T > kHistCap) chunk *= 2;
  return {tb, chunk};
}
inline LevelGeom choose_geom(uint64_t n, uint64_t target_tiles = kTargetTiles,
                             uint64_t target_chunks = kTargetChunks, unsigned max_tb = kTileMaxBits) {
  return choose_geom_sz(n, 64 * level_words(n ? n : 1), target_tiles, target_chunks, max_tb);
}

// Device status flags.
constexpr unsigned kStKeyZero = 1u;       // some FNV-1a key hash == 0
constexpr unsigned kStTooManyLevels = 2u;  // level budget exhausted (duplicates)
constexpr unsigned kStOverflow = 4u;       // workspace capacity exceeded
constexpr unsigned kStRank = 8u;           // a position landed outside [0, N)
constexpr unsigned kStRouteOverflow = 256u;  // a multi-GPU send region overflowed (rerun bigger)
constexpr unsigned kStBitmapBound = 512u;    // bitmap decomposition: a level outgrew the host's size bound
// Any of these ends the level pipeline: later kernels return at once.
constexpr unsigned kStStop = kStGeometry | kStOverflow | kStLookback | kStTooManyLevels;

// Levels whose active-key count is at most this run inside one workgroup with
// LDS-resident bit vectors (k_tail); larger levels run as full-grid kernels.
constexpr unsigned long long kTailKeys = 12288;
// Mid-size levels (above the tail, at most kMidMaxKeys keys) run inside one persistent
// kernel of kMidG cooperating workgroups (s3imph_binned.hip, k_mid_levels): records in
// registers, routed to the workgroup owning their position's words, grid barriers.
constexpr int kMidG = 64;
constexpr int kMidT = 1024;
constexpr int kMidR = 8;                   // records per thread (registers)
constexpr unsigned kMidSeg = 512;          // exchange records per (owner, sender)
constexpr unsigned kMidStage = 6144;       // settled records staged per owner (LDS)
constexpr unsigned long long kMidMaxKeys = 440ull << 10;  // owners average <= 6.9k of 8k slots
constexpr uint64_t kMidW32 = 2 * ((2 * kMidMaxKeys + 63) / 64);  // u32 words of the largest mid level
// scratch (u32 units): 64 unused (the barrier counter is LevelState::mid_bar), segment counts [kMidG][kMidG], per-owner
// totals [kMidG] u64, then the exchange area [kMidG][kMidG][kMidSeg] Rec
constexpr uint64_t kMidXc = 64;
constexpr uint64_t kMidTot = kMidXc + (uint64_t)kMidG * kMidG;  // even: u64-aligned
constexpr uint64_t kMidXb = kMidTot + 2 * kMidG + 16;          // 16-byte aligned
constexpr uint64_t kMidScratchU32 = kMidXb + (uint64_t)kMidG * kMidG * kMidSeg * 6;
constexpr double kMidMargin = 1.15;  // a level predicted above kMidMaxKeys / kMidMargin stays binned
// The same kernel over every CU (k_mid_levels<kMidGBig>) for the levels above kMidMaxKeys up to
// kMidMaxKeysBig (owners again average <= 6.9k of 8k slots; a level's size is predicted within
// 2 % + 6 sigma, the bound the binned geometry uses): per-(owner, sender) segments of kMidSegBig
// records (a sender's <= 8192 records over 256 owners: 32 on average), its own barrier counter.
constexpr int kMidGBig = 256;
constexpr unsigned kMidSegBig = 128;
constexpr unsigned long long kMidMaxKeysBig = 1750ull << 10;
constexpr uint64_t kMidBigMinKeys = 1ull << 20;  // sets this big get the 256-workgroup scratch
template <int G>
struct MidCfg {
  static constexpr unsigned kSeg = G == kMidG ? kMidSeg : kMidSegBig;
  static constexpr unsigned long long kMax = G == kMidG ? kMidMaxKeys : kMidMaxKeysBig;
  static constexpr uint64_t kW32 = 2 * ((2 * kMax + 63) / 64);  // u32 words of the largest level
  // scratch (u32 units): 64 unused, segment counts [G][G], per-owner totals [G] u64, exchange [G][G][kSeg] Rec
  static constexpr uint64_t kXc = 64;
  static constexpr uint64_t kTot = kXc + (uint64_t)G * G;
  static constexpr uint64_t kXb = kTot + 2 * G + 16;
  static constexpr uint64_t kScratchU32 = kXb + (uint64_t)G * G * kSeg * 6;
};
static_assert(MidCfg<kMidG>::kXb == kMidXb && MidCfg<kMidG>::kScratchU32 == kMidScratchU32, "mid scratch layout");
static_assert(MidCfg<kMidGBig>::kTot % 2 == 0 && MidCfg<kMidGBig>::kXb % 4 == 0, "mid scratch alignment");
constexpr int kTailThreads = 1024;
constexpr int kTailLdsWords32 = 2 * 2 * ((kGammaNum * kTailKeys + 63) / 64);  // A and C, u32 words

struct KernelArgs;  // fwd

// ---- launchers (s3imph_kernels.hip) -------------------------------------------
void launch_init_state(LevelState* st, uint64_t n, uint64_t out_cap, hipStream_t s,
                       const uint64_t* offsets = nullptr);
void launch_rank_scan(const uint64_t* bits, uint64_t cap_words, uint64_t* rank_base,
                      unsigned long long* block_sums, uint64_t max_blocks, LevelState* st,
                      hipStream_t s);
void launch_lookup(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const uint64_t* bits,
                   const uint64_t* rank_base, const LevelState* st, const uint64_t* fp,
                   const uint64_t* pos, uint64_t count, uint64_t* result, int grid, hipStream_t s);

int default_grid(uint64_t work, int block);

// ---- binned pipeline launchers (s3imph_binned.hip) ---------------------------------
// One key in flight between levels: FNV-1a key hash, FNV-1 fingerprint, position
// (the preorder pos the reference's Add received, mphf_streaming.go:68).
struct Rec {
  uint64_t k, f, p;
};

// The host build's key bytes arriving over PCIe (build_from_host): ensure(k) returns once
// keys [0, k) — and the 16 bytes after them, which the hash's wide loads may touch — are on
// the device, ordered before anything enqueued on the build stream afterwards.  The level-0
// hash is then launched in `pieces` launches, each as soon as its keys have arrived, so it
// runs beside the rest of the copy.
struct HashFeed {
  std::function<void(uint64_t)> ensure;
  int pieces = 16;
};

struct BinBuffers {
  uint64_t *kh, *fp;                    // level-0 hashes (key order)
  const uint64_t* pos;                  // caller positions (nullable: identity)
  uint64_t pos_base;
  Rec* bucket;                          // records grouped by position tile
  Rec* list[2];                         // next-level records (ping-pong)
  unsigned *hist, *off;                 // tiles x chunks histogram and its exclusive scan
  unsigned* tile_start;                 // kMaxTiles + 1
  unsigned* scan_sums;                  // scan block sums
  unsigned long long* flags;            // decoupled look-back words, one per tile
  unsigned long long* sflags;           // look-back words of the histogram scan
  unsigned* tcnt;                       // reservation-path shard fills, kResLevels x kScatterTiles x kResShards
  uint64_t bucket_cap;                  // bucket capacity in records
  unsigned long long* tile_prof;        // debug: per (level, tile) phase timestamps, or null
  uint64_t* bits;
  uint64_t cap_words;
  uint64_t* fp_out;
  uint64_t* pos_out;
  LevelState* st;
  bool dist;                            // multi-GPU owner levels: level 0 reads list[1] too
  bool padded = false;                  // list levels hold k = 0 padding records (fixed exchange regions)
  uint32_t* mid;                        // k_mid_levels scratch (kMidScratchU32)
  Rec* split;                           // k_tile_split scratch (split_scratch_records()), or null
  int scat_cfg = 2;                     // k_scatter_res forms (launch_binned_scatter_res)
  bool pipe_tiles = false;              // 2^14 reservation tiles on k_tile_p0 (else k_tile_reg)
  int skew_cfg = 2;                     // k_hash_skew block / group shape (launch_hash_skew)
  // bit L (L >= 1): level L's input list holds R20 records (k, f, key index; identity
  // positions) instead of Rec: its producer (k_tile_p0 / k_tile_split of level L - 1) writes
  // them, its reservation scatter reads them and keeps them R20 in the slots, and its tile
  // kernel (k_tile_p0 / k_tile_split) reads R20 — 4 bytes less per record on every pass
  unsigned l20 = 0;
  bool list20(int L) const { return L >= 1 && L < 32 && ((l20 >> L) & 1u); }
  const HashFeed* feed = nullptr;  // level 0's key bytes still arriving (host build), or null
};
uint64_t split_scratch_records();  // sub-tile segments of the split big-tile kernel

// ---- P0: level 0 of a big set in 2^14-position register tiles (s3imph_binned.hip) ----
// Sets whose level 0 has more than kP0MinTiles 2^14-position tiles (the ones the split
// kernel took) with identity positions: the level's tiles are grouped into S super-tiles of
// tps tiles (tps <= kP0MaxTps); records (R20: k, f, key index) go to per-(super-tile, XCD
// shard) slots of `sup`, then to per-(tile, shard) slots of `bucket`, then k_tile_reg.
constexpr uint64_t kP0MinTiles = 2048;
constexpr uint64_t kP0MaxTps = 1024;
// tiles per super-tile aimed at: fewer super-tiles give the fused hash partition longer region
// runs (C3 hash 2.69 -> 2.67 ms at 24 super-tiles vs 64), and the super-tile scatter's blocks
// (kP0ScatterBlocks in all) still reach ~12 records per tile and round
constexpr uint64_t kP0TargetTps = 512;
// the super-tile scatter's blocks: three waves of 1024-thread blocks over the 256 CUs, blocks per
// super-tile a multiple of the 8 XCD shards (C3: 24 x 32; 6.55-6.57 ms against 6.63-6.67 for
// 64 x 8 in two same-box sweeps, `gpurun_out` r4_sweep / r4_sweep2)
constexpr unsigned kP0ScatterBlocks = 768;
// at most 64 super-tiles (C3: 64).  k_scatter_p0 gives each one max(256 / S, 8) blocks of 1024
// threads, a multiple of 8 (past 32 super-tiles: 512 blocks in two waves over the CUs; with
// S3IMPH_P0_BIG=0, 8 blocks of 512 threads, two per CU), so the records of a tile arrive through
// all kResShards XCD shards (4 blocks per super-tile filled only 4 of a tile's 8 shard slots:
// twice their capacity on average, C3 overflowed into the rerun).  S3IMPH_P0_MAXS lowers the cap.
constexpr uint64_t kP0MaxS = 64;
constexpr unsigned kP0OneBlockS = 32;  // the most super-tiles the 256 blocks of one wave cover
constexpr uint64_t kP0MaxKeys = 1ull << 31;  // bucket slot indices stay below 2^32
// A level-0 record with an identity position: k (2 dwords), f (2), key index i (p = pos_base + i).
struct R20 {
  uint32_t w[5];
};
struct P0Bufs {
  unsigned S = 0, tps = 0;     // super-tiles, 2^14 tiles per super-tile
  R20* sup = nullptr;          // the super-tiles' records: per-(hash block, super-tile) regions of reg_cap
                               // (fused hash), or S x kResShards slots of sup_cap / (S kResShards) (pass)
  uint64_t sup_cap = 0;        // R20 records in sup
  uint64_t reg_cap = 0;
  uint64_t reg_cap_skew = 0;   // the same for k_hash_skew's p0_skew_blocks blocks (a skewed set)
  unsigned* pcnt = nullptr;    // region fills (kH0Grid x S), written by the hash
  unsigned* scnt = nullptr;    // super-tile slot fills (S x kResShards), zeroed before the build
  R20* bucket = nullptr;       // tile slots (T x kResShards)
  uint64_t bucket_cap = 0;     // R20 records in bucket
  unsigned* tcnt = nullptr;    // tile slot fills (T x kResShards), zeroed before the build
  unsigned long long* flags = nullptr;  // look-back words, one per tile
  // tile bits: kRegTileMaxBits for k_tile_p0; the bitmap decomposition's level 0 takes 2^tb
  // positions per tile (up to kBmP0MaxTb), so a rank's share of a tile stays ~8k records
  unsigned tb = kRegTileMaxBits;
  uint16_t* x = nullptr;       // bitmap decomposition: each slot's position in its tile (the mark's input)
  unsigned nb = 0;             // the regions' producer blocks (0: the level-0 hash's grid; a bitmap
                               // list level fed by the previous settle: its grid, NextPart)
  // level 0 with the super-tile scatter overlapped on the hash (single GPU, fused regions):
  // each hash block's XCD (kH0GridHost) and the parts the overlapped launch finished
  // (8 kP0OvChunks x S); null otherwise
  unsigned* hxcc = nullptr;
  unsigned* ov_done = nullptr;
  // super-tiles in 2^14-position units (tps tiles of 2^tb): the partition passes cut
  // (position >> 14) by this, so they need not know tb
  unsigned tps_sub() const { return tps << (tb - kRegTileMaxBits); }
};
void launch_p0_partition(const BinBuffers& b, const P0Bufs& p, hipStream_t s, bool only_skew);
// level 0's hash with the first partition fused in where it can be (else hash, then partition)
void launch_p0_hash(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                    const P0Bufs& p, hipStream_t s);
// level > 0 (the bitmap decomposition's R20 list levels): after launch_p0_partition_list
void launch_p0_scatter(const BinBuffers& b, const P0Bufs& p, bool fused, hipStream_t s, int level = 0);
void launch_p0_partition_list(int level, const BinBuffers& b, const P0Bufs& p, hipStream_t s);
bool p0_fused(const uint8_t* blob, const P0Bufs& p);  // the hash partitions (aligned blob, S <= kMaxRanks)
uint64_t p0_region_cap(uint64_t n, unsigned S, unsigned blocks);  // records per (hash block, super-tile) region
unsigned p0_skew_blocks(int skew_cfg);               // k_hash_skew's grid (its fused partition's blocks)
constexpr int kH0GridHost = 4096;                    // = k_hash0_pair's grid (kH0Grid)
constexpr int kP0FedGrid = 256;                      // P0F: level 0's tile kernel blocks (level 1's region producers)
void launch_p0_tile(const BinBuffers& b, const P0Bufs& p, hipStream_t s);
// level 0's super-tile scatter in its direct form: ov, the persistent launch beside the hash;
// otherwise the follow-up over the parts it left (or all of them)
constexpr unsigned kP0OvChunks = 8;  // hash-block chunks per XCD (kH0GridHost / 64 blocks each)
void launch_p0_scatter_direct(const BinBuffers& b, const P0Bufs& p, bool ov, hipStream_t s);
// P0F: level 1 fed by level 0's tile kernel (s3imph_binned.hip).  launch_p0_count: level 0's
// settled keys from the slots' in-tile positions (p.x), then level 1 sized on the device;
// launch_p0_tile_fed: level 0's tiles with the collided records into level 1's super-tile
// regions (np); launch_p0_tile_level: a list level's 2^14 tiles from the super-tile slots
void launch_p0_count(const BinBuffers& b, const P0Bufs& p, hipStream_t s);
struct NextPart;
void launch_p0_tile_fed(const BinBuffers& b, const P0Bufs& p, const NextPart& np, hipStream_t s);
void launch_p0_tile_level(int level, const BinBuffers& b, const P0Bufs& p, hipStream_t s);
void binned_set_lds_limits();
void launch_binned_count(int level, const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b,
                         LevelGeom g, int grid_chunks, hipStream_t s, bool histogram = true);
void launch_binned_scan(int level, const BinBuffers& b, int grid, hipStream_t s);
void launch_binned_scatter(int level, const BinBuffers& b, LevelGeom g, hipStream_t s);
void launch_binned_tile(int level, const BinBuffers& b, LevelGeom g, int grid_tiles, hipStream_t s,
                        bool reserved = false);
// tmax: an upper bound on the level's tiles (0: unknown, the 4096-tile kernel)
void launch_binned_scatter_res(int level, const BinBuffers& b, LevelGeom g, int grid, hipStream_t s,
                               uint64_t i_lo = 0, uint64_t i_hi = 0, uint64_t tmax = 0);
void launch_binned_tail(int first_level, int big_launched, const BinBuffers& b, hipStream_t s);
// levels L0..L1 (each predicted above the tail and at most kMidMaxKeys keys; big: at most
// kMidMaxKeysBig, over kMidGBig workgroups) in one launch
void launch_binned_mid(int L0, int L1, const BinBuffers& b, hipStream_t s, bool big = false);

// ---- multi-GPU launchers (s3imph_dist.hip) ------------------------------------------
constexpr int kMaxRanks = 64;
// Level-0 routing of the multi-GPU build (k_route, or fused into the level-0 hash kernel):
// record (kh, fp, pos) of key i goes to its owner's send region [o*cap, (o+1)*cap), this
// rank's own records to self_dst (capacity self_cap), counted in scnt like any owner's.
// mat_prev (nullable) holds the gathered (P + 1) x P counts of the key chunks routed
// before: self_dst then starts past the records received for them (chunked level 0).
struct Route0 {
  const uint64_t* pos;  // caller positions of these keys, or null: pos_base + i
  uint64_t pos_base;
  Rec* send;
  uint64_t cap;
  unsigned long long* scnt;
  Rec* self_dst;
  uint64_t self_cap;
  const unsigned long long* mat_prev;
  int P, rank;
};
// The level-0 hash with the route fused in (no kh / fp arrays; a skewed set, decided on
// the device, goes through k_hash_count0 + k_route instead).  b.kh / b.fp are scratch
// for that fallback.
void launch_hash0_route(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                        int grid, const Route0& rt, hipStream_t s);
// Records owned by `rank` itself go straight to self_dst (capacity self_cap), not to a send region.
// level-0 records from the hash kernel's kh / fp arrays (multi-GPU build)
void launch_route0_arrays(const uint64_t* kh, const uint64_t* fp, const uint64_t* pos, uint64_t pos_base, uint64_t n,
                          Rec* send, uint64_t cap, unsigned long long* scnt, LevelState* st, int P, int rank,
                          Rec* self_dst, uint64_t self_cap, hipStream_t s);
// the same from a Route0 (only_skew: nothing to do unless st->skew, i.e. unless the fused
// hash kernel left this set to k_hash_count0)
void launch_route0_arrays(const uint64_t* kh, const uint64_t* fp, uint64_t n, const Route0& rt, LevelState* st,
                          bool only_skew, hipStream_t s);
// the level-0 hash kernel alone (kh, fp in key order; no histogram)
void launch_hash0_only(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                       int grid, hipStream_t s);
void launch_route(int level, const Rec* list, uint64_t n_pred, Rec* send, uint64_t cap, unsigned long long* scnt,
                  LevelState* st, int P, int rank, Rec* self_dst, uint64_t self_cap, hipStream_t s);
void launch_dist_setup(LevelState* st, int L, const unsigned long long* gcount, uint64_t n_value, int rank, int P,
                       hipStream_t s);
void launch_set_u64(unsigned long long* p, uint64_t v, hipStream_t s);
void launch_route_flag(LevelState* st, unsigned long long* scnt, int P, hipStream_t s);
void launch_route_pad(Rec* send, uint64_t C, const unsigned long long* scnt, int P, int rank, Rec* self_region,
                      hipStream_t s);
void launch_dist_replicate(LevelState* st, int L, uint64_t n_all, uint64_t skip_from, hipStream_t s);

// ---- the bitmap decomposition of the multi-GPU build (s3imph_bitmap.hip) --------------
void launch_bm_check(LevelState* st, int level, uint64_t wmax, hipStream_t s);
// k_dist_setup (setup: from *gcount), k_bm_range and k_bm_check of level L in one launch
void launch_bm_level_begin(LevelState* st, int L, bool setup, const unsigned long long* gcount, int rank, int P,
                           uint64_t wmax, hipStream_t s);
// nib: count lanes are nibbles (two positions per byte; P <= kBmNibRanks), else bytes
constexpr int kBmNibRanks = 7;
// What crosses xGMI per position and level: a count byte, a count nibble (both summed by an
// RCCL reduce-scatter), or the 2-bit (A, C) planes (an all-to-all and k_bm_merge; default)
constexpr int kBmBytes = 0, kBmNibbles = 1, kBmPlanes = 2;
void launch_bm_decide(const uint8_t* slice, uint64_t S, uint64_t* out, const LevelState* st, bool nib, hipStream_t s);
// Bitmap levels are scattered into tiles of 2^tb positions, kBmMinTb <= tb <= kBmMaxTb, at
// most kScatterTiles of them (levels of up to 2^31 positions); the settle kernel keeps 18 B
// per tile word in LDS: 144 KiB at 2^19 positions.
constexpr unsigned kBmMinTb = 14, kBmMaxTb = 19;
// the largest tile whose settle stages its settled keys in LDS and the largest tile of the
// bitmap level 0 through P0 (2^16 positions: in-tile positions are u16; a rank's ~4k records
// of a tile at P = 8)
constexpr unsigned kBmP0MaxTb = 16;
constexpr uint64_t kBmP0MinTiles = 256;  // the bitmap level 0 takes P0 from this many tiles (one per CU)
// tiles of a bitmap level: kScatterTiles from the reservation scatter, or up to kBmMaxTiles
// 2^14-position tiles from the P0 super-tile scatter (level 0)
constexpr uint64_t kBmMaxTiles = 32768;
// level end: per-tile totals of the final bits -> tbase[2t] (rank within the level), tbase[2t+1]
// (first slot in this rank's settled list, continuing *out_cnt, which it then advances)
void launch_bm_level_end(int level, const uint64_t* g, const uint64_t* A, unsigned tb, uint64_t tiles, uint64_t* bits,
                         unsigned long long* tsum, unsigned long long* tbase, LevelState* st,
                         unsigned long long* gslot, unsigned long long* out_cnt, hipStream_t s);
void bm_set_lds_limits();
void launch_bm_range(LevelState* st, int level, hipStream_t s);
// bucket: Rec slots, or (r20) the P0 super-tile scatter's R20 slots of 2^14-position tiles
// (level 0 with identity positions p = pos_base + key index)
// xs (nullable): each slot's position (P0's level 0, R20 slots)
void launch_bm_tile_mark(int level, const void* bucket, bool r20, const unsigned* tc, uint64_t bucket_cap, unsigned tb,
                         uint64_t tiles, const LevelState* st, uint64_t wpad, uint8_t* lanes, uint64_t* A, int mode,
                         uint64_t S, hipStream_t s, const uint16_t* xs = nullptr);
// the all-to-all's (A, C) plane slices (P of them, 2 S words each) -> this rank's final bits
void launch_bm_merge(const uint64_t* recv, uint64_t S, int P, uint64_t* out, const LevelState* st, hipStream_t s);
// This rank's output slice [lo, lo + cnt) of the global outputs (slices of `slice` keys,
// mslice = level_magic(slice)): settled keys with p in it go straight to fp_out / pos_out;
// scnt[t] (P + 1 counters, zeroed before the first level) counts every settled key of slice t.
struct OwnSlice {
  uint64_t lo, cnt, slice, mslice;
  int rank, P;
  uint64_t *fp_out, *pos_out;
  unsigned long long* scnt;
};
// A bitmap level's settle partitioning its collided records straight into the NEXT level's
// super-tile regions, as the level-0 hash does for level 0 (the next level then skips
// launch_p0_partition_list): R20 records in per-(settle block, super-tile) regions of reg_cap,
// fills to pcnt[block][S].  The next level's exact size is known by then: gnext, its global key
// count, is written by this level's tile scan, which runs before the settle.
struct NextPart {
  R20* sup = nullptr;
  uint64_t reg_cap = 0;
  unsigned* pcnt = nullptr;
  unsigned tps_sub = 0, S = 0;  // super-tiles in 2^14-position units (P0Bufs::tps_sub), their count
  const unsigned long long* gnext = nullptr;
};
int bm_settle_threads(unsigned tb, int P, bool staged);  // the settle's block size
unsigned bm_settle_grid(uint64_t tiles, int threads);     // ... and its blocks (the regions' producers)
void launch_bm_flag(LevelState* st, unsigned flags, hipStream_t s);  // or device status flags
void launch_bm_tile_settle(int level, const void* bucket, bool r20, uint64_t pos_base, const unsigned* tc,
                           uint64_t bucket_cap, unsigned tb, uint64_t tiles, LevelState* st, const uint64_t* g,
                           const uint64_t* A, const unsigned long long* tbase, Rec* out, uint64_t out_cap, Rec* next,
                           uint64_t next_cap, bool next20, const OwnSlice& os, hipStream_t s, bool staged = false,
                           const uint16_t* xs = nullptr, bool o16 = false, const NextPart* np = nullptr);
// a settled key crossing to its output slice's owner with identity positions (16 B instead
// of a 24-B Rec): p - the slice's first p, the sending rank's key index, the fingerprint
struct BmT16 {
  uint32_t off, idx;
  uint64_t f;
};

// P > 1: the slice's settled keys from the P p-sorted runs (runs: device array of P
// {base, n, key_base}) merged through LDS windows over slice offsets [first, limit) (a group of
// levels' keys, below the replicated tail); bnd: scratch of bm_place_bound_words(P, limit) u32
void launch_bm_place_merge(const void* runs, bool k16, int P, uint64_t lo, uint64_t first, uint64_t limit,
                           uint32_t* bnd, uint64_t* fp_out, uint64_t* pos_out, LevelState* st, hipStream_t s);
uint64_t bm_place_bound_words(int P, uint64_t limit);
void launch_bm_tail_copy(const uint64_t* sfp, const uint64_t* spos, uint64_t g0, uint64_t total, uint64_t lo,
                         uint64_t cnt, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s);

// ---- host-memory builds (s3imph_build.hip, s3imph_multi.hip) -------------------------
// Where a host build puts mph.bin: a vector (resized to fit), the caller's buffer of cap
// bytes (reused across calls: no fresh pages), or (alloc) a malloc'd buffer of its exact
// size that the caller frees (s3imph_build_host's contract).  len is set on success.
struct MphOut {
  std::vector<uint8_t>* vec = nullptr;
  uint8_t* buf = nullptr;
  uint64_t cap = 0;
  bool alloc = false;
  uint64_t len = 0;
};
int build_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n,
                    uint64_t* fp_out, uint64_t* pos_out, MphOut* mph, std::string* msg);
int build_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n,
                    uint64_t* fp_out, uint64_t* pos_out, std::vector<uint8_t>* mph, std::string* msg);
// mph.bin's size bound for n keys (the caller buffer of s3imph_build_host_into)
uint64_t mph_bin_bound(uint64_t n);
int build_from_host_multi(const std::vector<int>& devs, unsigned flags, const uint8_t* blob, const uint64_t* offsets,
                          const uint64_t* pos, uint64_t n, uint64_t* fp_out, uint64_t* pos_out,
                          std::vector<uint8_t>* mph, std::string* msg);

// ---- the builder mirror's key store and feed (s3imph_feed.hip) ----------------------
// Keys appended by Add are copied once into pooled pinned chunks (the builder's host copy)
// and DMA'd to device arrays chunk by chunk; Build runs on those, then streams mph_fp
// (array 0) / mph_pos (array 1) to a sink chunk by chunk, one thread per array.
struct FeedSink {
  virtual ~FeedSink() = default;
  virtual bool put(int arr, const uint64_t* v, uint64_t cnt) = 0;  // false: stop taking data
  virtual std::string error() const = 0;
};
struct Feed;
Feed* feed_new(int device, bool use_gpu);  // use_gpu false: host chunks only (multi-GPU, no GPU)
void feed_free(Feed* f);
void feed_drop_device(Feed* f);  // stop feeding the device (the host copy stays)
int feed_reserve(Feed* f, uint64_t n_keys, uint64_t n_bytes, std::string* msg);
bool feed_add(Feed* f, const uint8_t* key, uint64_t len, uint64_t pos);  // false: out of host memory
// n keys of the caller's blob (offsets[0..n], any base); pos NULL -> count, count+1, ...
bool feed_add_batch(Feed* f, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n);
uint64_t feed_count(const Feed* f);
void feed_flush(Feed* f);              // enqueue the partial chunks (may turn the device path off)
bool feed_on_device(const Feed* f);
// contiguous copies (offsets N+1 from 0; blob padded to whole words + 16 B) for the host
// builds, MOVED out of the chunks (each chunk is released as it is copied, so the host copy
// never exists twice); the feed takes no more keys afterwards
void feed_take_host(Feed* f, std::vector<uint8_t>* blob, std::vector<uint64_t>* offsets, std::vector<uint64_t>* pos);
int feed_write_prefix_files(const Feed* f, const std::string& dir, std::string* msg);
// the single-GPU build on the fed arrays; open_sink() is called only once the build succeeded
int feed_build(Feed* f, std::vector<uint8_t>* mph, const std::function<FeedSink*()>& open_sink, std::string* msg);

// ---- host helpers (s3imph_host.cpp) -------------------------------------------
void set_err(char* err, size_t errlen, const std::string& msg);
void s3id_header(uint8_t out[kS3idHeaderSize], uint64_t count, uint32_t width);  // format.go:25-32
// a file made of `count` pieces, piece(i, &p, &n, &off) giving bytes p[0..n) at file offset
// off; the pieces are pwrite()-n by up to 8 threads
bool write_pieces(const std::string& path, size_t count,
                  const std::function<void(size_t, const uint8_t**, uint64_t*, uint64_t*)>& piece, std::string* msg);
int write_index_files(const std::string& dir, const uint8_t* mph_bin, uint64_t mph_len,
                      const uint64_t* fp, const uint64_t* pos, uint64_t n, const uint8_t* blob,
                      const uint64_t* offsets, std::string* msg);

}  // namespace s3imph
