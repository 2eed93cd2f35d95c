// s3imph_ctx.h — the device context and the pieces of the build orchestration shared by
// s3imph_build.hip (single-GPU and per-rank builds, the device-side C ABI) and
// s3imph_multi.hip (multi-GPU builds behind the host-memory boundary).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "s3imph.h"
#include "s3imph_internal.h"

namespace s3imph {

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

// Collectives of the multi-GPU build, on device buffers, ordered on stream s.
struct Comm {
  int rank = 0, nranks = 1;
  virtual ~Comm() = default;
  // d_recv[r * bytes ..) <- rank r's d_send[0 .. bytes)
  virtual void allgather(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) = 0;
  // d_recv[0 .. bytes) <- byte-wise sum over ranks of their d_send[rank * bytes ..) (u8, mod 256)
  virtual void reduce_scatter_u8(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) = 0;
  // element-wise u64 sum over ranks
  virtual void allreduce_u64(const unsigned long long* d_in, unsigned long long* d_out, uint64_t count,
                             hipStream_t s) = 0;
  // d_send + soff[q] (sbytes[q] bytes) -> rank q; rank q's bytes -> d_recv + roff[q] (rbytes[q]); host arrays
  virtual void alltoallv(const void* d_send, const uint64_t* soff, const uint64_t* sbytes, void* d_recv,
                         const uint64_t* roff, const uint64_t* rbytes, hipStream_t s) = 0;
  // a peer failed: make every pending and future collective of this rank return (RCCL:
  // ncclCommAbort, whose kernels then exit); the communicator is unusable afterwards
  virtual void abort() {}
  // this rank has its GPU to itself (RCCL: one rank per device); the host transports let
  // ranks share one, so no kernel of a rank may wait for all of the GPU's CUs at once
  virtual bool owns_gpu() const { return false; }
};

constexpr uint64_t kDistSwitchKeysDefault = 2ull << 20;  // levels below this run replicated

// Decomposition of the multi-GPU levels (s3imph_ctx_set_dist_mode / S3IMPH_DIST_MODE).
constexpr int kDistRoute = 0;   // records routed to the owner of their position range (s3imph_dist.hip)
constexpr int kDistBitmap = 1;  // count-lane reduction of the collision bitmap (s3imph_bitmap.hip)

struct DistState {
  Comm* comm = nullptr;
  int rank = 0, nranks = 1;
  uint64_t cap_list = 0, cap_send = 0, cap_stage_words = 0;
  Rec* send = nullptr;                       // per-owner send regions / replicated gather staging
  uint64_t* stage_bits = nullptr;            // level bit-vector all-gather staging
  unsigned long long* scnt = nullptr;        // per-owner send counts (nranks)
  unsigned long long* mat = nullptr;         // all-gathered send counts (nranks x nranks)
  unsigned long long* gslot = nullptr;       // per-level global counts (kMaxLevels + 2)
  unsigned long long* small = nullptr;       // scratch for tiny collectives (2 x 64 x 64)
  unsigned long long* h_pinned = nullptr;    // host staging (64 x 64 + 256 u64)
  std::vector<uint64_t> seg;                 // last build: (p_lo, count, local_off) triples
  uint64_t out_n = 0;
  // bitmap decomposition workspace: local A / C marks, count lanes, this rank's summed
  // slice, the gathered final bits, their word prefix and block sums
  uint64_t *bm_a = nullptr, *bm_g = nullptr, *bm_dec = nullptr;
  uint8_t *bm_lanes = nullptr, *bm_slice = nullptr, *bm_recv = nullptr;
  unsigned long long* bm_tsum = nullptr;   // per-tile totals of a level (kScatterTiles)
  unsigned long long* bm_tbase = nullptr;  // per-tile (rank, slot) bases (2 kScatterTiles)
  uint64_t bm_cap_words = 0;
  Rec* bm_out = nullptr;  // this rank's settled (p, fp, pos) triples (the tail's tile kernels own the bucket)
  uint64_t bm_cap_out = 0;
  uint32_t* bm_bnd = nullptr;  // the output merge's window bounds (launch_bm_place_merge)
  uint64_t bm_bnd_cap = 0;
  int mode = kDistRoute;
  bool strict = false;  // S3IMPH_DIST_STRICT: the bitmap decomposition may not fall back to routing
  // level 0's exchange runs on its own stream, chunk by chunk, beside the next chunk's hash
  hipStream_t xs = nullptr;
  hipEvent_t ev_route = nullptr, ev_counts = nullptr, ev_x = nullptr;
  // the bitmap decomposition's output exchange by level group (levels 0 and 1 as soon as they
  // are settled, then the rest): per group the settle's per-slice counts, gathered
  // (device + pinned mirror), the merge's run descriptors; the received entries; the exchange's
  // stream, its group events and its completion; its communicator (RCCL: split from `comm`, so
  // the exchange runs beside the next levels' collectives; null: `comm` on the build's stream)
  unsigned long long* xch = nullptr;
  unsigned long long* h_xch = nullptr;
  uint8_t* xrecv = nullptr;
  uint64_t cap_xrecv = 0;  // bytes
  hipStream_t xo = nullptr;
  hipEvent_t ev_xg[4] = {}, ev_xdone = nullptr;
  Comm* xcomm = nullptr;
  std::string agree_msg;  // message of a failure agreed inside route0_chunked
};

// RCCL over xGMI: all-to-all as grouped point-to-point send/recv (xGMI is a full mesh
// of point-to-point links, so every pair streams on its own link), all-gathers and
// all-reduces as RCCL collectives; the rank's own share is a device-to-device copy.
struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;  // written once, before any collective; never reset (abort keeps it)
  std::atomic<bool> aborted{false};
  ~RcclComm() override {
    if (comm && !aborted.load()) (void)ncclCommDestroy(comm);
  }
  // Called from a failing peer's thread (s3imph_multi.hip): ncclCommAbort makes this rank's
  // pending collectives return.  The handle is left as it is — the owning rank thread may be
  // reading it — and the owning thread's next collective throws instead of enqueueing on the
  // aborted communicator (a collective already being enqueued when the abort lands fails
  // inside RCCL and throws the same way).
  void abort() override {
    bool expected = false;
    if (comm && aborted.compare_exchange_strong(expected, true)) (void)ncclCommAbort(comm);
  }
  bool owns_gpu() const override { return true; }
  void live() const {
    if (aborted.load(std::memory_order_acquire))
      throw Fail{S3IMPH_ERR_RCCL, "RCCL communicator aborted: a peer rank failed"};
  }
  void allgather(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    live();
    NCCLCHECK(ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, s));
  }
  void reduce_scatter_u8(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    live();
    NCCLCHECK(ncclReduceScatter(d_send, d_recv, bytes, ncclUint8, ncclSum, comm, s));
  }
  void allreduce_u64(const unsigned long long* d_in, unsigned long long* d_out, uint64_t count,
                     hipStream_t s) override {
    live();
    NCCLCHECK(ncclAllReduce(d_in, d_out, count, ncclUint64, ncclSum, comm, s));
  }
  void alltoallv(const void* d_send, const uint64_t* soff, const uint64_t* sbytes, void* d_recv,
                 const uint64_t* roff, const uint64_t* rbytes, hipStream_t s) override {
    live();
    const char* sb = static_cast<const char*>(d_send);
    char* rb = static_cast<char*>(d_recv);
    NCCLCHECK(ncclGroupStart());
    for (int q = 0; q < nranks; ++q) {
      if (q == rank) continue;
      if (sbytes[q]) NCCLCHECK(ncclSend(sb + soff[q], sbytes[q], ncclUint8, q, comm, s));
      if (rbytes[q]) NCCLCHECK(ncclRecv(rb + roff[q], rbytes[q], ncclUint8, q, comm, s));
    }
    NCCLCHECK(ncclGroupEnd());
    if (sbytes[rank])
      HIPCHECK(hipMemcpyAsync(rb + roff[rank], sb + soff[rank], sbytes[rank], hipMemcpyDeviceToDevice, s));
  }
};

// Pinned staging for host-memory builds (the Go caller's buffers are pageable):
// kStageWorkers threads, each with its own pinned chunk buffer and stream, move the
// data through pinned memory, so the CPU copies of one worker overlap the DMA of the
// others and the PCIe link runs at its pinned rate.
constexpr int kStageWorkers = 8;
constexpr int kCopyPieces = 16;  // the host build's blob H2D pieces (at most; 256 MiB or more each)
constexpr uint64_t kStageChunk = 8ull << 20;

struct Stager {
  void* pin[kStageWorkers][2] = {};  // double-buffered: one chunk in DMA while the other is copied
  hipStream_t st[kStageWorkers] = {};
  hipEvent_t ev[kStageWorkers][2] = {};
  bool ready = false;
};

}  // namespace s3imph

using s3imph::DistState;
using s3imph::LevelState;
using s3imph::Rec;
using s3imph::Stager;

namespace s3imph {
struct FinScratch;  // s3imph_finalize.hip
}

struct s3imph_ctx {
  int device = 0;
  s3imph::FinScratch* fin = nullptr;  // finalize-pass scratch (s3imph_finalize.hip), lazily made
  uint32_t* mid = nullptr;            // k_mid_levels scratch (kMidScratchU32, or the 256-workgroup form's), lazily made
  uint64_t mid_cap = 0;               // ... its u32 words
  Rec* split = nullptr;               // k_tile_split scratch, made for sets big enough for 2^15+ tiles
  hipStream_t own_stream = nullptr;
  std::mutex mu;

  uint64_t cap_keys = 0, cap_words = 0, cap_blocks = 0;
  uint64_t *kh = nullptr, *fp = nullptr, *bits = nullptr, *rank_base = nullptr;
  uint64_t rank_base_cap = 0;  // words of rank_base (the Lookup directory, made on first lookup)
  unsigned long long* block_sums = nullptr;
  LevelState* d_st = nullptr;
  LevelState* h_st = nullptr;
  bool rank_valid = false;                   // rank_base matches the last build

  // single-GPU binned pipeline (s3imph_binned.hip)
  Rec* bucket = nullptr;
  Rec* list[2] = {nullptr, nullptr};
  uint64_t bucket_cap = 0;                   // records in bucket / each list
  unsigned *hist = nullptr, *hoff = nullptr, *tile_start = nullptr, *scan_sums = nullptr;
  unsigned long long* flags = nullptr;
  unsigned long long* sflags = nullptr;
  unsigned* tcnt = nullptr;  // reservation-path shard fills, kResLevels x kScatterTiles x kResShards
  uint64_t res_max_keys = s3imph::kResMaxKeys;
  // reservation slots hold >= 4x a tile's mean fill, 2x on levels above kResSmallKeys
  // (full 256-block grids: every XCD shard of a slot then fills evenly)
  uint64_t res_fill = 2;
  // test knobs (S3IMPH_RES_MAX / S3IMPH_RES0 / S3IMPH_RES_FILL) that force the fallback paths:
  // res0 = 0 puts level 0 on the counted path, 2 on the reservation path whatever its fill
  int res0 = 1;  // level 0 through the reservation scatter when its tiles are large
  bool route_self = false;  // S3IMPH_DIST_ROUTE_SELF: a one-rank sharded build routes like P > 1 (tests)
  int scat_cfg = 2;         // S3IMPH_SCAT_CFG: reservation-scatter forms (launch_binned_scatter_res)
  int skew_cfg = 2;         // S3IMPH_SKEW_CFG: skewed-length hash block / group shape (launch_hash_skew)
  bool loose_geom = false;  // S3IMPH_LOOSE_GEOM: list levels sized from 1.1x (not 1.02x + 6 sigma) bounds
  // P0 level 0 (s3imph_internal.h): tile slot fills / look-back words for up to p0_tiles
  // 2^14-position tiles, super-tile slot fills; made on first use.  S3IMPH_P0=0 keeps such
  // sets on the split kernel (A/B knob).
  int p0 = 1;
  uint64_t p0_tiles = 0;
  unsigned* p0_tcnt = nullptr;
  unsigned long long* p0_flags = nullptr;
  unsigned* p0_scnt = nullptr;
  unsigned* p0_pcnt = nullptr;  // the fused hash's region fills (kH0GridHost x kMaxRanks)
  s3imph::R20* p0_sup = nullptr;  // the super-tiles' records
  uint64_t p0_sup_cap = 0;
  uint16_t* p0_x = nullptr;       // bitmap decomposition: in-tile position of each level-0 R20 slot
  uint64_t p0_x_cap = 0;
  // level 0's super-tile scatter overlapped on the hash: its stream, the events that order it
  // (after the build's state init / before the follow-up scatter), and the hash blocks' XCDs +
  // the finished parts (kH0GridHost + 8 kP0OvChunks kMaxRanks u32)
  hipStream_t ov_stream = nullptr;
  hipEvent_t ov_ev[2] = {};
  unsigned* p0_ov = nullptr;
  // R20 list levels (BinBuffers::l20): on unless S3IMPH_L20=0 (A/B knob); l20_mask is the
  // last build's mask (classify_stop reads its stop level's list in that format)
  bool l20 = true;
  unsigned l20_mask = 0;
  bool bm_counts = false;   // S3IMPH_BM_LANES=counts: the bitmap decomposition sums count lanes (A/B knob)
  bool debug = false;
  bool fault_dup = false;   // S3IMPH_FAULT_DUP_REC: test hook, duplicates a record mid-build (fault_dup_record)
  unsigned long long* tile_prof = nullptr;  // debug: tile phase timestamps
  bool lds_attr_set = false;

  // staging for host-memory builds
  hipStream_t copy_stream = nullptr;  // the blob's H2D pieces (build_from_host), beside the hash
  hipEvent_t copy_evs[s3imph::kCopyPieces] = {};
  const s3imph::HashFeed* feed = nullptr;  // set for the duration of one host build
  uint8_t* s_blob = nullptr;
  uint64_t s_blob_cap = 0;
  uint64_t *s_offsets = nullptr, *s_pos = nullptr, *s_fp = nullptr, *s_posout = nullptr;
  uint64_t s_cap = 0;
  uint64_t s_pos_cap = 0;  // s_pos is made only for builds with caller positions
  Stager stager;

  bool have_build = false;
  uint64_t last_n = 0;
  s3imph_build_info info{};

  int profiling = 0;  // 0 off, 1 every stage, 2 the level-0 hash (or route) stage only
  std::vector<hipEvent_t> events;
  std::vector<std::string> ev_names;
  int ev_used = 0;
  std::vector<float> stage_ms;
  std::vector<std::string> stage_names;

  std::string last_msg;  // message of the last failed device-resident call
  bool dist = false;
  uint64_t dist_switch = s3imph::kDistSwitchKeysDefault;  // global keys below which levels run replicated
  DistState d;
};

namespace s3imph {

// Builds (s3imph_build.hip).  Both return an s3imph_status and throw Fail on HIP/RCCL errors.
int build_single(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n,
                 uint64_t* fp_out, uint64_t* pos_out, hipStream_t s, s3imph_build_info* info, std::string* msg);
int build_dist(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n_local,
               uint64_t key_base, uint64_t* fp_out, uint64_t* pos_out, uint64_t out_cap, uint64_t* out_n,
               hipStream_t s, s3imph_build_info* info, std::string* msg);
uint64_t dist_out_cap(const s3imph_ctx* c, uint64_t n_global);
// Chunked host <-> device copy through the ctx's pinned stager (h2d: device dst <- host src;
// with `bias`, src holds u64 words stored minus bias).
// conv 1: host u64 -> device u32 (h2d), conv 2: device u32 -> host u64 (d2h), conv 3: host
// u64 offsets -> device u16 key lengths (h2d; a length past 65535 sets *wide and stops the
// copy); `bytes` are device bytes.
void staged_copy(s3imph_ctx* c, bool h2d, void* dst, const void* src, uint64_t bytes, uint64_t bias = 0,
                 int conv = 0, std::atomic<bool>* wide = nullptr);
void launch_widen32(const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s);
void launch_narrow32(const uint64_t* in, uint32_t* out, uint64_t n, hipStream_t s);
// u16 key lengths -> u64 offsets (n + 1 of them); sums: len16_scratch_words(n) words
uint64_t len16_scratch_words(uint64_t n);
void launch_len16_offsets(const uint16_t* len, uint64_t n, uint64_t* sums, uint64_t* out, hipStream_t s);
// FNV-1a of keys [0, n) into out (the error path's recount of the original key hashes)
void launch_key_hashes(const uint8_t* blob, const uint64_t* offsets, uint64_t n, uint64_t* out, hipStream_t s);
int marshal_locked(s3imph_ctx* c, uint8_t* out, uint64_t cap, uint64_t* len, std::string* msg);
void ensure_s_pos(s3imph_ctx* c, uint64_t n);
void release_multi_sets();  // s3imph_multi.hip
int release_idle_multi_sets(const void* keep);  // s3imph_multi.hip: idle sets other than `keep`
// A build that ran out of HBM: free the workspaces this process caches for OTHER builds — the
// host builds' per-device default contexts and the idle multi-GPU sets (`keep_set` excepted)
// — plus `keep`'s finalize scratch; contexts or sets another thread is building on are left
// alone.  Returns whether anything was freed (s3imph_build.hip).
bool reclaim_cached(s3imph_ctx* keep, const void* keep_set = nullptr);
// Run the build step f (returns a status, may throw Fail); when it runs out of HBM, drain the
// stream, reclaim_cached(keep) and run it once more (cached workspaces of earlier
// builds must not fail a later, larger one).
template <class F>
int retry_on_nomem(s3imph_ctx* keep, hipStream_t s, std::string* msg, F&& f) {
  int rc;
  try {
    rc = f();
  } catch (const Fail& e) {
    if (e.code != S3IMPH_ERR_NOMEM) throw;
    rc = e.code;
    *msg = e.msg;
  }
  if (rc != S3IMPH_ERR_NOMEM) return rc;
  if (s) (void)hipStreamSynchronize(s);
  (void)hipGetLastError();
  if (!reclaim_cached(keep)) return rc;
  msg->clear();
  return f();
}
// Index finalize arrays (s3imph_finalize.hip): device pass over keys in HBM, and the
// host-memory form that writes the five files.
int finalize_device(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths, uint64_t n,
                    uint32_t* depth, uint64_t* subtree_end, uint32_t* max_depth_sub, uint64_t* depth_positions,
                    uint64_t* depth_offsets, uint64_t doff_cap, uint32_t* max_depth, hipStream_t s, std::string* msg);
int finalize_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths, uint64_t n,
                       const std::string& dir, std::string* msg);
void fin_scratch_free(s3imph_ctx* c);
// A context (s3imph_ctx_create) whose multi-GPU collectives go through `comm` (owned).
s3imph_ctx* make_dist_ctx(int device, Comm* comm, int rank, int nranks, std::string* msg);

}  // namespace s3imph
