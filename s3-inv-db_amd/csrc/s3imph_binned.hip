// s3imph_binned.hip — the single-GPU MPHF build as a position-binned level pipeline.
//
// Reference work replaced (/root/reference):
//   StreamingMPHFBuilder.Add hashing (pkg/format/mphf_streaming.go:73,80; mphf.go:349-369),
//   bbhash.New level construction (mphf_streaming.go:141; relab/bbhash restated in SURVEY App. A),
//   computeHashPositionsReverseMap + the fingerprint/position scatter (mphf_streaming.go:176-204).
//
// Per big level L (n_L keys, 64*words_L positions, tiles of 2^tb positions):
//   count    keys -> per-(tile, chunk) histogram (LDS atomics)
//   hscan    exclusive scan of the histogram, tile-major -> bucket offsets
//   scatter  records (kh, fp, pos) -> tile buckets.  Each 4096-key round is sorted by
//            tile in LDS and written run by run, so consecutive lanes store consecutive
//            slots; chunks are dealt to blocks XCD-contiguously so one L2 sees each
//            bucket region.  No global atomics.
//   tile     one workgroup per tile (ticket order): A/C bit vectors in LDS, final
//            bits A & ~C written once; the tile's global rank prefix comes from a
//            decoupled look-back over earlier tiles; settled keys write fp_out[p] /
//            pos_out[p] directly (a tile's keys cover one contiguous p range);
//            collided records go to the next level's list, one atomic per tile.
// Small levels run in one workgroup (k_bin_tail) with everything in LDS.
// Level bit vectors depend only on the SET of keys at each level, so every schedule
// (bucket order, LDS atomic order, tile order) yields the same bytes.
#include <hip/hip_runtime.h>

#include "s3imph_device.h"
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>

#include "s3imph_internal.h"


namespace s3imph {

namespace {

constexpr int kCB = 1024;             // count block
constexpr int kH0T = 256;             // k_hash0_pair: threads (2 keys each per round)
constexpr int kH0B = 32 << 10;        // ... window bytes per round (4 blocks per CU)
constexpr int kH0Grid = kH0GridHost;  // ... blocks: 4 per resident slot, a contiguous key range each
constexpr int kSB = 1024;             // scatter block
constexpr int kTailT = 1024;          // tail block
constexpr unsigned kLenBuckets = 256;  // key-length classes (4 B each) of the level-0 hash sort
constexpr uint64_t kTcntWords = (uint64_t)kResLevels * kTcntStride;
constexpr uint64_t kLdsTiles = kScatterTiles;  // count / start / cursor entries of the LDS-staged scatters
constexpr unsigned long long kGate = kTailKeys;
constexpr int kTailW32 = (int)(2 * ((kGammaNum * kTailKeys + 63) / 64));  // A/C words of the largest tail level
constexpr unsigned long long kFlagAgg = 1ull << 62;
constexpr unsigned long long kFlagInc = 2ull << 62;
constexpr unsigned long long kFlagVal = (1ull << 62) - 1;

__host__ __device__ __forceinline__ uint64_t ntiles_of(uint64_t words, unsigned tb) {
  return (64 * words + (1ull << tb) - 1) >> tb;
}

// Sum over the block (NT a multiple of 64, <= 1024).
template <int NT>
__device__ __forceinline__ uint64_t block_sum(uint64_t v) {
  __shared__ uint64_t s_red[NT / 64];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_down(v, d);
  if (lane_id() == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += s_red[w];
  __syncthreads();
  return t;
}

// Exclusive scan over the block; *total receives the block sum.
template <int NT>
__device__ __forceinline__ uint64_t block_exscan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t s_w[NT / 64];
  const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d);
    if (lane >= (unsigned)d) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    if ((unsigned)w < wave) pre += s_w[w];
    tot += s_w[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

__device__ __forceinline__ bool geom_ok(LevelState* st, uint64_t T, uint64_t B) {
  if (T > kMaxTiles || T * B > kHistCap) {
    if (threadIdx.x == 0) atomicOr(&st->status, kStGeometry);
    return false;
  }
  return true;
}

__device__ __forceinline__ bool level_active(int level, const LevelState* st) {
  return (st->preset[level] || level == 0 || st->n[level] > kGate) &&
         !(st->status & kStStop);
}

// A whole level that placed no key: its keys all collide again at every level (only
// duplicate key hashes do that at these sizes), so the build stops here instead of
// running out the level budget; the host then looks for duplicates among the n[level]
// records left in the level's input list.  (Sharded levels, preset, count this rank's
// share only and are not judged.)
__device__ __forceinline__ bool no_progress(LevelState* st, int level, uint64_t n) {
  if (level < 1 || st->preset[level] || st->preset[level - 1] || n == 0 || n != st->n[level - 1]) return false;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->stop_level = level;
    atomicOr(&st->status, kStTooManyLevels);
  }
  return true;
}

// ---------------------------------------------------------------- level 0 count ----
// Hash every key (FNV-1a key hash + FNV-1 fingerprint, one pass over the bytes),
// store both in key order, and (counted path) histogram the level-0 tiles per chunk.
// A key is read with aligned 8-byte loads pipelined two words ahead (fnv_both_pf), or
// with 16-byte loads (fnv_both_16) inside length-sorted groups.
// smode 3: sort a group when the set is skewed (st->skew, sampled by k_init_state);
// smode 5: the same, and a no-op launch unless skewed (k_hash0_pair hashed the set).
__global__ __launch_bounds__(kCB, 8) void k_hash_count0(const uint8_t* __restrict__ blob,
                                                     const uint64_t* __restrict__ offsets, uint64_t n,
                                                     uint64_t* __restrict__ kh, uint64_t* __restrict__ fp,
                                                     unsigned* __restrict__ hist,
                                                     unsigned long long* __restrict__ flags,
                                                     unsigned long long* __restrict__ sflags, LevelState* st,
                                                     unsigned tb, uint64_t chunk, unsigned* __restrict__ tcnt,
                                                     int smode) {
  __shared__ unsigned sh[kMaxTiles];
  __shared__ unsigned lcnt[kLenBuckets];
  __shared__ unsigned short sidx[kCB];
  __shared__ uint64_t sb0[kCB], sb1[kCB], sh1[kCB], sh2[kCB];
  __shared__ uint64_t s_lmax[kCB / 64], s_lsum[kCB / 64];
  if (smode == 5 && !st->skew) return;  // k_hash0_pair hashed this near-uniform set
  const bool sort = st->skew != 0;
  const uint64_t words = st->words[0], magic = st->magic[0];
  const uint64_t T = ntiles_of(words, tb), B = (n + chunk - 1) / chunk;
  if (!geom_ok(st, T, B)) return;
  const unsigned tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) {
    st->ntiles[0] = T;
    st->nchunks[0] = B;
  }
  for (uint64_t t = (uint64_t)blockIdx.x * kCB + tid; t < T; t += (uint64_t)gridDim.x * kCB) flags[t] = 0;
  const uint64_t nseg = (T * B + kScanSeg - 1) / kScanSeg;
  for (uint64_t q = (uint64_t)blockIdx.x * kCB + tid; q < nseg; q += (uint64_t)gridDim.x * kCB) sflags[q] = 0;
  for (uint64_t q = (uint64_t)blockIdx.x * kCB + tid; q < kTcntWords; q += (uint64_t)gridDim.x * kCB) tcnt[q] = 0;
  const uint64_t seed = level_seed(0);
  bool zero = false;
  for (uint64_t b = blockIdx.x; b < B; b += gridDim.x) {
    for (uint64_t t = tid; t < T; t += kCB) sh[t] = 0;
    const uint64_t lo = b * chunk, hi = min(n, lo + chunk);
    if (!sort) {
      __syncthreads();
      for (uint64_t i = lo + tid; i < hi; i += kCB) {
        uint64_t h1, h2;
        fnv_both_pf(blob, offsets[i], offsets[i + 1], h1, h2);
        kh[i] = h1;
        fp[i] = h2;
        zero |= (h1 == 0);
        if (hist) atomicAdd(&sh[bb_index(seed, h1, words, magic) >> tb], 1u);
      }
    } else {
    for (uint64_t g = lo; g < hi; g += kCB) {
      // Counting-sort the group's keys by length so that each wave hashes keys of one
      // length: FNV is one dependent multiply chain per byte, and a wave runs as long as
      // its longest lane.  Results return to key order through LDS.
      const uint64_t i = g + tid;
      uint64_t b0 = 0, b1 = 0;
      if (i < hi) {
        b0 = offsets[i];
        b1 = offsets[i + 1];
      }
      if (tid < kLenBuckets) lcnt[tid] = 0;
      // Sort only a skewed group (longest key > 2x the mean + 16 B): for near-uniform
      // lengths the shuffle costs more than the idle lanes it saves.
      {
        uint64_t mx = b1 - b0, sm = b1 - b0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          mx = max(mx, (uint64_t)__shfl_xor(mx, d));
          sm += __shfl_xor(sm, d);
        }
        if (lane_id() == 0) {
          s_lmax[tid >> 6] = mx;
          s_lsum[tid >> 6] = sm;
        }
      }
      __syncthreads();
      uint64_t gmax = 0, gsum = 0;
#pragma unroll
      for (int w = 0; w < kCB / 64; ++w) {
        gmax = max(gmax, s_lmax[w]);
        gsum += s_lsum[w];
      }
      const uint64_t gcnt = min<uint64_t>(kCB, hi - g);
      if (gmax * gcnt <= 2 * gsum + 16 * gcnt) {
        if (i < hi) {
          uint64_t h1, h2;
          fnv_both_16(blob, b0, b1, h1, h2);
          kh[i] = h1;
          fp[i] = h2;
          zero |= (h1 == 0);
          if (hist) atomicAdd(&sh[bb_index(seed, h1, words, magic) >> tb], 1u);
        }
        __syncthreads();
        continue;
      }
      const unsigned lb = (unsigned)min<uint64_t>((b1 - b0) >> 2, kLenBuckets - 1);
      const unsigned rk = atomicAdd(&lcnt[lb], 1u);
      __syncthreads();
      uint64_t tot;
      const uint64_t ex = block_exscan<kCB>(tid < kLenBuckets ? lcnt[tid] : 0u, &tot);
      if (tid < kLenBuckets) lcnt[tid] = (unsigned)ex;
      __syncthreads();
      const unsigned slot = lcnt[lb] + rk;
      sidx[slot] = (unsigned short)tid;
      sb0[slot] = b0;
      sb1[slot] = b1;
      __syncthreads();
      const unsigned j = sidx[tid];
      if (g + j < hi) {
        uint64_t h1, h2;
        fnv_both_16(blob, sb0[tid], sb1[tid], h1, h2);
        sh1[j] = h1;
        sh2[j] = h2;
        zero |= (h1 == 0);
        if (hist) atomicAdd(&sh[bb_index(seed, h1, words, magic) >> tb], 1u);
      }
      __syncthreads();
      if (i < hi) {
        kh[i] = sh1[tid];
        fp[i] = sh2[tid];
      }
    }
    }
    __syncthreads();
    if (hist)
      for (uint64_t t = tid; t < T; t += kCB) hist[t * B + b] = sh[t];
    __syncthreads();
  }
  if (zero) atomicOr(&st->status, kStKeyZero);
}

// Streamed loads and stores (ld_stream16, st_stream): s3imph_device.h.

// R20 (s3imph_internal.h): a level-0 record with an identity position, in five dwords.
__device__ __forceinline__ R20 r20_make(uint64_t k, uint64_t f, uint32_t i) {
  return R20{{(uint32_t)k, (uint32_t)(k >> 32), (uint32_t)f, (uint32_t)(f >> 32), i}};
}
__device__ __forceinline__ void r20_split(const R20& r, uint64_t pos_base, uint64_t& k, uint64_t& f, uint64_t& p) {
  k = (uint64_t)r.w[0] | ((uint64_t)r.w[1] << 32);
  f = (uint64_t)r.w[2] | ((uint64_t)r.w[3] << 32);
  p = pos_base + r.w[4];
}
// A collided record into the next list: Rec, or (o20: the next level's list is R20, see
// BinBuffers::l20) R20 with the key index p - pos_base.  o20 is a kernel argument: a uniform
// branch.
__device__ __forceinline__ void next_put(Rec* next, bool o20, uint64_t i, uint64_t k, uint64_t f, uint64_t p,
                                         uint64_t pos_base) {
  if (o20) reinterpret_cast<R20*>(next)[i] = r20_make(k, f, (uint32_t)(p - pos_base));
  else next[i] = Rec{k, f, p};
}

// ------------------------------------------------ level-0 hash, LDS-staged ----------
// FNV-1a + FNV-1 of every key (StreamingMPHFBuilder.Add, mphf_streaming.go:73,80;
// mphf.go:349-369) for near-uniform key lengths (st->skew == 0; skewed sets go to
// k_hash_count0).  A block works through its contiguous key range in rounds of up to 2 NT
// keys.  A round's bytes — one contiguous range of prefix_blob — come in with coalesced
// 16-byte loads, issued into registers while the PREVIOUS round is hashed, and are staged
// in LDS.  The round's keys are counting-sorted by length and lane t hashes sorted slot t
// (the shorter half), then slot m - 1 - t (the longer half): within a wave the keys of each
// half have nearly one length (no lane idles behind a longer key), and every lane, so every
// wave, carries about twice the mean length (no wave waits behind another at the round's
// barrier).  Each lane walks its key's aligned LDS words through a byte funnel.  Keys past
// the window budget BB wait for the next round; a key longer than BB is hashed from global
// memory by one lane.  (kh, fp) land in key order; no level-0 histogram (the reservation
// path needs none).  The grid is many blocks per resident slot (kH0Grid): a block that
// finishes early is replaced, so every SIMD keeps its waves to the end instead of running
// the last blocks' load / sort phases exposed.
// prof (S3IMPH_DEBUG): per wave, shader cycles total / hashing / barrier wait / rest, and
// the real-time clock span, for the phase report of print_tile_profile.
//
// RT (multi-GPU build): the level-0 route is fused in.  A round's (kh, fp, pos) records
// never reach kh / fp: they are counting-sorted by owner rank in LDS (staged in the
// round's byte window, free once every lane has hashed), one atomic per (round, owner)
// reserves the owner's run, and the runs are written out whole — k_route's work without
// its 16-byte-per-key read and the hash's 16-byte-per-key write.  The reservations are
// the kernel's limit: same-address device atomics serialise at ~12 ns each
// (tools/ubench_atomics.hip); 1024-key rounds (512 threads, 64 KiB windows) halve them
// but measured slower (C3 3.02 -> 3.51 ms: register spills, the larger rounds' tail).
//
// PT (P0 level 0, s3imph_internal.h): the same in-LDS counting sort, by SUPER-TILE (the
// record's level-0 position >> 14, divided by tps), and each run is appended to the block's
// OWN region for that super-tile as R20 records (k, f, key index): no global atomic per
// round (returning slot reservations stalled every round: hash 2.36 -> 4.15 ms on C3), the
// region fills are written once at the block's end.  The first of P0's two partition passes
// rides on the hash, whose HBM share is half idle, instead of a pass that reads kh / fp back.
struct P0Part {
  R20* sup;
  uint64_t reg_cap;  // records per (hash block, super-tile) region
  unsigned* pcnt;    // region fills, written at each block's end
  unsigned tps, S;
  // overlapped scatter (k_scatter_p0d<kOv>, beside this kernel): each block's XCD, published
  // with its fills once its region runs are in that XCD's L2; null: no publication
  unsigned* hxcc = nullptr;
};
template <int NT, int BB, bool PF, bool RT = false, bool PT = false>
__global__ __launch_bounds__(NT, 2048 / NT * NT / 256 / 2) void k_hash0_pair(const uint8_t* __restrict__ blob,
                                                  const uint64_t* __restrict__ offsets, uint64_t n,
                                                  uint64_t* __restrict__ kh, uint64_t* __restrict__ fp,
                                                  unsigned long long* __restrict__ flags,
                                                  unsigned long long* __restrict__ sflags, LevelState* st,
                                                  unsigned tb, uint64_t chunk, unsigned* __restrict__ tcnt,
                                                  unsigned long long* __restrict__ prof = nullptr,
                                                  Route0 rt = Route0{}, P0Part pt = P0Part{}, unsigned blk0 = 0,
                                                  unsigned nblk = 0) {
  // blocks [blk0, blk0 + gridDim.x) of an nblk-block decomposition of the keys (nblk 0: this
  // grid alone): the host build launches the hash in pieces, each once its keys' bytes have
  // crossed PCIe (launch_hash_pieces)
  static_assert(!(RT && PT), "route or partition, not both");
  const unsigned bid = blk0 + blockIdx.x, NBK = nblk ? nblk : gridDim.x;
  unsigned long long pt0 = __builtin_amdgcn_s_memtime(), ph = 0, pw = 0;  // debug phase clock
  const unsigned long long prt0 = __builtin_amdgcn_s_memrealtime();
  constexpr int G = 2 * NT;                    // keys per round
  constexpr int KW = (BB / 16 + NT - 1) / NT;  // 16-byte window chunks per thread
  constexpr unsigned kLB = 256;                // length classes of the sort
  constexpr int NW = NT / 64;
  // S3IMPH_FNV_PAIR: the window starts kWP words in, so >= 8 bytes precede every key (the
  // zero-prefixed first word of fnv_window_pair reads them, masked)
  constexpr unsigned kWP = S3IMPH_FNV_PAIR ? 2u : 0u;
  __shared__ uint64_t sw[BB / 8 + 2 + kWP];    // the round's window (+ 16 B: a lane may read one word past)
  // sorted slot -> key's window offset (< BB) | length (<= BB) << 16: one LDS word per key
  static_assert(BB <= 32768, "offset and length in 16 bits each");
  __shared__ unsigned sol[G];
  __shared__ unsigned short sidx[G];           // sorted slot -> key index in the round
  __shared__ unsigned lcnt[kLB];
  __shared__ unsigned s_cnt[NW];
  // RT: per-owner counts / run starts of the round, the owners' reserved run bases (record
  // offsets into self_dst or send), the block's sticky overflow flag
  __shared__ unsigned r_cnt[RT || PT ? kMaxRanks : 1], r_start[RT || PT ? kMaxRanks : 1];
  __shared__ uint64_t r_base[RT || PT ? kMaxRanks : 1];
  __shared__ unsigned r_over;
  __shared__ unsigned p_cur[PT ? kMaxRanks : 1];  // PT: this block's fill of each super-tile region
  __shared__ uint64_t s_fnv_init[S3IMPH_FNV_PAIR ? 8 : 1];  // fnv_prefixed_basis(pad), pad 0..7
  if (st->skew) return;  // k_hash_count0 hashes skewed sets (and clears the tile state)
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  if (S3IMPH_FNV_PAIR && tid < 8) {  // (ordered before the first hash by the round's barriers)
    constexpr uint64_t kInit[8] = {fnv_prefixed_basis(0), fnv_prefixed_basis(1), fnv_prefixed_basis(2),
                                   fnv_prefixed_basis(3), fnv_prefixed_basis(4), fnv_prefixed_basis(5),
                                   fnv_prefixed_basis(6), fnv_prefixed_basis(7)};
    s_fnv_init[tid] = kInit[tid];
  }
  static_assert(!RT || G * sizeof(Rec) + G <= sizeof(sw), "the route stage aliases the byte window");
  // RT: level 0's geometry and owner ranges; this rank's own-record shift (records received
  // for earlier key chunks sit before its own ones)
  uint64_t r_words = 0, r_magic = 0, r_S = 1, r_mS = 0, r_rb = 0;
  uint32_t p_mul = 0;
  if (PT) {
    if (tid == 0) r_over = 0;
    if (tid < kMaxRanks) p_cur[tid] = 0;
    r_words = st->words[0];
    r_magic = st->magic[0];
    p_mul = 0xffffffffu / pt.tps + 1;  // exact for (position >> 14) < 2^18, tps <= 2^14
  }
  if (RT) {
    if (tid == 0) r_over = 0;
    r_words = st->words[0];
    r_magic = st->magic[0];
    r_S = st->dS[0];
    r_mS = st->dmagic[0];
    uint64_t v = rt.mat_prev && lane < (unsigned)rt.P && (int)lane != rt.rank
                     ? rt.mat_prev[(uint64_t)lane * (rt.P + 1) + rt.rank] : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    r_rb = uniform64(v);
  }
  {
    const uint64_t T = ntiles_of(st->words[0], tb), B = (n + chunk - 1) / chunk;
    const uint64_t nseg = (T * B + kScanSeg - 1) / kScanSeg;
    const uint64_t g0 = (uint64_t)blockIdx.x * NT + tid, gs = (uint64_t)gridDim.x * NT;
    if (blk0 == 0 && blockIdx.x == 0 && tid == 0) {
      st->ntiles[0] = T;
      st->nchunks[0] = B;
    }
    if (blk0 == 0) {  // (the first piece's grid covers them all)
      for (uint64_t t = g0; t < T; t += gs) flags[t] = 0;
      for (uint64_t q = g0; q < nseg; q += gs) sflags[q] = 0;
      for (uint64_t q = g0; q < kTcntWords; q += gs) tcnt[q] = 0;
    }
  }
  // overlap: this block's XCD at once (the overlapped scatter learns which hash blocks share
  // its XCD from the first ones: the dispatcher deals blocks to the XCDs round-robin)
  if (PT && pt.hxcc && tid == 0) __hip_atomic_store(&pt.hxcc[bid], xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t per = (n + NBK - 1) / NBK;
  uint64_t g = (uint64_t)bid * per;
  const uint64_t gend = min(n, g + per);
  if (g >= gend) {
    if (PT && pt.hxcc) {  // (no region runs: published at once)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
      if (tid < pt.S) __hip_atomic_store(&pt.pcnt[(uint64_t)bid * pt.S + tid], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&st->h0_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (PT && tid < pt.S) pt.pcnt[(uint64_t)bid * pt.S + tid] = 0;
    return;
  }
  const uint64_t end8 = (offsets[n] + 7) & ~7ull;
  bool zero = false;
  // ---- the round at r0: keys r0 + tid and r0 + NT + tid, its window [wlo, wend) in wr
  uint64_t kb0[2], kb1[2], wlo = 0, wend = 0;
  bool kin[2];
  uint4 wr[KW];
  // the window as whole 16-byte chunks [0, nfull) below end8 & ~15, plus, in the blob's last
  // round only, the 8 bytes at end8 - 8 (chunk nfull) when end8 = 8 mod 16: per chunk a 32-bit
  // compare against a uniform count instead of two 64-bit address compares (119 VGPRs instead
  // of 128, C3 6.495 -> 6.460 ms, profiles/r5_hash/window_u32_ab_r5ar.txt)
  unsigned nfull = 0;
  bool tail8 = false;
  auto prefetch = [&](uint64_t r0) {
    const uint64_t last = min(gend, r0 + G);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t i = r0 + tid + (unsigned)h * NT;
      kin[h] = i < last;
      kb0[h] = kin[h] ? offsets[i] : 0;
      kb1[h] = kin[h] ? offsets[i + 1] : 0;
    }
    wlo = uniform64(offsets[r0] & ~15ull);
    wend = uniform64(min((offsets[last] + 15) & ~15ull, wlo + (uint64_t)BB));
    {
      const uint64_t e16 = min(wend, end8 & ~15ull);
      nfull = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(e16 > wlo ? (e16 - wlo) >> 4 : 0));
      tail8 = (end8 & 8) && end8 - 8 >= wlo && end8 - 8 < wend;
    }
    const uint8_t* wb = blob + wlo;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const unsigned c = tid + (unsigned)k * NT;
      wr[k] = make_uint4(0, 0, 0, 0);
      if (c < nfull) wr[k] = ld_stream16(wb + 16u * c);
    }
  };
  if (PF) prefetch(g);
  for (;;) {
    if (!PF) prefetch(g);
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const unsigned c = tid + (unsigned)k * NT;
      if (c < nfull) {
        sw[kWP + 2 * c] = (uint64_t)wr[k].x | ((uint64_t)wr[k].y << 32);
        sw[kWP + 2 * c + 1] = (uint64_t)wr[k].z | ((uint64_t)wr[k].w << 32);
      }
    }
    if (tail8 && tid == 0) {  // once per blob: the last 8 readable bytes (a blocking load)
      sw[kWP + 2 * nfull] = *reinterpret_cast<const uint64_t*>(blob + (end8 - 8));
      sw[kWP + 2 * nfull + 1] = 0;
    }
    for (unsigned b = tid; b < kLB; b += NT) lcnt[b] = 0;
    if ((RT || PT) && tid < kMaxRanks) r_cnt[tid] = 0;
    const uint64_t rw = wlo;
    const uint64_t t_b0[2] = {kb0[0], kb0[1]}, t_b1[2] = {kb1[0], kb1[1]};
    // keys whose bytes all lie in the window: a prefix of the round (offsets ascend)
    bool fits[2];
    unsigned mine = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      fits[h] = kin[h] && t_b1[h] - rw <= (uint64_t)BB;
      const uint64_t fb = __ballot(fits[h]);
      mine += (unsigned)__popcll(fb);
    }
    if (lane == 0) s_cnt[wave] = mine;
    __syncthreads();
    unsigned m = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) m += s_cnt[w];
    const bool alone = m == 0;  // the round's first key is longer than the window
    if (alone) m = 1;
    // ---- counting sort of the round's keys by length
    unsigned cls[2] = {0, 0}, rk[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (fits[h]) {
        cls[h] = (unsigned)min<uint64_t>(t_b1[h] - t_b0[h], kLB - 1);
        rk[h] = atomicAdd(&lcnt[cls[h]], 1u);
      }
    __syncthreads();
    if (tid < 64) {
      unsigned v[kLB / 64], sum = 0;
#pragma unroll
      for (int q = 0; q < (int)(kLB / 64); ++q) {
        v[q] = lcnt[tid * (kLB / 64) + q];
        sum += v[q];
      }
      unsigned x = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned y = __shfl_up(x, d);
        if (tid >= (unsigned)d) x += y;
      }
      unsigned ex = x - sum;
#pragma unroll
      for (int q = 0; q < (int)(kLB / 64); ++q) {
        lcnt[tid * (kLB / 64) + q] = ex;
        ex += v[q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (fits[h]) {
        const unsigned slot = lcnt[cls[h]] + rk[h];
        sidx[slot] = (unsigned short)(tid + (unsigned)h * NT);
        sol[slot] = ((unsigned)(t_b0[h] - rw) + 8u * kWP) | ((unsigned)(t_b1[h] - t_b0[h]) << 16);
      }
    __syncthreads();
    const uint64_t r0 = g;
    g += m;
    const bool more = g < gend;
    if (PF && more) prefetch(g);  // the next round's loads land while this one is hashed
    unsigned long long pta = prof ? __builtin_amdgcn_s_memtime() : 0;
    // ---- hash: slot tid (shorter half), then slot m - 1 - tid (longer half)
    uint64_t ra[2] = {0, 0}, rb[2] = {0, 0};
    unsigned rj[2] = {0, 0};
    bool rv[2] = {false, false};
    if (alone) {
      if (tid == 0) {
        uint64_t a, b;
        fnv_both_pf(blob, t_b0[0], t_b1[0], a, b);
        if (RT || PT) {
          ra[0] = a;
          rb[0] = b;
          rj[0] = 0;
          rv[0] = true;
        } else {
          kh[r0] = a;
          fp[r0] = b;
        }
        zero |= (a == 0);
      }
    } else if (S3IMPH_FNV_PAIR) {
      // the lane's two keys as one word loop (fnv_window_pair)
      const bool vA = tid < (m + 1) / 2, vB = tid < m / 2;
      if (vA) {
        const unsigned olA = sol[tid], olB = vB ? sol[m - 1 - tid] : 0u;
        rj[0] = sidx[tid];
        rj[1] = vB ? sidx[m - 1 - tid] : 0u;
        fnv_window_pair(reinterpret_cast<const uint32_t*>(sw), olA & 0xffffu, olA >> 16, olB & 0xffffu, olB >> 16, vB,
                        s_fnv_init, ra[0], rb[0], ra[1], rb[1]);
        rv[0] = true;
        rv[1] = vB;
        zero |= ra[0] == 0 || (vB && ra[1] == 0);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned slot = h == 0 ? tid : m - 1 - tid;
        if (h == 0 ? tid < (m + 1) / 2 : tid < m / 2) {
          uint64_t a, b;
          const unsigned j = sidx[slot];
          const unsigned ol = sol[slot];
          fnv_window(reinterpret_cast<const uint32_t*>(sw), ol & 0xffffu, ol >> 16, a, b);
          ra[h] = a;
          rb[h] = b;
          rj[h] = j;
          rv[h] = true;
          zero |= (a == 0);
        }
      }
    }
    if (!RT && !PT && !alone) {  // ---- (kh, fp) back to key order through LDS, then coalesced stores
      static_assert(2 * G * sizeof(uint64_t) <= sizeof(sw), "the result stage aliases the byte window");
      __syncthreads();  // every lane has hashed: the window is free
      uint64_t* sa = sw;
      uint64_t* sb = sw + G;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (rv[h]) {
          sa[rj[h]] = ra[h];
          sb[rj[h]] = rb[h];
        }
      __syncthreads();
      for (unsigned j = tid; j < m; j += NT) {
        st_stream(kh + r0 + j, sa[j]);
        st_stream(fp + r0 + j, sb[j]);
      }
    }
    if (RT) {  // ---- route the round's records to their owners (k_route's scheme)
      unsigned od[2] = {0, 0}, ork[2] = {0, 0};
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (rv[h]) {
          const uint64_t x = bb_index(level_seed(0), ra[h], r_words, r_magic);
          od[h] = owner_of(x >> 6, r_S, r_mS);
          if (od[h] >= (unsigned)rt.P) od[h] = rt.P - 1;  // unreachable: x < 64 words <= 64 P S
          ork[h] = atomicAdd(&r_cnt[od[h]], 1u);
        }
      __syncthreads();  // every lane has hashed (the window is free) and counted
      if (tid < 64) {
        const unsigned c = tid < (unsigned)rt.P ? r_cnt[tid] : 0u;
        unsigned x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned y = __shfl_up(x, o);
          if (tid >= (unsigned)o) x += y;
        }
        r_start[tid] = x - c;
        if (c) {
          const unsigned long long at = atomicAdd(&rt.scnt[tid], (unsigned long long)c);
          const bool self = (int)tid == rt.rank;
          if (self ? r_rb + at + c > rt.self_cap : at + c > rt.cap) r_over = 1;
          r_base[tid] = self ? r_rb + at : (uint64_t)tid * rt.cap + at;
        }
      }
      __syncthreads();
      Rec* stg = reinterpret_cast<Rec*>(sw);
      unsigned char* sdst = reinterpret_cast<unsigned char*>(stg + G);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (rv[h]) {
          const unsigned slot = r_start[od[h]] + ork[h];
          const uint64_t i = r0 + rj[h];
          stg[slot] = Rec{ra[h], rb[h], rt.pos ? rt.pos[i] : rt.pos_base + i};
          sdst[slot] = (unsigned char)od[h];
        }
      __syncthreads();
      if (!r_over) {
        for (unsigned j = tid; j < m; j += NT) {
          const unsigned o = sdst[j];
          Rec* dst = ((int)o == rt.rank ? rt.self_dst : rt.send) + r_base[o];
          dst[j - r_start[o]] = stg[j];
        }
      }
    }
    if (PT) {  // ---- the round's R20 records straight to their slots of this block's super-tile regions
      unsigned od[2] = {0, 0}, ork[2] = {0, 0};
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (rv[h]) {
          uint64_t x;  // (r_words: uniform; P0 levels have >= 2^19 words, the general form is a guard)
          if (r_words >= (1ull << 19)) x = bb_index_big(level_seed(0), ra[h], r_words, r_magic);
          else x = bb_index(level_seed(0), ra[h], r_words, r_magic);
          od[h] = __umulhi((uint32_t)(x >> kRegTileMaxBits), p_mul);
          if (od[h] >= pt.S) od[h] = pt.S - 1;  // unreachable: positions < 64 words
          ork[h] = atomicAdd(&r_cnt[od[h]], 1u);
        }
      __syncthreads();  // every lane has hashed (the window is free) and counted
      // 32-bit arithmetic only (offsets within this block's S regions, a uniform base): a
      // 64-bit result in a VGPR pair made wave 0 wait here for the next round's prefetch
      const unsigned rcap = (unsigned)pt.reg_cap;
      unsigned* r_off = reinterpret_cast<unsigned*>(r_base);
      if (tid < 64) {
        // (the thread index opaque here: its LDS addresses recomputed, not hoisted out of
        // the round loop and spilled — a scratch reload waits for every load in flight)
        unsigned me = tid;
        asm volatile("" : "+v"(me));
        const unsigned c = me < pt.S ? r_cnt[me] : 0u;
        unsigned x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned y = __shfl_up(x, o);
          if (me >= (unsigned)o) x += y;
        }
        r_start[me] = x - c;
        if (c) {
          const unsigned at = p_cur[me];
          if (at + c > rcap) r_over = 1;
          p_cur[me] = at + c;
          r_off[me] = me * rcap + at;
        }
      }
      __syncthreads();
      // each record straight to its slot of the round's run in its region (the run is one
      // contiguous range, written whole by the block within the round)
      if (!r_over) {
        R20* const blk = pt.sup + (uint64_t)__builtin_amdgcn_readfirstlane(bid) * pt.S * pt.reg_cap;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (rv[h]) blk[r_off[od[h]] + ork[h]] = r20_make(ra[h], rb[h], (uint32_t)(r0 + rj[h]));
      }
    }
    unsigned long long ptb = prof ? __builtin_amdgcn_s_memtime() : 0;
    if (!more) break;
    __syncthreads();  // every lane is done with sw / sidx before the next round overwrites them
    if (prof) {
      ph += ptb - pta;
      pw += __builtin_amdgcn_s_memtime() - ptb;
    }
  }
  if (prof && lane == 0 && (uint64_t)bid * NW + wave < 8192) {
    const unsigned long long tot = __builtin_amdgcn_s_memtime() - pt0;
    unsigned long long* q = prof + ((uint64_t)bid * NW + wave) * 8;
    q[0] = tot;
    q[1] = ph;
    q[2] = pw;
    q[3] = tot - ph - pw;
    const unsigned long long prt1 = __builtin_amdgcn_s_memrealtime();
    q[4] = prt1 - prt0;
    q[5] = prt0;
    q[6] = prt1;
  }
  if (zero) atomicOr(&st->status, kStKeyZero);
  if (RT && tid == 0 && r_over) atomicOr(&st->status, kStRouteOverflow);
  if (PT && tid == 0 && r_over) atomicOr(&st->status, kStOverflow | kStResOverflow);
  if (PT && pt.hxcc) {
    // publication for the overlapped scatter, which reads this block's regions through the
    // same XCD's L2 while the hash runs on: every thread's region stores complete (in L2)
    // before the barrier, the fills after it, then the block counts as done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (tid < pt.S)
      __hip_atomic_store(&pt.pcnt[(uint64_t)bid * pt.S + tid], p_cur[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&st->h0_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (PT && tid < pt.S) pt.pcnt[(uint64_t)bid * pt.S + tid] = p_cur[tid];  // wave 0 updated p_cur
}

// ------------------------------------------- level-0 hash, skewed key lengths --------
// FNV-1a + FNV-1 of every key (mphf.go:349-369) for sets whose sampled lengths are skewed
// (st->skew: C5's log-uniform 1-1024 B).  FNV is one dependent multiply chain per byte, so
// one lane hashes one key, and a wave runs as long as its longest lane: the wave's 64 keys
// must have (nearly) one length.  A block takes its contiguous key range in groups of kSkG
// keys; each group is counting-sorted by length (4-byte classes) in LDS and cut into
// batches of 64 consecutive sorted keys, which the block's waves take longest first from
// an LDS ticket (LPT: the last batches to start are the shortest, so the waves reach the
// group's barrier together).  A batch's key bytes are staged through a wave-private LDS
// buffer kSkC bytes per key at a time: lanes 4m..4m+3 of load t fetch the 16-byte units of
// key 16t+m's next chunk (one contiguous 64-byte run per key, issued while the previous
// chunk is hashed), so every key's bytes cross HBM / L2 once in whole segments instead of
// one lane's 16-byte stream per key (k_hash_count0: ~0.30 of the FNV ceiling on C5, its L1
// thrashed by 1024 interleaved streams).  Each lane then hashes its key's bytes of the
// chunk from LDS with the funnel step of fnv_window.  Results go to LDS by key and leave
// in key order with coalesced stores.  (Simulated over C5's lengths: 95 % of lane-steps do
// work with 4096-key groups, 82 % with 1024.)
constexpr int kSkC = 64;               // chunk bytes per key per step
constexpr int kSkS = kSkC + 16;        // LDS stride per key (16-B aligned for ds_write_b128)
constexpr int kSkU = kSkC / 16;        // 16-byte units per key chunk = loads per step
constexpr unsigned kSkLB = 256;        // length classes (4 B each)
// kSkT threads, kSkG keys per sorted group: 768 / 5120 (one block per CU, three waves per
// SIMD), 1024 / 4096 (four waves per SIMD) or 512 / 2048 (two blocks per CU: one block's
// sort and group barrier overlap the other's hashing).  A group's makespan is at least its
// longest batch (C5: 16 chunk steps for 1024-byte keys); 4096 keys give each of 16 waves
// ~12.5 steps on average, so the group barrier waited ~17 % of a wave's life; 5120 keys
// over 12 waves give ~21 (C5 hash 1.65-1.66 -> 1.60-1.62 ms, `profiles/r3_skew*/`; 11, 10 and
// 13 waves, and 8 waves with 4096 keys, measured slower).
// kRes false: the partition form only (P0's level 0, pt.sup set), whose records leave for
// their super-tile regions as each batch ends: no per-key result arrays in LDS, so two
// blocks fit a CU with 5120-key groups (S3IMPH_SKEW_CFG 3; 16 waves per CU instead of 12).
template <int kSkT, int kSkG>
constexpr size_t sk_stage_bytes() { return (size_t)(kSkT / 64) * 64 * kSkS; }
template <int kSkT, int kSkG, bool kRes = true>
constexpr size_t sk_lds_bytes() {
  return sk_stage_bytes<kSkT, kSkG>() + (kRes ? 2 * kSkG * sizeof(uint64_t) : 0) + kSkG * sizeof(unsigned short) +
         kSkLB * sizeof(unsigned) + 16;
}
static_assert(sk_lds_bytes<1024, 4096>() <= 160 * 1024, "k_hash_skew's LDS");
static_assert(2 * sk_lds_bytes<512, 2048>() <= 160 * 1024, "k_hash_skew's LDS, two blocks per CU");
static_assert(sk_lds_bytes<768, 5120>() <= 160 * 1024, "k_hash_skew's LDS, 12 waves");
static_assert(2 * sk_lds_bytes<512, 5120, false>() <= 160 * 1024, "k_hash_skew's LDS, partition form, two blocks per CU");
static_assert(kSkU * 16 == 64, "a load instruction covers 16 keys x 64 B");

template <int kSkT, int kSkG, bool kRes = true>
__global__ __launch_bounds__(kSkT, 4) void k_hash_skew(const uint8_t* __restrict__ blob,
                                                       const uint64_t* __restrict__ offsets, uint64_t n,
                                                       uint64_t* __restrict__ kh, uint64_t* __restrict__ fp,
                                                       unsigned long long* __restrict__ flags,
                                                       unsigned long long* __restrict__ sflags, LevelState* st,
                                                       unsigned tb, uint64_t chunk, unsigned* __restrict__ tcnt,
                                                       unsigned long long* __restrict__ prof, int order,
                                                       P0Part pt = P0Part{}) {
  extern __shared__ __align__(16) unsigned char sk_lds[];
  // pt.sup (P0's level 0): each group's records (R20) go to this block's region of their
  // super-tile through an LDS cursor per super-tile, instead of kh / fp in key order
  __shared__ unsigned sk_pcur[kMaxRanks];
  if (!st->skew) return;  // k_hash0_pair hashed this near-uniform set
  const bool part = kRes ? pt.sup != nullptr : true;
  if (!kRes && pt.sup == nullptr) {  // (the host launches the partition form only with regions)
    if (threadIdx.x == 0) atomicOr(&st->status, kStGeometry);
    return;
  }
  const uint32_t p_mul = part ? 0xffffffffu / pt.tps + 1 : 0u;
  const uint64_t p_words = st->words[0], p_magic = st->magic[0];
  bool p_over = false;
  if (part && threadIdx.x < kMaxRanks) sk_pcur[threadIdx.x] = 0;  // (the first group's barriers order it)
  const bool interleave = order == 0;
  // prof (S3IMPH_DEBUG): per wave, shader cycles total / hashing / waiting for a chunk's
  // loads / the rest (sort, tickets, barriers, write-back)
  const unsigned long long pt0 = __builtin_amdgcn_s_memtime(), prt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long p_hash = 0, p_wait = 0, p_sort = 0, p_end = 0;
  uint4* stage = reinterpret_cast<uint4*>(sk_lds);
  constexpr size_t kSkStage = sk_stage_bytes<kSkT, kSkG>();
  uint64_t* res_a = reinterpret_cast<uint64_t*>(sk_lds + kSkStage);
  uint64_t* res_b = res_a + (kRes ? kSkG : 0);
  unsigned short* sidx = reinterpret_cast<unsigned short*>(res_b + (kRes ? kSkG : 0));
  unsigned* cnt = reinterpret_cast<unsigned*>(sidx + kSkG);
  unsigned* next = cnt + kSkLB;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  {  // the level-0 tile state the reservation path starts from (as k_hash0_pair)
    const uint64_t T = ntiles_of(st->words[0], tb), B = (n + chunk - 1) / chunk;
    const uint64_t nseg = (T * B + kScanSeg - 1) / kScanSeg;
    const uint64_t g0 = (uint64_t)blockIdx.x * kSkT + tid, gs = (uint64_t)gridDim.x * kSkT;
    if (blockIdx.x == 0 && tid == 0) {
      st->ntiles[0] = T;
      st->nchunks[0] = B;
    }
    for (uint64_t t = g0; t < T; t += gs) flags[t] = 0;
    for (uint64_t q = g0; q < nseg; q += gs) sflags[q] = 0;
    for (uint64_t q = g0; q < kTcntWords; q += gs) tcnt[q] = 0;
  }
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t gbeg = min(n, (uint64_t)blockIdx.x * per), gend = min(n, gbeg + per);
  const uint64_t end8 = (offsets[n] + 7) & ~7ull;
  uint4* wst = stage + (size_t)wave * 64 * (kSkS / 16);  // this wave's 64 key regions
  const uint32_t* wst32 = reinterpret_cast<const uint32_t*>(wst);
  bool zero = false;
  constexpr int KPT = (kSkG + kSkT - 1) / kSkT;  // keys per thread in the sort
  for (uint64_t grp = gbeg; grp < gend; grp += kSkG) {
    const unsigned long long g0t = prof ? __builtin_amdgcn_s_memtime() : 0;
    const unsigned m = (unsigned)min<uint64_t>(kSkG, gend - grp);
    // ---- counting sort of the group's keys by length (ascending)
    for (unsigned c = tid; c < kSkLB; c += kSkT) cnt[c] = 0;
    if (tid == 0) *next = 0;
    __syncthreads();
    unsigned cls[KPT], rk[KPT];
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      const unsigned k = tid + (unsigned)q * kSkT;
      if (k < m) {
        const uint64_t len = offsets[grp + k + 1] - offsets[grp + k];
        cls[q] = (unsigned)min<uint64_t>(len >> 2, kSkLB - 1);
        rk[q] = atomicAdd(&cnt[cls[q]], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {
      unsigned v[kSkLB / 64], sum = 0;
#pragma unroll
      for (int q = 0; q < (int)(kSkLB / 64); ++q) {
        v[q] = cnt[tid * (kSkLB / 64) + q];
        sum += v[q];
      }
      unsigned x = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned y = __shfl_up(x, d);
        if (tid >= (unsigned)d) x += y;
      }
      unsigned ex = x - sum;
#pragma unroll
      for (int q = 0; q < (int)(kSkLB / 64); ++q) {
        cnt[tid * (kSkLB / 64) + q] = ex;
        ex += v[q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      const unsigned k = tid + (unsigned)q * kSkT;
      if (k < m) sidx[cnt[cls[q]] + rk[q]] = (unsigned short)k;
    }
    __syncthreads();
    // ---- batches of 64 sorted keys, longest first, one wave each.  The wave takes its next
    // ticket, reads that batch's keys and issues its first chunk's loads before it hashes the
    // current batch's last chunk, so the dependent ticket -> sidx -> offsets -> bytes chain
    // of a batch hides behind the previous batch's hashing.
    const unsigned nb = (m + 63) / 64;
    const unsigned u = lane & 3u;
    // Key offsets relative to the group's 16-byte aligned first byte gb fit 32 bits (a group
    // of more than 4 GiB of key bytes is refused), which keeps two batches in registers.
    const uint64_t gb = uniform64(offsets[grp] & ~15ull);
    const uint64_t gspan = offsets[grp + m] - gb;
    if (gspan >= 0xffff0000ull) {
      if (tid == 0) atomicOr(&st->status, kStGeometry);
      break;
    }
    const uint8_t* gblob = blob + gb;
    const uint32_t end8r = (uint32_t)min<uint64_t>(end8 - gb, 0xffffffffull);
    struct Batch {
      unsigned b, k, steps;
      bool valid;
      uint32_t ks, ke, kbase;
      uint32_t lb[kSkU], le[kSkU];  // the keys this lane loads for: key 16t + lane/4, unit lane%4
    };
    // issue: the ticket, the batch's sorted slots and its keys' offsets (loads in flight)
    auto take_issue = [&](Batch& x) {
      unsigned t = 0;
      if (lane == 0) t = atomicAdd(next, 1u);
      t = __shfl(t, 0);
      // longest batch first (LPT); the alternative alternates the longest and the shortest
      // batch left (measured worse on C5: the group barrier waited 33 % vs 17 %)
      x.b = t >= nb ? nb : (!interleave ? t : (t & 1u) ? nb - 1 - (t >> 1) : (t >> 1));
      if (x.b >= nb) return;
      const int hi = (int)m - 64 * (int)x.b;  // sorted slots [hi - 64, hi)
      const int slot = hi - 64 + (int)lane;
      x.valid = slot >= 0;
      x.k = x.valid ? sidx[slot] : 0u;
      x.ks = x.valid ? (uint32_t)(offsets[grp + x.k] - gb) : 0u;
      x.ke = x.valid ? (uint32_t)(offsets[grp + x.k + 1] - gb) : 0u;
    };
    // finish (uses the offsets): the wave's step count and the cooperative load addresses
    auto take_finish = [&](Batch& x) {
      if (x.b >= nb) return;
      x.kbase = x.ks & ~15u;
      const uint32_t span = x.valid ? x.ke - x.kbase : 0u;
      unsigned steps = (span + kSkC - 1) / kSkC;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) steps = max(steps, (unsigned)__shfl_xor(steps, d));
      x.steps = max(steps, 1u);  // >= 1: the step loop takes the next ticket
#pragma unroll
      for (int t = 0; t < kSkU; ++t) {
        const int src = 16 * t + (int)(lane >> 2);
        x.lb[t] = __shfl(x.kbase, src);
        x.le[t] = __shfl(x.valid ? x.ke : 0u, src);
      }
    };
    uint4 r[kSkU];
    // One 16-byte load per unit.  Units are 16-byte aligned; only a unit at end8 - 8 (when
    // end8 = 8 mod 16) would run past the readable blob: it takes the 8 bytes left in a
    // separate (non-temporal) load, so the compiler cannot fold the two into one split load.
    auto load = [&](const Batch& x, unsigned step) {
#pragma unroll
      for (int t = 0; t < kSkU; ++t) {
        const uint32_t a = x.lb[t] + step * kSkC + 16u * u;
        const bool in = a < x.le[t], full = (uint64_t)a + 16 <= end8r;
        uint4 v = make_uint4(0, 0, 0, 0);
#if S3IMPH_NT_SKEW
        if (in && full) v = ld_stream16(gblob + a);
#else
        if (in && full) v = *reinterpret_cast<const uint4*>(gblob + a);
#endif
        if (in && !full) {
          const uint64_t h = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(gblob + a));
          v = make_uint4((uint32_t)h, (uint32_t)(h >> 32), 0u, 0u);
        }
        r[t] = v;
      }
    };
    if (prof) p_sort += __builtin_amdgcn_s_memtime() - g0t;
    // Two batches in flight: the next batch's ticket and offsets are requested at the current
    // batch's first step, its first chunk at the current batch's last step (before hashing it).
    Batch cur, nxt;
    take_issue(cur);
    take_finish(cur);
    if (cur.b < nb) load(cur, 0);
    while (cur.b < nb) {
      uint32_t alo = (uint32_t)kFnvOffset, ahi = (uint32_t)(kFnvOffset >> 32), blo = alo, bhi = ahi;
      for (unsigned step = 0; step < cur.steps; ++step) {
        if (prof) {
          const unsigned long long w0 = __builtin_amdgcn_s_memtime();
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          p_wait += __builtin_amdgcn_s_memtime() - w0;
        }
#pragma unroll
        for (int t = 0; t < kSkU; ++t) wst[(16 * t + (lane >> 2)) * (kSkS / 16) + u] = r[t];
        // LDS operations of one wave complete in order: the lanes' reads below see every
        // lane's writes above, and the next step's writes follow this step's reads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (step == 0) take_issue(nxt);
        if (step + 1 < cur.steps) {
          load(cur, step + 1);
        } else {
          take_finish(nxt);
          if (nxt.b < nb) load(nxt, 0);
        }
        const uint32_t clo = cur.kbase + step * kSkC;
        const unsigned long long h0 = prof ? __builtin_amdgcn_s_memtime() : 0;
        if (cur.ke > clo) {
          const unsigned o = step == 0 ? cur.ks - cur.kbase : 0u;
          const unsigned top = min(cur.ke - clo, (uint32_t)kSkC);
          fnv_window_cont(wst32 + lane * (kSkS / 4), o, top - o, alo, ahi, blo, bhi);
        }
        if (prof) p_hash += __builtin_amdgcn_s_memtime() - h0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      if (cur.valid) {
        const uint64_t a = (uint64_t)alo | ((uint64_t)ahi << 32), f = (uint64_t)blo | ((uint64_t)bhi << 32);
        if (part) {
          // the key's record to its super-tile region right after its last chunk, while the
          // next batch's first chunk is in flight (at the group's end, after its barrier, this
          // phase ran with no hashing beside it)
          zero |= a == 0;
          uint64_t x;  // (as k_hash0_pair's partition)
          if (p_words >= (1ull << 19)) x = bb_index_big(level_seed(0), a, p_words, p_magic);
          else x = bb_index(level_seed(0), a, p_words, p_magic);
          unsigned od = __umulhi((uint32_t)(x >> kRegTileMaxBits), p_mul);
          if (od >= pt.S) od = pt.S - 1;  // unreachable: positions < 64 words
          const unsigned at = atomicAdd(&sk_pcur[od], 1u);
          if (at < (unsigned)pt.reg_cap)
            pt.sup[((uint64_t)blockIdx.x * pt.S + od) * pt.reg_cap + at] = r20_make(a, f, (uint32_t)(grp + cur.k));
          else
            p_over = true;
        } else if (kRes) {
          // results by key in LDS, written back in key order with coalesced stores (each
          // lane's own 8-byte stores cost more: they count against vmcnt, which every step
          // waits on, 1.64 -> 2.11 ms on C5 even with 8192-key groups in the freed LDS)
          res_a[cur.k] = a;
          res_b[cur.k] = f;
        }
      }
      cur = nxt;
    }
    const unsigned long long e0t = prof ? __builtin_amdgcn_s_memtime() : 0;
    __syncthreads();
    if (kRes && !part) {
      for (unsigned k = tid; k < m; k += kSkT) {
        const uint64_t a = res_a[k];
        kh[grp + k] = a;
        fp[grp + k] = res_b[k];
        zero |= a == 0;
      }
    }
    __syncthreads();  // the next group reuses cnt / sidx / res
    if (prof) p_end += __builtin_amdgcn_s_memtime() - e0t;
  }
  if (prof && lane == 0 && (uint64_t)blockIdx.x * (kSkT / 64) + wave < 8192) {
    const unsigned long long tot = __builtin_amdgcn_s_memtime() - pt0, prt1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* q = prof + ((uint64_t)blockIdx.x * (kSkT / 64) + wave) * 8;
    q[0] = tot;
    q[1] = p_hash;
    q[2] = p_wait;
    q[3] = tot - p_hash - p_wait;
    q[4] = prt1 - prt0;
    q[5] = prt0;
    q[6] = prt1;
    q[7] = (p_sort << 32) | (p_end & 0xffffffffull);  // group phases: sort | barrier + write-back
  }
  if (zero) atomicOr(&st->status, kStKeyZero);
  if (part) {
    __syncthreads();  // every cursor atomic done (the last group's barrier preceded the stores only)
    if (tid < pt.S) pt.pcnt[(uint64_t)blockIdx.x * pt.S + tid] = min<unsigned>(sk_pcur[tid], (unsigned)pt.reg_cap);
    if (p_over) atomicOr(&st->status, kStOverflow | kStResOverflow);
  }
}

// ------------------------------------------------------------- level L setup ---------
// Size level L from the redo count the previous level produced and carry its word
// offset (the rank base lvl_base[L] was published by the previous level's last tile).
// Runs only after a big level (the tail sizes its own levels).
__device__ void level_setup(int level, LevelState* st) {
  const int p = level - 1;
  if (p > 0 && !st->preset[p] && st->n[p] <= kGate) return;
  if (st->status & kStStop) return;
  const uint64_t n = st->n[level];
  const uint64_t w = n ? level_words(n) : 0;
  st->words[level] = w;
  st->magic[level] = level_magic(w);
  st->woff[level] = st->woff[p] + st->words[p];
  st->woff[level + 1] = st->woff[level] + w;
  st->nlevels = level;  // levels 0..level-1 are complete; raised again if level runs
}

// ------------------------------------------------------------ level L count ----------
__global__ __launch_bounds__(kCB) void k_count(int level, const Rec* __restrict__ list,
                                               unsigned* __restrict__ hist,
                                               unsigned long long* __restrict__ flags,
                                               unsigned long long* __restrict__ sflags, LevelState* st,
                                               unsigned tb, uint64_t chunk, uint64_t cap_words) {
  __shared__ unsigned sh[kMaxTiles];
  const int p = level - 1;
  const bool preset = st->preset[level] != 0;
  if (!preset && p > 0 && !st->preset[p] && st->n[p] <= kGate) return;  // previous level ran in the tail
  if (st->status & kStStop) return;
  const uint64_t n = st->n[level];
  uint64_t words, magic, woff;
  if (preset) {  // sized by the multi-GPU build: global words, this rank's records
    words = st->words[level];
    magic = st->magic[level];
    woff = st->woff[level];
  } else {  // level setup (every block derives it; block 0 publishes it)
    words = n ? level_words(n) : 0;
    magic = level_magic(words);
    woff = st->woff[p] + st->words[p];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->words[level] = words;
      st->magic[level] = magic;
      st->woff[level] = woff;
      st->woff[level + 1] = woff + words;
      st->nlevels = level;
    }
    if (n <= kGate) return;
    if (no_progress(st, level, n)) return;
  }
  const LevelRange rg = level_range(st, level, words);
  const uint64_t T = ntiles_of(rg.rw, tb), B = (n + chunk - 1) / chunk;
  if (!geom_ok(st, T, B)) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->ntiles[level] = T;
    st->nchunks[level] = B;
    if (woff + words > cap_words) atomicOr(&st->status, kStOverflow);
  }
  for (uint64_t t = (uint64_t)blockIdx.x * kCB + threadIdx.x; t < T; t += (uint64_t)gridDim.x * kCB) flags[t] = 0;
  const uint64_t nseg = (T * B + kScanSeg - 1) / kScanSeg;
  for (uint64_t q = (uint64_t)blockIdx.x * kCB + threadIdx.x; q < nseg; q += (uint64_t)gridDim.x * kCB) sflags[q] = 0;
  const uint64_t seed = level_seed(level);
  for (uint64_t b = blockIdx.x; b < B; b += gridDim.x) {
    for (uint64_t t = threadIdx.x; t < T; t += kCB) sh[t] = 0;
    __syncthreads();
    const uint64_t lo = b * chunk, hi = min(n, lo + chunk);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kCB)
      atomicAdd(&sh[(bb_index(seed, list[i].k, words, magic) - rg.plo) >> tb], 1u);
    __syncthreads();
    for (uint64_t t = threadIdx.x; t < T; t += kCB) hist[t * B + b] = sh[t];
    __syncthreads();
  }
}

// ------------------------------------------------------------------ scatter --------
// LDS: 4096 staged records (96 KiB) + tile ids + per-round count/start + chunk cursors.
constexpr int kScatterKPT = (int)(kSubRound / kSB);  // 4 keys per thread per round

__global__ __launch_bounds__(kSB) void k_scatter(int level, const uint64_t* __restrict__ ik,
                                                 const uint64_t* __restrict__ ifp,
                                                 const uint64_t* __restrict__ ipos, uint64_t pos_base,
                                                 const Rec* __restrict__ ilist,
                                                 const unsigned* __restrict__ off, Rec* __restrict__ bucket,
                                                 LevelState* st, unsigned tb, uint64_t chunk) {
  __shared__ Rec stage[kSubRound];
  __shared__ unsigned short stile[kSubRound];
  __shared__ unsigned cnt[kLdsTiles];
  __shared__ unsigned start[kLdsTiles];
  __shared__ unsigned cur[kLdsTiles];
  if (!level_active(level, st)) return;
  const uint64_t n = st->n[level];
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = st->ntiles[level], B = st->nchunks[level];
  if (T > kLdsTiles) {  // the host predicted fewer tiles: rerun (k_scatter_direct takes any T)
    if (threadIdx.x == 0) atomicOr(&st->status, kStGeometry);
    return;
  }
  const uint64_t plo = level_range(st, level, words).plo;
  const uint64_t seed = level_seed(level);
  // Blocks b, b+8, b+16, ... (one XCD under round-robin dispatch) share one contiguous
  // eighth of the chunks and take them interleaved, so at any moment an XCD's blocks
  // append adjacent runs of every bucket and its L2 completes whole lines.  Speed only.
  const unsigned groups = gridDim.x >= 8 ? 8 : 1;
  const uint64_t xcd = blockIdx.x % groups, r = blockIdx.x / groups, R = gridDim.x / groups;
  const uint64_t per = (B + groups - 1) / groups;
  const uint64_t g0 = min(B, xcd * per), g1 = min(B, g0 + per);
  const unsigned tid = threadIdx.x;
  // The block's work is the sequence of rounds (chunk b, keys [r0, r0 + kSubRound)).
  // Software pipeline: round i+1's records are loaded into registers right after
  // round i has been staged in LDS, so their latency hides behind round i's writes.
  uint64_t b = g0 + r;
  if (b >= g1) return;
  uint64_t r0 = b * chunk, hi = min(n, r0 + chunk);
  Rec rec[kScatterKPT];
  auto load_round = [&](uint64_t base, uint64_t end) {
#pragma unroll
    for (int q = 0; q < kScatterKPT; ++q) {
      const uint64_t i = base + (uint64_t)q * kSB + tid;
      if (i < end) {
        if (ilist) {
          rec[q] = ilist[i];
        } else {
          rec[q].k = ik[i];
          rec[q].f = ifp[i];
          rec[q].p = ipos ? ipos[i] : pos_base + i;
        }
      }
    }
  };
  load_round(r0, hi);
  for (uint64_t t = tid; t < T; t += kSB) {
    cnt[t] = 0;
    cur[t] = off[t * B + b];
  }
  __syncthreads();
  for (;;) {
    unsigned tt[kScatterKPT], rk[kScatterKPT];
#pragma unroll
    for (int q = 0; q < kScatterKPT; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kSB + tid;
      if (i < hi) {
        tt[q] = (unsigned)((bb_index(seed, rec[q].k, words, magic) - plo) >> tb);
        rk[q] = atomicAdd(&cnt[tt[q]], 1u);
      }
    }
    __syncthreads();
    // exclusive scan of the round's per-tile counts (kLdsTiles / kSB tiles per thread)
    constexpr int kTPT = (int)(kLdsTiles / kSB);
    const uint64_t t0 = (uint64_t)kTPT * tid;
    unsigned a[kTPT];
    uint64_t sum = 0;
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      a[q] = t0 + q < T ? cnt[t0 + q] : 0u;
      sum += a[q];
    }
    uint64_t tot;
    uint64_t ex = block_exscan<kSB>(sum, &tot);
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      if (t0 + q < T) start[t0 + q] = (unsigned)ex;
      ex += a[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kScatterKPT; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kSB + tid;
      if (i < hi) {
        const unsigned slot = start[tt[q]] + rk[q];
        stage[slot] = rec[q];
        stile[slot] = (unsigned short)tt[q];
      }
    }
    // advance to the next round and prefetch it
    const unsigned m = (unsigned)min<uint64_t>(kSubRound, hi - r0);
    const uint64_t pb = b;
    r0 += kSubRound;
    if (r0 >= hi) {
      b += R;
      if (b < g1) {
        r0 = b * chunk;
        hi = min(n, r0 + chunk);
      }
    }
    const bool more = b < g1;
    if (more) load_round(r0, hi);
    __syncthreads();
    for (unsigned j = tid; j < m; j += kSB) {
      const unsigned t = stile[j];
      bucket[cur[t] + (j - start[t])] = stage[j];
    }
    __syncthreads();
    if (!more) break;
    if (b != pb) {
      for (uint64_t t = tid; t < T; t += kSB) {
        cnt[t] = 0;
        cur[t] = off[t * B + b];
      }
    } else {
      for (uint64_t t = tid; t < T; t += kSB) {
        cur[t] += cnt[t];
        cnt[t] = 0;
      }
    }
    __syncthreads();
  }
}

constexpr unsigned kSplitSubBitsDev = 14;  // = kSplitSubBits (sub-tile of the split kernel)

// ------------------------------------------------------ 20-byte level-0 records ------
// Level 0 with identity positions (pos_out = pos_base + key index, the builder's case):
// a bucket / scratch record is (k, f, i) in 20 bytes — five dwords, i the key's index —
// instead of Rec's 24, so the level-0 scatter writes and the split kernel's bucket reads,
// scratch writes and scratch reads move 4 bytes less per key (1.6 GB less at C3).  Only
// the reservation scatter and the split big-tile kernel use it; the next list stays Rec.

// ---------------------------------------------------------- reservation scatter ------
// Small levels (a few 10^5 .. 10^6 keys) skip the count and histogram-scan kernels:
// tile t owns the fixed bucket slot [t * cap, (t + 1) * cap), cap = bucket_cap / T
// (several times the ~n/T keys a tile receives), cut into kResShards shards, and each
// block reserves its run in its shard of a tile with one atomic per (round, tile).  Record order inside a tile is then
// arbitrary, which nothing downstream depends on (ranks come from positions).  A slot
// overflow sets kStOverflow and the build reruns on the counted path.
// kR records per round, at most kT tiles (<4096, 4096>: one block per CU, 152 KiB of LDS).
// <2048, 2048> (two blocks per CU, so one block's atomics and barriers overlap the other's
// memory phases) measured slower on C2: level-0 scatter 0.156 -> 0.214 ms.
// kSrc: 0 records from ilist; 1 level-0 arrays ik / ifp with caller positions ipos;
// 2 level-0 arrays with identity positions; 3 records from ilist with padding records
// (k = 0) to skip: the multi-GPU build's fixed-size exchange regions (k_route_pad).  A compile-time source keeps the loads
// straight-line: with run-time selects the compiler waited out every record's loads
// before issuing the next record's (four round trips per round).
// kP20 (kSrc 2 / 4): bucket records are R20 (the split kernel reads them).  kSrc 4: records
// from ilist as R20 (a list level with identity positions, BinBuffers::l20).
template <int kR, int kT, int kSrc, bool kP20 = false>
__global__ __launch_bounds__(kSB) void k_scatter_res(int level, const Rec* __restrict__ ilist,
                                                     const uint64_t* __restrict__ ik, const uint64_t* __restrict__ ifp,
                                                     const uint64_t* __restrict__ ipos, uint64_t pos_base,
                                                     unsigned* __restrict__ tcnt, Rec* __restrict__ bucket,
                                                     uint64_t bucket_cap, unsigned long long* __restrict__ flags,
                                                     LevelState* st, unsigned tb, uint64_t cap_words,
                                                     unsigned long long* __restrict__ prof, uint64_t i_lo,
                                                     uint64_t i_hi, unsigned ts, unsigned gate) {
  constexpr int kKPT = kR / kSB;
  if (gate && !st->skew) return;  // gate: only for a skewed set (the fused P0 hash partitioned the rest)
  static_assert(!kP20 || kSrc == 2 || kSrc == 4, "20-byte records carry identity positions");
  static_assert(kSrc != 4 || kP20, "an R20 list scatters into R20 slots");
  __shared__ uint64_t stage_raw[kP20 ? (kR * 5 + 1) / 2 : kR * 3];  // kR Rec, or kR R20
  Rec* const stage = reinterpret_cast<Rec*>(stage_raw);
  R20* const stage20 = reinterpret_cast<R20*>(stage_raw);
  R20* const bucket20 = reinterpret_cast<R20*>(bucket);
  __shared__ unsigned short stile[kR];
  __shared__ unsigned cnt[kT];
  __shared__ unsigned start[kT];
  __shared__ unsigned cur[kT];  // bucket indices fit u32 (n < 2^32 per GPU)
  __shared__ unsigned s_over;
  const int p = level - 1;
  const bool preset = st->preset[level] != 0;
  if (!preset && p > 0 && !st->preset[p] && st->n[p] <= kGate) return;  // previous level ran in the tail
  if (st->status & kStStop) return;
  // [i_lo, i_hi): one chunk of level 0's key-order arrays (pipelined level 0); else all
  const uint64_t n = i_hi ? min<uint64_t>(st->n[level], i_hi) : st->n[level];
  const unsigned tid = threadIdx.x;
  uint64_t words, magic, woff;
  if (level == 0 || preset) {  // level 0: sized by k_init_state; preset: by the multi-GPU build
    words = st->words[level];
    magic = st->magic[level];
    woff = st->woff[level];
  } else {  // level setup (every block derives it; block 0 publishes it)
    words = n ? level_words(n) : 0;
    magic = level_magic(words);
    woff = st->woff[p] + st->words[p];
    if (blockIdx.x == 0 && tid == 0) {
      st->words[level] = words;
      st->magic[level] = magic;
      st->woff[level] = woff;
      st->woff[level + 1] = woff + words;
      st->nlevels = level;
    }
    if (n <= kGate) {
      // an R20 list (planned before level 0, BinBuffers::l20) for a level that turned out
      // small enough for the mid / tail kernels, which read Rec: rerun conservatively
      if (kSrc == 4 && blockIdx.x == 0 && tid == 0) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 1u));
      return;
    }
    if (no_progress(st, level, n)) return;
  }
  const LevelRange rg = level_range(st, level, words);
  const uint64_t T = tiles_of(rg.rw, tb, ts);
  // ts tiles: tile = (position offset >> 14) / ts by a 32-bit reciprocal (exact: the
  // quotient's operand is < 2^18 and ts <= 16)
  const uint32_t ts_mul = ts ? 0xffffffffu / ts + 1 : 0;
  if (T > kT) {
    if (tid == 0) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 2u));
    return;
  }
  if (blockIdx.x == 0 && tid == 0) {
    st->ntiles[level] = T;
    st->nchunks[level] = 0;
    if (woff + words > cap_words) atomicOr(&st->status, kStOverflow);
  }
  for (uint64_t t = (uint64_t)blockIdx.x * kSB + tid; t < T; t += (uint64_t)gridDim.x * kSB) flags[t] = 0;
  // tile t's slot is cut into kResShards shards, one per XCD under round-robin dispatch,
  // so a counter sees ~1/8 of the blocks: returning atomics on one address serialize
  const uint64_t cap = bucket_cap / T, scap = cap / kResShards;
  const unsigned shard = blockIdx.x % kResShards;
  const uint64_t seed = level_seed(level);
  const uint64_t stride = (uint64_t)gridDim.x * kR;
  uint64_t r0 = i_lo + (uint64_t)blockIdx.x * kR;
  if (r0 >= n) return;
  // debug: this block's time per phase summed over all its rounds, in prof row 32 + level
  // (stored as cumulative stamps: p[0] start, p[i] = p[i-1] + time of phase i)
  unsigned long long* tp =
      prof && blockIdx.x < kMaxTiles ? prof + ((uint64_t)(32 + level) * kMaxTiles + blockIdx.x) * 8 : nullptr;
  unsigned long long t_last = 0, t_first = 0, acc[4] = {0, 0, 0, 0};
#define SPROF(i)                                                       \
  do {                                                                 \
    if (tp && tid == 0) {                                              \
      const unsigned long long now_ = wall_clock64();                  \
      if ((i) == 0) t_first = now_;                                    \
      else if ((i) <= 4) acc[(i) > 0 ? (i) - 1 : 0] += now_ - t_last;    \
      t_last = now_;                                                   \
    }                                                                  \
  } while (0)
  SPROF(0);
  // records as three scalar arrays: a conditionally loaded Rec[] would live in scratch.
  // Level 0 reads the hash kernel's key-order arrays instead of a record list.
  uint64_t rk_[kKPT], rf_[kKPT], rp_[kKPT];
  auto load = [&](uint64_t i, int q) {
    if constexpr (kSrc == 4) {
      const R20 r = reinterpret_cast<const R20*>(ilist)[i];
      rk_[q] = (uint64_t)r.w[0] | ((uint64_t)r.w[1] << 32);
      rf_[q] = (uint64_t)r.w[2] | ((uint64_t)r.w[3] << 32);
      rp_[q] = r.w[4];
    } else if constexpr (kSrc == 0 || kSrc == 3) {
      rk_[q] = ilist[i].k;
      rf_[q] = ilist[i].f;
      rp_[q] = ilist[i].p;
    } else {
      rk_[q] = ik[i];
      rf_[q] = ifp[i];
      if constexpr (kSrc == 1) rp_[q] = ipos[i];
    }
  };
#pragma unroll
  for (int q = 0; q < kKPT; ++q) {
    const uint64_t i = r0 + (uint64_t)q * kSB + tid;
    rk_[q] = rf_[q] = rp_[q] = 0;
    if (i < n) load(i, q);
  }
  for (uint64_t t = tid; t < T; t += kSB) cnt[t] = 0;
  if (tid == 0) s_over = 0;
  __syncthreads();
  for (;;) {
    // a record's tile (< 2^12) and its rank among the round's records of that tile (< 2^13)
    // packed into one register: tt << 13 | rk
    static_assert(kT <= 4096 && kR <= 8192, "tile / rank packing");
    unsigned trk[kKPT];
#pragma unroll
    for (int q = 0; q < kKPT; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kSB + tid;
      if (i < n && (kSrc != 3 || rk_[q] != 0)) {  // kSrc 3: k = 0 is a padding record (k_route_pad)
        const uint64_t lp = bb_index(seed, rk_[q], words, magic) - rg.plo;
        const unsigned t = ts ? __umulhi((uint32_t)(lp >> kSplitSubBitsDev), ts_mul) : (unsigned)(lp >> tb);
        trk[q] = (t << 13) | atomicAdd(&cnt[t], 1u);
      }
    }
    __syncthreads();
    SPROF(1);
    constexpr int kTPT = (int)(kT / kSB);
    // The round's returning reservation atomics (one per tile present; thread tid takes
    // tiles q kSB + tid) go out as soon as the counts are final, so their round trip
    // overlaps the count scan, the stage writes and the next round's loads.  Counts are
    // re-read from LDS where they are used (cnt[] holds them until the next round) rather
    // than kept in registers: the 2048 / 4096-tile forms spilled 8-13 VGPRs in this loop.
    unsigned at[kTPT];
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      const uint64_t t = (uint64_t)q * kSB + tid;
      const unsigned c = t < T ? cnt[t] : 0u;
      at[q] = 0;
      if (c) at[q] = atomicAdd(&tcnt[t * kResShards + shard], c);
    }
    const uint64_t t0 = (uint64_t)kTPT * tid;
    uint64_t sum = 0;
#pragma unroll
    for (int q = 0; q < kTPT; ++q) sum += t0 + q < T ? cnt[t0 + q] : 0u;
    uint64_t tot;
    uint64_t ex = block_exscan<kSB>(sum, &tot);
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      if (t0 + q < T) {
        start[t0 + q] = (unsigned)ex;
        ex += cnt[t0 + q];
      }
    }
    __syncthreads();  // start[] complete
    SPROF(2);
#pragma unroll
    for (int q = 0; q < kKPT; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kSB + tid;
      if (i < n && (kSrc != 3 || rk_[q] != 0)) {
        const unsigned t = trk[q] >> 13, slot = start[t] + (trk[q] & 8191u);
        // identity positions (kSrc 2) are the record's index, recomputed rather than held
        if constexpr (kP20) stage20[slot] = r20_make(rk_[q], rf_[q], (uint32_t)(kSrc == 4 ? rp_[q] : i));
        else stage[slot] = Rec{rk_[q], rf_[q], kSrc == 2 ? pos_base + i : rp_[q]};
        stile[slot] = (unsigned short)t;
      }
    }
    // The next round's loads are issued before any atomic result is used, so the two
    // latencies overlap; one tile at a time waited out each round trip in turn (C3 level
    // 0: ~10 of ~20 us per round).
    // the round's staged records (kSrc 3: its padding records were not staged)
    const unsigned m = kSrc == 3 ? start[T - 1] + cnt[T - 1] : (unsigned)min<uint64_t>(kR, n - r0);
    r0 += stride;
    const bool more = r0 < n;
#pragma unroll
    for (int q = 0; q < kKPT; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kSB + tid;
      if (i < n) load(i, q);
    }
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      const uint64_t t = (uint64_t)q * kSB + tid;
      const unsigned c = t < T ? cnt[t] : 0u;
      if (c) {
        if (at[q] + c > scap) s_over = 1;
        cur[t] = (unsigned)(t * cap + shard * scap + at[q]);
      }
    }
    __syncthreads();
    SPROF(3);
    if (s_over) break;
    for (unsigned j = tid; j < m; j += kSB) {
      const unsigned t = stile[j];
      if constexpr (kP20) bucket20[cur[t] + (j - start[t])] = stage20[j];
      else bucket[cur[t] + (j - start[t])] = stage[j];
    }
    __syncthreads();
    SPROF(4);
    if (!more) break;
    for (uint64_t t = tid; t < T; t += kSB) cnt[t] = 0;
    __syncthreads();
  }
  if (s_over && tid == 0) atomicOr(&st->status, kStOverflow | kStResOverflow);
  if (tp && tid == 0) {
    unsigned long long c = t_first;
    tp[0] = c;
    for (int i = 0; i < 4; ++i) tp[i + 1] = (c += acc[i]);
    tp[7] = c;
  }
#undef SPROF
}

// ------------------------------------------- level 0 in 2^14-position tiles (P0) --------
// Level 0 of a set with more than kP0MinTiles 2^14-position tiles (C3: 12.2k) takes
// register-resident tiles too, without the split kernel's 2^14 sub-tile scratch round trip:
// its positions are cut into S super-tiles of tps tiles each (tps <= kT), the level-0 records
// (R20: k, f, key index) first land in the super-tiles: in per-(hash block, super-tile)
// regions written by the level-0 hash itself (k_hash0_pair<..., PT>), or, for skewed /
// unaligned sets, in per-(super-tile, XCD shard) slots written by a k_scatter_res pass over
// kh / fp — and this kernel gives each super-tile bps blocks that
// scatter its records into the slots of their 2^14-position tiles: an LDS counting sort by
// tile inside the super-tile's window, one reservation atomic per (round, tile, XCD shard),
// runs written whole (k_scatter_res's scheme).  A record reads 20 B and writes 20 B here, and
// k_tile_p0 reads it once more: the 40 B per record of the split kernel's scratch are gone.
struct P0In {
  const R20* sup;
  uint64_t reg_cap;        // regions: records per (hash block, super-tile) region
  const unsigned* pcnt;    // ... their fills, [hash block][super-tile]
  unsigned NB, S;          // hash blocks, super-tiles
  unsigned NB_skew;        // a skewed set: k_hash_skew's blocks and region size
  uint64_t reg_cap_skew;
  uint64_t sup_cap;        // slots: R20 records in sup (the partition pass's bucket capacity)
  const unsigned* scnt;    // ... their fills
  bool fused;              // the hash wrote regions (unless it found the set skewed)
};

// tb: the tiles' position bits (kRegTileMaxBits for the single-GPU k_tile_p0; the bitmap
// decomposition scales them with the rank count, P0Bufs::tb <= 16).  kX: each record's
// position within its tile (u16) also goes to xo at its slot (the bitmap mark reads 2 B per
// record instead of its 20, and the settle skips bb_index), staged beside the tile.
template <int kR, int kT, int NT = kSB, bool kX = false>  // (512 threads, 2560-record rounds, two blocks per CU: slower)
__global__ __launch_bounds__(NT) void k_scatter_p0(P0In in, unsigned bps, unsigned tps, R20* __restrict__ bucket,
                                                    uint64_t bcap, unsigned* __restrict__ tcnt,
                                                    unsigned long long* __restrict__ flags, LevelState* st,
                                                    unsigned long long* __restrict__ prof, unsigned tb = kRegTileMaxBits,
                                                    uint16_t* __restrict__ xo = nullptr, int level = 0) {
  constexpr int kKPT = kR / NT;
  constexpr unsigned kMaxRuns = kH0Grid / 8 + 1;  // bps >= 8 (launch_p0_scatter)
  __shared__ uint64_t stage_raw[(kR * 5 + 1) / 2];
  R20* const stage = reinterpret_cast<R20*>(stage_raw);
  __shared__ unsigned short stile[kR];    // slot -> tile in the window
  __shared__ uint16_t sx[kX ? kR : 1];    // kX: slot -> position in the tile
  __shared__ unsigned cnt[kT];
  __shared__ unsigned start[kT];
  __shared__ unsigned cur[kT];
  __shared__ unsigned rp[kMaxRuns + 1];  // regions: the block's runs' exclusive prefix
  __shared__ unsigned s_over;
  if (st->status & kStStop) return;
  const unsigned tid = threadIdx.x;
  // (level > 0: a bitmap list level's records, partitioned into the super-tiles' slots first)
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = tiles_of(words, tb, 0);
  if (blockIdx.x == 0 && tid == 0) {
    st->ntiles[level] = T;
    st->nchunks[level] = 0;
  }
  for (uint64_t t = (uint64_t)blockIdx.x * NT + tid; t < T; t += (uint64_t)gridDim.x * NT) flags[t] = 0;
  const unsigned sidx = blockIdx.x / bps, part = blockIdx.x % bps;
  const uint64_t t0 = (uint64_t)sidx * tps;
  if (t0 >= T) return;
  const unsigned tn = (unsigned)min<uint64_t>(tps, T - t0);
  if (tn > (unsigned)kT) {
    if (tid == 0) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 3u));
    return;
  }
  // This block's records, index j in [lo, hi): the super-tile's kResShards slots back to back
  // (a skewed set, partitioned by k_scatter_res), or the runs its part of the hash blocks left
  // in their regions (prefix rp; record j of run i at region (b0 + i, sidx) + j - rp[i]).
  // regions: the fused partition of either level-0 hash (k_hash_skew's for a skewed set)
  // (a list level's regions come from the previous level's settle, whatever the key lengths)
  const bool regions = in.fused, skw = st->skew && level == 0;
  const unsigned NB = skw ? in.NB_skew : in.NB;
  const uint64_t reg_cap = skw ? in.reg_cap_skew : in.reg_cap;
  unsigned pre[kResShards + 1];
  uint64_t lo = 0, hi = 0;
  unsigned b0 = 0, nr = 0;
  if (regions) {
    b0 = (unsigned)((uint64_t)NB * part / bps);
    nr = (unsigned)((uint64_t)NB * (part + 1) / bps) - b0;
    if (nr > (unsigned)NT || nr > kMaxRuns) {  // (the host keeps bps >= NB / NT)
      if (tid == 0) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 4u));
      return;
    }
    const unsigned c = tid < nr ? in.pcnt[(uint64_t)(b0 + tid) * in.S + sidx] : 0u;
    uint64_t tot;
    const uint64_t ex = block_exscan<NT>(c, &tot);
    if (tid < nr) rp[tid] = (unsigned)ex;
    if (tid == 0) rp[nr] = (unsigned)tot;
    hi = tot;
    __syncthreads();
  } else {
    pre[0] = 0;
#pragma unroll
    for (int x = 0; x < kResShards; ++x) pre[x + 1] = pre[x] + in.scnt[sidx * kResShards + x];
    const uint64_t m = pre[kResShards];
    lo = m * part / bps;
    hi = m * (part + 1) / bps;
  }
  // the partition pass's slot layout (k_scatter_res over ceil(T / tps) super-tiles: cap
  // = sup_cap / that many per super-tile, cut into kResShards shard slots)
  const uint64_t sup_each = in.sup_cap / ((T + tps - 1) / tps), slot_cap = sup_each / kResShards;
  const R20* sbase = in.sup + (uint64_t)sidx * sup_each;
  // record j's address (the loads themselves run in straight-line code: a load inside the
  // search's divergent branches was waited for on the spot, five HBM latencies per round)
  auto src = [&](uint64_t j) -> const R20* {
    if (regions) {
      unsigned a = 0, z = nr;  // the run holding j: rp[a] <= j < rp[a + 1]
      while (z - a > 1) {
        const unsigned mid = (a + z) >> 1;
        if (rp[mid] <= (unsigned)j) a = mid;
        else z = mid;
      }
      return in.sup + ((uint64_t)(b0 + a) * in.S + sidx) * reg_cap + ((unsigned)j - rp[a]);
    }
    uint64_t o = j;
#pragma unroll
    for (int x = 1; x < kResShards; ++x)
      if (j >= pre[x]) o = (uint64_t)x * slot_cap + (j - pre[x]);
    return sbase + o;
  };
  // records live as (dwords 0-3, dword 4) register pairs: an R20[] copied whole into the stage
  // stayed a memory array (its f / i words spilled to LDS and scratch, each load waited for)
  uint4 rq[kKPT];
  uint32_t rz[kKPT];
  auto fetch = [&](uint64_t r) {
    const uint32_t* a[kKPT];
#pragma unroll
    for (int u = 0; u < kKPT; ++u) {
      const uint64_t j = r + (uint64_t)u * NT + tid;
      a[u] = (j < hi ? src(j) : in.sup)->w;  // (a past-the-end lane reads record 0; trk skips it)
    }
#pragma unroll
    for (int u = 0; u < kKPT; ++u) {
      rq[u] = *reinterpret_cast<const uint4*>(a[u]);  // dword-aligned 16-B load
      rz[u] = a[u][4];
    }
  };
  const uint64_t cap = bcap / T, scap = cap / kResShards;
  const unsigned shard = blockIdx.x % kResShards;
  const uint64_t seed = level_seed(level);
  uint64_t r0 = lo;
  if (r0 >= hi) return;
  // debug: phase times summed over the block's rounds, k_scatter_res's row 32 (level 0) layout
  unsigned long long* tp = prof && blockIdx.x < kMaxTiles ? prof + ((uint64_t)32 * kMaxTiles + blockIdx.x) * 8 : nullptr;
  unsigned long long t_last = 0, t_first = 0, acc[4] = {0, 0, 0, 0};
#define P0PROF(i)                                                      \
  do {                                                                 \
    if (tp && tid == 0) {                                              \
      const unsigned long long now_ = wall_clock64();                  \
      if ((i) == 0) t_first = now_;                                    \
      else acc[(i) > 0 ? (i) - 1 : 0] += now_ - t_last;                \
      t_last = now_;                                                   \
    }                                                                  \
  } while (0)
  P0PROF(0);
  fetch(r0);
  for (unsigned t = tid; t < kT; t += NT) cnt[t] = 0;
  if (tid == 0) s_over = 0;
  __syncthreads();
  bool geo = false;
  for (;;) {
    unsigned trk[kKPT];  // tile in the window << 13 | rank in the round's run of that tile
    uint16_t xr[kX ? kKPT : 1];
#pragma unroll
    for (int u = 0; u < kKPT; ++u) {
      const uint64_t j = r0 + (uint64_t)u * NT + tid;
      trk[u] = 0xffffffffu;
      if (j < hi) {
        const uint64_t k = (uint64_t)rq[u].x | ((uint64_t)rq[u].y << 32);
        const uint64_t x = bb_index(seed, k, words, magic);
        if constexpr (kX) xr[u] = (uint16_t)(x & ((1u << tb) - 1));
        const uint64_t t = (x >> tb) - t0;
        if (t < tn) trk[u] = ((unsigned)t << 13) | atomicAdd(&cnt[t], 1u);
        else geo = true;
      }
    }
    __syncthreads();
    P0PROF(1);
    constexpr int kTPT = (int)((kT + NT - 1) / NT);
    unsigned at[kTPT];
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      const unsigned t = (unsigned)q * NT + tid;
      const unsigned c = t < tn ? cnt[t] : 0u;
      at[q] = 0;
      if (c) at[q] = atomicAdd(&tcnt[(t0 + t) * kResShards + shard], c);
    }
    const unsigned tb0 = (unsigned)kTPT * tid;
    uint64_t sum = 0;
#pragma unroll
    for (int q = 0; q < kTPT; ++q) sum += tb0 + q < tn ? cnt[tb0 + q] : 0u;
    uint64_t tot;
    uint64_t ex = block_exscan<NT>(sum, &tot);
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      if (tb0 + q < tn) {
        start[tb0 + q] = (unsigned)ex;
        ex += cnt[tb0 + q];
      }
    }
    __syncthreads();  // start[] complete
    P0PROF(2);
#pragma unroll
    for (int u = 0; u < kKPT; ++u) {
      if (trk[u] != 0xffffffffu) {
        const unsigned t = trk[u] >> 13, slot = start[t] + (trk[u] & 8191u);
        uint32_t* d = stage[slot].w;
        d[0] = rq[u].x;
        d[1] = rq[u].y;
        d[2] = rq[u].z;
        d[3] = rq[u].w;
        d[4] = rz[u];
        if constexpr (kX) sx[slot] = xr[u];
        stile[slot] = (unsigned short)t;
      }
    }
    const unsigned mr = (unsigned)tot;
    r0 += kR;
    const bool more = r0 < hi;
#pragma unroll
    for (int q = 0; q < kTPT; ++q) {
      const unsigned t = (unsigned)q * NT + tid;
      const unsigned c = t < tn ? cnt[t] : 0u;
      if (c) {
        if (at[q] + c > scap) s_over = 1;
        cur[t] = (unsigned)((t0 + t) * cap + shard * scap + at[q]);
      }
    }
    __syncthreads();
    P0PROF(3);
    if (s_over) break;
    for (unsigned j = tid; j < mr; j += NT) {
      const unsigned t = stile[j];
      const unsigned o = cur[t] + (j - start[t]);
      bucket[o] = stage[j];
      if constexpr (kX) xo[o] = sx[j];
    }
    // The next round's records, in flight over the barriers below.  (Issued before the write
    // above, they were waited for at once: a 64-bit address write to a VGPR pair that a
    // pending load still read, s_waitcnt vmcnt(0), in the store's address computation.)
    if (more) fetch(r0);

    __syncthreads();
    P0PROF(4);
    if (!more) break;
    for (unsigned t = tid; t < tn; t += NT) cnt[t] = 0;
    __syncthreads();
  }
  if (tp && tid == 0) {
    unsigned long long c = t_first;
    tp[0] = c;
    for (int i = 0; i < 4; ++i) tp[i + 1] = (c += acc[i]);
    tp[7] = c;
  }
#undef P0PROF
  if (geo) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 5u));
  if (s_over && tid == 0) atomicOr(&st->status, kStOverflow | kStResOverflow);
}

// ---- the super-tile scatter, direct form; overlapped with the level-0 hash --------------
// A round's records stay in registers and go straight to their tiles' slots: LDS holds only
// the per-tile counts and run bases (~5 KB), so a block fits beside three hash blocks on a CU.
// A super-tile's records are cut into parts by hash block: part x C + c (XCD x, chunk c)
// holds the regions of hash blocks x + 8 (c R + i), i < R = NB / 8C, and its records take
// reservation shard x.
// kOv: persistent blocks launched beside the level-0 hash (k_hash0_pair with P0Part::hxcc).
// A block takes the parts of the residue class of hash blocks that runs on its own XCD (the
// dispatcher deals a launch's blocks to the XCDs round-robin, from a varying first XCD: the
// class is learned from the first eight hash blocks' published XCDs, each part's checked) by
// ticket, chunk-major, and waits for the part's hash blocks: they wrote their region runs through its L2, so their fills — published with agent-scope
// stores after a workgroup release — make the runs readable here without an L2 write-back.  A
// part whose hash blocks ran elsewhere or are not done within the spin bound, and every part
// still open when the hash has finished, is left to the follow-up launch (!kOv: one block per
// (super-tile, part), after the hash, so across a kernel boundary), which skips the parts the
// overlapped launch marked done.
struct P0Ov {
  const unsigned* hxcc = nullptr;  // each hash block's XCD (kOv)
  unsigned* done = nullptr;        // [part][super-tile] scattered by the overlapped launch
  unsigned C = 8;                  // chunks per XCD
};
constexpr int kDT = 256;
constexpr int kDU = 16;                       // records per thread and round (4096 per round)
constexpr unsigned kPcntOpen = 0xffffffffu;   // a region fill not yet published
constexpr unsigned kOvSpin = 1u << 20;        // wait rounds for a part's hash blocks (~s_sleep 8 each)

template <int kT, bool kOv>
__global__ __launch_bounds__(kDT) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_scatter_p0d(P0In in, unsigned tps, R20* __restrict__ bucket, uint64_t bcap,
                                                     unsigned* __restrict__ tcnt, unsigned long long* __restrict__ flags,
                                                     LevelState* st, P0Ov ov) {
  __shared__ unsigned cnt[kT];
  __shared__ unsigned cur[kT];
  __shared__ unsigned rp[65];
  __shared__ unsigned s_item, s_ok, s_over;
  if (st->status & kStStop) return;
  const unsigned tid = threadIdx.x, lane = lane_id();
  const uint64_t words = st->words[0], magic = st->magic[0];
  const uint64_t T = tiles_of(words, kRegTileMaxBits, 0);
  const bool skw = st->skew != 0;
  if (kOv && skw) return;  // the skewed hash's regions come after this launch: the follow-up's
  if (!kOv) {
    if (blockIdx.x == 0 && tid == 0) {
      st->ntiles[0] = T;
      st->nchunks[0] = 0;
    }
    for (uint64_t t = (uint64_t)blockIdx.x * kDT + tid; t < T; t += (uint64_t)gridDim.x * kDT) flags[t] = 0;
  }
  const unsigned NB = skw ? in.NB_skew : in.NB;
  const uint64_t reg_cap = skw ? in.reg_cap_skew : in.reg_cap;
  const unsigned C = ov.C, R = NB / (8 * C), parts = 8 * C;
  const uint64_t cap = bcap / T, scap = cap / kResShards;
  const uint64_t seed = level_seed(0);
  // kOv: the residue class r (hash blocks r, r + 8, ...) that runs on this block's XCD, from
  // the XCDs the first eight hash blocks publish at their start
  unsigned x_me = 0;
  if (kOv) {
    if (tid < 64) {
      const unsigned me = xcc_id();
      unsigned hx = kPcntOpen;
      uint64_t m = 0;
      for (unsigned spin = 0; spin < kOvSpin; ++spin) {
        if (lane < 8) hx = __hip_atomic_load(const_cast<unsigned*>(ov.hxcc) + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = __ballot(lane < 8 && hx == me);
        if (m) break;
        __builtin_amdgcn_s_sleep(8);
      }
      if (lane == 0) s_item = m ? (unsigned)__builtin_ctzll(m) : ~0u;
    }
    __syncthreads();
    x_me = s_item;
    if (x_me >= 8) return;  // no class found: the follow-up takes every part
    __syncthreads();
  }
  if (tid == 0) s_over = 0;
  for (unsigned t = tid; t < (unsigned)kT; t += kDT) cnt[t] = 0;
  __syncthreads();
  bool geo = false;
  for (;;) {
    unsigned sidx, part;
    if (kOv) {
      if (tid == 0) {
        unsigned it = ~0u;
        if (__hip_atomic_load(&st->h0_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < NB)
          it = (unsigned)atomicAdd(&st->ov_ticket[x_me], 1ull);
        s_item = it;
      }
      __syncthreads();
      const unsigned it = s_item;
      if (it >= C * in.S) break;
      sidx = it % in.S;
      part = x_me * C + it / in.S;
    } else {
      sidx = blockIdx.x / parts;
      part = blockIdx.x % parts;
      if (ov.done && ov.done[(uint64_t)part * in.S + sidx]) break;
    }
    const unsigned x = part / C, c = part % C;
    const uint64_t t0 = (uint64_t)sidx * tps;
    if (t0 >= T) {
      if (kOv) continue;
      break;
    }
    const unsigned tn = (unsigned)min<uint64_t>(tps, T - t0);
    if (tn > (unsigned)kT) {
      geo = true;
      break;
    }
    // the part's runs: lane i of wave 0 reads hash block x + 8 (c R + i)'s fill
    if (tid < 64) {
      const unsigned hb = x + 8 * (c * R + lane);
      unsigned* const pp = const_cast<unsigned*>(in.pcnt) + (uint64_t)hb * in.S + sidx;
      unsigned v = 0;
      bool ok = true;
      if (kOv) {
        if (lane < R) v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (unsigned spin = 0;; ++spin) {
          const bool open = lane < R && v == kPcntOpen;
          if (!__ballot(open)) break;
          if (spin >= kOvSpin) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(8);
          if (open) v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (ok) {  // every hash block of the part ran on this XCD
          const unsigned me = xcc_id();
          const unsigned hx =
              lane < R ? __hip_atomic_load(const_cast<unsigned*>(ov.hxcc) + hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : me;
          if (__ballot(hx != me)) ok = false;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      } else if (lane < R) {
        v = *pp;
      }
      if (!ok || lane >= R) v = 0;
      unsigned incl = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned y = __shfl_up(incl, d);
        if (lane >= (unsigned)d) incl += y;
      }
      rp[lane] = incl - v;
      if (lane == 63) rp[64] = incl;
      if (lane == 0) s_ok = ok ? 1u : 0u;
    }
    __syncthreads();
    if (kOv && !s_ok) break;  // left to the follow-up launch
    const unsigned tot = rp[64];
    const R20* const rbase = in.sup;
    for (unsigned r0 = 0; r0 < tot; r0 += kDT * kDU) {
      uint4 rq[kDU];
      uint32_t rz[kDU];
      unsigned trk[kDU];
      // the round's loads straight-line, all in flight together (indices clamped, not guarded)
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        const unsigned j = min(r0 + (unsigned)u * kDT + tid, tot - 1);
        unsigned a = 0, z = R;  // the run holding j: rp[a] <= j < rp[a + 1]
        while (z - a > 1) {
          const unsigned mid = (a + z) >> 1;
          if (rp[mid] <= j) a = mid;
          else z = mid;
        }
        const unsigned hb = x + 8 * (c * R + a);
        const uint32_t* w = (rbase + ((uint64_t)hb * in.S + sidx) * reg_cap + (j - rp[a]))->w;
        rq[u] = *reinterpret_cast<const uint4*>(w);  // dword-aligned 16-B load
        rz[u] = w[4];
      }
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        trk[u] = ~0u;
        if (r0 + (unsigned)u * kDT + tid < tot) {
          const uint64_t k = (uint64_t)rq[u].x | ((uint64_t)rq[u].y << 32);
          const uint64_t t = (bb_index(seed, k, words, magic) >> kRegTileMaxBits) - t0;
          if (t < tn) trk[u] = ((unsigned)t << 13) | atomicAdd(&cnt[t], 1u);
          else geo = true;
        }
      }
      __syncthreads();
      for (unsigned t = tid; t < tn; t += kDT) {
        const unsigned n = cnt[t];
        if (n) {
          const unsigned at = atomicAdd(&tcnt[(t0 + t) * kResShards + x], n);
          if (at + n > scap) s_over = 1;
          cur[t] = (unsigned)((t0 + t) * cap + x * scap + at);
          cnt[t] = 0;
        }
      }
      __syncthreads();
      if (s_over) break;
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        if (trk[u] != ~0u) {
          uint32_t* d = bucket[cur[trk[u] >> 13] + (trk[u] & 8191u)].w;
          *reinterpret_cast<uint4*>(d) = rq[u];
          d[4] = rz[u];
        }
      }
    }
    if (s_over) break;
    if (kOv && tid == 0) ov.done[(uint64_t)part * in.S + sidx] = 1u;
    if (!kOv) break;
  }
  if (geo) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 6u));
  if (s_over && tid == 0) atomicOr(&st->status, kStOverflow | kStResOverflow);
}

// --------------------------------------------------------------------- tile --------
// dyn LDS: A[tpw], C[tpw] u32 (C becomes the per-word rank prefix after finalize);
// for tiles of <= 2^kCacheBits positions also loc[kCache] u16 (each record's
// in-tile position), ridx[kRank] u16 (rank -> record) and a redo bitmask.
constexpr unsigned kCacheBits = 16;
// Records cached per tile: a tile of 2^tb positions holds 2^tb / 2 keys on average
// (gamma = 2), so 5/8 of 2^tb covers it with > 30 sigma to spare.
__host__ __device__ constexpr unsigned cache_keys(unsigned tb) { return (5u << tb) / 8; }
// Rank table entries: every cached record up to 2^15-position tiles; for 2^16 (149 KiB of
// LDS in all) 3/8 of 2^tb, against ~0.30 x 2^tb settled keys (a tile that settles more
// writes its outputs in record order instead).
__host__ __device__ constexpr unsigned rank_keys(unsigned tb) { return tb < 16 ? cache_keys(tb) : (3u << tb) / 8; }
constexpr int kTU = 4;                         // loads in flight per lane

// Decoupled look-back run by one wave: lane i inspects tile (t-1-i) of the current
// 64-tile window; the window's aggregates up to the nearest inclusive prefix are summed
// with one ballot, otherwise the window slides back 64 tiles.  Returns the exclusive
// prefix of tile t and publishes its inclusive prefix.
__device__ __forceinline__ unsigned long long look_back_wave(unsigned long long* flags, uint64_t t, uint64_t pop,
                                                             LevelState* st) {
  const unsigned lane = lane_id();
  if (t == 0) {
    if (lane == 0) __hip_atomic_store(&flags[0], kFlagInc | pop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&flags[t], kFlagAgg | pop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t excl = 0;
  int64_t top = (int64_t)t - 1;  // newest tile of the window
  uint64_t spins = 0;
  while (top >= 0) {
    const int64_t q = top - (int64_t)lane;
    unsigned long long v = kFlagInc;  // lanes past tile 0 act as an inclusive zero
    if (q >= 0) v = __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t not_ready = __ballot((v & ~kFlagVal) == 0);
    const uint64_t inc = __ballot((v & ~kFlagVal) == kFlagInc);
    // lanes up to (and including) the first inclusive one, if every one of them is ready
    const uint64_t upto = inc ? (inc & (~inc + 1)) * 2 - 1 : ~0ull;
    if (not_ready & upto) {
      if (++spins > (1ull << 24)) {  // bounded: a lost predecessor must not hang the GPU
        if (lane == 0) atomicOr(&st->status, kStLookback);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t part = ((upto >> lane) & 1ull) && q >= 0 ? (v & kFlagVal) : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d);
    excl += part;
    if (inc) break;
    top -= 64;
  }
  if (lane == 0) __hip_atomic_store(&flags[t], kFlagInc | (excl + pop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// --------------------------------------------------- histogram scan (tile-major) -----
// One pass: segments of kScanSeg entries in ticket order, prefix by wave look-back.
constexpr int kHST = 1024;
constexpr int kHSPer = (int)(kScanSeg / kHST);  // 8 entries per thread

__global__ __launch_bounds__(kHST) void k_hscan(int level, const unsigned* __restrict__ hist,
                                                unsigned* __restrict__ off, unsigned* __restrict__ tile_start,
                                                unsigned long long* sflags, LevelState* st) {
  __shared__ unsigned long long s_seg, s_prefix;
  if (!level_active(level, st)) return;
  const uint64_t T = st->ntiles[level], B = st->nchunks[level], M = T * B;
  const uint64_t nseg = (M + kScanSeg - 1) / kScanSeg;
  const unsigned tid = threadIdx.x;
  if (B == 0) {  // no records (a multi-GPU rank whose range received none): empty tiles
    for (uint64_t t = (uint64_t)blockIdx.x * kHST + tid; t <= T; t += (uint64_t)gridDim.x * kHST) tile_start[t] = 0;
    return;
  }
  for (;;) {
    if (tid == 0) s_seg = atomicAdd(&st->sticket[level], 1ull);
    __syncthreads();
    const uint64_t g = s_seg;
    if (g >= nseg) break;
    const uint64_t e0 = g * kScanSeg + (uint64_t)tid * kHSPer;
    unsigned v[kHSPer];
    uint64_t sum = 0;
#pragma unroll
    for (int q = 0; q < kHSPer; ++q) {
      v[q] = (e0 + q < M) ? hist[e0 + q] : 0u;
      sum += v[q];
    }
    uint64_t tot;
    const uint64_t ex = block_exscan<kHST>(sum, &tot);
    if (tid < 64) {
      const uint64_t pre = look_back_wave(sflags, g, tot, st);
      if (tid == 0) s_prefix = pre;
    }
    __syncthreads();
    uint64_t run = s_prefix + ex;
#pragma unroll
    for (int q = 0; q < kHSPer; ++q) {
      const uint64_t e = e0 + q;
      if (e < M) {
        off[e] = (unsigned)run;
        if (e % B == 0) tile_start[e / B] = (unsigned)run;
      }
      run += v[q];
    }
    if (g == 0 && tid == 0) tile_start[T] = (unsigned)st->n[level];
    __syncthreads();
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_tile(int level, const Rec* __restrict__ bucket,
                                              const unsigned* __restrict__ tile_start,
                                              const unsigned* __restrict__ tcnt, uint64_t bucket_cap,
                                              unsigned long long* flags, uint64_t* __restrict__ bits,
                                              Rec* __restrict__ next, uint64_t* __restrict__ fp_out,
                                              uint64_t* __restrict__ pos_out, LevelState* st, unsigned tb,
                                              unsigned long long* __restrict__ prof) {
  extern __shared__ uint32_t dyn[];
  __shared__ unsigned long long s_t, s_prefix;
  __shared__ unsigned s_wc[NT / 64];
  __shared__ unsigned long long s_wbase[NT / 64];
  if (!level_active(level, st)) return;
  const uint64_t N = st->out_cap;
  const bool out_on = level_out_on(st, level);
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = st->ntiles[level];
  const LevelRange rg = level_range(st, level, words);
  const uint64_t w32_level = 2 * rg.rw;
  const unsigned tpw = 1u << (tb - 5);
  const unsigned per = (tpw + NT - 1) / NT;
  uint32_t* sA = dyn;
  uint32_t* sC = dyn + tpw;
  const bool small = tb <= kCacheBits;
  const unsigned kcap = small ? cache_keys(tb) : 0;
  const unsigned rcap = small ? rank_keys(tb) : 0;
  unsigned short* sloc = reinterpret_cast<unsigned short*>(dyn + 2 * tpw);
  unsigned short* sridx = sloc + kcap;
  uint64_t* srm = reinterpret_cast<uint64_t*>(sridx + rcap);  // kcap / 64 words
  uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + st->woff[level] + rg.plo / 64);
  const uint64_t seed = level_seed(level);
  const uint64_t lvl_base = st->lvl_base[level];
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  bool bad = false;
  for (;;) {
    if (tid == 0) s_t = atomicAdd(&st->ticket[level], 1ull);
    for (unsigned w = tid; w < tpw; w += NT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    __syncthreads();
    const uint64_t t = s_t;
    if (t >= T) break;
    // phase timestamps of this tile (debug builds of the schedule only: prof != null)
    unsigned long long* tp = prof ? prof + ((uint64_t)level * kMaxTiles + (t < kMaxTiles ? t : 0)) * 8 : nullptr;
#define TPROF(i)                                 \
  do {                                           \
    if (tp && tid == 0) tp[i] = wall_clock64(); \
  } while (0)
    TPROF(0);
    // bucket range: from the histogram scan, or (reservation path) the kResShards shard
    // ranges of the tile's fixed slot; record j lives at rb[RB(j)]
    uint64_t lo, nk, shcap = 0;
    unsigned pre[kResShards];
    if (tcnt) {
      const uint64_t cap = bucket_cap / T;
      shcap = cap / kResShards;
      lo = t * cap;
      unsigned acc = 0;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) {
        pre[x] = acc;
        acc += tcnt[t * kResShards + x];
      }
      nk = acc;
    } else {
      lo = tile_start[t];
      nk = tile_start[t + 1] - lo;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) pre[x] = x ? 0xffffffffu : 0u;
    }
    const Rec* rb = bucket + lo;
    auto shard_off = [&](uint64_t j) -> uint64_t {
      uint64_t o = j;
#pragma unroll
      for (int x = 1; x < kResShards; ++x)
        if (j >= pre[x]) o = (uint64_t)x * shcap + (j - pre[x]);
      return o;
    };
#define RB(j) rb[shard_off(j)]
    const uint64_t tbase = rg.plo + (t << tb);
    const bool cached = small && nk <= kcap;
    // ---- mark: A/C in LDS (and each record's in-tile position, when cached)
    for (uint64_t j0 = tid; j0 < nk; j0 += (uint64_t)NT * kTU) {
      uint64_t k[kTU];
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const uint64_t j = j0 + (uint64_t)u * NT;
        k[u] = j < nk ? RB(j).k : 0;
      }
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const uint64_t j = j0 + (uint64_t)u * NT;
        if (j < nk) {
          const unsigned loc = (unsigned)(bb_index(seed, k[u], words, magic) - tbase);
          if (cached) sloc[j] = (unsigned short)loc;
          const uint32_t bit = 1u << (loc & 31);
          const uint32_t old = atomicOr(&sA[loc >> 5], bit);
          if (old & bit) atomicOr(&sC[loc >> 5], bit);
        }
      }
    }
    __syncthreads();
    TPROF(1);
    // ---- finalize: A & ~C -> LDS + global bits; per-word rank prefix into C
    const unsigned w0 = tid * per;
    uint64_t cntw = 0;
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        const uint32_t v = sA[w] & ~sC[w];
        sA[w] = v;
        const uint64_t gw = (uint64_t)t * tpw + w;
        if (gw < w32_level) g32[gw] = v;
        cntw += __popc(v);
      }
    }
    uint64_t pop;
    uint64_t run = block_exscan<NT>(cntw, &pop);
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        sC[w] = (uint32_t)run;
        run += __popc(sA[w]);
      }
    }
    TPROF(2);
    if (wave == 0) {
      const uint64_t excl = look_back_wave(flags, t, pop, st);
      if (lane == 0) {
        if (t == T - 1) st->lvl_base[level + 1] = lvl_base + excl + pop;
        s_prefix = excl;
      }
    }
    __syncthreads();
    TPROF(3);
    const uint64_t base = lvl_base + s_prefix;
    unsigned wc = 0;
    if (cached && pop > rcap) {
      // ---- more settled keys than the rank table holds: outputs in record order from the
      // cached locs (no rehash), redo bitmask by ballot
      if (base + pop > N && out_on) bad = true;
      const bool wr = out_on && base + pop <= N;
      for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
        const uint64_t j = jb + lane;
        bool redo = false;
        if (j < nk) {
          const unsigned loc = sloc[j];
          const uint32_t wv = sA[loc >> 5];
          const uint32_t bit = 1u << (loc & 31);
          if (wv & bit) {
            if (wr) {
              const uint64_t p = base + sC[loc >> 5] + __popc(wv & (bit - 1));
              fp_out[p] = RB(j).f;
              pos_out[p] = RB(j).p;
            }
          } else {
            redo = true;
          }
        }
        const uint64_t m = __ballot(redo);
        if (lane == 0) srm[jb >> 6] = m;
        wc += __popcll(m);
      }
    } else if (cached) {
      // ---- rank pass (LDS only): rank -> record index; redo bitmask by ballot
      for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
        const uint64_t j = jb + lane;
        bool redo = false;
        if (j < nk) {
          const unsigned loc = sloc[j];
          const uint32_t wv = sA[loc >> 5];
          const uint32_t bit = 1u << (loc & 31);
          if (wv & bit) {
            sridx[sC[loc >> 5] + __popc(wv & (bit - 1))] = (unsigned short)j;
          } else {
            redo = true;
          }
        }
        const uint64_t m = __ballot(redo);
        if (lane == 0) srm[jb >> 6] = m;
        wc += __popcll(m);
      }
      __syncthreads();
      TPROF(4);
      // ---- outputs: consecutive ranks -> consecutive fp_out/pos_out slots
      if (base + pop > N && out_on) bad = true;
      for (uint64_t r0 = tid; out_on && r0 < pop && base + pop <= N; r0 += (uint64_t)NT * kTU) {
        uint64_t cf[kTU], cp[kTU];  // only f and p are needed for a settled key
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
          const uint64_t r = r0 + (uint64_t)u * NT;
          cf[u] = cp[u] = 0;
          if (r < pop) {
            const Rec* src = &RB(sridx[r]);
            cf[u] = src->f;
            cp[u] = src->p;
          }
        }
#pragma unroll
        for (int u = 0; u < kTU; ++u) {
          const uint64_t r = r0 + (uint64_t)u * NT;
          if (r < pop) {
            fp_out[base + r] = cf[u];
            pos_out[base + r] = cp[u];
          }
        }
      }
    } else {
      // ---- generic path (tiles too big to cache): rehash, write outputs in place
      for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
        const uint64_t j = jb + lane;
        bool redo = false;
        if (j < nk) {
          const Rec rc = RB(j);
          const unsigned loc = (unsigned)(bb_index(seed, rc.k, words, magic) - tbase);
          const uint32_t wv = sA[loc >> 5];
          const uint32_t bit = 1u << (loc & 31);
          if (wv & bit) {
            const uint64_t p = base + sC[loc >> 5] + __popc(wv & (bit - 1));
            if (p < N) {
              if (out_on) {
                fp_out[p] = rc.f;
                pos_out[p] = rc.p;
              }
            } else if (out_on) {
              bad = true;
            }
          } else {
            redo = true;
          }
        }
        wc += __popcll(__ballot(redo));
      }
    }
    // ---- collided records -> next level (one reservation per tile, per-wave offsets)
    if (tp) __syncthreads();
    TPROF(5);
    if (lane == 0) s_wc[wave] = wc;
    __syncthreads();
    if (tid == 0) {
      unsigned tot = 0;
      for (int w = 0; w < NT / 64; ++w) tot += s_wc[w];
      unsigned long long b0 = tot ? atomicAdd(&st->n[level + 1], (unsigned long long)tot) : 0;
      for (int w = 0; w < NT / 64; ++w) {
        s_wbase[w] = b0;
        b0 += s_wc[w];
      }
    }
    __syncthreads();
    TPROF(6);
    if (wc) {
      uint64_t o = s_wbase[wave];
      const uint64_t lt = lanemask_lt();
      if (cached) {
        // kRU 64-record steps per iteration: all their loads in flight before the stores
        constexpr int kRU = 2;
        for (uint64_t jb0 = wave * 64; jb0 < nk; jb0 += (uint64_t)NT * kRU) {
          uint64_t m[kRU], ck[kRU], cf[kRU], cp[kRU];
#pragma unroll
          for (int u = 0; u < kRU; ++u) {
            const uint64_t jb = jb0 + (uint64_t)u * NT;
            m[u] = jb < nk ? srm[jb >> 6] : 0ull;
            ck[u] = cf[u] = cp[u] = 0;
            if ((m[u] >> lane) & 1ull) {
              const Rec* q = &RB(jb + lane);
              ck[u] = q->k;
              cf[u] = q->f;
              cp[u] = q->p;
            }
          }
#pragma unroll
          for (int u = 0; u < kRU; ++u) {
            if ((m[u] >> lane) & 1ull) next[o + __popcll(m[u] & lt)] = Rec{ck[u], cf[u], cp[u]};
            o += __popcll(m[u]);
          }
        }
      } else {
        for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
          const uint64_t j = jb + lane;
          bool redo = false;
          uint64_t ck = 0;
          if (j < nk) {
            ck = RB(j).k;
            const unsigned loc = (unsigned)(bb_index(seed, ck, words, magic) - tbase);
            redo = !((sA[loc >> 5] >> (loc & 31)) & 1u);
          }
          const uint64_t m = __ballot(redo);
          if (redo) next[o + __popcll(m & lt)] = Rec{ck, RB(j).f, RB(j).p};
          o += __popcll(m);
        }
      }
    }
    __syncthreads();
    TPROF(7);
#undef RB
#undef TPROF
  }
  if (bad) atomicOr(&st->status, kStRank);
}

// ------------------------------------------------------------- split big tile -----
// Tiles of 2^15 / 2^16 positions (C3/C4's first levels, where a tile holds ~16k / ~33k
// records and the rank permutation of its settled keys does not fit a CU's LDS).  One
// persistent 1024-thread workgroup per CU takes tiles by ticket:
//   split     the tile's records are read once (coalesced), A / C marked in LDS, and each
//             record appended to the scratch segment of its 2^14-position sub-tile (an
//             LDS cursor per sub-tile: a wave's lanes with one sub-tile land on one run);
//   finalize  A & ~C -> LDS + global bits, per-word rank prefix; wave look-back for the
//             tile's rank base; the tile's next-list slots (nk - pop) reserved at once;
//   per sub-tile: its records come back into registers (kSplitR per thread, coalesced),
//             settled (f, p) are staged by rank in LDS and written as one run, collided
//             records go to the next list.
// Every record is read twice and written once more than in a register tile, all in
// runs, instead of k_tile's rank-order gathers of (f, p) (16-byte random reads) and its
// second pass for the collided records.
constexpr unsigned kSplitSubBits = kSplitSubBitsDev;
constexpr unsigned kSplitMaxSub = 1u << (kSplitMaxBits - kSplitSubBits);  // 16 sub-tiles of a 2^18 tile
constexpr int kSplitR = 9;                  // sub-tile records per thread in registers (9216 >= 8192 + 11 sigma)
constexpr unsigned kSplitStage = 5120;      // settled records staged per sub-tile (mean ~4970, sigma ~44)
constexpr unsigned kSplitSeg = 10240;       // scratch records per sub-tile (mean 8192, sigma ~90)
constexpr int kSplitT = 1024;
constexpr int kSplitGrid = kSplitGridHost;  // one workgroup per CU (its LDS takes ~144 KiB)
__host__ __device__ constexpr uint64_t split_scratch_recs() { return (uint64_t)kSplitGrid * kSplitMaxSub * kSplitSeg; }

// kP20: the bucket holds R20 records (p = pos_base + i: level 0, or a list level whose list
// is R20); the scratch segments then hold R20 too.  o20: collided records leave as R20.
template <bool kP20, bool kO20>
__global__ __launch_bounds__(kSplitT) void k_tile_split(int level, const Rec* __restrict__ bucket,
                                                        const unsigned* __restrict__ tile_start,
                                                        const unsigned* __restrict__ tcnt, uint64_t bucket_cap,
                                                        unsigned long long* flags, uint64_t* __restrict__ bits,
                                                        Rec* __restrict__ next, uint64_t* __restrict__ fp_out,
                                                        uint64_t* __restrict__ pos_out, LevelState* st, unsigned tb,
                                                        Rec* __restrict__ scratch, unsigned long long* __restrict__ prof,
                                                        uint64_t pos_base, unsigned ts) {
  constexpr bool o20 = kO20;  // (a template argument: as a run-time flag the kernel spilled 7 more VGPRs)
  constexpr int kSU = 3;  // split-phase records per thread per batch (the batch is staged in sfp)
  static_assert((size_t)kSU * kSplitT * sizeof(Rec) <= 2 * kSplitStage * sizeof(uint64_t), "split stage fits sf/sp");
  __shared__ uint32_t sA[1u << (kSplitMaxBits - 5)], sC[1u << (kSplitMaxBits - 5)];
  __shared__ uint64_t sfp[2 * kSplitStage];  // phase 2: settled (f, p) by rank; split phase: the batch by sub-tile
  __shared__ unsigned char stq[kSU * kSplitT];
  __shared__ unsigned s_q[kSplitMaxSub], s_cnt[kSplitMaxSub], s_start[kSplitMaxSub], s_base[kSplitMaxSub];
  __shared__ unsigned s_m;
  uint64_t* const sf = sfp;
  uint64_t* const sp = sfp + kSplitStage;
  Rec* const stg = reinterpret_cast<Rec*>(sfp);
  R20* const stg20 = reinterpret_cast<R20*>(sfp);
  __shared__ unsigned s_wc[kSplitT / 64];
  __shared__ unsigned long long s_t, s_prefix, s_b0, s_run;
  if (!level_active(level, st)) return;
  const uint64_t N = st->out_cap;
  const bool out_on = level_out_on(st, level);
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = st->ntiles[level];
  const LevelRange rg = level_range(st, level, words);
  const uint64_t w32_level = 2 * rg.rw;
  const unsigned nsub = ts ? ts : 1u << (tb - kSplitSubBits);  // 2^14-position sub-tiles per tile
  const unsigned tpw = nsub << (kSplitSubBits - 5);
  uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + st->woff[level] + rg.plo / 64);
  const uint64_t seed = level_seed(level);
  const uint64_t lvl_base = st->lvl_base[level];
  Rec* seg = scratch + (uint64_t)blockIdx.x * kSplitMaxSub * kSplitSeg;  // this workgroup's sub-tile segments
  R20* seg20 = reinterpret_cast<R20*>(scratch) + (uint64_t)blockIdx.x * kSplitMaxSub * kSplitSeg;
  // record j of a bucket / scratch array as (k, f, p)
  auto rec_get = [&](const Rec* a, const R20* a20, uint64_t j, uint64_t& k, uint64_t& f, uint64_t& p) {
    if constexpr (kP20) {
      r20_split(a20[j], pos_base, k, f, p);
    } else {
      const Rec* q = a + j;
      k = q->k;
      f = q->f;
      p = q->p;
    }
  };
  bool bad = false;
  for (;;) {
    // the thread index, opaque per tile: its derived addresses are recomputed each tile
    // instead of hoisted, spilled and reloaded from scratch on each tile's critical path
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const unsigned lane = tid & 63u, wave = tid >> 6;
    const uint64_t lt = lane ? ~0ull >> (64 - lane) : 0ull;
    if (tid == 0) s_t = atomicAdd(&st->ticket[level], 1ull);
    for (unsigned w = tid; w < tpw; w += kSplitT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    if (tid < kSplitMaxSub) {
      s_q[tid] = 0;
      s_cnt[tid] = 0;
    }
    __syncthreads();
    const uint64_t t = s_t;
    if (t >= T) break;
    // debug: phase stamps (split, finalize, look-back, then one per sub-tile)
    unsigned long long* tp = prof ? prof + ((uint64_t)level * kMaxTiles + (t < kMaxTiles ? t : 0)) * 8 : nullptr;
#define SPROF2(i)                                \
  do {                                           \
    if (tp && tid == 0) tp[i] = wall_clock64(); \
  } while (0)
    SPROF2(0);
    // bucket range: histogram scan, or the kResShards shard ranges of the tile's slot
    uint64_t lo, nk, shcap = 0;
    unsigned pre[kResShards];
    if (tcnt) {
      const uint64_t cap = bucket_cap / T;
      shcap = cap / kResShards;
      lo = t * cap;
      unsigned acc = 0;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) {
        pre[x] = acc;
        acc += tcnt[t * kResShards + x];
      }
      nk = acc;
    } else {
      lo = tile_start[t];
      nk = tile_start[t + 1] - lo;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) pre[x] = x ? 0xffffffffu : 0u;
    }
    const Rec* rb = bucket + lo;
    const R20* rb20 = reinterpret_cast<const R20*>(bucket) + lo;
    auto shard_off = [&](uint64_t j) -> uint64_t {
      uint64_t o = j;
#pragma unroll
      for (int x = 1; x < kResShards; ++x)
        if (j >= pre[x]) o = (uint64_t)x * shcap + (j - pre[x]);
      return o;
    };
    const uint64_t tbase = rg.plo + t * ((uint64_t)nsub << kSplitSubBits);
    // ---- split: mark A / C, append each record to its sub-tile's scratch segment.
    // Batches of kSU records per thread, the next batch's loads in flight while one is
    // processed (double-buffered registers; workgroup-uniform trip count and clamped
    // indices keep the loads unconditional).  A batch is counting-sorted by sub-tile in
    // LDS and written to the segments as runs of ~kSU kSplitT / nsub records, so the
    // scratch stores are whole lines (lane-order appends gave runs of ~4 records).
    bool over = false;
    auto load_batch = [&](uint64_t jb, uint64_t (&k)[kSU], uint64_t (&f)[kSU], uint64_t (&p)[kSU]) {
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const uint64_t j = min(jb + (uint64_t)u * kSplitT + tid, nk - 1);
        rec_get(rb, rb20, shard_off(j), k[u], f[u], p[u]);
      }
    };
    auto split_batch = [&](uint64_t jb, const uint64_t (&k)[kSU], const uint64_t (&f)[kSU],
                           const uint64_t (&p)[kSU]) {
      unsigned qs[kSU], rk[kSU];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const uint64_t j = jb + (uint64_t)u * kSplitT + tid;
        qs[u] = kSplitMaxSub;
        if (j < nk) {
          const unsigned loc = (unsigned)(bb_index(seed, k[u], words, magic) - tbase);
          qs[u] = loc >> kSplitSubBits;
          const uint32_t bit = 1u << (loc & 31);
          const uint32_t old = atomicOr(&sA[loc >> 5], bit);
          if (old & bit) atomicOr(&sC[loc >> 5], bit);
        }
      }
      // rank inside the batch's sub-tile run: one LDS count per (wave, sub-tile) present; a
      // lane's peers (lanes of its sub-tile) come from one ballot per bit of the index
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const unsigned q = qs[u];
        uint64_t peers = __ballot(true);
#pragma unroll
        for (unsigned bq = 1; bq <= kSplitMaxSub; bq <<= 1) {
          const uint64_t m1 = __ballot((q & bq) != 0);
          peers &= (q & bq) ? m1 : ~m1;
        }
        const unsigned lead = (unsigned)__builtin_ctzll(peers);
        unsigned b = 0;
        if (lane == lead && q < kSplitMaxSub) b = atomicAdd(&s_cnt[q], (unsigned)__popcll(peers));
        rk[u] = __shfl(b, lead) + (unsigned)__popcll(peers & lt);
      }
      __syncthreads();
      if (wave == 0) {  // run starts in the stage, segment reservations
        const unsigned c = lane < kSplitMaxSub ? s_cnt[lane] : 0u;
        unsigned x = c;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
          const unsigned y = __shfl_up(x, d);
          if (lane >= (unsigned)d) x += y;
        }
        if (lane < kSplitMaxSub) {
          s_start[lane] = x - c;
          s_base[lane] = s_q[lane];
          s_q[lane] += c;
          s_cnt[lane] = 0;
        }
        if (lane == kSplitMaxSub - 1) s_m = x;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        if (qs[u] < kSplitMaxSub) {
          const unsigned slot = s_start[qs[u]] + rk[u];
          if constexpr (kP20) stg20[slot] = r20_make(k[u], f[u], (uint32_t)(p[u] - pos_base));
          else stg[slot] = Rec{k[u], f[u], p[u]};
          stq[slot] = (unsigned char)qs[u];
        }
      }
      __syncthreads();
      const unsigned m = s_m;
      for (unsigned jj = tid; jj < m; jj += kSplitT) {
        const unsigned q = stq[jj];
        const unsigned d = s_base[q] + (jj - s_start[q]);
        if (d >= kSplitSeg) over = true;
        else if constexpr (kP20) seg20[(uint64_t)q * kSplitSeg + d] = stg20[jj];
        else seg[(uint64_t)q * kSplitSeg + d] = stg[jj];
      }
    };
    constexpr uint64_t kBatch = (uint64_t)kSplitT * kSU;
    if (nk) {
      uint64_t kA[kSU], fA[kSU], pA[kSU], kB[kSU], fB[kSU], pB[kSU];
      load_batch(0, kA, fA, pA);
      for (uint64_t jb = 0; jb < nk; jb += 2 * kBatch) {
        load_batch(jb + kBatch, kB, fB, pB);
        split_batch(jb, kA, fA, pA);
        if (jb + kBatch >= nk) break;
        load_batch(jb + 2 * kBatch, kA, fA, pA);
        split_batch(jb + kBatch, kB, fB, pB);
      }
    }
    if (over) atomicOr(&st->status, kStOverflow);
    __syncthreads();
    SPROF2(1);
    // ---- finalize: A & ~C -> LDS + global bits; per-word rank prefix into C
    const unsigned per = (tpw + kSplitT - 1) / kSplitT, w0 = tid * per;
    uint64_t cntw = 0;
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        const uint32_t v = sA[w] & ~sC[w];
        sA[w] = v;
        const uint64_t gw = (uint64_t)t * tpw + w;
        if (gw < w32_level) g32[gw] = v;
        cntw += __popc(v);
      }
    }
    uint64_t pop;
    uint64_t run = block_exscan<kSplitT>(cntw, &pop);
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        sC[w] = (uint32_t)run;
        run += __popc(sA[w]);
      }
    }
    SPROF2(2);
    if (tid == 64) {
      s_b0 = nk > pop ? atomicAdd(&st->n[level + 1], (unsigned long long)(nk - pop)) : 0ull;
      s_run = 0;
    }
    if (wave == 0) {
      const uint64_t excl = look_back_wave(flags, t, pop, st);
      if (lane == 0) {
        if (t == T - 1) st->lvl_base[level + 1] = lvl_base + excl + pop;
        s_prefix = excl;
      }
    }
    __syncthreads();
    SPROF2(3);
    const uint64_t base = lvl_base + s_prefix;
    const bool ok = base + pop <= N;
    if (!ok && out_on) bad = true;
    // ---- per sub-tile: records back into registers, staged outputs, collided -> next
    for (unsigned sq = 0; sq < nsub; ++sq) {
      const unsigned m = min(s_q[sq], kSplitSeg);
      const Rec* sr = seg + (uint64_t)sq * kSplitSeg;
      const R20* sr20 = seg20 + (uint64_t)sq * kSplitSeg;
      const unsigned qw = sq << (kSplitSubBits - 5);              // first word of the sub-tile
      const unsigned qrank = sC[qw];                               // its first rank in the tile
      const unsigned qend = sq + 1 < nsub ? sC[qw + (1u << (kSplitSubBits - 5))] : (unsigned)pop;
      const bool fits = m <= (unsigned)kSplitR * kSplitT;
      unsigned wc = 0;
      if (fits) {
        uint64_t k[kSplitR], f[kSplitR], p[kSplitR];
#pragma unroll
        for (int r = 0; r < kSplitR; ++r) {
          const unsigned j = r * kSplitT + tid;
          k[r] = f[r] = p[r] = 0;
          if (j < m) rec_get(sr, sr20, j, k[r], f[r], p[r]);
        }
        unsigned redo = 0;
#pragma unroll
        for (int r = 0; r < kSplitR; ++r) {
          const unsigned j = r * kSplitT + tid;
          bool rd = false;
          if (j < m) {
            const unsigned loc = (unsigned)(bb_index(seed, k[r], words, magic) - tbase);
            const uint32_t wv = sA[loc >> 5];
            const uint32_t bit = 1u << (loc & 31);
            if (wv & bit) {
              const unsigned local = sC[loc >> 5] + __popc(wv & (bit - 1)) - qrank;
              if (local < kSplitStage) {
                sf[local] = f[r];
                sp[local] = p[r];
              } else if (ok && out_on) {
                fp_out[base + qrank + local] = f[r];
                pos_out[base + qrank + local] = p[r];
              }
            } else {
              rd = true;
              redo |= 1u << r;
            }
          }
          wc += __popcll(__ballot(rd));
        }
        if (lane == 0) s_wc[wave] = wc;
        __syncthreads();
        uint64_t o = s_b0 + s_run;
        for (unsigned w = 0; w < wave; ++w) o += s_wc[w];
#pragma unroll
        for (int r = 0; r < kSplitR; ++r) {
          const bool rd = (redo >> r) & 1u;
          const uint64_t mm = __ballot(rd);
          if (rd) next_put(next, o20, o + __popcll(mm & lt), k[r], f[r], p[r], pos_base);
          o += __popcll(mm);
        }
      } else {
        // more records than registers hold (never at load 1/2): straight from scratch
        for (unsigned jb = wave * 64; jb < m; jb += kSplitT) {
          const unsigned j = jb + lane;
          bool rd = false;
          if (j < m) {
            uint64_t jk, jf, jp;
            rec_get(sr, sr20, j, jk, jf, jp);
            const unsigned loc = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
            const uint32_t wv = sA[loc >> 5];
            const uint32_t bit = 1u << (loc & 31);
            if (wv & bit) {
              if (ok && out_on) {
                const uint64_t q = base + sC[loc >> 5] + __popc(wv & (bit - 1));
                fp_out[q] = jf;
                pos_out[q] = jp;
              }
            } else {
              rd = true;
            }
          }
          wc += __popcll(__ballot(rd));
        }
        if (lane == 0) s_wc[wave] = wc;
        __syncthreads();
        uint64_t o = s_b0 + s_run;
        for (unsigned w = 0; w < wave; ++w) o += s_wc[w];
        for (unsigned jb = wave * 64; jb < m; jb += kSplitT) {
          const unsigned j = jb + lane;
          bool rd = false;
          uint64_t jk = 0, jf = 0, jp = 0;
          if (j < m) {
            rec_get(sr, sr20, j, jk, jf, jp);
            const unsigned loc = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
            rd = !((sA[loc >> 5] >> (loc & 31)) & 1u);
          }
          const uint64_t mm = __ballot(rd);
          if (rd) next_put(next, o20, o + __popcll(mm & lt), jk, jf, jp, pos_base);
          o += __popcll(mm);
        }
      }
      if (ok && out_on && fits) {
        const unsigned ns = min(qend - qrank, kSplitStage);
        for (unsigned i = tid; i < ns; i += kSplitT) {
          st_stream(fp_out + base + qrank + i, sf[i]);
          st_stream(pos_out + base + qrank + i, sp[i]);
        }
      }
      __syncthreads();  // stage / s_wc reused by the next sub-tile
      if (tid == 0) {
        unsigned long long c = 0;
        for (int w = 0; w < kSplitT / 64; ++w) c += s_wc[w];
        s_run += c;
      }
      __syncthreads();
      if (sq < 4) SPROF2(4 + sq);
    }
#undef SPROF2
  }
  if (bad) atomicOr(&st->status, kStRank);
}

// ------------------------------------------------------- register-resident tile -----
// Tiles of at most 2^kRegMaxBits positions hold ~2^(tb-1) records, at most kRegR per
// thread (record r NT + i belongs to thread i, so every load instruction is coalesced):
// each thread loads its records once (all loads in flight together) and keeps
// (k, f, p, in-tile position) in registers through mark -> finalize -> look-back.
// Settled records go to an LDS stage indexed by rank (copied out coalesced), collided
// ones straight from registers to the next list: the bucket is read exactly once.
// A tile with more records than fit takes a streaming fallback (never at load 1/2).
constexpr unsigned kRegMaxBits = 14;
// Settled-record stage: a tile settles ~0.30 x 2^tb keys (gamma 2); 3/8 x 2^tb covers
// it with a wide margin, ranks past it are written directly.
__host__ __device__ constexpr unsigned reg_stage(unsigned tb) { return (3u << tb) / 8; }
size_t tile_reg_lds_bytes(unsigned tb) {
  return (size_t)reg_stage(tb) * 16 + 2ull * (1ull << (tb - 5)) * sizeof(uint32_t);
}

template <int NT, int kRegR, int kWaves, bool kShard>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(kWaves))) void k_tile_reg(int level, const Rec* __restrict__ bucket,
                                                  const unsigned* __restrict__ tile_start,
                                                  const unsigned* __restrict__ tcnt, uint64_t bucket_cap,
                                                  unsigned long long* flags, uint64_t* __restrict__ bits,
                                                  Rec* __restrict__ next, uint64_t* __restrict__ fp_out,
                                                  uint64_t* __restrict__ pos_out, LevelState* st, unsigned tb,
                                                  unsigned long long* __restrict__ prof) {
  extern __shared__ uint64_t dyn64[];
  __shared__ unsigned long long s_t, s_prefix, s_b0;
  __shared__ unsigned s_wc[NT / 64];
  if (!level_active(level, st)) return;
  const uint64_t N = st->out_cap;
  const bool out_on = level_out_on(st, level);
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = st->ntiles[level];
  const LevelRange rg = level_range(st, level, words);
  const uint64_t w32_level = 2 * rg.rw;
  const unsigned tpw = 1u << (tb - 5);
  const unsigned per = (tpw + NT - 1) / NT;
  const unsigned scap = reg_stage(tb);
  uint64_t* sf = dyn64;
  uint64_t* sp = dyn64 + scap;
  uint32_t* sA = reinterpret_cast<uint32_t*>(dyn64 + 2 * scap);
  uint32_t* sC = sA + tpw;
  uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + st->woff[level] + rg.plo / 64);
  const uint64_t seed = level_seed(level);
  const uint64_t lvl_base = st->lvl_base[level];
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t lt = lanemask_lt();
  bool bad = false;
  for (;;) {
    if (tid == 0) s_t = atomicAdd(&st->ticket[level], 1ull);
    for (unsigned w = tid; w < tpw; w += NT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    __syncthreads();
    const uint64_t t = s_t;
    if (t >= T) break;
    unsigned long long* tp = prof ? prof + ((uint64_t)level * kMaxTiles + (t < kMaxTiles ? t : 0)) * 8 : nullptr;
#define TPROF(i)                                 \
  do {                                           \
    if (tp && tid == 0) tp[i] = wall_clock64(); \
  } while (0)
    TPROF(0);
    // bucket range: contiguous from the histogram scan, or kResShards shard ranges
    // (reservation path); record j lives at rb[shard_off(j)]
    uint64_t lo, nk, shcap = 0;  // shcap: records per reservation shard
    unsigned pre[kResShards];  // exclusive prefix of the shard fills (uniform)
    if (kShard) {
      const uint64_t cap = bucket_cap / T;
      shcap = cap / kResShards;
      lo = t * cap;
      unsigned acc = 0;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) {
        pre[x] = acc;
        acc += tcnt[t * kResShards + x];
      }
      nk = acc;
    } else {
      lo = tile_start[t];
      nk = tile_start[t + 1] - lo;
#pragma unroll
      for (int x = 0; x < kResShards; ++x) pre[x] = x ? 0xffffffffu : 0u;
    }
    const Rec* rb = bucket + lo;
    auto shard_off = [&](unsigned j) -> uint64_t {
      uint64_t o = j;
      if (kShard) {
#pragma unroll
        for (int x = 1; x < kResShards; ++x)
          if (j >= pre[x]) o = (uint64_t)x * shcap + (j - pre[x]);
      }
      return o;
    };
    const uint64_t tbase = rg.plo + (t << tb);
    const bool fits = nk <= (uint64_t)kRegR * NT;
    uint64_t k[kRegR], f[kRegR], p[kRegR];
    unsigned loc2[(kRegR + 1) / 2];  // in-tile positions (< 2^14), two per register
#define LOC(r) ((loc2[(r) >> 1] >> (((r) & 1) * 16)) & 0xffffu)
    // ---- load + mark
    if (fits) {
#pragma unroll
      for (int r = 0; r < kRegR; ++r) {
        const unsigned j = r * NT + tid;
        k[r] = f[r] = p[r] = 0;
        if (j < nk) {
          const Rec* q = rb + shard_off(j);
          k[r] = q->k;
          f[r] = q->f;
          p[r] = q->p;
        }
      }

#pragma unroll
      for (int r = 0; r < (kRegR + 1) / 2; ++r) loc2[r] = 0;
#pragma unroll
      for (int r = 0; r < kRegR; ++r) {
        const unsigned j = r * NT + tid;
        if (j < nk) {
          const unsigned x = (unsigned)(bb_index(seed, k[r], words, magic) - tbase);
          loc2[r >> 1] |= x << ((r & 1) * 16);
          const uint32_t bit = 1u << (x & 31);
          const uint32_t old = atomicOr(&sA[x >> 5], bit);
          if (old & bit) atomicOr(&sC[x >> 5], bit);
        }
      }
    } else {
      for (uint64_t j = tid; j < nk; j += NT) {
        const unsigned x = (unsigned)(bb_index(seed, rb[shard_off((unsigned)j)].k, words, magic) - tbase);
        const uint32_t bit = 1u << (x & 31);
        const uint32_t old = atomicOr(&sA[x >> 5], bit);
        if (old & bit) atomicOr(&sC[x >> 5], bit);
      }
    }
    __syncthreads();
    TPROF(1);
    // ---- finalize: A & ~C -> LDS + global bits; per-word rank prefix into C
    const unsigned w0 = tid * per;
    uint64_t cntw = 0;
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        const uint32_t v = sA[w] & ~sC[w];
        sA[w] = v;
        const uint64_t gw = (uint64_t)t * tpw + w;
        if (gw < w32_level) g32[gw] = v;
        cntw += __popc(v);
      }
    }
    uint64_t pop;
    uint64_t run = block_exscan<NT>(cntw, &pop);
    for (unsigned q = 0; q < per; ++q) {
      const unsigned w = w0 + q;
      if (w < tpw) {
        sC[w] = (uint32_t)run;
        run += __popc(sA[w]);
      }
    }
    __syncthreads();  // every word's A & ~C and rank prefix in LDS before any record reads them
    TPROF(2);
    // Every record settles or collides, so the tile's collided count nk - pop is known
    // now: wave 1 reserves the next list's slots while wave 0 runs the look-back, and
    // every wave classifies its records (neither needs the tile's rank prefix).
    if (tid == 64) s_b0 = nk > pop ? atomicAdd(&st->n[level + 1], (unsigned long long)(nk - pop)) : 0ull;
    if (wave == 0) {
      const uint64_t excl = look_back_wave(flags, t, pop, st);
      if (lane == 0) {
        if (t == T - 1) st->lvl_base[level + 1] = lvl_base + excl + pop;
        s_prefix = excl;
      }
    }
    // ---- classify: settled -> stage[rank] (ranks past the stage are written below);
    // collided -> counted per wave
    unsigned wc = 0;
    uint32_t late = 0;  // bit r: settled with a rank past the stage
    if (fits) {
#pragma unroll
      for (int r = 0; r < kRegR; ++r) {
        const unsigned j = r * NT + tid;
        bool redo = false;
        if (j < nk) {
          const unsigned x = LOC(r);
          const uint32_t wv = sA[x >> 5];
          const uint32_t bit = 1u << (x & 31);
          if (wv & bit) {
            const unsigned rank = sC[x >> 5] + __popc(wv & (bit - 1));
            if (rank < scap) {
              sf[rank] = f[r];
              sp[rank] = p[r];
            } else {
              late |= 1u << r;
            }
          } else {
            redo = true;
          }
        }
        wc += __popcll(__ballot(redo));
      }
    } else {
      for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
        const uint64_t j = jb + lane;
        bool redo = false;
        if (j < nk) {
          const unsigned x = (unsigned)(bb_index(seed, rb[shard_off((unsigned)j)].k, words, magic) - tbase);
          redo = !((sA[x >> 5] >> (x & 31)) & 1u);
        }
        wc += __popcll(__ballot(redo));
      }
    }
    TPROF(3);
    if (lane == 0) s_wc[wave] = wc;
    __syncthreads();
    TPROF(4);
    const uint64_t base = lvl_base + s_prefix;
    const bool ok = base + pop <= N;
    if (!ok && out_on) bad = true;
    TPROF(5);
    TPROF(6);
    // ---- collided records -> next level; settled records -> outputs
    uint64_t o = s_b0;
    for (unsigned w = 0; w < wave; ++w) o += s_wc[w];
    if (fits) {
      if (wc) {
#pragma unroll
        for (int r = 0; r < kRegR; ++r) {
          const unsigned j = r * NT + tid;
          const unsigned x = LOC(r);
          const bool redo = j < nk && !((sA[x >> 5] >> (x & 31)) & 1u);
          const uint64_t m = __ballot(redo);
          if (redo) next[o + __popcll(m & lt)] = Rec{k[r], f[r], p[r]};
          o += __popcll(m);
        }
      }
      if (late && ok && out_on) {
#pragma unroll
        for (int r = 0; r < kRegR; ++r) {
          if ((late >> r) & 1u) {
            const unsigned x = LOC(r);
            const uint32_t wv = sA[x >> 5];
            const uint64_t q = base + sC[x >> 5] + __popc(wv & ((1u << (x & 31)) - 1));
            fp_out[q] = f[r];
            pos_out[q] = p[r];
          }
        }
      }
      if (ok && out_on) {
        const uint64_t ns = min<uint64_t>(pop, scap);
        for (uint64_t i = tid; i < ns; i += NT) {
          fp_out[base + i] = sf[i];
          pos_out[base + i] = sp[i];
        }
      }
    } else {
      for (uint64_t jb = wave * 64; jb < nk; jb += NT) {
        const uint64_t j = jb + lane;
        bool redo = false;
        const Rec* q = rb + shard_off((unsigned)j);
        uint64_t ck = 0;
        if (j < nk) {
          ck = q->k;
          const unsigned x = (unsigned)(bb_index(seed, ck, words, magic) - tbase);
          const uint32_t wv = sA[x >> 5];
          const uint32_t bit = 1u << (x & 31);
          if (wv & bit) {
            if (ok && out_on) {
              const uint64_t rank = sC[x >> 5] + __popc(wv & (bit - 1));
              fp_out[base + rank] = q->f;
              pos_out[base + rank] = q->p;
            }
          } else {
            redo = true;
          }
        }
        const uint64_t m = __ballot(redo);
        if (redo) next[o + __popcll(m & lt)] = Rec{ck, q->f, q->p};
        o += __popcll(m);
      }
    }
    __syncthreads();
    TPROF(7);
#undef TPROF
#undef LOC
  }
  if (bad) atomicOr(&st->status, kStRank);
}

// ----------------------------------------------------- P0 level-0 register tiles ------
// Level 0's 2^14-position tiles after k_scatter_p0 (R20 records, identity positions): one
// persistent 1024-thread workgroup per CU takes tiles by ticket, nine records per thread in
// registers, and overlaps each tile's memory traffic with LDS phases of its own:
//   mark      A / C of tile t in LDS (its records arrived during the previous tile's work)
//   finalize  A & ~C -> LDS + global bits, per-word rank prefix; the tile's aggregate is
//             published for the look-back at once, its collided records' slots reserved
//   classify  settled (f, i) -> the LDS stage by in-tile rank; collided -> the next list
//   prefetch  the next tile's records into the registers just freed (its ticket was taken
//             and its slot fills read during the mark)
//   resolve   tile t's look-back, well after its predecessors published: its rank base
//   write     the stage -> fp_out / pos_out[base + rank] in runs, beside the prefetch
// k_tile_reg keeps one tile per CU and leaves HBM idle through every finalize, look-back and
// output phase.  A tile holding more records than the registers (never at load 1/2: 11
// sigma) or more settled keys than the stage (30 sigma) is finished from the bucket with
// its base resolved first.
constexpr int kP0T = 768;
constexpr int kP0R = 12;                                  // 9216 >= 8192 + 11 sigma
constexpr unsigned kP0Stage = 6144;                       // settled ranks staged (mean ~4965)
constexpr unsigned kP0W32 = 1u << (kRegTileMaxBits - 5);  // A / C words of a tile

__device__ __forceinline__ void lb_publish(unsigned long long* flags, uint64_t t, uint64_t pop) {
  __hip_atomic_store(&flags[t], (t == 0 ? kFlagInc : kFlagAgg) | pop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// look_back_wave without its first store (the aggregate went out with lb_publish)
__device__ __forceinline__ uint64_t lb_resolve(unsigned long long* flags, uint64_t t, uint64_t pop, LevelState* st) {
  if (t == 0) return 0;
  const unsigned lane = lane_id();
  uint64_t excl = 0;
  int64_t top = (int64_t)t - 1;
  uint64_t spins = 0;
  while (top >= 0) {
    const int64_t q = top - (int64_t)lane;
    unsigned long long v = kFlagInc;
    if (q >= 0) v = __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t not_ready = __ballot((v & ~kFlagVal) == 0);
    const uint64_t inc = __ballot((v & ~kFlagVal) == kFlagInc);
    const uint64_t upto = inc ? (inc & (~inc + 1)) * 2 - 1 : ~0ull;
    if (not_ready & upto) {
      if (++spins > (1ull << 24)) {
        if (lane == 0) atomicOr(&st->status, kStLookback);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t part = ((upto >> lane) & 1ull) && q >= 0 ? (v & kFlagVal) : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d);
    excl += part;
    if (inc) break;
    top -= 64;
  }
  if (lane == 0) __hip_atomic_store(&flags[t], kFlagInc | (excl + pop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// k20: R20 records (identity positions: p = pos_base + key index, 12-B stage entries);
// otherwise Rec records of any level whose tiles are 2^14 positions (16-B stage entries).
// o20: the collided records leave as R20 (the next level's list is R20, BinBuffers::l20).
// kPN (P0F, level 0 of a single-GPU build): the collided records go straight to level 1's
// super-tile regions (NextPart: per (block, super-tile) regions of R20, the level-0 hash's
// scheme) instead of level 1's list; level 1's size came from k_p0_count before this kernel.
template <bool k20, bool kPN = false>
__global__ __launch_bounds__(kP0T) void k_tile_p0(int level, const void* __restrict__ bucket_v, uint64_t bucket_cap,
                                                  const unsigned* __restrict__ tcnt, unsigned long long* flags,
                                                  uint64_t* __restrict__ bits, Rec* __restrict__ next,
                                                  uint64_t* __restrict__ fp_out, uint64_t* __restrict__ pos_out,
                                                  LevelState* st, uint64_t pos_base, bool o20, NextPart pn = NextPart{}) {
  static_assert(!kPN || k20, "the next level's regions hold R20 records");
  using PT = std::conditional_t<k20, uint32_t, uint64_t>;  // key index, or p
  __shared__ uint64_t sf[kP0Stage];
  __shared__ PT si[kP0Stage];
  __shared__ uint32_t sA[kP0W32], sC[kP0W32];
  __shared__ unsigned s_wc[kP0T / 64];
  __shared__ unsigned s_cnt[2][kResShards];
  __shared__ unsigned long long s_t[2], s_b0, s_excl;
  __shared__ unsigned s_late;
  __shared__ unsigned p_cur[kPN ? kMaxRanks : 1];  // kPN: this block's fill of each level-1 region
  if (!level_active(level, st)) {
    if constexpr (kPN)  // (the next level's scatter reads every block's fills)
      for (unsigned q = threadIdx.x; q < pn.S; q += kP0T) pn.pcnt[(uint64_t)blockIdx.x * pn.S + q] = 0;
    return;
  }
  const uint64_t N = st->out_cap;
  const bool out_on = level_out_on(st, level);
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t T = st->ntiles[level];
  const LevelRange rg = level_range(st, level, words);
  const uint64_t w32_level = 2 * rg.rw;
  uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + st->woff[level] + rg.plo / 64);
  const uint64_t seed = level_seed(level);
  const uint64_t lvl_base = st->lvl_base[level];
  auto pos_of = [&](PT v) -> uint64_t { return k20 ? pos_base + v : (uint64_t)v; };
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t lt = lanemask_lt();
  const uint64_t cap = bucket_cap / T, shcap = cap / kResShards;
  constexpr unsigned kCntT = kP0T - kResShards;  // the last wave's lanes read a tile's slot fills
  // a tile's slot fills as wave-uniform exclusive prefixes (scalar registers)
  struct Fills {
    unsigned pre[kResShards];
    unsigned n;
  };
  auto fills = [&](const unsigned* c) {
    Fills F;
    unsigned a = 0;
#pragma unroll
    for (int x = 0; x < kResShards; ++x) {
      F.pre[x] = a;
      a += __builtin_amdgcn_readfirstlane(c[x]);
    }
    F.n = a;
    return F;
  };
  // tile t's record j as (k, f, key index or p)
  auto rec = [&](uint64_t t, const Fills& F, unsigned j, uint64_t& k_, uint64_t& f_, PT& p_) {
    uint32_t o = j;
#pragma unroll
    for (int x = 1; x < kResShards; ++x)
      if (j >= F.pre[x]) o = (uint32_t)(x * shcap) + (j - F.pre[x]);
    if constexpr (k20) {
      const R20 r = static_cast<const R20*>(bucket_v)[t * cap + o];
      k_ = (uint64_t)r.w[0] | ((uint64_t)r.w[1] << 32);
      f_ = (uint64_t)r.w[2] | ((uint64_t)r.w[3] << 32);
      p_ = r.w[4];
    } else {
      const Rec* q = static_cast<const Rec*>(bucket_v) + t * cap + o;
      k_ = q->k;
      f_ = q->f;
      p_ = q->p;
    }
  };
  // kPN: level 1's geometry (sized by k_p0_level1_setup) and this block's region appends
  uint64_t w1 = 0, m1 = 0, seed1 = 0;
  uint32_t pmul = 0;
  unsigned rcap = 0;
  bool rover = false;
  if constexpr (kPN) {
    if (threadIdx.x < (unsigned)kMaxRanks) p_cur[threadIdx.x] = 0;  // (ordered by the barrier below)
    w1 = st->words[level + 1];
    m1 = st->magic[level + 1];
    seed1 = level_seed(level + 1);
    pmul = 0xffffffffu / pn.tps_sub + 1;  // exact for (position >> 14) < 2^18 (the hash's partition)
    rcap = (unsigned)pn.reg_cap;
  }
  // a collided record into its level-1 super-tile's region of this block
  auto put_region = [&](uint64_t kk, uint64_t ff, uint32_t ii) {
    const uint64_t x1 = w1 >= (1ull << 19) ? bb_index_big(seed1, kk, w1, m1) : bb_index(seed1, kk, w1, m1);
    unsigned sp = __umulhi((uint32_t)(x1 >> kRegTileMaxBits), pmul);
    if (sp >= pn.S) sp = pn.S - 1;  // a level past its bound: the scatter flags the geometry
    const unsigned at = atomicAdd(&p_cur[sp], 1u);
    if (at < rcap)
      pn.sup[((uint64_t)blockIdx.x * pn.S + sp) * rcap + at] = r20_make(kk, ff, ii);
    else
      rover = true;
  };
  uint64_t k[kP0R], f[kP0R];
  PT p[kP0R];
  auto load_regs = [&](uint64_t t, const Fills& F, unsigned me) {
#pragma unroll
    for (int r = 0; r < kP0R; ++r) {
      const unsigned j = (unsigned)r * kP0T + me;
      k[r] = f[r] = 0;
      p[r] = 0;
      if (j < F.n) rec(t, F, j, k[r], f[r], p[r]);
    }
  };
  // Tickets run one tile ahead of the prefetch: tile i + 2's is taken beside tile i's look-back
  // (before any prefetch load of tid 0's wave, so its return does not wait behind them:
  // vmcnt counts in order).  Here: the first two.
  if (tid == 0) {
    s_t[0] = atomicAdd(&st->ticket[level], 1ull);
    s_t[1] = atomicAdd(&st->ticket[level], 1ull);
  }
  for (unsigned w = tid; w < kP0W32; w += kP0T) {
    sA[w] = 0;
    sC[w] = 0;
  }
  __syncthreads();
  uint64_t t = s_t[0];
  if (tid >= kCntT && t < T) s_cnt[0][tid - kCntT] = tcnt[t * kResShards + (tid - kCntT)];
  __syncthreads();
  int cb = 0;
  Fills F = fills(s_cnt[0]);
  if (t < T && F.n <= (unsigned)kP0R * kP0T) load_regs(t, F, tid);
  bool bad = false;
  while (t < T) {
    const int nb = cb ^ 1;
    const unsigned nk = F.n;
    // the thread index, opaque per iteration: per-thread record indices and addresses are
    // recomputed each tile instead of hoisted out of the loop and kept live (they spilled)
    unsigned me = tid;
    asm volatile("" : "+v"(me));
    const bool fits = nk <= (unsigned)kP0R * kP0T;
    const uint64_t tbase = rg.plo + (t << kRegTileMaxBits);
    // ---- mark
    unsigned loc2[(kP0R + 1) / 2];
#define LOC(r) ((loc2[(r) >> 1] >> (((r) & 1) * 16)) & 0xffffu)
#pragma unroll
    for (int r = 0; r < (kP0R + 1) / 2; ++r) loc2[r] = 0;
    if (fits) {
#pragma unroll
      for (int r = 0; r < kP0R; ++r) {
        const unsigned j = (unsigned)r * kP0T + me;
        if (j < nk) {
          const unsigned x = (unsigned)(bb_index(seed, k[r], words, magic) - tbase);
          loc2[r >> 1] |= x << ((r & 1) * 16);
          const uint32_t bit = 1u << (x & 31);
          const uint32_t old = atomicOr(&sA[x >> 5], bit);
          if (old & bit) atomicOr(&sC[x >> 5], bit);
        }
      }
    } else {
      #pragma unroll 1
      for (unsigned j = me; j < nk; j += kP0T) {
        uint64_t jk, jf;
        PT jp;
        rec(t, F, j, jk, jf, jp);
        const unsigned x = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
        const uint32_t bit = 1u << (x & 31);
        const uint32_t old = atomicOr(&sA[x >> 5], bit);
        if (old & bit) atomicOr(&sC[x >> 5], bit);
      }
    }
    __syncthreads();  // A / C complete; the next tile's ticket is in s_t[nb] (taken a tile ago)
    const uint64_t tn = s_t[nb];
    if (tid >= kCntT && tn < T) s_cnt[nb][tid - kCntT] = tcnt[tn * kResShards + (tid - kCntT)];
    // ---- finalize: A & ~C -> LDS + global bits; per-word rank prefix into C
    uint64_t cntw = 0;
    uint32_t v = 0;
    if (tid < kP0W32) {
      v = sA[tid] & ~sC[tid];
      sA[tid] = v;
      const uint64_t gw = t * kP0W32 + tid;
      if (gw < w32_level) g32[gw] = v;
      cntw = __popc(v);
    }
    uint64_t pop;
    const uint64_t run = block_exscan<kP0T>(cntw, &pop);
    if (tid < kP0W32) sC[tid] = (uint32_t)run;
    if (tid == 0) {
      lb_publish(flags, t, pop);
      s_late = 0;
    }
    if (tid == 64) s_b0 = nk > pop ? atomicAdd(&st->n[level + 1], (unsigned long long)(nk - pop)) : 0ull;
    __syncthreads();  // rank prefix, slot reservation
    // ---- classify: settled -> stage[rank]; collided counted per wave
    unsigned wc = 0;
    uint32_t late = 0;
    if (fits) {
#pragma unroll
      for (int r = 0; r < kP0R; ++r) {
        const unsigned j = (unsigned)r * kP0T + me;
        bool redo = false;
        if (j < nk) {
          const unsigned x = LOC(r);
          const uint32_t wv = sA[x >> 5];
          const uint32_t bit = 1u << (x & 31);
          if (wv & bit) {
            const unsigned rank = sC[x >> 5] + __popc(wv & (bit - 1));
            if (rank < kP0Stage) {
              sf[rank] = f[r];
              si[rank] = p[r];
            } else {
              late |= 1u << r;
            }
          } else {
            redo = true;
          }
        }
        wc += __popcll(__ballot(redo));
      }
      if (late) s_late = 1;
    } else {
      #pragma unroll 1
      for (unsigned jb = wave * 64; jb < nk; jb += kP0T) {
        const unsigned j = jb + lane;
        bool redo = false;
        if (j < nk) {
          uint64_t jk, jf;
          PT jp;
          rec(t, F, j, jk, jf, jp);
          const unsigned x = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
          redo = !((sA[x >> 5] >> (x & 31)) & 1u);
        }
        wc += __popcll(__ballot(redo));
      }
    }
    if (lane == 0) s_wc[wave] = wc;
    __syncthreads();
    // ---- collided records -> next level
    {
      uint64_t o = s_b0;
      #pragma unroll 1
      for (unsigned w = 0; w < wave; ++w) o += s_wc[w];
      if (fits) {
#pragma unroll
        for (int r = 0; r < kP0R; ++r) {
          const unsigned j = (unsigned)r * kP0T + me;
          const unsigned x = LOC(r);
          const bool redo = j < nk && !((sA[x >> 5] >> (x & 31)) & 1u);
          if constexpr (kPN) {
            if (redo) put_region(k[r], f[r], (uint32_t)p[r]);
          } else {
            const uint64_t m = __ballot(redo);
            if (redo) next_put(next, o20, o + __popcll(m & lt), k[r], f[r], pos_of(p[r]), pos_base);
            o += __popcll(m);
          }
        }
      } else {
        #pragma unroll 1
        for (unsigned jb = wave * 64; jb < nk; jb += kP0T) {
          const unsigned j = jb + lane;
          bool redo = false;
          uint64_t jk = 0, jf = 0;
          PT jp = 0;
          if (j < nk) {
            rec(t, F, j, jk, jf, jp);
            const unsigned x = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
            redo = !((sA[x >> 5] >> (x & 31)) & 1u);
          }
          if constexpr (kPN) {
            if (redo) put_region(jk, jf, (uint32_t)jp);
          } else {
            const uint64_t m = __ballot(redo);
            if (redo) next_put(next, o20, o + __popcll(m & lt), jk, jf, pos_of(jp), pos_base);
            o += __popcll(m);
          }
        }
      }
    }
    // ---- the rare tiles: base first, then the records the stage does not hold
    const bool early = !fits || s_late;
    if (early) {
      // the tile after tn: its ticket in flight beside the look-back's flag loads
      unsigned long long tk = 0;
      if (tid == 0) tk = atomicAdd(&st->ticket[level], 1ull);
      if (wave == 0) {
        const uint64_t excl = lb_resolve(flags, t, pop, st);
        if (lane == 0) {
          if (t == T - 1) st->lvl_base[level + 1] = lvl_base + excl + pop;
          s_excl = excl;
        }
      }
      if (tid == 0) s_t[cb] = tk;
      __syncthreads();
      const uint64_t base = lvl_base + s_excl;
      const bool wr = out_on && base + pop <= N;
      if (fits) {
#pragma unroll
        for (int r = 0; r < kP0R; ++r)
          if (wr && ((late >> r) & 1u)) {
            const unsigned x = LOC(r);
            const uint32_t wv = sA[x >> 5];
            const uint64_t q = base + sC[x >> 5] + __popc(wv & ((1u << (x & 31)) - 1));
            fp_out[q] = f[r];
            pos_out[q] = pos_of(p[r]);
          }
      } else {
        #pragma unroll 1
        for (unsigned j = me; wr && j < nk; j += kP0T) {
          uint64_t jk, jf;
          PT jp;
          rec(t, F, j, jk, jf, jp);
          const unsigned x = (unsigned)(bb_index(seed, jk, words, magic) - tbase);
          const uint32_t wv = sA[x >> 5];
          const uint32_t bit = 1u << (x & 31);
          if (wv & bit) {
            const uint64_t q = base + sC[x >> 5] + __popc(wv & (bit - 1));
            fp_out[q] = jf;
            pos_out[q] = pos_of(jp);
          }
        }
      }
    }
#undef LOC
    __syncthreads();  // s_cnt[nb] visible; every register record consumed
    // ---- prefetch the next tile's records (wave 0, which polls the look-back, after it:
    // its flag loads would otherwise wait behind its own prefetch, in order, and hold the
    // barrier that every wave then waits at)
    const Fills Fn = fills(s_cnt[nb]);
    const bool pf = tn < T && Fn.n <= (unsigned)kP0R * kP0T;
    if (pf && (wave != 0 || early)) load_regs(tn, Fn, me);
    // ---- resolve the look-back, write the stage
    if (!early) {
      // the tile after tn: its ticket in flight beside the look-back's flag loads
      unsigned long long tk = 0;
      if (tid == 0) tk = atomicAdd(&st->ticket[level], 1ull);
      if (wave == 0) {
        const uint64_t excl = lb_resolve(flags, t, pop, st);
        if (lane == 0) {
          if (t == T - 1) st->lvl_base[level + 1] = lvl_base + excl + pop;
          s_excl = excl;
        }
      }
      if (tid == 0) s_t[cb] = tk;
      __syncthreads();
      if (pf && wave == 0) load_regs(tn, Fn, me);
    }
    const uint64_t base = lvl_base + s_excl;
    if (base + pop > N && out_on) bad = true;
    if (fits && out_on && base + pop <= N) {
      const unsigned ns = (unsigned)min<uint64_t>(pop, kP0Stage);
      #pragma unroll 1
      for (unsigned i = me; i < ns; i += kP0T) {
        st_stream(fp_out + base + i, sf[i]);
        st_stream(pos_out + base + i, pos_of(si[i]));
      }
    }
    for (unsigned w = tid; w < kP0W32; w += kP0T) {
      sA[w] = 0;
      sC[w] = 0;
    }
    __syncthreads();  // stage read, A / C cleared before the next mark
    t = tn;
    F = Fn;
    cb = nb;
  }
  if (bad) atomicOr(&st->status, kStRank);
  if constexpr (kPN) {  // (the tile loop ended on a barrier: every append is in p_cur)
    __syncthreads();
    for (unsigned q = tid; q < pn.S; q += kP0T) pn.pcnt[(uint64_t)blockIdx.x * pn.S + q] = min(p_cur[q], rcap);
    if (rover) atomicOr(&st->status, kStResOverflow);  // a region overflowed: the build reruns
  }
}

// ---- P0F: level 1 fed by level 0's tile kernel -------------------------------------------
// Level 1's geometry needs its exact size, which the single-GPU build otherwise learns only
// once level 0's tile kernel has finished; k_p0_count gets it first.  Per 2^14-position tile
// of level 0 it marks A / C in LDS from each slot's in-tile position (a u16 the super-tile
// scatter wrote beside the record: 2 B per key read instead of 20) and counts the settled keys,
// popcount(A & ~C), into st->settled0; k_p0_level1_setup then sizes level 1 from N minus
// them, and k_tile_p0<true, true> writes level 1's records straight into its super-tile regions
// (the level-0 hash's scheme).  Level 1 then reaches 2^14-position register tiles through the
// super-tile scatter, instead of the reservation scatter and the split kernel's sub-tile
// scratch (40 B per record written and read back).
constexpr int kCntT = 512;
constexpr int kCntU = 4;  // slot positions in flight per thread
__global__ __launch_bounds__(kCntT) void k_p0_count(const uint16_t* __restrict__ xs, const unsigned* __restrict__ tcnt,
                                                   uint64_t bucket_cap, LevelState* st) {
  __shared__ uint32_t sA[kP0W32], sC[kP0W32];
  __shared__ unsigned s_fo[kResShards + 1];
  __shared__ unsigned long long s_w[kCntT / 64];
  if (st->status & kStStop) return;
  const uint64_t T = st->ntiles[0];
  if (T == 0) return;
  const uint64_t cap = bucket_cap / T, scap = cap / kResShards;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  unsigned long long settled = 0;
  for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
    for (unsigned w = tid; w < kP0W32; w += kCntT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    if (wave == 0) {  // the tile's slot fills: exclusive prefix over lanes 0-7
      const unsigned c = lane < (unsigned)kResShards ? tcnt[t * kResShards + lane] : 0u;
      unsigned x = c;
#pragma unroll
      for (int d = 1; d < kResShards; d <<= 1) {
        const unsigned y = __shfl_up(x, d);
        if (lane >= (unsigned)d) x += y;
      }
      if (lane < (unsigned)kResShards) s_fo[lane] = x - c;
      if (lane == (unsigned)kResShards - 1) s_fo[kResShards] = x;
    }
    __syncthreads();
    unsigned fo[kResShards + 1];
#pragma unroll
    for (int q = 0; q <= kResShards; ++q) fo[q] = s_fo[q];
    const unsigned nrec = fo[kResShards];
    for (unsigned i0 = 0; i0 < nrec; i0 += kCntT * kCntU) {
      unsigned x[kCntU];
#pragma unroll
      for (int u = 0; u < kCntU; ++u) {  // straight-line, clamped: all loads in flight together
        const unsigned i = min(i0 + u * kCntT + tid, nrec - 1);
        unsigned sh = 0;
#pragma unroll
        for (int q = 1; q < kResShards; ++q) sh += i >= fo[q] ? 1u : 0u;
        unsigned b = fo[0];
#pragma unroll
        for (int q = 1; q < kResShards; ++q)
          if (sh == (unsigned)q) b = fo[q];
        x[u] = xs[t * cap + (uint64_t)sh * scap + (i - b)];
      }
#pragma unroll
      for (int u = 0; u < kCntU; ++u) {
        if (i0 + u * kCntT + tid >= nrec) continue;
        const uint32_t bit = 1u << (x[u] & 31);
        const uint32_t old = atomicOr(&sA[x[u] >> 5], bit);
        if (old & bit) atomicOr(&sC[x[u] >> 5], bit);
      }
    }
    __syncthreads();
    for (unsigned w = tid; w < kP0W32; w += kCntT) settled += (unsigned)__popc(sA[w] & ~sC[w]);
    __syncthreads();
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) settled += __shfl_xor(settled, d);
  if (lane == 0) s_w[wave] = settled;
  __syncthreads();
  if (tid == 0) {
    unsigned long long sum = 0;
#pragma unroll
    for (int w = 0; w < kCntT / 64; ++w) sum += s_w[w];
    if (sum) atomicAdd(&st->settled0, sum);
  }
}

// Level 1's words, Barrett reciprocal and word offsets from its exact size (n[0] minus level 0's
// settled keys), as k_scatter_res's level setup would write them; n[1] itself is still counted
// by level 0's tile kernel (the same value).
__global__ void k_p0_level1_setup(LevelState* st, uint64_t cap_words) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || (st->status & kStStop)) return;
  const uint64_t n1 = st->n[0] - st->settled0;
  const uint64_t w = level_words(n1);
  st->words[1] = w;
  st->magic[1] = level_magic(w);
  st->woff[1] = st->woff[0] + st->words[0];
  st->woff[2] = st->woff[1] + w;
  st->nlevels = 1;
  if (st->woff[2] > cap_words) atomicOr(&st->status, kStOverflow);
  if (n1 <= kGate) (atomicOr(&st->status, kStGeometry), atomicCAS(&st->pad0_, 0u, 6u));  // (never at P0 sizes)
}

// ------------------------------------------------------------ mid-size levels --------
// Levels between the single-workgroup tail (<= kTailKeys keys) and the binned pipeline's
// scatter + tile kernels, where the latter pay mostly fixed latency (two launches, a
// reservation round trip, a look-back chain: ~20-40 us per level of 10^4-10^5 keys).
// kMidG workgroups of kMidT threads, all resident, run every such level in one launch.
// Workgroup g owns the level words [g sl, (g+1) sl) (sl = ceil(words32 / kMidG)), and the
// records a workgroup holds stay in its registers (kMidR per thread) from level to level:
//   route     each record goes to the owner of its position: counted per owner in LDS and
//             written to the (owner, sender) segment of an exchange area (kMidSeg records);
//   own       the owner gathers its segments into its registers, marks A / C for its
//             words in LDS, writes the level's bits A & ~C and its words' rank prefix,
//             publishes its settled and collided counts in one tagged word;
//   settle    once every owner's word is in (an all-gather polled by one wave, no fence):
//             rank = level base + settled counts of the owners before it + in-slice rank:
//             settled (f, p) are staged by rank in LDS and written as one contiguous run;
//             collided records stay in registers for the next level and are also written to
//             the next list at the collided count of the owners before it (no atomic), where
//             the tail finds them;
// with a grid barrier after the route phase only (round 5: the second barrier and the
// next-list reservation atomic became the all-gather, C2 levels 0.296 -> 0.287 ms,
// profiles/r5_levels/mid_gather_ab_r5ah.txt; the next level's key count is derived from the
// counts).  Every decision derives from the same
// level state, so all workgroups take the same branches; an overflow (a segment or an owner
// past its capacity, predicted not to happen) is flagged and the build reruns on the
// conservative path.  Level bookkeeping mirrors k_scatter_res + k_tile_reg (words, woff,
// nlevels, lvl_base, n[L+1]); a level of <= kTailKeys keys is left to the tail.
// Grid barrier (MI355X_MICROARCH.md, inter-workgroup visibility): every wave waits for its
// own stores and atomics, the workgroup meets, then ONE release (one L2 write-back per
// workgroup, not per wave) and the arrival; after the count is reached, one agent-scope
// acquire for the CU before anyone loads.
__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned target, LevelState* st, int* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++spins > (1u << 22)) {  // bounded: a missing workgroup must not hang the GPU.  Workgroups
        // that never become resident (another build's persistent kernel holds the CUs) are the
        // likely cause: the attempt reruns on the conservative path, which has no grid barrier.
        atomicOr(&st->status, kStTailOverflow);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1 invalidated for the loads after
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

template <int kG>
__global__ __launch_bounds__(kMidT) void k_mid_levels(int L0, int L1, Rec* list0, Rec* list1, uint64_t* bits,
                                                      uint64_t cap_words, uint64_t* __restrict__ fp_out,
                                                      uint64_t* __restrict__ pos_out, LevelState* st,
                                                      uint32_t* mid, Rec* __restrict__ xb,
                                                      unsigned long long* __restrict__ prof, unsigned seq) {
  // debug (prof != null): phase stamps of the first and last workgroup, 8 per level
  unsigned long long* tp =
      prof && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1)
          ? prof + (uint64_t)(kMaxLevels - 4) * kMaxTiles * 8 + (blockIdx.x ? 512 : 0)
          : nullptr;
#define MPROF(li, i)                                                              \
  do {                                                                            \
    if (tp && threadIdx.x == 0 && (li) < 64) tp[(li) * 8 + (i)] = wall_clock64(); \
  } while (0)
  using Cfg = MidCfg<kG>;
  constexpr unsigned kSeg = Cfg::kSeg;
  constexpr int kE = kG / 64;  // owners (senders) per lane in wave 0's scans
  static_assert(kG % 64 == 0 && kG <= 256, "mid workgroups");
  constexpr unsigned kSlW = (unsigned)((Cfg::kW32 + kG - 1) / kG);  // owner slice, u32 words
  static_assert(kSlW <= (unsigned)kMidT, "one owner word per thread");
  __shared__ uint32_t sA[kSlW], sC[kSlW], sP[kSlW];
  __shared__ uint64_t sf[kMidStage], sp[kMidStage];
  __shared__ unsigned s_cnt[kG], s_spre[kG + 1];
  __shared__ unsigned long long s_pre[kG + 1];
  __shared__ unsigned s_cpre[kG + 1];  // collided records of the owners before
  __shared__ unsigned s_wc[kMidT / 64];
  __shared__ unsigned long long s_wbase[kMidT / 64];
  __shared__ int s_go, s_ok;

  const unsigned g = blockIdx.x, G = gridDim.x;
  // zeroed by k_init_state: one launch of each form per build attempt
  unsigned* bar = kG == kMidG ? &st->mid_bar : &st->mid_bar2;
  unsigned* xc = mid + Cfg::kXc;  // [owner][sender] segment counts
  unsigned long long* tot = reinterpret_cast<unsigned long long*>(mid + Cfg::kTot);
  const uint64_t N = st->out_cap;
  unsigned target = 0;
  bool bad = false;
  uint64_t k[kMidR], f[kMidR], pp[kMidR];
  unsigned valid = 0;  // bit r: k/f/pp[r] hold a record of the current level
  // key counts of the current and previous level after L0: every workgroup derives them
  // from the settled totals (n[L+1] = n[L] - settled), so no barrier waits for the
  // next-list atomics and no decision reads state another workgroup may still be writing
  uint64_t n_loc = 0, n_prev = 0;
  for (int L = L0; L <= L1; ++L) {
    // The thread index, opaque per level: addresses derived from it are recomputed each
    // level instead of hoisted out of the loop, where they spilled to scratch and every
    // level waited for their reloads on its critical path
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const unsigned lane = tid & 63u, wave = tid >> 6;
    const uint64_t lt = lane ? ~0ull >> (64 - lane) : 0ull;
    // ---- level setup: the same values in every workgroup, workgroup 0 publishes
    if (tid == 0) {
      const int p = L - 1;
      int go = L > L0 || (!(st->status & kStStop) && !(p > 0 && !st->preset[p] && st->n[p] <= kGate));
      if (go) {
        const uint64_t n = L > L0 ? n_loc : st->n[L];
        const uint64_t words = n ? level_words(n) : 0;
        const uint64_t woff = st->woff[p] + st->words[p];
        if (g == 0) {
          st->words[L] = words;
          st->magic[L] = level_magic(words);
          st->woff[L] = woff;
          st->woff[L + 1] = woff + words;
          st->nlevels = L;
          if (woff + words > cap_words) atomicOr(&st->status, kStOverflow);
        }
        if (n <= kGate || woff + words > cap_words) {
          go = 0;  // the tail takes this level (or the workspace is too small: rerun)
        } else if (n > Cfg::kMax) {
          if (g == 0) atomicOr(&st->status, kStTailOverflow);  // bigger than predicted: rerun
          go = 0;
        } else if (!st->preset[L] && !st->preset[p] && n == (L > L0 ? n_prev : st->n[p])) {
          if (g == 0) {  // no key placed at the previous level: duplicates (no_progress)
            st->stop_level = L;
            atomicOr(&st->status, kStTooManyLevels);
          }
          go = 0;
        }
      }
      s_go = go;
    }
    __syncthreads();
    if (!s_go) break;
    const uint64_t n = L > L0 ? n_loc : st->n[L];
    const uint64_t words = level_words(n), magic = level_magic(words);
    const uint64_t woff = st->woff[L - 1] + st->words[L - 1];
    const uint64_t seed = level_seed(L);
    const unsigned W32 = (unsigned)(2 * words);
    const unsigned sl = (W32 + G - 1) / G, w0 = min(W32, g * sl), w1 = min(W32, w0 + sl);
    const int li = L - L0;
    MPROF(li, 0);
    if (L == L0) {  // the first level's records: this workgroup's share of the input list
      const Rec* in = (L & 1) ? list0 : list1;  // list[(L - 1) & 1]
      const uint64_t per = (n + G - 1) / G, r0 = (uint64_t)g * per, r1 = min(n, r0 + per);
      valid = 0;
#pragma unroll
      for (int r = 0; r < kMidR; ++r) {
        const uint64_t j = r0 + (uint64_t)r * kMidT + tid;
        if (j < r1) {
          const Rec* q = in + j;
          k[r] = q->k;
          f[r] = q->f;
          pp[r] = q->p;
          valid |= 1u << r;
        }
      }
    }
    // ---- route: records -> (owner, sender) segments
    if (tid < (unsigned)kG) s_cnt[tid] = 0;
    __syncthreads();
    {
      bool over = false;
#pragma unroll
      for (int r = 0; r < kMidR; ++r) {
        if ((valid >> r) & 1u) {
          const unsigned x = (unsigned)bb_index(seed, k[r], words, magic);
          const unsigned o = (x >> 5) / sl;
          const unsigned slot = atomicAdd(&s_cnt[o], 1u);
          if (slot < kSeg)
            xb[((uint64_t)o * kG + g) * kSeg + slot] = Rec{k[r], f[r], pp[r]};
          else
            over = true;
        }
      }
      if (over) atomicOr(&st->status, kStTailOverflow);
    }
    __syncthreads();
    if (tid < G) xc[tid * kG + g] = min(s_cnt[tid], kSeg);
    MPROF(li, 1);
    target += G;
    if (!grid_sync(bar, target, st, &s_ok)) break;
    MPROF(li, 2);
    // ---- own: gather this slice's records, mark A / C, bits, word rank prefix, total
    if (wave == 0) {  // segment prefix over the senders (kE consecutive senders per lane)
      unsigned v[kE], sum = 0;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const unsigned q = lane * kE + e;
        v[e] = q < G ? xc[g * kG + q] : 0u;
        sum += v[e];
      }
      unsigned xs = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned y = __shfl_up(xs, d);
        if (lane >= (unsigned)d) xs += y;
      }
      unsigned ex = xs - sum;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const unsigned q = lane * kE + e;
        if (q <= G) s_spre[q] = ex;  // (q == G: the total, when G ends inside this lane's run)
        ex += v[e];
      }
      if (lane == 63) s_spre[G] = xs;
    }
    for (unsigned w = tid; w < sl; w += kMidT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    __syncthreads();
    const unsigned m = s_spre[G];
    if (m > (unsigned)kMidR * kMidT && tid == 0) atomicOr(&st->status, kStTailOverflow);
    unsigned lx[kMidR];
    valid = 0;
#pragma unroll
    for (int r = 0; r < kMidR; ++r) {
      const unsigned j = r * kMidT + tid;
      lx[r] = 0;
      if (j < m) {
        unsigned lo = 0, hi = G;  // last sender b with s_spre[b] <= j
        while (hi - lo > 1) {
          const unsigned mid2 = (lo + hi) >> 1;
          if (s_spre[mid2] <= j) lo = mid2;
          else hi = mid2;
        }
        const Rec* q = xb + ((uint64_t)g * kG + lo) * kSeg + (j - s_spre[lo]);
        k[r] = q->k;
        f[r] = q->f;
        pp[r] = q->p;
        valid |= 1u << r;
      }
    }
#pragma unroll
    for (int r = 0; r < kMidR; ++r) {
      if ((valid >> r) & 1u) {
        lx[r] = (unsigned)bb_index(seed, k[r], words, magic) - 32u * w0;
        const uint32_t bit = 1u << (lx[r] & 31);
        const uint32_t old = atomicOr(&sA[lx[r] >> 5], bit);
        if (old & bit) atomicOr(&sC[lx[r] >> 5], bit);
      }
    }
    __syncthreads();
    {
      uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + woff);
      const unsigned w = tid;  // sl <= kSlW <= kMidT words
      uint32_t v = 0;
      if (w0 + w < w1) {
        v = sA[w] & ~sC[w];
        sA[w] = v;
        g32[w0 + w] = v;
      }
      uint64_t total;
      const uint64_t ex = block_exscan<kMidT>((uint64_t)__popc(v), &total);
      if (w0 + w < w1) sP[w] = (uint32_t)ex;
      // this owner's settled and collided counts (< 2^14 each), tagged with the launch and
      // level, in ONE word: the all-gather below needs no fence, only the word itself
      if (tid == 0) {
        const unsigned held = min(m, (unsigned)kMidR * kMidT);
        const unsigned long long wv = ((unsigned long long)((seq << 6) | (unsigned)li) << 32) |
                                      ((unsigned long long)(held - (unsigned)total) << 16) | total;
        __hip_atomic_store(&tot[g], wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    MPROF(li, 3);
    // All-gather of the owners' counts instead of a second grid barrier: wave 0 polls the G
    // tagged words (one per lane) until every one carries this level's tag.  No data crosses
    // workgroups in the settle except these counts (ranks, outputs and the next list's runs
    // are placed from them), and a sender overwrites an owner's exchange segments only after
    // the next level's first barrier, which follows every owner's reads here.
    if (wave == 0) {  // (kE consecutive owners per lane)
      const unsigned tagv = (seq << 6) | (unsigned)li;
      unsigned long long v[kE];
      unsigned spins = 0;
      int okv = 1;
      for (;;) {
        bool mine = true;
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const unsigned q = lane * kE + e;
          v[e] = q < G ? __hip_atomic_load(&tot[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : ((unsigned long long)tagv << 32);
          mine = mine && (unsigned)(v[e] >> 32) == tagv;
        }
        if (__all(mine)) break;
        if (++spins > (1u << 22)) {  // bounded, as grid_sync
          if (lane == 0) atomicOr(&st->status, kStTailOverflow);
          okv = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      unsigned long long sv[kE], ssum = 0;
      unsigned cv[kE], csum = 0;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const bool in = lane * kE + e < G;
        sv[e] = in ? (v[e] & 0xffffu) : 0ull;
        cv[e] = in ? (unsigned)((v[e] >> 16) & 0xffffu) : 0u;
        ssum += sv[e];
        csum += cv[e];
      }
      unsigned long long xs = ssum;
      unsigned xc2 = csum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(xs, d);
        const unsigned y2 = __shfl_up(xc2, d);
        if (lane >= (unsigned)d) {
          xs += y;
          xc2 += y2;
        }
      }
      unsigned long long exs = xs - ssum;
      unsigned exc = xc2 - csum;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const unsigned q = lane * kE + e;
        if (q <= G) {
          s_pre[q] = exs;
          s_cpre[q] = exc;
        }
        exs += sv[e];
        exc += cv[e];
      }
      if (lane == 63) {
        s_pre[G] = xs;
        s_cpre[G] = xc2;
      }
      if (lane == 0) s_ok = okv;
    }
    __syncthreads();
    if (!s_ok) break;
    MPROF(li, 4);
    const uint64_t lvl_base = st->lvl_base[L];
    if (g == 0 && tid == 0) st->lvl_base[L + 1] = lvl_base + s_pre[G];
    const bool out_on = level_out_on(st, L);
    const uint64_t base = lvl_base + s_pre[g];
    const uint64_t mine = s_pre[g + 1] - s_pre[g];
    const bool ok = lvl_base + s_pre[G] <= N;
    if (!ok && out_on) bad = true;
    unsigned wc = 0, keep = 0;
#pragma unroll
    for (int r = 0; r < kMidR; ++r) {
      bool redo = false;
      if ((valid >> r) & 1u) {
        const uint32_t wv = sA[lx[r] >> 5];
        const uint32_t bit = 1u << (lx[r] & 31);
        if (wv & bit) {
          const unsigned rank = sP[lx[r] >> 5] + __popc(wv & (bit - 1));
          if (rank < kMidStage) {
            sf[rank] = f[r];
            sp[rank] = pp[r];
          } else if (ok && out_on) {
            fp_out[base + rank] = f[r];
            pos_out[base + rank] = pp[r];
          }
        } else {
          redo = true;
          keep |= 1u << r;
        }
      }
      wc += __popcll(__ballot(redo));
    }
    if (lane == 0) s_wc[wave] = wc;
    __syncthreads();
    if (tid == 0) {
      // the next list's runs in owner order: no returning atomic, and the same order every run
      unsigned long long b0 = s_cpre[g];
      if (g == 0) st->n[L + 1] = s_cpre[G];
      for (int w = 0; w < kMidT / 64; ++w) {
        s_wbase[w] = b0;
        b0 += s_wc[w];
      }
    }
    __syncthreads();
    if (ok && out_on) {
      const uint64_t ns = min<uint64_t>(mine, kMidStage);
      for (uint64_t i = tid; i < ns; i += kMidT) {
        fp_out[base + i] = sf[i];
        pos_out[base + i] = sp[i];
      }
    }
    if (wc) {
      Rec* next = (L & 1) ? list1 : list0;  // list[L & 1]
      uint64_t o = s_wbase[wave];
#pragma unroll
      for (int r = 0; r < kMidR; ++r) {
        const bool redo = (keep >> r) & 1u;
        const uint64_t mm = __ballot(redo);
        if (redo) next[o + __popcll(mm & lt)] = Rec{k[r], f[r], pp[r]};
        o += __popcll(mm);
      }
    }
    valid = keep;
    // No barrier here: the next level's route writes only exchange segments and counts its
    // owners read after that level's first grid barrier (which this workgroup's settle
    // precedes), n[L + 1] is derived, and lvl_base[L + 1] / the tot[] totals are read only
    // after later barriers.  An overflow flagged above leaves garbage the host discards
    // (the conservative rerun); every access stays within its capacity meanwhile.
    n_prev = n;
    n_loc = n - s_pre[G];
    MPROF(li, 5);
  }
  if (bad) atomicOr(&st->status, kStRank);
#undef MPROF
}

// --------------------------------------------------------------------- tail --------
constexpr unsigned kWaveKeys = 64;  // tail levels this small run in one wave
// The wave tail holds key i in lane i, compacts with 64-bit ballots and reads the level's
// A/C words (<= level_words(64) * 2 u32) with lane shuffles: all of it is wave64-only.
static_assert(kWaveKeys == 64, "the wave tail assumes one key per lane of a 64-lane wave");
static_assert(2 * ((kGammaNum * kWaveKeys + 63) / 64) <= kWaveKeys, "wave tail: A/C words must fit one per lane");

// Orders one wave's LDS accesses across lanes (a wave's LDS operations execute in order;
// this keeps the compiler from moving them across the point).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every remaining level in one workgroup, with the live records in LDS: the first tail
// level's key hashes (and their input indices) are loaded once; each level marks A/C
// in LDS, finalizes and ranks, records each settled key's input index at its rank in an
// LDS table shared by all tail levels, and compacts the collided records in place for the
// next level; the outputs of every tail level go out in one rank-order pass at the end
// (f, p fetched from the first tail level's input list through that table).  No level after the
// first reads or writes a record list.
__global__ __launch_bounds__(kTailT) void k_bin_tail(int first_level, int big_launched, Rec* list0, Rec* list1, uint64_t* bits,
                                                     uint64_t cap_words, uint64_t* __restrict__ fp_out,
                                                     uint64_t* __restrict__ pos_out, LevelState* st,
                                                     unsigned long long* __restrict__ prof) {
  __shared__ uint64_t ck[kTailKeys];           // live keys, as mix64(key hash)
  __shared__ unsigned short cj[kTailKeys];     // ... and their index in the input list
  __shared__ unsigned short srank[kTailKeys];  // tail rank (every tail level) -> input index
  __shared__ uint32_t sA[kTailW32];
  __shared__ uint32_t sC[kTailW32];
  __shared__ uint32_t spre[kTailW32];
  __shared__ unsigned s_wc[kTailT / 64];
  __shared__ unsigned long long s_n;
  __shared__ unsigned long long s_wbase0, s_wout;  // wave-level tail: base0 / out_end for the block
  __shared__ int s_level;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  if (tid == 0) {
    level_setup(big_launched + 1, st);  // size the level after the last big one
    int L = first_level > 1 ? first_level : 1;
    while (L <= big_launched && st->n[L] > kGate) ++L;
    s_level = L;
    s_n = st->n[L];
    if (st->status & kStStop) s_n = 0;
    if (s_n > kTailKeys) {
      atomicOr(&st->status, kStTailOverflow);
      s_n = 0;
    }
    st->tail_first = L;
  }
  __syncthreads();
  const uint64_t N = st->out_cap;
  bool bad = false;
  const Rec* in = (s_level & 1) ? list0 : list1;  // written by the level before
  {
    constexpr int kR = (int)((kTailKeys + kTailT - 1) / kTailT);
    const unsigned n0 = (unsigned)s_n;
    uint64_t k[kR];
#pragma unroll
    for (int u = 0; u < kR; ++u) {  // every load in flight before the first LDS store
      const unsigned i = tid + u * kTailT;
      k[u] = i < n0 ? in[i].k : 0;
    }
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const unsigned i = tid + u * kTailT;
      if (i < n0) {
        ck[i] = mix64(k[u]);  // the level-independent half of key_mix, once
        cj[i] = (unsigned short)i;
      }
    }
  }
  __syncthreads();
  // Outputs of every tail level go out in one pass after the last level: the tail's ranks
  // are contiguous from the first tail level's base, so one rank -> input-index table
  // covers them all and the (f, p) gathers from `in` pay one memory round trip, not one
  // per level.  Levels with outputs on are a prefix of the tail (out_skip_from).
  uint64_t base0 = ~0ull, out_end = 0;
  bool wave_levels = false;
  for (;;) {
    const int L = s_level;
    const unsigned n = (unsigned)s_n;
    // debug: level start times in the last prof row
    if (prof && tid == 0 && L < kMaxLevels) prof[(uint64_t)(kMaxLevels - 1) * kMaxTiles * 8 + L] = wall_clock64();
    if (n == 0) break;
    if (L >= kMaxLevels) {
      // level budget exhausted: leave the unplaced keys in level L's list, where the host
      // looks for duplicates (as mix64(key hash): a bijection, so duplicates are preserved)
      if (tid == 0) {
        st->stop_level = L;
        atomicOr(&st->status, kStTooManyLevels);
      }
      Rec* out = (L & 1) ? list0 : list1;
      for (unsigned i = tid; i < n; i += kTailT) out[i] = Rec{ck[i], 0, 0};
      break;
    }
    if (n <= kWaveKeys) {  // the rest runs in wave 0 alone, below
      wave_levels = true;
      break;
    }
    const uint64_t words = st->words[L], magic = st->magic[L], woff = st->woff[L];
    const uint64_t base = st->lvl_base[L];
    if (base0 == ~0ull) base0 = base;
    const unsigned rb0 = (unsigned)(base - base0);  // this level's first slot in srank
    const unsigned w32 = (unsigned)(2 * words);
    for (unsigned w = tid; w < w32; w += kTailT) {
      sA[w] = 0;
      sC[w] = 0;
    }
    __syncthreads();
    const uint64_t seed = level_seed(L);
    for (unsigned i = tid; i < n; i += kTailT) {
      const uint32_t x = (uint32_t)bb_index_mk(seed, ck[i], words, magic);
      const uint32_t bit = 1u << (x & 31);
      const uint32_t old = atomicOr(&sA[x >> 5], bit);
      if (old & bit) atomicOr(&sC[x >> 5], bit);
    }
    __syncthreads();
    constexpr unsigned kPer = (kTailW32 + kTailT - 1) / kTailT;
    uint64_t cnt = 0;
    uint32_t* g32 = reinterpret_cast<uint32_t*>(bits + woff);
#pragma unroll
    for (unsigned q = 0; q < kPer; ++q) {
      const unsigned w = tid * kPer + q;
      if (w < w32) {
        const uint32_t v = sA[w] & ~sC[w];
        sA[w] = v;
        g32[w] = v;
        cnt += __popc(v);
      }
    }
    uint64_t tot;
    uint64_t run = block_exscan<kTailT>(cnt, &tot);
#pragma unroll
    for (unsigned q = 0; q < kPer; ++q) {
      const unsigned w = tid * kPer + q;
      if (w < w32) {
        spre[w] = (uint32_t)run;
        run += __popc(sA[w]);
      }
    }
    __syncthreads();
    // settled -> rank table; collided -> compacted in place, one block-wide segment of
    // kTailT records at a time (a record only moves down, never past its segment's end)
    unsigned n1 = 0;
    for (unsigned i0 = 0; i0 < n; i0 += kTailT) {
      const unsigned i = i0 + tid;
      bool coll = false;
      uint64_t k = 0;
      unsigned j = 0;
      if (i < n) {
        k = ck[i];
        j = cj[i];
        const uint32_t x = (uint32_t)bb_index_mk(seed, k, words, magic);
        const uint32_t wv = sA[x >> 5];
        const uint32_t bit = 1u << (x & 31);
        if (wv & bit) srank[rb0 + spre[x >> 5] + __popc(wv & (bit - 1))] = (unsigned short)j;
        else coll = true;
      }
      const uint64_t m = __ballot(coll);
      if (lane == 0) s_wc[wave] = (unsigned)__popcll(m);
      __syncthreads();  // also: every read of this segment precedes the writes below
      unsigned pre = n1, all = 0;
#pragma unroll
      for (int w = 0; w < kTailT / 64; ++w) {
        pre += (unsigned)w < wave ? s_wc[w] : 0u;
        all += s_wc[w];
      }
      if (coll) {
        const unsigned d = pre + (unsigned)__popcll(m & lanemask_lt());
        ck[d] = k;
        cj[d] = (unsigned short)j;
      }
      n1 += all;
      __syncthreads();
    }
    if (level_out_on(st, L)) out_end = rb0 + tot;
    if (tot == 0) {
      // No key placed: these keys collide again at every level (duplicate hashes); stop and
      // leave them, as mix64(key hash) (a bijection: duplicates stay duplicates), where the
      // host looks: list[(stop_level - 1) & 1]
      Rec* out = (L & 1) ? list1 : list0;
      for (unsigned i = tid; i < n; i += kTailT) out[i] = Rec{ck[i], 0, 0};
      if (tid == 0) {
        st->n[L + 1] = n;
        st->stop_level = L + 1;
        atomicOr(&st->status, kStTooManyLevels);
        s_level = L + 1;
        s_n = 0;
      }
      __syncthreads();
      break;
    }
    if (tid == 0) {
      const uint64_t w1 = n1 ? level_words(n1) : 0;
      st->n[L + 1] = n1;
      st->words[L + 1] = w1;
      st->magic[L + 1] = level_magic(w1);
      st->woff[L + 1] = woff + words;
      st->woff[L + 2] = woff + words + w1;
      st->lvl_base[L + 1] = base + tot;
      st->nlevels = L + 1;
      if (woff + words + w1 > cap_words) {
        atomicOr(&st->status, kStOverflow);
        s_n = 0;
      } else {
        s_n = n1;
      }
      s_level = L + 1;
    }
    __syncthreads();
  }
  // Levels of at most kWaveKeys keys: wave 0 alone, lane i holding key i, so a level costs
  // wave-local LDS ops and ballots instead of the block's barriers (~3 us per level).
  // Level parameters are carried in registers (the same values the block path writes).
  if (wave_levels) {
    if (wave == 0) {
      if (__builtin_amdgcn_wavefrontsize() != 64) __builtin_trap();  // gfx950 only: wave64
      int L = s_level;
      unsigned n = (unsigned)s_n;
      uint64_t words = st->words[L], magic = st->magic[L], woff = st->woff[L], base = st->lvl_base[L];
      if (base0 == ~0ull) base0 = base;
      uint32_t* g32 = nullptr;
      for (;;) {
        if (prof && lane == 0 && L < kMaxLevels) prof[(uint64_t)(kMaxLevels - 1) * kMaxTiles * 8 + L] = wall_clock64();
        if (n == 0) break;
        const bool act = lane < n;
        if (L >= kMaxLevels) {  // as in the block path
          if (lane == 0) {
            st->stop_level = L;
            atomicOr(&st->status, kStTooManyLevels);
          }
          Rec* out = (L & 1) ? list0 : list1;
          if (act) out[lane] = Rec{ck[lane], 0, 0};
          break;
        }
        const uint64_t k = act ? ck[lane] : 0;
        const unsigned short j = act ? cj[lane] : (unsigned short)0;
        const unsigned w32 = (unsigned)(2 * words);  // <= 4 for <= 64 keys
        const unsigned rb0 = (unsigned)(base - base0);
        if (lane < w32) {
          sA[lane] = 0;
          sC[lane] = 0;
        }
        wave_lds_sync();
        uint32_t x = 0;
        if (act) {
          x = (uint32_t)bb_index_mk(level_seed(L), k, words, magic);
          const uint32_t bit = 1u << (x & 31);
          const uint32_t old = atomicOr(&sA[x >> 5], bit);
          if (old & bit) atomicOr(&sC[x >> 5], bit);
        }
        wave_lds_sync();
        g32 = reinterpret_cast<uint32_t*>(bits + woff);
        uint32_t v = 0;
        if (lane < w32) {
          v = sA[lane] & ~sC[lane];
          g32[lane] = v;
        }
        unsigned tot = 0, pre = 0;
        uint32_t vx = 0;
        for (unsigned q = 0; q < w32; ++q) {
          const uint32_t vq = (uint32_t)__shfl((int)v, (int)q);
          tot += __popc(vq);
          if (q < (x >> 5)) pre += __popc(vq);
          if (q == (x >> 5)) vx = vq;
        }
        const uint32_t bit = 1u << (x & 31);
        const bool settled = act && (vx & bit);
        if (settled) srank[rb0 + pre + __popc(vx & (bit - 1))] = j;
        const uint64_t cm = __ballot(act && !settled);
        const unsigned n1 = (unsigned)__popcll(cm);
        if (n1 == n) {
          // No key placed.  Stop only if every key has a twin (duplicate hashes never
          // resolve); distinct keys this few can all collide by chance, and go on.
          bool twin = false;
          for (unsigned q = 0; q < n; ++q) {
            const uint64_t kq = __shfl(k, (int)q);
            twin |= act && q != lane && kq == k;
          }
          if (__ballot(act && !twin) == 0) {
            Rec* out = (L & 1) ? list1 : list0;  // list[(stop_level - 1) & 1]
            if (act) out[lane] = Rec{k, 0, 0};
            if (lane == 0) {
              st->n[L + 1] = n;
              st->stop_level = L + 1;
              atomicOr(&st->status, kStTooManyLevels);
            }
            ++L;
            break;
          }
        }
        wave_lds_sync();
        if (act && !settled) {
          const unsigned d = (unsigned)__popcll(cm & lanemask_lt());
          ck[d] = k;
          cj[d] = j;
        }
        wave_lds_sync();
        if (level_out_on(st, L)) out_end = rb0 + tot;
        const uint64_t w1 = n1 ? level_words(n1) : 0;
        const bool over = woff + words + w1 > cap_words;
        if (lane == 0) {
          st->n[L + 1] = n1;
          st->words[L + 1] = w1;
          st->magic[L + 1] = level_magic(w1);
          st->woff[L + 1] = woff + words;
          st->woff[L + 2] = woff + words + w1;
          st->lvl_base[L + 1] = base + tot;
          st->nlevels = L + 1;
          if (over) atomicOr(&st->status, kStOverflow);
        }
        woff += words;
        words = w1;
        magic = level_magic(w1);
        base += tot;
        n = over ? 0 : n1;
        ++L;
      }
      if (lane == 0) {
        s_level = L;
        s_wbase0 = base0;
        s_wout = out_end;
      }
    }
    __syncthreads();
    base0 = s_wbase0;
    out_end = s_wout;
  }
  // On kStTooManyLevels the unplaced keys were written over a record list (possibly `in`):
  // the build fails and fp_out / pos_out are undefined, so nothing is gathered.
  if (st->status & kStTooManyLevels) out_end = 0;
  if (out_end) {
    if (base0 + out_end > N) {
      bad = true;
    } else {
#pragma unroll 4
      for (uint64_t i = tid; i < out_end; i += kTailT) {
        const Rec* src = in + srank[i];
        fp_out[base0 + i] = src->f;
        pos_out[base0 + i] = src->p;
      }
    }
  }
  if (bad) atomicOr(&st->status, kStRank);
  if (tid == 0) st->rank_total = st->lvl_base[s_level];
}

size_t tile_lds_bytes(unsigned tb) {
  const size_t ac = 2ull * (1ull << (tb - 5)) * sizeof(uint32_t);
  const size_t kc = cache_keys(tb);
  if (tb <= kCacheBits) return ac + (kc + rank_keys(tb)) * sizeof(unsigned short) + (kc / 64 + 1) * sizeof(uint64_t);
  return ac;
}

}  // namespace

uint64_t split_scratch_records() { return split_scratch_recs(); }

// The skewed-length level-0 hash (a no-op launch unless st->skew).  A/B knobs:
// b.skew_cfg (S3IMPH_SKEW_CFG at context creation) selects the block / group shape: 2
// (default) one 768-thread block per CU with 5120-key groups, 1 one 1024-thread block with
// 4096-key groups (C5 1.65 vs 1.61 ms), 0 two 512-thread blocks per CU with 2048-key groups
// (1.75 ms), 3 (partition form only, else 2) two 512-thread blocks per CU with 5120-key groups
// and no result arrays; S3IMPH_SKEW_ORDER=0 alternates the longest and the shortest batch instead of
// longest first.
void launch_hash_skew(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                      unsigned long long* prof, hipStream_t s, const P0Part& pt = P0Part{}) {
  const int cfg = b.skew_cfg;
  static const int order = [] {  // 1: longest first; 0: alternating longest / shortest
    const char* e = dev_env("S3IMPH_SKEW_ORDER");
    return e ? std::atoi(e) : 1;
  }();
  if (cfg == 3 && pt.sup)  // the partition form, two blocks per CU (p0_skew_blocks sized its regions)
    k_hash_skew<512, 5120, false><<<512, 512, sk_lds_bytes<512, 5120, false>(), s>>>(
        blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st, g.tb, g.chunk, b.tcnt, prof, order, pt);
  else if (cfg == 1)
    k_hash_skew<1024, 4096><<<256, 1024, sk_lds_bytes<1024, 4096>(), s>>>(
        blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st, g.tb, g.chunk, b.tcnt, prof, order, pt);
  else if (cfg == 2 || cfg == 3)
    k_hash_skew<768, 5120><<<256, 768, sk_lds_bytes<768, 5120>(), s>>>(
        blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st, g.tb, g.chunk, b.tcnt, prof, order, pt);
  else
    k_hash_skew<512, 2048><<<512, 512, sk_lds_bytes<512, 2048>(), s>>>(
        blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st, g.tb, g.chunk, b.tcnt, prof, order, pt);
}

void binned_set_lds_limits() {
  (void)hipFuncSetAttribute((const void*)k_hash_skew<1024, 4096>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sk_lds_bytes<1024, 4096>());
  (void)hipFuncSetAttribute((const void*)k_hash_skew<512, 2048>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sk_lds_bytes<512, 2048>());
  (void)hipFuncSetAttribute((const void*)k_hash_skew<768, 5120>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sk_lds_bytes<768, 5120>());
  (void)hipFuncSetAttribute((const void*)k_hash_skew<512, 5120, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sk_lds_bytes<512, 5120, false>());
  (void)hipFuncSetAttribute((const void*)k_tile<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)std::max(tile_lds_bytes(kTileMaxBits), tile_lds_bytes(kCacheBits)));
  (void)hipFuncSetAttribute((const void*)k_tile_reg<512, 20, 2, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)tile_reg_lds_bytes(kRegMaxBits));
  (void)hipFuncSetAttribute((const void*)k_tile_reg<512, 20, 2, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)tile_reg_lds_bytes(kRegMaxBits));
}

// The level-0 pair hash over all kH0Grid blocks: one launch, or (b.feed: the host build's key
// bytes still crossing PCIe) one launch per piece of the blocks, each after feed->ensure(its
// keys), so the hash of the arrived keys runs beside the rest of the copy.
template <bool PT>
void launch_hash_pieces(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                        unsigned long long* prof, const P0Part& pt, hipStream_t s) {
  // A/B knob S3IMPH_H0_PAD: dynamic LDS bytes added to each block (3072: three blocks per CU
  // instead of four, leaving the LDS of one co-resident 256-thread super-tile scatter block)
  // The overlapped scatter (pt.hxcc) takes the fourth slot: 3072 B by default (S3IMPH_OV_PAD)
  static const unsigned pad = [] {
    const char* e = dev_env("S3IMPH_H0_PAD");
    return e ? (unsigned)std::atoi(e) : 0u;
  }();
  static const unsigned ov_pad = [] {
    const char* e = dev_env("S3IMPH_OV_PAD");
    return e ? (unsigned)std::atoi(e) : 3072u;
  }();
  const unsigned pd = PT && pt.hxcc ? ov_pad : pad;
  auto go = [&](unsigned b0, unsigned nb) {
    k_hash0_pair<kH0T, kH0B, true, false, PT><<<nb, kH0T, pd, s>>>(blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st,
                                                                 g.tb, g.chunk, b.tcnt, prof, Route0{}, pt, b0,
                                                                 (unsigned)kH0Grid);
  };
  if (!b.feed) {
    go(0, kH0Grid);
    return;
  }
  const unsigned P = (unsigned)std::max(1, std::min(b.feed->pieces, kH0Grid));
  const uint64_t per = (n + kH0Grid - 1) / kH0Grid;  // the kernel's key range per block
  for (unsigned j = 0; j < P; ++j) {
    const unsigned b0 = (unsigned)((uint64_t)kH0Grid * j / P), b1 = (unsigned)((uint64_t)kH0Grid * (j + 1) / P);
    b.feed->ensure(std::min<uint64_t>(n, (uint64_t)b1 * per));
    go(b0, b1 - b0);
  }
}

void launch_binned_count(int level, const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b,
                         LevelGeom g, int grid_chunks, hipStream_t s, bool histogram) {
  if (level == 0 && !b.dist) {
    // a set whose sampled lengths are skewed (k_init_state) hashes 1024-key groups
    // length-sorted in k_hash_count0 (16-byte loads); so does a caller's unaligned blob
    if (!histogram && ((uintptr_t)blob & 15) == 0) {
      // near-uniform lengths: LDS-staged, length-sorted rounds; skewed sets (decided on the
      // device from sampled lengths) fall through to k_hash_count0's length-sorted groups
      unsigned long long* prof = b.tile_prof ? b.tile_prof + (uint64_t)(kMaxLevels - 3) * kMaxTiles * 8 : nullptr;
      launch_hash_pieces<false>(blob, offsets, n, b, g, prof, P0Part{}, s);
      if (b.feed) b.feed->ensure(n);
      launch_hash_skew(blob, offsets, n, b, g, prof, s);
      return;
    }
    if (b.feed) b.feed->ensure(n);
    k_hash_count0<<<grid_chunks, kCB, 0, s>>>(blob, offsets, n, b.kh, b.fp, histogram ? b.hist : nullptr,
                                                  b.flags, b.sflags, b.st, g.tb, g.chunk, b.tcnt, 3);
  } else {
    k_count<<<grid_chunks, kCB, 0, s>>>(level, b.list[(level - 1) & 1], b.hist, b.flags, b.sflags, b.st, g.tb,
                                        g.chunk, b.cap_words);
  }
}

void launch_hash0_only(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                       int grid, hipStream_t s) {
  if (((uintptr_t)blob & 15) == 0) {  // as the single-GPU level 0: pair rounds unless st->skew
    k_hash0_pair<kH0T, kH0B, true><<<kH0Grid, kH0T, 0, s>>>(blob, offsets, n, b.kh, b.fp, b.flags, b.sflags, b.st,
                                                           g.tb, g.chunk, b.tcnt, nullptr);
    launch_hash_skew(blob, offsets, n, b, g, nullptr, s);
    return;
  }
  k_hash_count0<<<grid, kCB, 0, s>>>(blob, offsets, n, b.kh, b.fp, nullptr, b.flags, b.sflags, b.st, g.tb,
                                           g.chunk, b.tcnt, 3);
}

void launch_hash0_route(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                        int grid, const Route0& rt, hipStream_t s) {
  if (((uintptr_t)blob & 15) == 0) {  // near-uniform lengths: hash + route in one pass
    k_hash0_pair<kH0T, kH0B, true, true><<<kH0Grid, kH0T, 0, s>>>(blob, offsets, n, b.kh, b.fp, b.flags, b.sflags,
                                                                 b.st, g.tb, g.chunk, b.tcnt, nullptr, rt);
    // a skewed set (st->skew): k_hash_skew's length-sorted batches, then k_route
    launch_hash_skew(blob, offsets, n, b, g, nullptr, s);
    launch_route0_arrays(b.kh, b.fp, n, rt, b.st, true, s);
    return;
  }
  k_hash_count0<<<grid, kCB, 0, s>>>(blob, offsets, n, b.kh, b.fp, nullptr, b.flags, b.sflags, b.st, g.tb,
                                           g.chunk, b.tcnt, 3);
  launch_route0_arrays(b.kh, b.fp, n, rt, b.st, false, s);
}

void launch_binned_scan(int level, const BinBuffers& b, int grid, hipStream_t s) {
  k_hscan<<<grid, kHST, 0, s>>>(level, b.hist, b.off, b.tile_start, b.sflags, b.st);
}

void launch_binned_scatter(int level, const BinBuffers& b, LevelGeom g, hipStream_t s) {
  const Rec* il = level == 0 && !b.dist ? nullptr : b.list[(level - 1) & 1];
  k_scatter<<<256, kSB, 0, s>>>(level, b.kh, b.fp, b.pos, b.pos_base, il, b.off, b.bucket, b.st, g.tb, g.chunk);
}

void launch_binned_tile(int level, const BinBuffers& b, LevelGeom g, int grid_tiles, hipStream_t s, bool reserved) {
  if (g.tb == kRegMaxBits && reserved && b.pipe_tiles) {
    // 2^14-position tiles from reservation slots: the persistent, pipelined register tiles
    // (level 0 with identity positions reads the scatter's R20 records)
    const unsigned* tc = b.tcnt + (uint64_t)level * kTcntStride;
    // R20 buckets: level 0 with identity positions, or a level whose list is R20
    if ((level == 0 && !b.dist && !b.pos) || b.list20(level))
      k_tile_p0<true><<<256, kP0T, 0, s>>>(level, b.bucket, b.bucket_cap, tc, b.flags, b.bits, b.list[level & 1],
                                           b.fp_out, b.pos_out, b.st, b.pos_base, b.list20(level + 1));
    else
      k_tile_p0<false><<<256, kP0T, 0, s>>>(level, b.bucket, b.bucket_cap, tc, b.flags, b.bits, b.list[level & 1],
                                            b.fp_out, b.pos_out, b.st, b.pos_base, b.list20(level + 1));
    return;
  }
  if (g.tb <= kRegMaxBits) {
    // records per tile ~2^(tb-1): pick the variant whose NT x R covers it with margin
    // (lighter variants keep several tiles resident per CU)
    const unsigned* tc = reserved ? b.tcnt + (uint64_t)level * kTcntStride : nullptr;
    const size_t lds = tile_reg_lds_bytes(g.tb);
#define S3_TILE_REG(NT_, R_, W_)                                                                             \
  (tc ? k_tile_reg<NT_, R_, W_, true> : k_tile_reg<NT_, R_, W_, false>)<<<grid_tiles, NT_, lds, s>>>(level, b.bucket, b.tile_start, tc, b.bucket_cap, b.flags, \
                                                   b.bits, b.list[level & 1], b.fp_out, b.pos_out, b.st, g.tb,  \
                                                   b.tile_prof)
    // A level with no more tiles than CUs runs one round whatever the variant, so it
    // takes twice the threads per tile (half the records per thread: a shorter chain).
    const bool one_round = grid_tiles <= 256;
    if (g.tb == 14) S3_TILE_REG(512, 20, 2);                     // 1 tile per CU
    else if (g.tb == 13 && one_round) S3_TILE_REG(512, 10, 2);
    else if (g.tb == 13) S3_TILE_REG(256, 20, 2);                // 2 tiles per CU
    else if (g.tb == 12 && one_round) S3_TILE_REG(512, 5, 2);
    else if (g.tb == 12) S3_TILE_REG(256, 10, 3);                // 3 tiles per CU
    else if (g.tb == 11 && one_round) S3_TILE_REG(512, 3, 2);
    else if (one_round) S3_TILE_REG(512, 2, 2);
    else S3_TILE_REG(256, 5, 5);                                 // 5 tiles per CU
#undef S3_TILE_REG
    return;
  }
  const unsigned* tc = reserved ? b.tcnt + (uint64_t)level * kTcntStride : nullptr;
  // 2^15 / 2^16 tiles: the split kernel (k_tile stays for contexts without its scratch
  // and for the 2^17+ tiles of oversized conservative reruns)
  if (b.split && g.tb > kRegMaxBits && g.tb <= kSplitMaxBits) {
    // level 0 through the reservation scatter with identity positions: R20 records
    // (or a list level whose list is R20: the scatter kept them R20)
    const bool p20 = (level == 0 && !b.dist && !b.pos && reserved) || b.list20(level);
    const bool o20 = b.list20(level + 1);
    (p20 ? (o20 ? k_tile_split<true, true> : k_tile_split<true, false>)
         : (o20 ? k_tile_split<false, true> : k_tile_split<false, false>))<<<kSplitGrid, kSplitT, 0, s>>>(
        level, b.bucket, b.tile_start, tc, b.bucket_cap, b.flags, b.bits, b.list[level & 1], b.fp_out, b.pos_out, b.st,
        g.tb, b.split, b.tile_prof, b.pos_base, reserved ? g.ts : 0u);
    return;
  }
  k_tile<1024><<<grid_tiles, 1024, tile_lds_bytes(g.tb), s>>>(level, b.bucket, b.tile_start, tc, b.bucket_cap, b.flags,
                                                          b.bits, b.list[level & 1], b.fp_out, b.pos_out, b.st, g.tb,
                                                          b.tile_prof);
}

void launch_binned_scatter_res(int level, const BinBuffers& b, LevelGeom g, int grid, hipStream_t s, uint64_t i_lo,
                               uint64_t i_hi, uint64_t tmax) {
  const bool l0 = level == 0 && !b.dist;
  const Rec* il = l0 ? nullptr : b.list[(level - 1) & 1];
  unsigned* tc = b.tcnt + (uint64_t)level * kTcntStride;
  // level 0 whose tiles go to the split kernel, identity positions: R20 records (the
  // split launch makes the same choice)
  const bool p20 = l0 && !b.pos && ((b.split && g.tb > kRegMaxBits && g.tb <= kSplitMaxBits) ||
                                    (b.pipe_tiles && g.tb == kRegMaxBits));
  // LDS count / start / cursor arrays sized to the level's tiles (tmax: the host's bound;
  // a level past it flags kStGeometry and reruns), the freed LDS taken by longer rounds
  // (more records per tile per round: longer runs, fewer reservation atomics per record).
  // b.scat_cfg (S3IMPH_SCAT_CFG at context creation; A/B knob and test hook): 0 the 4096-tile /
  // 4096-record kernel for every level; 1 tiles by tmax, 4096-record rounds; 2 (default) tiles
  // by tmax, longer rounds.
  const int cfg = b.scat_cfg;
  const int kt = cfg == 0 || tmax == 0 || tmax > 2048 ? 4096 : tmax > 1024 ? 2048 : 1024;
  // (longer rounds with 2048 counters too: they spill 6-8 VGPRs against 0-4, yet measured
  // faster on C2's level 0 than 4096-record rounds there, 0.144-0.149 vs 0.152-0.154 ms)
  auto pick = [&](auto r4096, auto r_long) {
    return cfg == 2 ? r_long : r4096;
  };
  using KFn = decltype(&k_scatter_res<kSubRound, kLdsTiles, 0>);
  KFn kern;
  const bool l20 = !l0 && b.list20(level);  // an R20 list (kSrc 4) into R20 slots
  if (l20) {
    kern = kt == 1024   ? pick(k_scatter_res<4096, 1024, 4, true>, k_scatter_res<6144, 1024, 4, true>)
           : kt == 2048 ? pick(k_scatter_res<4096, 2048, 4, true>, k_scatter_res<6144, 2048, 4, true>)
                        : k_scatter_res<kSubRound, kLdsTiles, 4, true>;
  } else if (kt == 1024) {
    kern = !l0    ? (b.padded ? pick(k_scatter_res<4096, 1024, 3>, k_scatter_res<5120, 1024, 3>)
                              : pick(k_scatter_res<4096, 1024, 0>, k_scatter_res<5120, 1024, 0>))
           : b.pos ? pick(k_scatter_res<4096, 1024, 1>, k_scatter_res<5120, 1024, 1>)
           : p20   ? pick(k_scatter_res<4096, 1024, 2, true>, k_scatter_res<6144, 1024, 2, true>)
                   : pick(k_scatter_res<4096, 1024, 2>, k_scatter_res<5120, 1024, 2>);
  } else if (kt == 2048) {
    kern = !l0    ? (b.padded ? pick(k_scatter_res<4096, 2048, 3>, k_scatter_res<5120, 2048, 3>)
                              : pick(k_scatter_res<4096, 2048, 0>, k_scatter_res<5120, 2048, 0>))
           : b.pos ? pick(k_scatter_res<4096, 2048, 1>, k_scatter_res<5120, 2048, 1>)
           : p20   ? pick(k_scatter_res<4096, 2048, 2, true>, k_scatter_res<6144, 2048, 2, true>)
                   : pick(k_scatter_res<4096, 2048, 2>, k_scatter_res<5120, 2048, 2>);
  } else {
    kern = !l0    ? (b.padded ? k_scatter_res<kSubRound, kLdsTiles, 3> : k_scatter_res<kSubRound, kLdsTiles, 0>)
           : b.pos ? k_scatter_res<kSubRound, kLdsTiles, 1>
           : p20   ? k_scatter_res<kSubRound, kLdsTiles, 2, true>
                   : k_scatter_res<kSubRound, kLdsTiles, 2>;
  }
  kern<<<grid, kSB, 0, s>>>(level, il, b.kh, b.fp, b.pos, b.pos_base, tc, b.bucket, b.bucket_cap, b.flags, b.st, g.tb,
                            b.cap_words, b.tile_prof, i_lo, i_hi, b.split ? g.ts : 0u, 0u);
}

// A per-launch tag for k_mid_levels' all-gather words (26 bits: a word left by a launch 2^26
// launches ago in the same scratch could alias)
static unsigned mid_seq() {
  static std::atomic<unsigned> q{0};
  return (q.fetch_add(1, std::memory_order_relaxed) + 1) & ((1u << 26) - 1);
}

void launch_binned_mid(int L0, int L1, const BinBuffers& b, hipStream_t s, bool big) {
  if (big)
    k_mid_levels<kMidGBig><<<kMidGBig, kMidT, 0, s>>>(L0, L1, b.list[0], b.list[1], b.bits, b.cap_words, b.fp_out,
                                                     b.pos_out, b.st, b.mid,
                                                     reinterpret_cast<Rec*>(b.mid + MidCfg<kMidGBig>::kXb),
                                                     b.tile_prof, mid_seq());
  else
    k_mid_levels<kMidG><<<kMidG, kMidT, 0, s>>>(L0, L1, b.list[0], b.list[1], b.bits, b.cap_words, b.fp_out,
                                                b.pos_out, b.st, b.mid, reinterpret_cast<Rec*>(b.mid + MidCfg<kMidG>::kXb),
                                                b.tile_prof, mid_seq());
}

void launch_binned_tail(int first_level, int big_launched, const BinBuffers& b, hipStream_t s) {
  k_bin_tail<<<1, kTailT, 0, s>>>(first_level, big_launched, b.list[0], b.list[1], b.bits, b.cap_words, b.fp_out, b.pos_out,
                                  b.st, b.tile_prof);
}

// ---- P0: level 0 through super-tiles into 2^14-position register tiles ----------------
// The records' first partition, into the super-tiles' slots of p.sup, when the level-0 hash
// did not write them there (kh / fp from k_hash_count0 or k_hash_skew): k_scatter_res with
// the super-tiles as its tiles (tile = (position >> 14) / tps, exact by the reciprocal).
// A bitmap list level's R20 list (level L's input, b.list[(L - 1) & 1]) into the super-tiles'
// slots: the same pass over the list (k_scatter_res, kSrc 4), which k_scatter_p0 then reads.
void launch_p0_partition_list(int level, const BinBuffers& b, const P0Bufs& p, hipStream_t s) {
  k_scatter_res<6144, 1024, 4, true><<<256, kSB, 0, s>>>(level, b.list[(level - 1) & 1], nullptr, nullptr, nullptr,
                                                         b.pos_base, p.scnt, reinterpret_cast<Rec*>(p.sup), p.sup_cap,
                                                         p.flags, b.st, kRegTileMaxBits, b.cap_words, nullptr, 0, 0,
                                                         p.tps_sub(), 0u);
}

void launch_p0_partition(const BinBuffers& b, const P0Bufs& p, hipStream_t s, bool only_skew) {
  k_scatter_res<5120, 1024, 2, true><<<256, kSB, 0, s>>>(0, nullptr, b.kh, b.fp, nullptr, b.pos_base, p.scnt,
                                                        reinterpret_cast<Rec*>(p.sup), p.sup_cap, p.flags, b.st,
                                                        kRegTileMaxBits, b.cap_words, nullptr, 0, 0, p.tps_sub(),
                                                        only_skew ? 1u : 0u);
}

bool p0_fused(const uint8_t* blob, const P0Bufs& p) {
  return ((uintptr_t)blob & 15) == 0 && p.S <= (unsigned)kMaxRanks;
}
uint64_t p0_region_cap(uint64_t n, unsigned S, unsigned blocks) {
  const double per = (double)((n + blocks - 1) / blocks), mean = per / S;
  return (uint64_t)(mean + 10.0 * std::sqrt(mean) + 32.0);
}
unsigned p0_skew_blocks(int skew_cfg) { return skew_cfg == 0 || skew_cfg == 3 ? 512u : 256u; }  // launch_hash_skew's grid

// P0 level 0's hash and first partition: fused (k_hash0_pair<..., PT>) for an aligned blob
// of up to kMaxRanks super-tiles, with k_hash_skew + the partition pass standing by for a
// set the device finds skewed; otherwise kh / fp, then the partition pass.
void launch_p0_hash(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const BinBuffers& b, LevelGeom g,
                    const P0Bufs& p, hipStream_t s) {
  if (p0_fused(blob, p)) {
    unsigned long long* prof = b.tile_prof ? b.tile_prof + (uint64_t)(kMaxLevels - 3) * kMaxTiles * 8 : nullptr;
    const P0Part pt{p.sup, p.reg_cap, p.pcnt, p.tps_sub(), p.S, p.hxcc};
    launch_hash_pieces<true>(blob, offsets, n, b, g, prof, pt, s);
    if (b.feed) b.feed->ensure(n);
    // a skewed set: k_hash_skew's groups partition the same way, into regions of its own
    // (fewer, larger: p0_skew_blocks blocks, reg_cap_skew records each)
    const P0Part pts{p.sup, p.reg_cap_skew, p.pcnt, p.tps_sub(), p.S};
    launch_hash_skew(blob, offsets, n, b, g, prof, s, pts);
    return;
  }
  launch_binned_count(0, blob, offsets, n, b, g, 256, s, false);
  launch_p0_partition(b, p, s, false);
}

__global__ void k_set_status(LevelState* st, unsigned f) {
  if (threadIdx.x == 0) atomicOr(&st->status, f);
}

void launch_p0_scatter(const BinBuffers& b, const P0Bufs& p, bool fused, hipStream_t s, int level) {
  const P0In in{p.sup, p.reg_cap, p.pcnt, p.nb ? p.nb : (unsigned)kH0Grid, p.S, p0_skew_blocks(b.skew_cfg),
                p.reg_cap_skew, p.sup_cap, p.scnt, fused};
  // blocks per super-tile: a multiple of kResShards, so every shard slot of a tile takes the
  // records of the same number of blocks (9 blocks put 2/9 of a super-tile's records on one
  // shard: 1.8x the mean fill, past the slot capacity at S = 26)
  // More than 32 super-tiles (C3: 64 of ~191 tiles) take the one-block form too: 8 blocks of
  // 1024 threads per super-tile, 512 blocks dispatched in two waves over the 256 CUs, 6144-record
  // rounds of ~32 records per tile (C3 scatter0_p0 1.22 -> 1.09-1.11 ms, the fused partition's
  // hash +0.09; step -0.05 ms over two same-box A/Bs).  S3IMPH_P0_BIG=0: the two-block form below.
  static const bool big = [] {
    const char* e = dev_env("S3IMPH_P0_BIG");
    return !(e && std::atoi(e) == 0);
  }();
  if (p.S > kP0OneBlockS && !big) {
    // more than 32 super-tiles: 8 blocks of 512 threads each (two per CU), 3072-record rounds
    // (2560 with 1024-tile counters, so two blocks' LDS fit a CU): shorter rounds than the
    // one-block form's 5120, but as many records per tile and round at S = 64 (tps ~ 191 vs
    // 382), and one block's count / scan / stage phases run beside the other's loads and stores
    constexpr unsigned bps = kResShards;
    if (p.tps <= 256)
      k_scatter_p0<3072, 256, 512><<<p.S * bps, 512, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags,
                                                             b.st, b.tile_prof, kRegTileMaxBits, nullptr, level);
    else if (p.tps <= 512)
      k_scatter_p0<3072, 512, 512><<<p.S * bps, 512, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags,
                                                             b.st, b.tile_prof, kRegTileMaxBits, nullptr, level);
    else
      k_scatter_p0<2560, 1024, 512><<<p.S * bps, 512, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags,
                                                              b.st, b.tile_prof, kRegTileMaxBits, nullptr, level);
    return;
  }
  static const unsigned bps_knob = [] {  // A/B knob S3IMPH_P0_BPS: blocks per super-tile (a multiple of 8)
    const char* e = dev_env("S3IMPH_P0_BPS");
    const unsigned v = e ? (unsigned)std::atoi(e) : 0u;
    return v / kResShards * kResShards;
  }();
  const unsigned bps = bps_knob ? bps_knob : std::max(1u, kP0ScatterBlocks / p.S / kResShards) * kResShards;
  // A/B knob S3IMPH_P0_SMALL: 256-thread blocks with 1280-record rounds (~33 KB of LDS, less than
  // three padded hash blocks leave on a CU), as many blocks per super-tile as keep a block's runs
  // <= 256
  static const bool small = [] {
    const char* e = dev_env("S3IMPH_P0_SMALL");
    return e && std::atoi(e) != 0;
  }();
  if (small && !p.x && p.tps <= 512) {
    const unsigned nb = fused ? in.NB : 0u;
    const unsigned bsm = std::max(bps, ((nb + 255) / 256 + kResShards - 1) / kResShards * kResShards);
    if (p.tps <= 256)
      k_scatter_p0<1280, 256, 256><<<p.S * bsm, 256, 0, s>>>(in, bsm, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags,
                                                             b.st, b.tile_prof, kRegTileMaxBits, nullptr, level);
    else
      k_scatter_p0<1280, 512, 256><<<p.S * bsm, 256, 0, s>>>(in, bsm, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags,
                                                             b.st, b.tile_prof, kRegTileMaxBits, nullptr, level);
    return;
  }
  if (p.x) {
    // the bitmap decomposition: tiles of 2^p.tb positions, each record's in-tile position to
    // p.x as well; its levels have at most kBmMaxTiles tiles in <= 64 super-tiles of <= 1024
    // (super-tiles of 513-1024 tiles: 5120-record rounds, ~137 KB of LDS)
    if (p.tps > 1024) {
      k_set_status<<<1, 64, 0, s>>>(b.st, kStGeometry);  // unreachable (p0_super_tiles); the build reruns
      return;
    }
    if (p.tps > 512)
      k_scatter_p0<5120, 1024, kSB, true><<<p.S * bps, kSB, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt,
                                                                     p.flags, b.st, b.tile_prof, p.tb, p.x, level);
    else
      k_scatter_p0<6144, 512, kSB, true><<<p.S * bps, kSB, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt,
                                                                    p.flags, b.st, b.tile_prof, p.tb, p.x, level);
    return;
  }
  if (p.tps <= 256)
    k_scatter_p0<6144, 256><<<p.S * bps, kSB, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.st,
                                                       b.tile_prof, kRegTileMaxBits, nullptr, level);
  else if (p.tps <= 512)
    k_scatter_p0<6144, 512><<<p.S * bps, kSB, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.st,
                                                       b.tile_prof, kRegTileMaxBits, nullptr, level);
  else
    k_scatter_p0<6144, 1024><<<p.S * bps, kSB, 0, s>>>(in, bps, p.tps, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.st,
                                                        b.tile_prof, kRegTileMaxBits, nullptr, level);
}

// The super-tile scatter's direct form (k_scatter_p0d): ov, the persistent launch beside the
// level-0 hash (one block per CU); otherwise one block per (super-tile, part), skipping the
// parts an overlapped launch finished (p.ov_done, or none).
void launch_p0_scatter_direct(const BinBuffers& b, const P0Bufs& p, bool ov, hipStream_t s) {
  const P0In in{p.sup, p.reg_cap, p.pcnt, (unsigned)kH0Grid, p.S, p0_skew_blocks(b.skew_cfg),
                p.reg_cap_skew, p.sup_cap, p.scnt, true};
  const P0Ov o{p.hxcc, p.ov_done, kP0OvChunks};
  const unsigned grid = ov ? 256u : p.S * 8u * kP0OvChunks;
#define S3_P0D(KT)                                                                                                  \
  (ov ? k_scatter_p0d<KT, true> : k_scatter_p0d<KT, false>)<<<grid, kDT, 0, s>>>(in, p.tps, p.bucket, p.bucket_cap,  \
                                                                                   p.tcnt, p.flags, b.st, o)
  if (p.tps <= 256) S3_P0D(256);
  else if (p.tps <= 512) S3_P0D(512);
  else S3_P0D(1024);
#undef S3_P0D
}

void launch_p0_tile(const BinBuffers& b, const P0Bufs& p, hipStream_t s) {
  k_tile_p0<true><<<256, kP0T, 0, s>>>(0, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.bits, b.list[0], b.fp_out,
                                       b.pos_out, b.st, b.pos_base, b.list20(1));
}

void launch_p0_count(const BinBuffers& b, const P0Bufs& p, hipStream_t s) {
  k_p0_count<<<1024, kCntT, 0, s>>>(p.x, p.tcnt, p.bucket_cap, b.st);
  k_p0_level1_setup<<<1, 64, 0, s>>>(b.st, b.cap_words);
}

void launch_p0_tile_fed(const BinBuffers& b, const P0Bufs& p, const NextPart& np, hipStream_t s) {
  k_tile_p0<true, true><<<kP0FedGrid, kP0T, 0, s>>>(0, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.bits, nullptr,
                                                    b.fp_out, b.pos_out, b.st, b.pos_base, true, np);
}

void launch_p0_tile_level(int level, const BinBuffers& b, const P0Bufs& p, hipStream_t s) {
  k_tile_p0<true><<<256, kP0T, 0, s>>>(level, p.bucket, p.bucket_cap, p.tcnt, p.flags, b.bits, b.list[level & 1],
                                       b.fp_out, b.pos_out, b.st, b.pos_base, b.list20(level + 1));
}

}  // namespace s3imph
