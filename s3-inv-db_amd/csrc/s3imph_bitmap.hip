// s3imph_bitmap.hip — kernels of the multi-GPU build's second decomposition: the
// north_star's per-level reduction of the collision bitmap over RCCL.
//
// Each rank keeps its key shard for the whole build.  At a distributed level L (global
// key count n_L, words_L = ceil(2 n_L / 64)) every rank hashes its active records over the
// WHOLE level and marks a local 2-bit count per position (A: >= 1 key, C: >= 2 keys) with
// in LDS; the count lanes min(local count, 2) are expanded to one nibble per position (P <= 7
// ranks: sums <= 14, no carry out of a nibble) or one byte (P >= 8: sums <= 2P <= 128) and
// summed over the ranks by an RCCL reduce-scatter (u8 sum), so rank r
// holds the global counts of its slice of the level's words; it decides the final bits
// there (exactly one key: count == 1) and an all-gather gives every rank the level's final
// bit vector — mph.bin's level L, the same bytes a single GPU writes.  Every rank then
// settles its own records against it: a record at position x is placed iff bit x is set
// (its own key is the one key there), at p = ranks[L] - 1 + popcount(A_L[0:x)) (SURVEY
// App. A.3), and the rest go to the next level.  Two collectives per level and no host
// round trip: the next level's global size is n_L - popcount(A_L), known to every rank.
// Settled (p, fp, pos) triples stay on the rank that hashed them; one all-to-all at the
// end moves them to the owner of p's output slice (contiguous ranges of [0, N)).
//
// Reference work replaced: bbhash.New's level loop (pkg/format/mphf_streaming.go:141,
// relab/bbhash restated in SURVEY App. A.2-A.3) + computeHashPositionsReverseMap and the
// fp/pos scatter (:176-204).
#include <hip/hip_runtime.h>

#include "s3imph_device.h"
#include "s3imph_internal.h"

#include <algorithm>
#include <cmath>
#include <type_traits>

namespace s3imph {

namespace {

constexpr int kBT = 256;
constexpr int kBTopT = 1024;                     // the single-block scan of tile totals

// The level's size is outside the host's bound (or the level flagged earlier): skip.
__device__ __forceinline__ bool bm_dead(const LevelState* st) { return (st->status & kStBitmapBound) != 0; }

// bytes of v equal to 1 -> their high bits (exact per byte)
__device__ __forceinline__ unsigned ones_mask(unsigned v) {
  const unsigned t = v ^ 0x01010101u;
  const unsigned y = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t | 0x7f7f7f7fu);
  return y;  // 0x80 in each byte that was 1
}
__device__ __forceinline__ unsigned gather4(unsigned m) {  // high bits of the 4 bytes -> 4 bits
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

// nibbles of v equal to 1 -> 8 bits (nibble j -> bit j)
__device__ __forceinline__ unsigned nib_ones8(unsigned v) {
  const unsigned t = v ^ 0x11111111u;
  const unsigned y = ~(((t & 0x77777777u) + 0x77777777u) | t | 0x77777777u);  // bit 3 of each zero nibble of t
  unsigned m = (y >> 3) & 0x11111111u;
  m = (m | (m >> 3)) & 0x03030303u;
  m = (m | (m >> 6)) & 0x000f000fu;
  return (m | (m >> 12)) & 0xffu;
}

// This rank's slice of the summed lanes (S words) -> final bits: exactly one key.  kNib: a
// lane is one nibble (two positions per byte: P <= 7 ranks sum to at most 14), else a byte.
template <bool kNib>
__global__ __launch_bounds__(kBT) void k_bm_decide(const uint4* __restrict__ slice, uint64_t S,
                                                   uint64_t* __restrict__ out, const LevelState* st) {
  if (bm_dead(st)) return;
  for (uint64_t w = (uint64_t)blockIdx.x * kBT + threadIdx.x; w < S; w += (uint64_t)gridDim.x * kBT) {
    uint64_t bits = 0;
    if (kNib) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint4 v = slice[2 * w + q];
        const uint64_t b32 = (uint64_t)nib_ones8(v.x) | ((uint64_t)nib_ones8(v.y) << 8) |
                             ((uint64_t)nib_ones8(v.z) << 16) | ((uint64_t)nib_ones8(v.w) << 24);
        bits |= b32 << (32 * q);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = slice[4 * w + q];
        const uint64_t b16 = gather4(ones_mask(v.x)) | (gather4(ones_mask(v.y)) << 4) |
                             (gather4(ones_mask(v.z)) << 8) | (gather4(ones_mask(v.w)) << 12);
        bits |= b16 << (16 * q);
      }
    }
    out[w] = bits;
  }
}

// The all-to-all's P (A, C) plane slices of this rank's words (rank q's at 2 S q) -> final
// bits: the associative merge (A, C) + (a, c) = (A | a, C | c | (A & a)) over the ranks,
// then exactly one key = A & ~C.  Two bits per position cross xGMI instead of a count byte.
__global__ __launch_bounds__(kBT) void k_bm_merge(const uint64_t* __restrict__ recv, uint64_t S, int P,
                                                  uint64_t* __restrict__ out, const LevelState* st) {
  if (bm_dead(st)) return;
  for (uint64_t w = (uint64_t)blockIdx.x * kBT + threadIdx.x; w < S; w += (uint64_t)gridDim.x * kBT) {
    uint64_t A = 0, C = 0;
    for (int q = 0; q < P; ++q) {
      const uint64_t a = recv[2 * S * q + w], c = recv[2 * S * q + S + w];
      C |= c | (A & a);
      A |= a;
    }
    out[w] = A & ~C;
  }
}

// ---- level end: tile totals over the gathered final bits -------------------------------
// Tile t (2^tb positions, W = 2^(tb-6) words) -> tsum[t] = popcount(g) << 32 | popcount(g & A)
// over its words (the level's keys placed in the tile, and this rank's share of them); g is
// also copied to bits + woff[L] (mph.bin's level L).
__global__ __launch_bounds__(kBT) void k_bm_tsum(int level, const uint64_t* __restrict__ g,
                                                 const uint64_t* __restrict__ A, unsigned tb,
                                                 uint64_t* __restrict__ bits, unsigned long long* __restrict__ tsum,
                                                 const LevelState* st) {
  if (bm_dead(st) || (st->status & kStStop)) return;
  const uint64_t words = st->words[level], woff = st->woff[level];
  const uint64_t W = 1ull << (tb - 6);
  const uint64_t T = (words + W - 1) / W;
  const unsigned lane = lane_id();
  // a wave per tile, 16-byte loads (W >= 256 words: whole word pairs; the level's last tile
  // may end on an odd word)
  const uint4* g2 = reinterpret_cast<const uint4*>(g);
  const uint4* A2 = reinterpret_cast<const uint4*>(A);
  for (uint64_t t = (uint64_t)blockIdx.x * (kBT / 64) + (threadIdx.x >> 6); t < T; t += (uint64_t)gridDim.x * (kBT / 64)) {
    const uint64_t w0 = t * W, w1 = min<uint64_t>(words, w0 + W);
    const uint64_t p1 = w1 >> 1;  // whole pairs below w1
    unsigned long long s = 0;
#pragma unroll 2
    for (uint64_t p = (w0 >> 1) + lane; p < p1; p += 64) {
      const uint4 v = g2[p], a = A2[p];
      const uint64_t v0 = (uint64_t)v.x | ((uint64_t)v.y << 32), v1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
      const uint64_t a0 = (uint64_t)a.x | ((uint64_t)a.y << 32), a1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
      s += ((unsigned long long)(__popcll(v0) + __popcll(v1)) << 32) | (unsigned)(__popcll(v0 & a0) + __popcll(v1 & a1));
      bits[woff + 2 * p] = v0;
      bits[woff + 2 * p + 1] = v1;
    }
    if ((w1 & 1) && lane == 0) {
      const uint64_t v = g[w1 - 1];
      s += ((unsigned long long)__popcll(v) << 32) | (unsigned)__popcll(v & A[w1 - 1]);
      bits[woff + w1 - 1] = v;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if (lane == 0) tsum[t] = s;
  }
}

// One block: exclusive scans of the tile totals -> tbase[2t] (the tile's first rank within
// the level) and tbase[2t + 1] (its first slot in this rank's settled list, which runs on
// from *out_cnt: the list is in (level, position) order, so sorted by p).  The level's
// total settles the next level's global size and rank base.
constexpr int kTsPer = (int)(kBmMaxTiles / kBTopT);
__global__ __launch_bounds__(kBTopT) void k_bm_tscan(int level, const unsigned long long* __restrict__ tsum,
                                                     unsigned tb, unsigned long long* __restrict__ tbase,
                                                     LevelState* st, unsigned long long* __restrict__ gslot,
                                                     unsigned long long* __restrict__ out_cnt) {
  __shared__ unsigned long long s_w[kBTopT / 64];
  __shared__ unsigned long long s_base;
  // the tile totals pass through LDS in 4096-entry rounds: each round's global loads are
  // coalesced (a thread's kTsPer consecutive entries straight from HBM touched a line per
  // lane and load: 40 us for C3's 12k tiles)
  constexpr int kRound = 4096;
  __shared__ unsigned long long s_t[kRound];
  if (bm_dead(st) || (st->status & kStStop)) return;
  const uint64_t words = st->words[level];
  const uint64_t W = 1ull << (tb - 6);
  const uint64_t T = (words + W - 1) / W;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  if (tid == 0) s_base = *out_cnt;
  unsigned long long v[kTsPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kTsPer; ++q) v[q] = 0;
  static_assert(kTsPer * kBTopT % kRound == 0 && kRound % kTsPer == 0, "tscan rounds");
  const int nr = (int)((T + kRound - 1) / kRound);  // rounds holding tiles (the rest are zeros)
  for (int r = 0; r < nr; ++r) {
    for (int j = (int)tid; j < kRound; j += kBTopT) {
      const uint64_t i = (uint64_t)r * kRound + j;
      s_t[j] = i < T ? tsum[i] : 0ull;
    }
    __syncthreads();
    // threads [r * kRound / kTsPer, (r + 1) * kRound / kTsPer) own this round's entries
    const unsigned own0 = (unsigned)(r * kRound / kTsPer);
    if (tid >= own0 && tid < own0 + kRound / kTsPer) {
#pragma unroll
      for (int q = 0; q < kTsPer; ++q) v[q] = s_t[(tid - own0) * kTsPer + q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < kTsPer; ++q) sum += v[q];
  unsigned long long x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(x, d);
    if (lane >= (unsigned)d) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  unsigned long long pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBTopT / 64; ++w) {
    if ((unsigned)w < wave) pre += s_w[w];
    tot += s_w[w];
  }
  unsigned long long ex = pre + x - sum;
  const unsigned long long ob = s_base;
#pragma unroll
  for (int q = 0; q < kTsPer; ++q) {
    const uint64_t i = (uint64_t)tid * kTsPer + q;
    if (i < T) {
      tbase[2 * i] = ex >> 32;
      tbase[2 * i + 1] = ob + (ex & 0xffffffffull);
    }
    ex += v[q];
  }
  if (tid == 0) {
    const unsigned long long n = st->gn[level], placed = tot >> 32;
    if (placed > n) atomicOr(&st->status, kStRank);  // cannot happen: each set bit is one key
    gslot[level + 1] = n - placed;                    // keys entering level L + 1, globally
    st->lvl_base[level + 1] = st->lvl_base[level] + placed;
    *out_cnt = ob + (tot & 0xffffffffull);
  }
}

// ---- per-tile kernels over the reservation scatter's buckets ---------------------------
// Level L's records were scattered by k_scatter_res into tiles of 2^tb positions over the
// level's WHOLE position range (tile t: kResShards shard slots of scap records from
// t * cap, fills in tc).  Marking and settling then touch only tile-local state in LDS.
// Both read a tile's records as one flattened index range over its shards, kU records
// per thread in flight.
constexpr int kTT = 1024;
// the mark: a tile per 256-thread block, eight blocks per CU (tiles in flight per CU, not
// threads per tile, hide its per-tile round trips and barriers)
constexpr int kMT = 256;
constexpr int kU = 4;

__device__ __forceinline__ uint32_t spread4(uint32_t v) {  // 4 bits -> 4 bytes (bit j -> byte j)
  return (v & 1u) | ((v & 2u) << 7) | ((v & 4u) << 14) | ((v & 8u) << 21);
}
__device__ __forceinline__ uint32_t spread8n(uint32_t v) {  // 8 bits -> 8 nibbles (bit j -> nibble j)
  v &= 0xffu;
  v = (v | (v << 12)) & 0x000f000fu;
  v = (v | (v << 6)) & 0x03030303u;
  return (v | (v << 3)) & 0x11111111u;
}

// shard fills of tile t -> exclusive prefix fo[0..8] (fo[8] = the tile's records)
__device__ __forceinline__ void shard_prefix(const unsigned* __restrict__ tc, uint64_t t, unsigned* fo) {
  unsigned a = 0;
#pragma unroll
  for (int sh = 0; sh < kResShards; ++sh) {
    fo[sh] = a;
    a += tc[t * kResShards + sh];
  }
  fo[kResShards] = a;
}
__device__ __forceinline__ uint64_t rec_index(unsigned i, const unsigned* fo, uint64_t tslot, uint64_t scap) {
  unsigned sh = 0;
#pragma unroll
  for (int k = 1; k < kResShards; ++k) sh += i >= fo[k] ? 1u : 0u;
  unsigned base = fo[0];
#pragma unroll
  for (int k = 1; k < kResShards; ++k)
    if (sh == (unsigned)k) base = fo[k];
  return tslot + (uint64_t)sh * scap + (i - base);
}

// Mark: this rank's records of tile t -> local A (>= 1 key) / C (>= 2 keys) in LDS ->
// the tile's lanes and its A words (kept for the settle).  Lanes of positions past the
// level's true size are zeroed here too.  kMode:
//   kBmBytes / kBmNibbles  count lanes, byte or nibble x = A + C = min(local count, 2),
//                          summed over the ranks by an RCCL reduce-scatter (u8);
//   kBmPlanes              the A and C bit planes themselves, 2 bits per position, laid out
//                          by output slice (slice t = words [t S, (t+1) S): S A words then S C
//                          words) for an all-to-all and k_bm_merge's associative merge
//                          (A, C) + (a, c) = (A | a, C | c | (A & a)).
// a record's k (offset 0 of both record types)
template <class RT>
__device__ __forceinline__ uint64_t rec_k(const RT* __restrict__ q) {
  const uint2 v = *reinterpret_cast<const uint2*>(q);
  return (uint64_t)v.x | ((uint64_t)v.y << 32);
}
// kX: the records' in-tile positions come from xs (u16 per slot, written by the super-tile
// scatter: 2 B per record read instead of the record's k and its bb_index)
template <int kMode, class RT, bool kX = false>
__global__ __launch_bounds__(kMT) void k_bm_tile_mark(int level, const RT* __restrict__ bucket,
                                                      const unsigned* __restrict__ tc, uint64_t bucket_cap,
                                                      unsigned tb, const LevelState* st, uint64_t wpad,
                                                      uint8_t* __restrict__ lanes, uint32_t* __restrict__ A32,
                                                      uint64_t S, uint64_t mS, const uint16_t* __restrict__ xs = nullptr) {
  constexpr bool kNib = kMode == kBmNibbles;
  extern __shared__ uint32_t bm_lds[];
  __shared__ unsigned s_fo[kResShards + 1];
  if (bm_dead(st) || (st->status & kStStop)) return;
  const uint64_t words = st->words[level], magic = st->magic[level], seed = level_seed(level);
  const uint64_t T = (64 * words + (1ull << tb) - 1) >> tb;
  const unsigned W32 = 1u << (tb - 5);  // u32 words of a tile's bit vector
  uint32_t* sA = bm_lds;
  uint32_t* sC = bm_lds + W32;
  const unsigned tid = threadIdx.x;
  // zero the lanes of [64 words, 64 wpad): no tile covers them (64 positions: 4 or 2 uint4,
  // or one A and one C word)
  if (kMode == kBmPlanes) {
    uint64_t* ac = reinterpret_cast<uint64_t*>(lanes);
    for (uint64_t w = words + (uint64_t)blockIdx.x * kMT + tid; w < wpad; w += (uint64_t)gridDim.x * kMT) {
      const uint64_t sl = owner_of(w, S, mS), j = w - sl * S;
      ac[2 * S * sl + j] = 0;
      ac[2 * S * sl + S + j] = 0;
    }
  } else {
    constexpr uint64_t kU4 = kNib ? 2 : 4;
    for (uint64_t q = kU4 * words + (uint64_t)blockIdx.x * kMT + tid; q < kU4 * wpad; q += (uint64_t)gridDim.x * kMT)
      reinterpret_cast<uint4*>(lanes)[q] = make_uint4(0, 0, 0, 0);
  }
  if (T == 0) return;
  const uint64_t cap = bucket_cap / T, scap = cap / kResShards;
  // a tile's slot fills come in one tile ahead (lanes 0-7 of wave 0), during the previous
  // tile's writes: a tile starts without a round trip of its own
  const unsigned lane = lane_id();
  unsigned nfill = 0;
  if (tid < (unsigned)kResShards && blockIdx.x < T) nfill = tc[(uint64_t)blockIdx.x * kResShards + tid];
  for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
    for (unsigned j = tid; j < W32; j += kMT) sA[j] = sC[j] = 0;
    if (tid < 64) {
      unsigned xf = tid < (unsigned)kResShards ? nfill : 0u;  // inclusive prefix over lanes 0-7
#pragma unroll
      for (int d = 1; d < kResShards; d <<= 1) {
        const unsigned y = __shfl_up(xf, d);
        if (lane >= (unsigned)d) xf += y;
      }
      if (tid < (unsigned)kResShards) s_fo[tid] = xf - nfill;
      if (tid == (unsigned)kResShards - 1) s_fo[kResShards] = xf;
    }
    __syncthreads();
    unsigned fo[kResShards + 1];
#pragma unroll
    for (int k = 0; k <= kResShards; ++k) fo[k] = s_fo[k];
    const uint64_t t0 = t << tb;
    const unsigned nrec = fo[kResShards];
    // the next kMT * kU records load while this batch is marked (loads straight-line, the
    // index clamped instead of guarded)
    uint64_t kk[kU], kn[kU];
    auto ld = [&](unsigned i0, uint64_t (&dst)[kU]) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const uint64_t ri = rec_index(min(i0 + u * kMT + tid, nrec - 1), fo, t * cap, scap);
        if constexpr (kX) dst[u] = xs[ri];
        else dst[u] = rec_k(bucket + ri);
      }
    };
    if (nrec) ld(0, kk);
    for (unsigned i0 = 0; i0 < nrec; i0 += kMT * kU) {
      const bool nx = i0 + kMT * kU < nrec;
      if (nx) ld(i0 + kMT * kU, kn);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (i0 + u * kMT + tid < nrec) {
          const uint64_t lx = kX ? kk[u] : bb_index(seed, kk[u], words, magic) - t0;
          const uint32_t bit = 1u << (lx & 31);
          if (atomicOr(&sA[lx >> 5], bit) & bit) atomicOr(&sC[lx >> 5], bit);
        }
      }
      if (nx) {
#pragma unroll
        for (int u = 0; u < kU; ++u) kk[u] = kn[u];
      }
    }
    __syncthreads();
    {  // the next tile's fills, in flight over this tile's writes
      const uint64_t tn = t + gridDim.x;
      if (tid < (unsigned)kResShards && tn < T) nfill = tc[tn * kResShards + tid];
    }
    // the tile's lanes and A words (positions below 64 words only); planes and A as whole u64
    // words (t0 is a multiple of 2^14: a pair of u32 words is one u64 word of its slice)
    const uint64_t wend = min<uint64_t>((uint64_t)W32, (64 * words - t0 + 31) / 32);
    if (kMode == kBmPlanes) {
      uint64_t* ac = reinterpret_cast<uint64_t*>(lanes);
      uint64_t* A64 = reinterpret_cast<uint64_t*>(A32);
      for (unsigned jp = tid; 2 * jp < wend; jp += kMT) {
        const unsigned j = 2 * jp;
        const uint64_t a = (uint64_t)sA[j] | ((uint64_t)(j + 1 < wend ? sA[j + 1] : 0u) << 32);
        const uint64_t c = (uint64_t)sC[j] | ((uint64_t)(j + 1 < wend ? sC[j + 1] : 0u) << 32);
        const uint64_t w = (t0 >> 6) + jp, sl = owner_of(w, S, mS), jw = w - sl * S;
        A64[w] = a;
        ac[2 * S * sl + jw] = a;
        ac[2 * S * sl + S + jw] = c;
      }
    } else {
      for (unsigned j = tid; j < wend; j += kMT) {
        const uint32_t a = sA[j], c = sC[j];
        A32[(t0 >> 5) + j] = a;
        if (kNib) {  // 32 lanes in 16 bytes
          uint4* dst = reinterpret_cast<uint4*>(lanes + t0 / 2 + 16ull * j);
          dst[0] = make_uint4(spread8n(a) + spread8n(c), spread8n(a >> 8) + spread8n(c >> 8),
                              spread8n(a >> 16) + spread8n(c >> 16), spread8n(a >> 24) + spread8n(c >> 24));
        } else {
          uint4* dst = reinterpret_cast<uint4*>(lanes + t0 + 32ull * j);
#pragma unroll
          for (int q = 0; q < 2; ++q) {  // bytes 16q .. 16q + 15 of this word's 32 lanes
            const uint32_t as = a >> (16 * q), cs = c >> (16 * q);
            dst[q] = make_uint4(spread4(as & 15u) + spread4(cs & 15u), spread4((as >> 4) & 15u) + spread4((cs >> 4) & 15u),
                                spread4((as >> 8) & 15u) + spread4((cs >> 8) & 15u),
                                spread4((as >> 12) & 15u) + spread4((cs >> 12) & 15u));
          }
        }
      }
    }
    __syncthreads();
  }
}

// Settle: with the tile's final bits g (gathered) and this rank's A bits a, a record at x is
// placed iff g bit x is set (exactly one key there, so this rank's); its
//   p    = lvl_base[L] + tbase[2t] + popcount(g over the tile below x)
//   slot = tbase[2t + 1] + popcount(g & a over the tile below x)
// so this rank's settled list is in p order whatever order the records arrive in.  The
// tile keeps g and g & a (16 B per word) and, per group of 4 words, both prefixes (2 B per
// word): 144 KiB at 2^19 positions.  Collided records go to the next level's list at one
// atomic per tile plus an LDS cursor.  A settled key whose p falls in this rank's own output
// slice [own_lo, own_lo + slice) is written to fp_out / pos_out at once (its list slot stays
// a hole no one reads); every settled key is counted per output slice in scnt, which is
// the output all-to-all's send counts (the list's runs by slice, holes included).
constexpr unsigned kGrp = 4;
// staged settled keys per tile, at most: the tiles of a staged level are sized so that a rank
// holds ~8k records of one (2^14 positions at one rank, 2^(14 + lg P) at P, kBmP0MaxTb at
// most): mean ~4970 settled, 9.9 sigma below this at one rank.  A launch stages
// bm_stage_entries(tb, P) (P = 8 at 2^16: 4k records, 3072 entries — the settle then fits two
// blocks per CU); a key past the stage is written directly.
constexpr unsigned kBmStage = 5632;
unsigned bm_stage_entries(unsigned tb, int P) {
  static const unsigned cap = [] {  // A/B knob S3IMPH_BM_STAGE_MAX: fewer entries (the rest written directly)
    const char* e = dev_env("S3IMPH_BM_STAGE_MAX");
    const unsigned v = e ? (unsigned)std::atoi(e) : kBmStage;
    return std::max(256u, std::min(kBmStage, v));
  }();
  const double m = std::ldexp(1.0, (int)tb - 1) / std::max(1, P) * 0.6066;  // e^-1/2 of the rank's records
  const unsigned e = (unsigned)(m + 10.0 * std::sqrt(m) + 256.0 + 255.0) & ~255u;
  return std::min(cap, std::max(256u, e));
}
// a staged settled key: its fingerprint, key index (p = pos_base + i) and rank in the tile
struct BmStaged {
  uint64_t f;
  uint32_t i, pg;
};
// a settled key bound for another rank's output slice: as Rec {p, f, pos}, or (identity
// positions) in 16 B — p as an offset in its slice, pos as this rank's key index
__device__ __forceinline__ void put_out(Rec* out, bool o16, uint64_t i, uint64_t p, uint64_t f, uint64_t pos,
                                        const OwnSlice& os, unsigned sl, uint64_t pos_base) {
  if (o16) reinterpret_cast<BmT16*>(out)[i] = BmT16{(uint32_t)(p - (uint64_t)sl * os.slice), (uint32_t)(pos - pos_base), f};
  else out[i] = Rec{p, f, pos};
}
// a slot from an LDS cursor for each active lane, one atomic per wave (lane order)
__device__ __forceinline__ unsigned wave_slot(unsigned* cur) {
  const uint64_t act = __ballot(1);
  unsigned b = 0;
  if ((lanemask_lt() & act) == 0) b = atomicAdd(cur, (unsigned)__popcll(act));
  b = __shfl(b, __builtin_ffsll((long long)act) - 1);
  return b + (unsigned)__popcll(act & lanemask_lt());
}
// one settled key of output slice sl counted in the block's LDS counters: the active lanes of a
// wave mostly share one slice (at one rank all of them; in p order, runs), so one atomic per
// wave then (a same-address LDS atomic per key serialised the whole wave)
__device__ __forceinline__ void count_slice(unsigned* s_sc, unsigned sl, int P) {
  if (sl >= (unsigned)P) sl = P - 1;
  const unsigned s0 = __builtin_amdgcn_readfirstlane(sl);
  const uint64_t act = __ballot(1), same = __ballot(sl == s0);
  if (same == act) {
    if ((lanemask_lt() & act) == 0) atomicAdd(&s_sc[s0], (unsigned)__popcll(act));
  } else {
    atomicAdd(&s_sc[sl], 1u);
  }
}
__device__ __forceinline__ void fp_out_own(const OwnSlice& os, uint64_t p, uint64_t f, uint64_t pos, bool& over) {
  const uint64_t o = p - os.lo;
  if (p < os.lo || o >= os.cnt) {
    over = true;
    return;
  }
  os.fp_out[o] = f;
  os.pos_out[o] = pos;
}
// kStaged (R20 records, identity positions, tiles of a rank's ~8k records: 2^14 to
// 2^kBmP0MaxTb positions): this rank's settled keys of a tile are staged in LDS (16 B each)
// behind the tile words.  kO20: the collided records leave as R20 (k, f, p - pos_base), the
// next bitmap level's list (BinBuffers::l20).  kX: positions from xs (the super-tile scatter's).
// kPN: the collided records go to the next level's super-tile regions (NextPart) instead of
// its list.
template <class RT, bool kStaged, bool kO20, bool kX = false, bool kPN = false, int NT = kTT>
__global__ __launch_bounds__(NT) void k_bm_tile_settle(int level, const RT* __restrict__ bucket, uint64_t pos_base,
                                                        const unsigned* __restrict__ tc, uint64_t bucket_cap,
                                                        unsigned tb, LevelState* st, const uint64_t* __restrict__ g,
                                                        const uint64_t* __restrict__ A,
                                                        const unsigned long long* __restrict__ tbase,
                                                        Rec* __restrict__ out, uint64_t out_cap,
                                                        Rec* __restrict__ next, uint64_t next_cap, OwnSlice os,
                                                        const uint16_t* __restrict__ xs, bool o16, unsigned stage,
                                                        NextPart pn) {
  static_assert(!kStaged || sizeof(RT) != sizeof(Rec), "staged settles read R20 tiles");
  static_assert(!kX || kStaged, "x positions come with P0's R20 tiles");
  static_assert(!kPN || kO20, "the next level's regions hold R20 records");
  extern __shared__ uint64_t bm_lds64[];
  __shared__ unsigned long long s_w[NT / 64];
  __shared__ unsigned s_sc[kMaxRanks];
  __shared__ unsigned s_fo[kResShards + 1];
  __shared__ unsigned long long s_nb, s_tg, s_ta;
  __shared__ unsigned s_ncur;
  __shared__ unsigned p_cur[kPN ? kMaxRanks : 1];  // kPN: this block's fill of each next-level region
  // kPN: a block that settles nothing still publishes empty regions (the next level's scatter
  // reads every block's fills)
  auto no_regions = [&]() {
    if constexpr (kPN)
      for (unsigned q = threadIdx.x; q < pn.S; q += NT) pn.pcnt[(uint64_t)blockIdx.x * pn.S + q] = 0;
  };
  if (bm_dead(st) || (st->status & kStStop)) {
    no_regions();
    return;
  }
  const uint64_t words = st->words[level], magic = st->magic[level], seed = level_seed(level);
  const uint64_t base = st->lvl_base[level];
  const uint64_t T = (64 * words + (1ull << tb) - 1) >> tb;
  if (T == 0) {
    no_regions();
    return;
  }
  const unsigned W = 1u << (tb - 6), G = W / kGrp;  // words, groups of a tile
  uint64_t* sg = bm_lds64;
  uint64_t* sga = sg + W;
  unsigned* gpg = reinterpret_cast<unsigned*>(sga + W);  // per group: popcount(g) before it
  unsigned* gpa = gpg + G;                               // ... popcount(g & a)
  BmStaged* stg = reinterpret_cast<BmStaged*>(gpa + G);  // kStaged: `stage` entries (8-B aligned: G even)
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t cap = bucket_cap / T, scap = cap / kResShards;
  constexpr int kGper = 2;  // groups per thread in the tile scan (G <= 2 NT)
  if (G > (unsigned)(NT * kGper)) {  // (the host takes NT = 512 for tiles of at most 2^16 positions)
    if (tid == 0) atomicOr(&st->status, kStGeometry);
    no_regions();
    return;
  }
  bool over = false, rover = false;
  if (tid < (unsigned)kMaxRanks) s_sc[tid] = 0;  // (the first tile's barriers order it before use)
  // kPN: level L + 1's geometry, from its global size (this level's tile scan wrote it)
  uint64_t w1 = 0, m1 = 0, seed1 = 0;
  uint32_t pmul = 0;
  unsigned rcap = 0;
  if constexpr (kPN) {
    if (tid < (unsigned)kMaxRanks) p_cur[tid] = 0;
    w1 = level_words(*pn.gnext);
    m1 = level_magic(w1);
    seed1 = level_seed(level + 1);
    pmul = 0xffffffffu / pn.tps_sub + 1;  // exact for (position >> 14) < 2^18 (as the hash's partition)
    rcap = (unsigned)pn.reg_cap;
  }
  unsigned long long coll = 0;  // kPN: this block's collided records (one atomic at the end)
  for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
    const uint64_t w0 = t * W;
    const unsigned nw = (unsigned)min<uint64_t>(W, words - w0);
    // the tile's slot fills (lanes 0-7 of wave 0) and its two bases (lanes 8-9), requested
    // before its bit words so that both round trips overlap
    unsigned mfill = 0;
    unsigned long long mbase = 0;
    if (wave == 0) {
      if (lane < (unsigned)kResShards) mfill = tc[t * kResShards + lane];
      else if (lane < (unsigned)kResShards + 2) mbase = tbase[2 * t + (lane - kResShards)];
    }
    unsigned long long c[kGper], sum = 0;
#pragma unroll
    for (int q = 0; q < kGper; ++q) {
      const unsigned grp = tid * kGper + q;
      unsigned cg = 0, ca = 0;
      if (grp < G) {
        const unsigned j0 = grp * kGrp;
        uint64_t gv[kGrp], av[kGrp];
        if (j0 + kGrp <= nw) {
          const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(g + w0 + j0);
          const ulonglong2* a2 = reinterpret_cast<const ulonglong2*>(A + w0 + j0);
          const ulonglong2 x0 = g2[0], x1 = g2[1], y0 = a2[0], y1 = a2[1];
          gv[0] = x0.x; gv[1] = x0.y; gv[2] = x1.x; gv[3] = x1.y;
          av[0] = y0.x; av[1] = y0.y; av[2] = y1.x; av[3] = y1.y;
        } else {
#pragma unroll
          for (int k = 0; k < (int)kGrp; ++k) {
            gv[k] = j0 + k < nw ? g[w0 + j0 + k] : 0ull;
            av[k] = j0 + k < nw ? A[w0 + j0 + k] : 0ull;
          }
        }
#pragma unroll
        for (int k = 0; k < (int)kGrp; ++k) {
          const uint64_t ga = gv[k] & av[k];
          sg[j0 + k] = gv[k];
          sga[j0 + k] = ga;
          cg += (unsigned)__popcll(gv[k]);
          ca += (unsigned)__popcll(ga);
        }
      }
      c[q] = ((unsigned long long)cg << 32) | ca;
      sum += c[q];
    }
    unsigned long long x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d);
      if (lane >= (unsigned)d) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      if ((unsigned)w < wave) pre += s_w[w];
      tot += s_w[w];
    }
    unsigned long long ex = pre + x - sum;
#pragma unroll
    for (int q = 0; q < kGper; ++q) {
      const unsigned grp = tid * kGper + q;
      if (grp < G) {
        gpg[grp] = (unsigned)(ex >> 32);
        gpa[grp] = (unsigned)ex;
      }
      ex += c[q];
    }
    if (wave == 0) {
      unsigned xf = lane < (unsigned)kResShards ? mfill : 0u;  // inclusive prefix over lanes 0-7
#pragma unroll
      for (int d = 1; d < kResShards; d <<= 1) {
        const unsigned y = __shfl_up(xf, d);
        if (lane >= (unsigned)d) xf += y;
      }
      if (lane < (unsigned)kResShards) s_fo[lane] = xf - mfill;
      if (lane == (unsigned)kResShards - 1) s_fo[kResShards] = xf;
      if (lane == (unsigned)kResShards) s_tg = mbase;
      if (lane == (unsigned)kResShards + 1) s_ta = mbase;
      const unsigned nrec = __shfl(xf, kResShards - 1), placed = (unsigned)tot;
      if (lane == 0) {
        if constexpr (kPN) {
          coll += nrec > placed ? nrec - placed : 0u;
        } else {
          s_nb = nrec > placed ? atomicAdd(&st->n[level + 1], (unsigned long long)(nrec - placed)) : 0ull;
        }
        s_ncur = 0;
      }
    }
    __syncthreads();
    unsigned fo[kResShards + 1];
#pragma unroll
    for (int k = 0; k <= kResShards; ++k) fo[k] = s_fo[k];
    const uint64_t t0 = t << tb, pb = base + s_tg, ob = s_ta, nb = s_nb;
    const unsigned nrec = fo[kResShards];
    for (unsigned i0 = 0; i0 < nrec; i0 += NT * kU) {
      Rec r[kU];
      uint16_t rx[kX ? kU : 1];
      // the batch's loads straight-line, all in flight together (the index clamped instead of
      // guarded: a guarded load per record waited for the previous one)
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const unsigned i = min(i0 + u * NT + tid, nrec - 1);
        const uint64_t ri = rec_index(i, fo, t * cap, scap);
        const RT* q = bucket + ri;
        if constexpr (kX) rx[u] = xs[ri];
        if constexpr (sizeof(RT) == sizeof(Rec)) {
          r[u] = *reinterpret_cast<const Rec*>(q);
        } else {  // R20: (k, f, key index), p = pos_base + index
          const uint32_t* w = reinterpret_cast<const uint32_t*>(q);
          const uint4 a = *reinterpret_cast<const uint4*>(w);  // dword-aligned 16-B load
          r[u] = Rec{(uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32), pos_base + w[4]};
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (i0 + u * NT + tid >= nrec) continue;
        const uint64_t lx = kX ? (uint64_t)rx[u] : bb_index(seed, r[u].k, words, magic) - t0;
        const unsigned j = (unsigned)(lx >> 6), b = (unsigned)(lx & 63), grp = j / kGrp;
        const uint64_t below = (1ull << b) - 1ull, v = sg[j];
        if ((v >> b) & 1ull) {
          const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(sg + grp * kGrp);
          const ulonglong2* a2 = reinterpret_cast<const ulonglong2*>(sga + grp * kGrp);
          const ulonglong2 x0 = g2[0], x1 = g2[1], y0 = a2[0], y1 = a2[1];
          const uint64_t gw[kGrp] = {x0.x, x0.y, x1.x, x1.y}, aw[kGrp] = {y0.x, y0.y, y1.x, y1.y};
          unsigned pg = gpg[grp], pa = gpa[grp];
          const unsigned jr = j % kGrp;
#pragma unroll
          for (int k = 0; k < (int)kGrp; ++k)
            if ((unsigned)k < jr) {
              pg += (unsigned)__popcll(gw[k]);
              pa += (unsigned)__popcll(aw[k]);
            }
          pg += (unsigned)__popcll(v & below);
          pa += (unsigned)__popcll(sga[j] & below);
          const uint64_t gp = pb + pg;
          const unsigned sl = owner_of(gp, os.slice, os.mslice);
          const bool staged = kStaged && pa < stage;  // (staged keys are counted at their write-out)
          if (!staged) count_slice(s_sc, sl, os.P);
          if (staged) {  // written out below in pa order
            stg[pa] = BmStaged{r[u].f, (uint32_t)(r[u].p - pos_base), pg};
          } else if ((int)sl == os.rank) {
            fp_out_own(os, gp, r[u].f, r[u].p, over);
          } else {
            const uint64_t slot = ob + pa;
            if (slot < out_cap)
              put_out(out, o16, slot, gp, r[u].f, r[u].p, os, sl, pos_base);
            else
              over = true;
          }
        } else if constexpr (kPN) {  // into this block's region of its level-(L+1) super-tile
          const uint64_t x1 = bb_index(seed1, r[u].k, w1, m1);
          unsigned sp = __umulhi((uint32_t)(x1 >> kRegTileMaxBits), pmul);
          if (sp >= pn.S) sp = pn.S - 1;  // unreachable: positions < 64 w1
          const unsigned at = atomicAdd(&p_cur[sp], 1u);
          if (at < rcap)
            pn.sup[((uint64_t)blockIdx.x * pn.S + sp) * rcap + at] =
                R20{{(uint32_t)r[u].k, (uint32_t)(r[u].k >> 32), (uint32_t)r[u].f, (uint32_t)(r[u].f >> 32),
                     (uint32_t)(r[u].p - pos_base)}};
          else
            rover = true;
        } else {
          const uint64_t slot = nb + wave_slot(&s_ncur);
          if (slot >= next_cap) over = true;
          else if constexpr (kO20) reinterpret_cast<R20*>(next)[slot] = R20{{(uint32_t)r[u].k, (uint32_t)(r[u].k >> 32),
                                                                          (uint32_t)r[u].f, (uint32_t)(r[u].f >> 32),
                                                                          (uint32_t)(r[u].p - pos_base)}};
          else next[slot] = r[u];
        }
      }
    }
    if constexpr (kStaged) {
      // this rank's settled keys of the tile in pa order: their p ascend, so own-slice keys
      // land in runs of fp_out / pos_out (at one rank: the whole tile, one run) and the
      // others in one run of the settled list, instead of one scattered 8-byte store each
      __syncthreads();
      const unsigned ns = (unsigned)min<unsigned long long>(tot & 0xffffffffull, stage);
      for (unsigned i = tid; i < ns; i += NT) {
        const BmStaged e = stg[i];
        const uint64_t gp = pb + e.pg, p = pos_base + e.i;
        const unsigned sl = owner_of(gp, os.slice, os.mslice);
        count_slice(s_sc, sl, os.P);
        if ((int)sl == os.rank) {
          fp_out_own(os, gp, e.f, p, over);
        } else if (ob + i < out_cap) {
          put_out(out, o16, ob + i, gp, e.f, p, os, sl, pos_base);
        } else {
          over = true;
        }
      }
    }
    __syncthreads();  // the tile's LDS state is reused by the next tile
  }
  if (tid < (unsigned)os.P && s_sc[tid]) atomicAdd(&os.scnt[tid], (unsigned long long)s_sc[tid]);
  if (over) atomicOr(&st->status, kStOverflow);
  if constexpr (kPN) {  // (the tile loop ended on a barrier: every append is in p_cur)
    if (tid == 0 && coll) atomicAdd(&st->n[level + 1], coll);  // this rank's records of level L + 1
    for (unsigned q = tid; q < pn.S; q += NT) pn.pcnt[(uint64_t)blockIdx.x * pn.S + q] = min(p_cur[q], rcap);
    if (rover) atomicOr(&st->status, kStResOverflow);  // a region overflowed: the build reruns
  }
}

// Bitmap levels cover the level's whole position range on every rank (the routed build's
// k_dist_setup gave this rank a slice): the scatter and the tile kernels see [0, 64 words).
__global__ void k_bm_range(LevelState* st, int level) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st->wlo[level] = 0;
    st->rw[level] = st->words[level];
  }
}

__global__ void k_bm_flag(LevelState* st, unsigned f) {
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicOr(&st->status, f);
}

// The level's true size against the host's bound (words_L <= wmax), after k_dist_setup.
__global__ void k_bm_check(LevelState* st, int level, uint64_t wmax) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && st->words[level] > wmax) atomicOr(&st->status, kStBitmapBound);
}

// ---- the output slices' assembly at P > 1: a P-way merge through LDS windows ---------------
// Every rank's settled list is sorted by p, so its run for this rank's slice (received, or its
// own run in place) is sorted by slice offset.  Window w covers slice offsets [w Wn, (w+1) Wn):
// its entries of run q are bnd[q][w] .. bnd[q][w+1] (k_bm_place_bounds: a binary search per
// (run, window)); k_bm_place_merge drops them into LDS by offset and writes the window's
// fp_out / pos_out as whole lines — one scattered 8-byte store per key (the first form: a line per
// store at P = 8, 3.5 ms for C3's 100M keys per rank) becomes two coalesced passes.
constexpr unsigned kPlaceWin = 2048;  // slice offsets per window (32 KB of LDS for fp + pos)
struct PlaceRun {
  const void* base;   // the run's first entry
  uint64_t n;         // entries
  uint64_t key_base;  // the sending rank's key base (16-B entries)
};
template <bool k16>
__device__ __forceinline__ uint64_t run_off(const void* base, uint64_t i, uint64_t lo) {
  if constexpr (k16) return static_cast<const BmT16*>(base)[i].off;
  else return static_cast<const Rec*>(base)[i].k - lo;
}
template <bool k16>
__global__ __launch_bounds__(kBT) void k_bm_place_bounds(const PlaceRun* __restrict__ runs, int P, uint64_t lo,
                                                         uint64_t first, uint64_t nwin, uint32_t* __restrict__ bnd) {
  const uint64_t gid = (uint64_t)blockIdx.x * kBT + threadIdx.x;
  if (gid >= (uint64_t)P * (nwin + 1)) return;
  const int q = (int)(gid / (nwin + 1));
  const uint64_t w = gid % (nwin + 1), key = first + w * kPlaceWin;
  const PlaceRun r = runs[q];
  uint64_t a = 0, b = r.n;  // first entry with offset >= key
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (run_off<k16>(r.base, m, lo) < key) a = m + 1;
    else b = m;
  }
  bnd[gid] = (uint32_t)a;
}
template <bool k16>
__global__ __launch_bounds__(kBT) void k_bm_place_merge(const PlaceRun* __restrict__ runs, int P, uint64_t lo,
                                                        uint64_t first, uint64_t limit, uint64_t nwin,
                                                        const uint32_t* __restrict__ bnd,
                                                        uint64_t* __restrict__ fp_out, uint64_t* __restrict__ pos_out,
                                                        LevelState* st) {
  __shared__ uint64_t sf[kPlaceWin], sp[kPlaceWin];
  __shared__ uint32_t s_i0[kMaxRanks], s_pre[kMaxRanks + 1];
  __shared__ const void* s_rb[kMaxRanks];  // the runs' bases and key bases, in LDS: an entry's
  __shared__ uint64_t s_kb[kMaxRanks];     // address waits on no global load but its own
  const uint64_t w = blockIdx.x, w0 = first + w * kPlaceWin;
  if (w >= nwin) return;
  const unsigned wn = (unsigned)min<uint64_t>(kPlaceWin, limit - w0), tid = threadIdx.x;
  // the window's entries over the runs, flattened: run q's part is [s_pre[q], s_pre[q + 1])
  if (tid < 64) {
    uint32_t i0 = 0, c = 0;
    if (tid < (unsigned)P) {
      i0 = bnd[(uint64_t)tid * (nwin + 1) + w];
      c = bnd[(uint64_t)tid * (nwin + 1) + w + 1] - i0;
    }
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (tid >= (unsigned)d) x += y;
    }
    if (tid < (unsigned)P) {
      s_i0[tid] = i0;
      s_pre[tid] = x - c;
      s_rb[tid] = runs[tid].base;
      s_kb[tid] = runs[tid].key_base;
    }
    if (tid == (unsigned)P - 1) s_pre[P] = x;
  }
  __syncthreads();
  const uint32_t have = s_pre[P];  // exactly one entry per offset, or a fault
  bool bad = have != wn;
  if (!bad) {
    // kPlaceWin / kBT entries per thread, their loads all in flight before the LDS drops: the
    // addresses first (LDS only; a thread past the window's entries re-reads the last one),
    // then straight-line loads through global (not flat) pointers, so no load waits on
    // another's LDS counter or branch
    constexpr int kE = (int)(kPlaceWin / kBT);
    using G64 = const __attribute__((address_space(1))) unsigned long long;
    uintptr_t ad[kE];
    uint64_t off[kE], f[kE], pos[kE], kb[kE];
    bool v[kE];
    int q = 0;  // (j ascends with e: the run index only advances)
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const uint32_t j0 = tid + (uint32_t)e * kBT, j = min(j0, have - 1);
      v[e] = j0 < have;
      while (q + 1 < P && s_pre[q + 1] <= j) ++q;
      const uint64_t i = s_i0[q] + (j - s_pre[q]);
      ad[e] = reinterpret_cast<uintptr_t>(s_rb[q]) + i * (k16 ? sizeof(BmT16) : sizeof(Rec));
      kb[e] = s_kb[q];
    }
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      G64* x = reinterpret_cast<G64*>(ad[e]);
      if constexpr (k16) {  // BmT16: off | idx << 32, f
        const uint64_t a = x[0];
        f[e] = x[1];
        off[e] = (uint32_t)a;
        pos[e] = kb[e] + (a >> 32);
      } else {  // Rec: k, f, p
        off[e] = x[0] - lo;
        f[e] = x[1];
        pos[e] = x[2];
      }
    }
#pragma unroll
    for (int e = 0; e < kE; ++e)
      if (v[e]) {
        const uint64_t j = off[e] - w0;
        if (j >= wn) bad = true;
        else {
          sf[j] = f[e];
          sp[j] = pos[e];
        }
      }
  }
  // (a window short of entries, or one off its window, leaves slots unwritten: flagged)
  if (__syncthreads_or(bad)) {
    if (tid == 0) atomicOr(&st->status, kStRank);
    return;
  }
  for (unsigned j = tid; j < wn; j += kBT) {
    fp_out[w0 + j] = sf[j];
    pos_out[w0 + j] = sp[j];
  }
}

// The replicated tail's outputs (global p in [g0, g0 + total), scratch index p - g0) that
// fall inside this rank's slice [lo, lo + cnt).
__global__ __launch_bounds__(kBT) void k_bm_tail_copy(const uint64_t* __restrict__ sfp, const uint64_t* __restrict__ spos,
                                                      uint64_t g0, uint64_t total, uint64_t lo, uint64_t cnt,
                                                      uint64_t* __restrict__ fp_out, uint64_t* __restrict__ pos_out) {
  const uint64_t a = max(g0, lo), b = min(g0 + total, lo + cnt);
  for (uint64_t p = a + (uint64_t)blockIdx.x * kBT + threadIdx.x; p < b; p += (uint64_t)gridDim.x * kBT) {
    fp_out[p - lo] = sfp[p - g0];
    pos_out[p - lo] = spos[p - g0];
  }
}

int grid_for(uint64_t n, int per_block, int cap = 4096) {
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)cap));
}

}  // namespace

void launch_bm_check(LevelState* st, int level, uint64_t wmax, hipStream_t s) {
  k_bm_check<<<1, 64, 0, s>>>(st, level, wmax);
}

void launch_bm_decide(const uint8_t* slice, uint64_t S, uint64_t* out, const LevelState* st, bool nib, hipStream_t s) {
  if (nib) k_bm_decide<true><<<grid_for(S, kBT, 8192), kBT, 0, s>>>(reinterpret_cast<const uint4*>(slice), S, out, st);
  else k_bm_decide<false><<<grid_for(S, kBT, 8192), kBT, 0, s>>>(reinterpret_cast<const uint4*>(slice), S, out, st);
}

void launch_bm_level_end(int level, const uint64_t* g, const uint64_t* A, unsigned tb, uint64_t tiles, uint64_t* bits,
                         unsigned long long* tsum, unsigned long long* tbase, LevelState* st,
                         unsigned long long* gslot, unsigned long long* out_cnt, hipStream_t s) {
  k_bm_tsum<<<(int)std::max<uint64_t>(1, std::min<uint64_t>((tiles + kBT / 64 - 1) / (kBT / 64), 4096)), kBT, 0, s>>>(
      level, g, A, tb, bits, tsum, st);
  k_bm_tscan<<<1, kBTopT, 0, s>>>(level, tsum, tb, tbase, st, gslot, out_cnt);
}

size_t bm_tile_lds(unsigned tb, bool settle) {
  const size_t W = (size_t)1 << (tb - 6);
  return settle ? W * 16 + (W / kGrp) * 8 : W * 16;
}

void bm_set_lds_limits() {
  for (const void* k : {(const void*)k_bm_tile_mark<kBmBytes, Rec>, (const void*)k_bm_tile_mark<kBmNibbles, Rec>,
                        (const void*)k_bm_tile_mark<kBmPlanes, Rec>, (const void*)k_bm_tile_mark<kBmBytes, R20>,
                        (const void*)k_bm_tile_mark<kBmNibbles, R20>, (const void*)k_bm_tile_mark<kBmPlanes, R20>,
                        (const void*)k_bm_tile_mark<kBmBytes, R20, true>, (const void*)k_bm_tile_mark<kBmNibbles, R20, true>,
                        (const void*)k_bm_tile_mark<kBmPlanes, R20, true>})
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bm_tile_lds(kBmMaxTb, false));
  for (const void* k : {(const void*)k_bm_tile_settle<Rec, false, false>, (const void*)k_bm_tile_settle<Rec, false, true>,
                        (const void*)k_bm_tile_settle<R20, false, false>, (const void*)k_bm_tile_settle<R20, false, true>})
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bm_tile_lds(kBmMaxTb, true));
  static_assert(((size_t)1 << (kBmP0MaxTb - 6)) * 18 + kBmStage * sizeof(BmStaged) <= 160 * 1024, "staged settle LDS");
  for (const void* k : {(const void*)k_bm_tile_settle<R20, true, false>, (const void*)k_bm_tile_settle<R20, true, true>,
                        (const void*)k_bm_tile_settle<R20, true, false, true>,
                        (const void*)k_bm_tile_settle<R20, true, true, true>,
                        (const void*)k_bm_tile_settle<R20, true, true, false, true>,
                        (const void*)k_bm_tile_settle<R20, true, true, true, true>,
                        (const void*)k_bm_tile_settle<R20, true, false, false, false, 512>,
                        (const void*)k_bm_tile_settle<R20, true, true, false, false, 512>,
                        (const void*)k_bm_tile_settle<R20, true, false, true, false, 512>,
                        (const void*)k_bm_tile_settle<R20, true, true, true, false, 512>,
                        (const void*)k_bm_tile_settle<R20, true, true, false, true, 512>,
                        (const void*)k_bm_tile_settle<R20, true, true, true, true, 512>})
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(bm_tile_lds(kBmP0MaxTb, true) + kBmStage * sizeof(BmStaged)));
}

void launch_bm_flag(LevelState* st, unsigned flags, hipStream_t s) { k_bm_flag<<<1, 64, 0, s>>>(st, flags); }

void launch_bm_range(LevelState* st, int level, hipStream_t s) { k_bm_range<<<1, 64, 0, s>>>(st, level); }

void launch_bm_tile_mark(int level, const void* bucket, bool r20, const unsigned* tc, uint64_t bucket_cap, unsigned tb,
                         uint64_t tiles, const LevelState* st, uint64_t wpad, uint8_t* lanes, uint64_t* A, int mode,
                         uint64_t S, hipStream_t s, const uint16_t* xs) {
  const int grid = (int)std::max<uint64_t>(256, std::min<uint64_t>(tiles, 4096));
  auto go = [&](auto rt, auto xt) {
    using RT = decltype(rt);
    constexpr bool kX = decltype(xt)::value;
    const RT* bk = static_cast<const RT*>(bucket);
    auto kern = mode == kBmPlanes    ? k_bm_tile_mark<kBmPlanes, RT, kX>
                : mode == kBmNibbles ? k_bm_tile_mark<kBmNibbles, RT, kX>
                                     : k_bm_tile_mark<kBmBytes, RT, kX>;
    kern<<<grid, kMT, bm_tile_lds(tb, false), s>>>(level, bk, tc, bucket_cap, tb, st, wpad, lanes,
                                                   reinterpret_cast<uint32_t*>(A), S, level_magic(S), xs);
  };
  if (xs) go(R20{}, std::true_type{});
  else if (r20) go(R20{}, std::false_type{});
  else go(Rec{}, std::false_type{});
}

void launch_bm_merge(const uint64_t* recv, uint64_t S, int P, uint64_t* out, const LevelState* st, hipStream_t s) {
  k_bm_merge<<<grid_for(S, kBT, 8192), kBT, 0, s>>>(recv, S, P, out, st);
}

// The settle's block: 512 threads (two blocks, two tiles in flight per CU) where the tile's
// LDS (bit words and the stage) leaves room for two blocks, else 1024
int bm_settle_threads(unsigned tb, int P, bool staged) {
  if (!staged || tb > kBmP0MaxTb) return kTT;
  const size_t lds = bm_tile_lds(tb, true) + bm_stage_entries(tb, P) * sizeof(BmStaged);
  return lds <= 80 * 1024 ? 512 : kTT;
}
unsigned bm_settle_grid(uint64_t tiles, int threads) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, threads == kTT ? 1024 : 2048));
}

void launch_bm_tile_settle(int level, const void* bucket, bool r20, uint64_t pos_base, const unsigned* tc,
                           uint64_t bucket_cap, unsigned tb, uint64_t tiles, LevelState* st, const uint64_t* g,
                           const uint64_t* A, const unsigned long long* tbase, Rec* out, uint64_t out_cap, Rec* next,
                           uint64_t next_cap, bool next20, const OwnSlice& os, hipStream_t s, bool staged,
                           const uint16_t* xs, bool o16, const NextPart* np) {
  // R20 tiles holding ~8k of this rank's records (the caller's `staged`: 2^14 positions per
  // rank, at most kBmP0MaxTb) stage their settled keys; larger tiles and Rec buckets write
  // them directly.  np (staged R20 levels whose next level is an R20 super-tile level): the
  // collided records into that level's regions.
  staged = staged && r20 && tb <= kBmP0MaxTb;
  const int nt = bm_settle_threads(tb, os.P, staged);
  const int grid = (int)bm_settle_grid(tiles, nt);
  const NextPart pn = np ? *np : NextPart{};
  auto go = [&](auto rt, auto stg, auto o20, auto xt, auto pt) {
    using RT = decltype(rt);
    constexpr bool kSt = decltype(stg)::value, kO = decltype(o20)::value, kX = decltype(xt)::value,
                   kP = decltype(pt)::value;
    const unsigned stage = kSt ? bm_stage_entries(tb, os.P) : 0u;
    const size_t lds = bm_tile_lds(tb, true) + stage * sizeof(BmStaged);
    if constexpr (kSt) {
      if (nt == 512) {
        k_bm_tile_settle<RT, kSt, kO, kX, kP, 512><<<grid, 512, lds, s>>>(level, static_cast<const RT*>(bucket),
                                                                           pos_base, tc, bucket_cap, tb, st, g, A, tbase,
                                                                           out, out_cap, next, next_cap, os, xs, o16,
                                                                           stage, pn);
        return;
      }
    }
    k_bm_tile_settle<RT, kSt, kO, kX, kP><<<grid, kTT, lds, s>>>(level, static_cast<const RT*>(bucket), pos_base, tc,
                                                                    bucket_cap, tb, st, g, A, tbase, out, out_cap, next,
                                                                    next_cap, os, xs, o16, stage, pn);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (np && !(staged && next20)) {  // (the host never asks for it) the next level would read no regions: rerun
    k_bm_flag<<<1, 64, 0, s>>>(st, kStGeometry);
    return;
  }
  if (np) xs ? go(R20{}, T_{}, T_{}, T_{}, T_{}) : go(R20{}, T_{}, T_{}, F_{}, T_{});
  else if (staged && xs) next20 ? go(R20{}, T_{}, T_{}, T_{}, F_{}) : go(R20{}, T_{}, F_{}, T_{}, F_{});
  else if (staged) next20 ? go(R20{}, T_{}, T_{}, F_{}, F_{}) : go(R20{}, T_{}, F_{}, F_{}, F_{});
  else if (r20) next20 ? go(R20{}, F_{}, T_{}, F_{}, F_{}) : go(R20{}, F_{}, F_{}, F_{}, F_{});
  else next20 ? go(Rec{}, F_{}, T_{}, F_{}, F_{}) : go(Rec{}, F_{}, F_{}, F_{}, F_{});
}


// runs: P device PlaceRun entries (this rank's own run included), each sorted by slice offset;
// [first, limit): the slice offsets the merge fills, exactly one entry each over the runs (a
// group of levels' settled keys below the replicated tail); bnd: P x (nwin + 1) u32 scratch
void launch_bm_place_merge(const void* runs, bool k16, int P, uint64_t lo, uint64_t first, uint64_t limit,
                           uint32_t* bnd, uint64_t* fp_out, uint64_t* pos_out, LevelState* st, hipStream_t s) {
  if (limit <= first) return;
  const uint64_t nwin = (limit - first + kPlaceWin - 1) / kPlaceWin;
  const PlaceRun* r = static_cast<const PlaceRun*>(runs);
  const int gb = grid_for((uint64_t)P * (nwin + 1), kBT, 1 << 20);
  if (k16) {
    k_bm_place_bounds<true><<<gb, kBT, 0, s>>>(r, P, lo, first, nwin, bnd);
    k_bm_place_merge<true><<<(int)nwin, kBT, 0, s>>>(r, P, lo, first, limit, nwin, bnd, fp_out, pos_out, st);
  } else {
    k_bm_place_bounds<false><<<gb, kBT, 0, s>>>(r, P, lo, first, nwin, bnd);
    k_bm_place_merge<false><<<(int)nwin, kBT, 0, s>>>(r, P, lo, first, limit, nwin, bnd, fp_out, pos_out, st);
  }
}
uint64_t bm_place_bound_words(int P, uint64_t limit) { return (uint64_t)P * ((limit + kPlaceWin - 1) / kPlaceWin + 1); }

void launch_bm_tail_copy(const uint64_t* sfp, const uint64_t* spos, uint64_t g0, uint64_t total, uint64_t lo,
                         uint64_t cnt, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s) {
  if (total && cnt) k_bm_tail_copy<<<grid_for(total, kBT, 4096), kBT, 0, s>>>(sfp, spos, g0, total, lo, cnt, fp_out, pos_out);
}

}  // namespace s3imph
