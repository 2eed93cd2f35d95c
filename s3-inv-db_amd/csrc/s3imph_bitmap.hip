// s3imph_bitmap.hip — kernels of the multi-GPU build's second decomposition: the
// north_star's per-level reduction of the collision bitmap over RCCL.
//
// Each rank keeps its key shard for the whole build.  At a distributed level L (global
// key count n_L, words_L = ceil(2 n_L / 64)) every rank hashes its active records over the
// WHOLE level and marks a local 2-bit count per position (A: >= 1 key, C: >= 2 keys) with
// atomics; the count lanes min(local count, 2) are expanded to one byte per position and
// summed over the ranks by an RCCL reduce-scatter (u8 sum: at most 2P <= 128), so rank r
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

namespace s3imph {

namespace {

constexpr int kBT = 256;
constexpr int kBScanPer = 8;                     // words per thread in the word-prefix passes
constexpr int kBScanBlock = kBT * kBScanPer;     // 2048 words per block
constexpr int kBTopT = 1024;                     // the single-block scan of block sums
constexpr int kBTopPer = 32;                     // ... 32 per thread: up to 32768 blocks (67M words)

// Level L's records: kSrc 2 = level 0 from the hash kernel's key-order arrays (n_keys of
// them, positions pos[i] or pos_base + i); kSrc 1 = the list of this rank's records that
// collided at L-1 (st->n[L] of them).
template <int kSrc>
__device__ __forceinline__ uint64_t bm_count(int level, uint64_t n_keys, const LevelState* st) {
  return kSrc == 2 ? n_keys : st->n[level];
}

// The level's size is outside the host's bound (or the level flagged earlier): skip.
__device__ __forceinline__ bool bm_dead(const LevelState* st) { return (st->status & kStBitmapBound) != 0; }

template <int kSrc>
__global__ __launch_bounds__(kBT) void k_bm_mark(int level, const uint64_t* __restrict__ kh, uint64_t n_keys,
                                                 const Rec* __restrict__ ilist, const LevelState* st,
                                                 unsigned* __restrict__ A32, unsigned* __restrict__ C32) {
  if (bm_dead(st)) return;
  const uint64_t n = bm_count<kSrc>(level, n_keys, st);
  const uint64_t words = st->words[level], magic = st->magic[level], seed = level_seed(level);
  for (uint64_t i = (uint64_t)blockIdx.x * kBT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBT) {
    const uint64_t k = kSrc == 2 ? kh[i] : ilist[i].k;
    const uint64_t x = bb_index(seed, k, words, magic);
    const unsigned bit = 1u << (x & 31);
    const unsigned old = atomicOr(&A32[x >> 5], bit);
    if (old & bit) atomicOr(&C32[x >> 5], bit);  // a second key here: local count >= 2
  }
}

// 4 bits -> 4 bytes (bit j of v -> byte j)
__device__ __forceinline__ unsigned spread4(unsigned v) {
  return (v & 1u) | ((v & 2u) << 7) | ((v & 4u) << 14) | ((v & 8u) << 21);
}

// Count lanes: byte x = A bit x + C bit x = min(local count, 2), for words [0, wpad).
__global__ __launch_bounds__(kBT) void k_bm_lanes(const uint64_t* __restrict__ A, const uint64_t* __restrict__ C,
                                                  uint64_t wpad, uint4* __restrict__ lanes, const LevelState* st) {
  if (bm_dead(st)) return;
  for (uint64_t w = (uint64_t)blockIdx.x * kBT + threadIdx.x; w < wpad; w += (uint64_t)gridDim.x * kBT) {
    const uint64_t a = A[w], c = C[w];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // bytes 16q .. 16q+15
      const unsigned as = (unsigned)(a >> (16 * q)), cs = (unsigned)(c >> (16 * q));
      uint4 v;
      v.x = spread4(as & 15u) + spread4(cs & 15u);
      v.y = spread4((as >> 4) & 15u) + spread4((cs >> 4) & 15u);
      v.z = spread4((as >> 8) & 15u) + spread4((cs >> 8) & 15u);
      v.w = spread4((as >> 12) & 15u) + spread4((cs >> 12) & 15u);
      lanes[4 * w + q] = v;
    }
  }
}

// bytes of v equal to 1 -> their high bits (exact per byte)
__device__ __forceinline__ unsigned ones_mask(unsigned v) {
  const unsigned t = v ^ 0x01010101u;
  const unsigned y = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t | 0x7f7f7f7fu);
  return y;  // 0x80 in each byte that was 1
}
__device__ __forceinline__ unsigned gather4(unsigned m) {  // high bits of the 4 bytes -> 4 bits
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

// This rank's slice of the summed lanes (S words) -> final bits: exactly one key.
__global__ __launch_bounds__(kBT) void k_bm_decide(const uint4* __restrict__ slice, uint64_t S,
                                                   uint64_t* __restrict__ out, const LevelState* st) {
  if (bm_dead(st)) return;
  for (uint64_t w = (uint64_t)blockIdx.x * kBT + threadIdx.x; w < S; w += (uint64_t)gridDim.x * kBT) {
    uint64_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = slice[4 * w + q];
      const uint64_t b16 = gather4(ones_mask(v.x)) | (gather4(ones_mask(v.y)) << 4) |
                           (gather4(ones_mask(v.z)) << 8) | (gather4(ones_mask(v.w)) << 12);
      bits |= b16 << (16 * q);
    }
    out[w] = bits;
  }
}

// Pass 1 over the gathered final bits: copy the level's words to bits + woff[L] (mph.bin's
// level L), and per 2048-word block the popcount total.
__global__ __launch_bounds__(kBT) void k_bm_pass1(int level, const uint64_t* __restrict__ g, uint64_t wpad,
                                                  uint64_t* __restrict__ bits, unsigned long long* __restrict__ bsum,
                                                  const LevelState* st) {
  __shared__ unsigned long long s_w[kBT / 64];
  if (bm_dead(st)) return;
  const uint64_t words = st->words[level], woff = st->woff[level];
  const uint64_t b0 = (uint64_t)blockIdx.x * kBScanBlock;
  unsigned long long s = 0;
#pragma unroll
  for (int t = 0; t < kBScanPer; ++t) {
    const uint64_t w = b0 + (uint64_t)t * kBT + threadIdx.x;
    if (w < wpad) {
      const uint64_t v = g[w];
      s += __popcll(v);
      if (w < words) bits[woff + w] = v;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  if (lane_id() == 0) s_w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < kBT / 64; ++k) t += s_w[k];
    bsum[blockIdx.x] = t;
  }
}

// Pass 2 (one block): exclusive scan of the block totals in place; the level's total
// settles the next level's global size and rank base.
__global__ __launch_bounds__(kBTopT) void k_bm_pass2(int level, unsigned long long* __restrict__ bsum, uint64_t nblk,
                                                     LevelState* st, unsigned long long* __restrict__ gslot) {
  __shared__ unsigned long long s_w[kBTopT / 64];
  if (bm_dead(st)) return;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  unsigned long long v[kBTopPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kBTopPer; ++q) {
    const uint64_t i = (uint64_t)tid * kBTopPer + q;
    v[q] = i < nblk ? bsum[i] : 0ull;
    sum += v[q];
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
  for (int w = 0; w < kBTopT / 64; ++w) {
    if ((unsigned)w < wave) pre += s_w[w];
    tot += s_w[w];
  }
  unsigned long long ex = pre + x - sum;
#pragma unroll
  for (int q = 0; q < kBTopPer; ++q) {
    const uint64_t i = (uint64_t)tid * kBTopPer + q;
    if (i < nblk) bsum[i] = ex;
    ex += v[q];
  }
  if (tid == 0) {
    const unsigned long long n = st->gn[level];
    if (tot > n) atomicOr(&st->status, kStRank);  // cannot happen: each set bit is one key
    gslot[level + 1] = n - tot;                   // keys entering level L + 1, globally
    st->lvl_base[level + 1] = st->lvl_base[level] + tot;
  }
}

// Pass 3: per-word exclusive prefix of set bits within the level (u32: n_L < 2^32).
__global__ __launch_bounds__(kBT) void k_bm_pass3(const uint64_t* __restrict__ g, uint64_t wpad,
                                                  const unsigned long long* __restrict__ bsum,
                                                  unsigned* __restrict__ wpre, const LevelState* st) {
  __shared__ unsigned s_w[kBT / 64];
  if (bm_dead(st)) return;
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kBScanBlock + (uint64_t)tid * kBScanPer;  // this thread's 8 words
  unsigned c[kBScanPer], sum = 0;
#pragma unroll
  for (int t = 0; t < kBScanPer; ++t) {
    const uint64_t w = b0 + t;
    c[t] = w < wpad ? (unsigned)__popcll(g[w]) : 0u;
    sum += c[t];
  }
  unsigned x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned y = __shfl_up(x, d);
    if (lane >= (unsigned)d) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  unsigned pre = 0;
#pragma unroll
  for (int w = 0; w < kBT / 64; ++w)
    if ((unsigned)w < wave) pre += s_w[w];
  unsigned ex = (unsigned)bsum[blockIdx.x] + pre + x - sum;
#pragma unroll
  for (int t = 0; t < kBScanPer; ++t) {
    const uint64_t w = b0 + t;
    if (w < wpad) wpre[w] = ex;
    ex += c[t];
  }
}

// Settle this rank's level-L records against the final bits: placed records leave as
// (p, fp, pos) triples (Rec with k = p) in `out`, the others go to the next level's list
// (st->n[L+1] counts them).  A block takes kSetQ x kBT consecutive records at a time:
// the first sweep counts each (wave, round)'s placed / collided records, one atomic per
// counter reserves the block's runs, and the second sweep (records and final-bit words
// again, from L2) writes every wave-round as one contiguous run.  Same-address device
// atomics serialise (~12 ns each): one per wave made this stage 20x slower.
constexpr int kSetQ = 16;
template <int kSrc>
__global__ __launch_bounds__(kBT) void k_bm_settle(int level, const uint64_t* __restrict__ kh,
                                                   const uint64_t* __restrict__ fp, const uint64_t* __restrict__ pos,
                                                   uint64_t pos_base, uint64_t n_keys, const Rec* __restrict__ ilist,
                                                   LevelState* st, const uint64_t* __restrict__ g,
                                                   const unsigned* __restrict__ wpre, Rec* __restrict__ out,
                                                   unsigned long long* __restrict__ out_cnt, uint64_t out_cap,
                                                   Rec* __restrict__ next, uint64_t next_cap) {
  constexpr int NW = kBT / 64;
  __shared__ unsigned s_cp[NW * kSetQ], s_cn[NW * kSetQ];
  __shared__ unsigned long long s_bp, s_bn;
  if (bm_dead(st)) return;
  const uint64_t n = bm_count<kSrc>(level, n_keys, st);
  const uint64_t words = st->words[level], magic = st->magic[level], seed = level_seed(level);
  const uint64_t base = st->lvl_base[level];
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  bool over = false;
  auto rec_at = [&](uint64_t i) -> Rec {
    if (kSrc == 2) return Rec{kh[i], fp[i], pos ? pos[i] : pos_base + i};
    return ilist[i];
  };
  for (uint64_t c0 = (uint64_t)blockIdx.x * kSetQ * kBT; c0 < n; c0 += (uint64_t)gridDim.x * kSetQ * kBT) {
    // sweep 1: counts per (wave, round)
#pragma unroll 4
    for (int q = 0; q < kSetQ; ++q) {
      const uint64_t i = c0 + (uint64_t)q * kBT + tid;
      bool placed = false;
      if (i < n) {
        const uint64_t x = bb_index(seed, kSrc == 2 ? kh[i] : ilist[i].k, words, magic);
        placed = (g[x >> 6] >> (x & 63)) & 1ull;
      }
      const uint64_t pm = __ballot(i < n && placed), nm = __ballot(i < n && !placed);
      if (lane == 0) {
        s_cp[wave * kSetQ + q] = (unsigned)__popcll(pm);
        s_cn[wave * kSetQ + q] = (unsigned)__popcll(nm);
      }
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scans of the NW x kSetQ (<= 64) entries, and the reservations
      const unsigned cp = tid < NW * kSetQ ? s_cp[tid] : 0u, cn = tid < NW * kSetQ ? s_cn[tid] : 0u;
      unsigned xp = cp, xn = cn;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned yp = __shfl_up(xp, d), yn = __shfl_up(xn, d);
        if (tid >= (unsigned)d) {
          xp += yp;
          xn += yn;
        }
      }
      if (tid < NW * kSetQ) {
        s_cp[tid] = xp - cp;
        s_cn[tid] = xn - cn;
      }
      const unsigned tp = __shfl(xp, 63), tn = __shfl(xn, 63);
      if (tid == 0) {
        s_bp = tp ? atomicAdd(out_cnt, (unsigned long long)tp) : 0ull;
        s_bn = tn ? atomicAdd(&st->n[level + 1], (unsigned long long)tn) : 0ull;
      }
    }
    __syncthreads();
    // sweep 2: every wave-round writes its runs
#pragma unroll 2
    for (int q = 0; q < kSetQ; ++q) {
      const uint64_t i = c0 + (uint64_t)q * kBT + tid;
      Rec r{0, 0, 0};
      bool placed = false;
      uint64_t p = 0;
      if (i < n) {
        r = rec_at(i);
        const uint64_t x = bb_index(seed, r.k, words, magic);
        const uint64_t v = g[x >> 6];
        const unsigned b = (unsigned)(x & 63);
        placed = (v >> b) & 1ull;
        if (placed) p = base + wpre[x >> 6] + (uint64_t)__popcll(v & ((1ull << b) - 1ull));
      }
      const uint64_t pm = __ballot(i < n && placed), nm = __ballot(i < n && !placed);
      const uint64_t lt = lanemask_lt();
      if (i < n) {
        if (placed) {
          const uint64_t slot = s_bp + s_cp[wave * kSetQ + q] + (uint64_t)__popcll(pm & lt);
          if (slot < out_cap)
            out[slot] = Rec{p, r.f, r.p};
          else
            over = true;
        } else {
          const uint64_t slot = s_bn + s_cn[wave * kSetQ + q] + (uint64_t)__popcll(nm & lt);
          if (slot < next_cap)
            next[slot] = r;
          else
            over = true;
        }
      }
    }
    __syncthreads();  // s_cp / s_cn / s_bp / s_bn are reused by the next chunk
  }
  if (over) atomicOr(&st->status, kStOverflow);
}

// The level's true size against the host's bound (words_L <= wmax), after k_dist_setup.
__global__ void k_bm_check(LevelState* st, int level, uint64_t wmax) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && st->words[level] > wmax) atomicOr(&st->status, kStBitmapBound);
}

// Settled triples -> per-owner send regions (owner of p = p / slice): rounds of kRR
// records counting-sorted by owner in LDS, one atomic per (round, owner), runs written
// whole (as k_route).
constexpr int kRR = 2048;
__global__ __launch_bounds__(1024) void k_bm_route_out(const Rec* __restrict__ in, const unsigned long long* n_in,
                                                       uint64_t slice, int P, Rec* __restrict__ send, uint64_t cap,
                                                       unsigned long long* __restrict__ scnt, LevelState* st) {
  __shared__ Rec stage[kRR];
  __shared__ unsigned char sdst[kRR];
  __shared__ unsigned cnt[kMaxRanks], start[kMaxRanks];
  __shared__ uint64_t rbase[kMaxRanks];
  __shared__ unsigned s_over;
  const unsigned tid = threadIdx.x;
  if (tid == 0) s_over = 0;
  const uint64_t n = *n_in;
  for (uint64_t r0 = (uint64_t)blockIdx.x * kRR; r0 < n; r0 += (uint64_t)gridDim.x * kRR) {
    if (tid < kMaxRanks) cnt[tid] = 0;
    __syncthreads();
    Rec rec[2];
    unsigned d[2] = {0, 0}, rk[2] = {0, 0};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint64_t i = r0 + (uint64_t)q * 1024 + tid;
      if (i < n) {
        rec[q] = in[i];
        d[q] = (unsigned)min<uint64_t>(rec[q].k / slice, (uint64_t)(P - 1));
        rk[q] = atomicAdd(&cnt[d[q]], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {
      const unsigned c = tid < (unsigned)P ? cnt[tid] : 0u;
      unsigned x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o);
        if (tid >= (unsigned)o) x += y;
      }
      start[tid] = x - c;
      if (c) {
        const unsigned long long at = atomicAdd(&scnt[tid], (unsigned long long)c);
        if (at + c > cap) s_over = 1;
        rbase[tid] = (uint64_t)tid * cap + at;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint64_t i = r0 + (uint64_t)q * 1024 + tid;
      if (i < n) {
        const unsigned slot = start[d[q]] + rk[q];
        stage[slot] = rec[q];
        sdst[slot] = (unsigned char)d[q];
      }
    }
    __syncthreads();
    const unsigned m = (unsigned)min<uint64_t>(kRR, n - r0);
    if (!s_over)
      for (unsigned j = tid; j < m; j += 1024) {
        const unsigned o = sdst[j];
        send[rbase[o] + (j - start[o])] = stage[j];
      }
    __syncthreads();
  }
  if (tid == 0 && s_over) atomicOr(&st->status, kStRouteOverflow);
}

// Received triples of this rank's output slice [lo, lo + cnt) -> fp_out / pos_out.
__global__ __launch_bounds__(kBT) void k_bm_place(const Rec* __restrict__ in, uint64_t n, uint64_t lo, uint64_t cnt,
                                                  uint64_t* __restrict__ fp_out, uint64_t* __restrict__ pos_out,
                                                  LevelState* st) {
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kBT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBT) {
    const Rec r = in[i];
    const uint64_t o = r.k - lo;
    if (r.k < lo || o >= cnt) {
      bad = true;
      continue;
    }
    fp_out[o] = r.f;
    pos_out[o] = r.p;
  }
  if (bad) atomicOr(&st->status, kStRank);
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

void launch_bm_mark(int level, const uint64_t* kh, uint64_t n_keys, const Rec* list, uint64_t n_pred,
                    const LevelState* st, uint64_t* A, uint64_t* C, hipStream_t s) {
  unsigned* a = reinterpret_cast<unsigned*>(A);
  unsigned* c = reinterpret_cast<unsigned*>(C);
  if (level == 0)
    k_bm_mark<2><<<grid_for(n_keys, kBT, 8192), kBT, 0, s>>>(0, kh, n_keys, nullptr, st, a, c);
  else
    k_bm_mark<1><<<grid_for(n_pred, kBT, 8192), kBT, 0, s>>>(level, nullptr, 0, list, st, a, c);
}

void launch_bm_lanes(const uint64_t* A, const uint64_t* C, uint64_t wpad, uint8_t* lanes, const LevelState* st,
                     hipStream_t s) {
  k_bm_lanes<<<grid_for(wpad, kBT, 8192), kBT, 0, s>>>(A, C, wpad, reinterpret_cast<uint4*>(lanes), st);
}

void launch_bm_decide(const uint8_t* slice, uint64_t S, uint64_t* out, const LevelState* st, hipStream_t s) {
  k_bm_decide<<<grid_for(S, kBT, 8192), kBT, 0, s>>>(reinterpret_cast<const uint4*>(slice), S, out, st);
}

uint64_t bm_scan_blocks(uint64_t wpad) { return (wpad + kBScanBlock - 1) / kBScanBlock; }
uint64_t bm_max_words() { return (uint64_t)kBTopT * kBTopPer * kBScanBlock; }

void launch_bm_level_end(int level, const uint64_t* g, uint64_t wpad, uint64_t* bits, unsigned long long* bsum,
                         unsigned* wpre, LevelState* st, unsigned long long* gslot, hipStream_t s) {
  const uint64_t nblk = bm_scan_blocks(wpad);
  k_bm_pass1<<<(int)std::max<uint64_t>(nblk, 1), kBT, 0, s>>>(level, g, wpad, bits, bsum, st);
  k_bm_pass2<<<1, kBTopT, 0, s>>>(level, bsum, nblk, st, gslot);
  k_bm_pass3<<<(int)std::max<uint64_t>(nblk, 1), kBT, 0, s>>>(g, wpad, bsum, wpre, st);
}

void launch_bm_settle(int level, const uint64_t* kh, const uint64_t* fp, const uint64_t* pos, uint64_t pos_base,
                      uint64_t n_keys, const Rec* list, uint64_t n_pred, LevelState* st, const uint64_t* g,
                      const unsigned* wpre, Rec* out, unsigned long long* out_cnt, uint64_t out_cap, Rec* next,
                      uint64_t next_cap, hipStream_t s) {
  if (level == 0)
    k_bm_settle<2><<<grid_for(n_keys, kBT * kSetQ, 2048), kBT, 0, s>>>(0, kh, fp, pos, pos_base, n_keys, nullptr, st,
                                                                        g, wpre, out, out_cnt, out_cap, next, next_cap);
  else
    k_bm_settle<1><<<grid_for(n_pred, kBT * kSetQ, 2048), kBT, 0, s>>>(level, nullptr, nullptr, nullptr, 0, 0, list,
                                                                        st, g, wpre, out, out_cnt, out_cap, next,
                                                                        next_cap);
}

void launch_bm_route_out(const Rec* in, const unsigned long long* n_in, uint64_t n_pred, uint64_t slice, int P,
                         Rec* send, uint64_t cap, unsigned long long* scnt, LevelState* st, hipStream_t s) {
  k_bm_route_out<<<grid_for(n_pred, kRR, 2048), 1024, 0, s>>>(in, n_in, slice, P, send, cap, scnt, st);
}

void launch_bm_place(const Rec* in, uint64_t n, uint64_t lo, uint64_t cnt, uint64_t* fp_out, uint64_t* pos_out,
                     LevelState* st, hipStream_t s) {
  if (n) k_bm_place<<<grid_for(n, kBT, 8192), kBT, 0, s>>>(in, n, lo, cnt, fp_out, pos_out, st);
}

void launch_bm_tail_copy(const uint64_t* sfp, const uint64_t* spos, uint64_t g0, uint64_t total, uint64_t lo,
                         uint64_t cnt, uint64_t* fp_out, uint64_t* pos_out, hipStream_t s) {
  if (total && cnt) k_bm_tail_copy<<<grid_for(total, kBT, 4096), kBT, 0, s>>>(sfp, spos, g0, total, lo, cnt, fp_out, pos_out);
}

}  // namespace s3imph
