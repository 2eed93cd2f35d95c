// s3imph_kernels.hip — hand-written gfx950 kernels for the MPHF build.
//
// What each kernel replaces in the reference (/root/reference):
//   k_hash_mark0  StreamingMPHFBuilder.Add's hashBytes + computeFingerprintBytes
//                 (pkg/format/mphf_streaming.go:73,80; mphf.go:349-369) fused with the first
//                 level pass of bbhash.New (mphf_streaming.go:141; SURVEY App. A.2 pass 1).
//   k_resolve     bbhash level pass 2 (peel collided positions, build the redo set).
//   k_mark        bbhash level pass 1 for levels >= 1.
//   k_finalize    A_L &= ~C_L, clear C, size the next level.
//   k_tail        all small levels in ONE workgroup with LDS-resident A/C bit vectors.
//   k_scan_*      level ranks (ranks[L] + in-level popcount prefix, App. A.3).
//   k_place       computeHashPositionsReverseMap + the scatter loop
//                 (mphf_streaming.go:176-204,237-261): p = Find(k)-1 computed from the
//                 (level, bit) the key settled at; fp_out[p], pos_out[p] written once.
//   k_lookup      MPHF.Lookup (mphf.go:275-302), batched.
//
// No MFMA anywhere: this is 64-bit integer hashing and bit-vector work.  Every
// level bit vector depends only on the SET of keys active at that level, so the
// atomic-OR construction is bit-exact whatever the schedule.
#include <hip/hip_runtime.h>

#include "s3imph_internal.h"

namespace s3imph {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
}

// Position of `key` in a level of 64*words bits: keyHash % (64*words), computed as
// 64*((h>>6) mod words) + (h & 63) with a Barrett step (q < 2^58, one correction).
__device__ __forceinline__ uint64_t bb_index(uint64_t seed, uint64_t key, uint64_t words,
                                             uint64_t magic) {
  uint64_t h = key_mix(seed, key);
  uint64_t q = h >> 6;
  uint64_t qe = __umul64hi(q, magic);
  uint64_t r = q - qe * words;
  if (r >= words) r -= words;
  return (r << 6) | (h & 63);
}

__device__ __forceinline__ void fnv_step(uint64_t& a, uint64_t& b, uint32_t byte) {
  a = (a ^ byte) * kFnvPrime;  // FNV-1a (hashBytes)
  b = (b * kFnvPrime) ^ byte;  // FNV-1  (computeFingerprintBytes)
}

// FNV-1a and FNV-1 of blob[b0, b1) in one pass over aligned 8-byte words.
// The blob must be readable up to round_up(b1, 8).
__device__ __forceinline__ void fnv_both(const uint8_t* __restrict__ blob, uint64_t b0, uint64_t b1,
                                         uint64_t& ha, uint64_t& hb) {
  uint64_t a = kFnvOffset, b = kFnvOffset;
  if (b1 > b0) {
    const uint64_t first = b0 & ~7ull;
    const uint64_t* w = reinterpret_cast<const uint64_t*>(blob + first);
    const uint64_t nw = (((b1 - 1) & ~7ull) - first) / 8 + 1;
    uint64_t v = w[0];
    unsigned s = (unsigned)(b0 & 7);
    for (uint64_t k = 0; k < nw; ++k) {
      uint64_t base = first + 8 * k;
      uint64_t nv = (k + 1 < nw) ? w[k + 1] : 0;  // prefetch next word
      unsigned e = (base + 8 <= b1) ? 8u : (unsigned)(b1 - base);
      if (s == 0 && e == 8) {
#pragma unroll
        for (int t = 0; t < 8; ++t) fnv_step(a, b, (uint32_t)(v >> (8 * t)) & 0xffu);
      } else {
        for (unsigned t = s; t < e; ++t) fnv_step(a, b, (uint32_t)(v >> (8 * t)) & 0xffu);
      }
      s = 0;
      v = nv;
    }
  }
  ha = a;
  hb = b;
}

__device__ __forceinline__ bool test_bit32(const uint32_t* v, uint64_t x) {
  return (v[x >> 5] >> (x & 31)) & 1u;
}

__device__ __forceinline__ void mark_bit(uint32_t* A, uint32_t* C, uint64_t x) {
  const uint32_t bit = 1u << (x & 31);
  const uint32_t old = atomicOr(&A[x >> 5], bit);
  if (old & bit) atomicOr(&C[x >> 5], bit);
}

// ----------------------------------------------------------------------------------
__global__ void k_init_state(LevelState* st, uint64_t n) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(st);
  for (size_t i = threadIdx.x; i < sizeof(LevelState) / 8; i += blockDim.x) p[i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t w = level_words(n);
    st->n[0] = n;
    st->words[0] = w;
    st->woff[0] = 0;
    st->woff[1] = w;
    st->magic[0] = level_magic(w);
  }
}

// Input segment s of a big level: level 0 splits the contiguous kh array into kNSeg
// equal ranges (idx = position in kh); level >= 1 reads segment s of the previous
// level's redo list (capacity seg_cap each, count st->seg[level][s]).
struct SegView {
  const uint64_t* keys;
  const uint32_t* idx;  // nullptr: idx = base + j
  uint64_t base;
  uint64_t cnt;
};

__device__ __forceinline__ SegView seg_view(int level, int s, const uint64_t* keys, const uint32_t* idx,
                                            uint64_t seg_cap, const LevelState* st) {
  SegView v;
  if (level == 0) {
    const uint64_t n = st->n[0];
    const uint64_t lo = n * (uint64_t)s / kNSeg, hi = n * (uint64_t)(s + 1) / kNSeg;
    v.keys = keys + lo;
    v.idx = nullptr;
    v.base = lo;
    v.cnt = hi - lo;
  } else {
    v.keys = keys + (uint64_t)s * seg_cap;
    v.idx = idx + (uint64_t)s * seg_cap;
    v.base = 0;
    v.cnt = st->seg[level][s];
  }
  return v;
}

// Level 0, fused with key hashing: one lane per key.
__global__ __launch_bounds__(kBlock) void k_hash_mark0(
    const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offsets, uint64_t n,
    uint64_t* __restrict__ kh, uint64_t* __restrict__ fp, uint32_t* A, uint32_t* C,
    uint64_t words, uint64_t magic, LevelState* st) {
  const uint64_t seed = level_seed(0);
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  bool zero = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    uint64_t h1, h2;
    fnv_both(blob, offsets[i], offsets[i + 1], h1, h2);
    kh[i] = h1;
    fp[i] = h2;
    zero |= (h1 == 0);
    mark_bit(A, C, bb_index(seed, h1, words, magic));
  }
  if (zero) atomicOr(&st->status, kStKeyZero);
}

// Level >= 1, pass 1 (full grid, gridDim a multiple of kNSeg).  Runs only while the
// level is big (n > gate).
__global__ __launch_bounds__(kBlock) void k_mark(int level, const uint64_t* __restrict__ keys,
                                                 uint64_t seg_cap, uint64_t* bits, uint32_t* C,
                                                 LevelState* st, unsigned long long gate) {
  const uint64_t n = st->n[level];
  if (n <= gate || (st->status & kStOverflow)) return;
  const uint64_t words = st->words[level], magic = st->magic[level];
  uint32_t* A = reinterpret_cast<uint32_t*>(bits + st->woff[level]);
  const uint64_t seed = level_seed(level);
  const int sgi = blockIdx.x % kNSeg;
  const uint64_t sub = blockIdx.x / kNSeg, nsub = gridDim.x / kNSeg;
  const SegView v = seg_view(level, sgi, keys, nullptr, seg_cap, st);
  for (uint64_t j = sub * kBlock + threadIdx.x; j < v.cnt; j += nsub * kBlock)
    mark_bit(A, C, bb_index(seed, v.keys[j], words, magic));
}

// Pass 2: settled keys record their global bit index; collided keys go to the
// next level's list.  Block b reads input segment b % kNSeg and appends to output
// segment b % kNSeg; one atomic per block tile (kResolveKPT*256 keys) reserves space.
constexpr int kResolveKPT = 4;

template <bool kLevel0>
__global__ __launch_bounds__(kBlock) void k_resolve(int level, const uint64_t* __restrict__ keys_in,
                                                    const uint32_t* __restrict__ idx_in,
                                                    const uint32_t* __restrict__ C,
                                                    uint64_t* __restrict__ keys_out,
                                                    uint32_t* __restrict__ idx_out, uint64_t seg_cap,
                                                    uint64_t* __restrict__ settle, LevelState* st,
                                                    unsigned long long gate) {
  __shared__ unsigned s_wcnt[kBlock / 64];
  __shared__ unsigned long long s_wbase[kBlock / 64];
  const uint64_t n = st->n[level];
  if ((!kLevel0 && n <= gate) || (st->status & kStOverflow)) return;
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t gbase = st->woff[level] * 64;
  const uint64_t seed = level_seed(level);
  const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
  const int sgi = blockIdx.x % kNSeg;
  const uint64_t sub = blockIdx.x / kNSeg, nsub = gridDim.x / kNSeg;
  const SegView v = seg_view(kLevel0 ? 0 : level, sgi, keys_in, idx_in, seg_cap, st);
  uint64_t* kout = keys_out + (uint64_t)sgi * seg_cap;
  uint32_t* iout = idx_out + (uint64_t)sgi * seg_cap;
  unsigned long long* seg_counter = &st->seg[level + 1][sgi];
  constexpr uint64_t kTile = (uint64_t)kBlock * kResolveKPT;
  for (uint64_t t0 = sub * kTile; t0 < v.cnt; t0 += nsub * kTile) {
    bool r[kResolveKPT];
    uint64_t k[kResolveKPT];
    uint32_t id[kResolveKPT];
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      const uint64_t j = t0 + (uint64_t)q * kBlock + threadIdx.x;
      r[q] = false;
      k[q] = 0;
      id[q] = 0;
      if (j < v.cnt) {
        k[q] = v.keys[j];
        id[q] = v.idx ? v.idx[j] : (uint32_t)(v.base + j);
        const uint64_t x = bb_index(seed, k[q], words, magic);
        r[q] = test_bit32(C, x);
        if (!r[q]) settle[id[q]] = gbase + x;
      }
    }
    uint64_t m[kResolveKPT];
    unsigned wc = 0;
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      m[q] = __ballot(r[q]);
      wc += __popcll(m[q]);
    }
    if (lane == 0) s_wcnt[wave] = wc;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned tot = 0;
      for (int w = 0; w < kBlock / 64; ++w) tot += s_wcnt[w];
      unsigned long long base = tot ? atomicAdd(seg_counter, (unsigned long long)tot) : 0;
      for (int w = 0; w < kBlock / 64; ++w) {
        s_wbase[w] = base;
        base += s_wcnt[w];
      }
    }
    __syncthreads();
    uint64_t o = s_wbase[wave];
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      if (r[q]) {
        const uint64_t slot = o + __popcll(m[q] & lanemask_lt());
        if (slot < seg_cap) {
          kout[slot] = k[q];
          iout[slot] = id[q];
        } else {
          atomicOr(&st->status, kStOverflow);
        }
      }
      o += __popcll(m[q]);
    }
  }
}

// A_L &= ~C_L and clear C for the next level; block 0 sizes level L+1.
__global__ __launch_bounds__(kBlock) void k_finalize(int level, uint64_t* bits, uint64_t* C,
                                                     uint64_t cap_words, LevelState* st,
                                                     unsigned long long gate) {
  const uint64_t n = st->n[level];
  if ((level > 0 && n <= gate) || (st->status & kStOverflow)) return;
  const uint64_t words = st->words[level];
  uint64_t* A = bits + st->woff[level];
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += stride) {
    A[w] &= ~C[w];
    C[w] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t n1 = 0;
    for (int g = 0; g < kNSeg; ++g) n1 += st->seg[level + 1][g];
    st->n[level + 1] = n1;
    const uint64_t w1 = n1 ? level_words(n1) : 0;
    const uint64_t off1 = st->woff[level] + words;
    st->words[level + 1] = w1;
    st->woff[level + 1] = off1;
    st->woff[level + 2] = off1 + w1;
    st->magic[level + 1] = level_magic(w1);
    st->nlevels = level + 1;
    if (off1 + w1 > cap_words) atomicOr(&st->status, kStOverflow);
  }
}

// All remaining levels in one workgroup.  A and C live in LDS while the level
// fits (n <= kTailKeys); larger levels (only if the host under-predicted the big
// levels) fall back to global bit vectors within the same workgroup.  The first
// tail level reads the segmented list of the last big level; later tail levels
// read a contiguous list.
__global__ __launch_bounds__(kTailThreads) void k_tail(int big_launched, uint64_t* bits,
                                                       uint64_t cap_words, uint32_t* Cg,
                                                       uint64_t* keys0, uint32_t* idx0,
                                                       uint64_t* keys1, uint32_t* idx1,
                                                       uint64_t seg_cap, uint64_t* settle,
                                                       LevelState* st) {
  __shared__ uint32_t sA[kTailLdsWords32 / 2];
  __shared__ uint32_t sC[kTailLdsWords32 / 2];
  __shared__ unsigned long long s_cnt[kNSeg];
  __shared__ unsigned long long s_n, s_words, s_woff, s_magic, s_next, s_stride;
  __shared__ int s_level, s_nseg;
  const unsigned tid = threadIdx.x;
  const unsigned lane = lane_id();

  if (tid == 0) {
    int L = 1;
    while (L <= big_launched && st->n[L] > kTailKeys) ++L;
    s_level = L;
    // Never touch level storage once a capacity overflow has been flagged.
    s_n = (st->status & kStOverflow) ? 0 : st->n[L];
    s_words = st->words[L];
    s_woff = st->woff[L];
    s_magic = st->magic[L];
    s_nseg = kNSeg;
    s_stride = seg_cap;
    st->tail_first = L;
  }
  __syncthreads();
  if (tid < kNSeg) s_cnt[tid] = st->seg[s_level][tid];
  __syncthreads();

  for (;;) {
    const int L = s_level;
    const uint64_t n = s_n;
    if (n == 0) break;
    if (L >= kMaxLevels) {
      if (tid == 0) atomicOr(&st->status, kStTooManyLevels);
      break;
    }
    const uint64_t words = s_words, woff = s_woff, magic = s_magic;
    const int nseg = s_nseg;
    const uint64_t stride = s_stride;
    const uint64_t w32 = 2 * words;
    const bool in_lds = w32 <= (uint64_t)(kTailLdsWords32 / 2);
    uint32_t* A = in_lds ? sA : reinterpret_cast<uint32_t*>(bits + woff);
    uint32_t* C = in_lds ? sC : Cg;
    const uint64_t* kin = (L & 1) ? keys0 : keys1;  // level L's keys were written by level L-1
    const uint32_t* iin = (L & 1) ? idx0 : idx1;
    uint64_t* kout = (L & 1) ? keys1 : keys0;
    uint32_t* iout = (L & 1) ? idx1 : idx0;

    for (uint64_t w = tid; w < w32; w += kTailThreads) {
      C[w] = 0;
      if (in_lds) A[w] = 0;
    }
    if (tid == 0) s_next = 0;
    __syncthreads();
    if (!in_lds) __threadfence();

    const uint64_t seed = level_seed(L);
    for (int g = 0; g < nseg; ++g) {
      const uint64_t* kk = kin + (uint64_t)g * stride;
      const uint64_t c = s_cnt[g];
      for (uint64_t j = tid; j < c; j += kTailThreads) mark_bit(A, C, bb_index(seed, kk[j], words, magic));
    }
    __syncthreads();
    if (!in_lds) __threadfence();

    for (int g = 0; g < nseg; ++g) {
      const uint64_t* kk = kin + (uint64_t)g * stride;
      const uint32_t* ii = iin + (uint64_t)g * stride;
      const uint64_t c = s_cnt[g];
      for (uint64_t wb = tid & ~63u; wb < c; wb += kTailThreads) {
        const uint64_t j = wb + lane;
        bool redo = false;
        uint64_t k = 0;
        uint32_t idx = 0;
        if (j < c) {
          k = kk[j];
          idx = ii[j];
          const uint64_t x = bb_index(seed, k, words, magic);
          // Fallback path: the atomics ran at the memory side, so read back with an
          // atomic as well (never a possibly stale cached line).
          const uint32_t cw = in_lds ? C[x >> 5] : atomicAdd(&C[x >> 5], 0u);
          redo = (cw >> (x & 31)) & 1u;
          if (!redo) settle[idx] = woff * 64 + x;
        }
        const uint64_t m = __ballot(redo);
        if (m) {
          unsigned long long base = 0;
          if (lane == 0) base = atomicAdd(&s_next, (unsigned long long)__popcll(m));
          base = __shfl(base, 0);
          if (redo) {
            const uint64_t o = base + __popcll(m & lanemask_lt());
            kout[o] = k;  // o < n <= buffer capacity
            iout[o] = idx;
          }
        }
      }
    }
    __syncthreads();

    uint32_t* gA = reinterpret_cast<uint32_t*>(bits + woff);
    for (uint64_t w = tid; w < w32; w += kTailThreads) {
      if (in_lds) {
        gA[w] = A[w] & ~C[w];
      } else {
        const uint32_t c = atomicAdd(&C[w], 0u);
        const uint32_t a = atomicAdd(&A[w], 0u);
        atomicAnd(&gA[w], a & ~c);
      }
    }
    __syncthreads();
    if (tid == 0) {
      const uint64_t n1 = s_next;
      const uint64_t w1 = n1 ? level_words(n1) : 0;
      const uint64_t off1 = woff + words;
      st->n[L + 1] = n1;
      st->words[L + 1] = w1;
      st->woff[L + 1] = off1;
      st->woff[L + 2] = off1 + w1;
      st->magic[L + 1] = level_magic(w1);
      st->nlevels = L + 1;
      if (off1 + w1 > cap_words) {
        atomicOr(&st->status, kStOverflow);
        s_n = 0;
      } else {
        s_n = n1;
      }
      s_level = L + 1;
      s_words = w1;
      s_woff = off1;
      s_magic = level_magic(w1);
      s_nseg = 1;
      s_stride = 0;
      s_cnt[0] = n1;
    }
    __syncthreads();
  }
}

// ---- rank scan over all level words (levels concatenated in order) -------------
constexpr int kScanPerThread = 8;
constexpr int kScanPerBlock = kBlock * kScanPerThread;  // 2048 words

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t s_wave[kBlock / 64];
  const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(x, d);
    if (lane >= (unsigned)d) x += y;
  }
  if (lane == 63) s_wave[wave] = x;
  __syncthreads();
  uint64_t wprefix = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w) {
    if ((unsigned)w < wave) wprefix += s_wave[w];
    tot += s_wave[w];
  }
  __syncthreads();
  *total = tot;
  return wprefix + x - v;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint64_t* __restrict__ bits,
                                                        const LevelState* st, const uint64_t* Wp,
                                                        uint64_t cap, unsigned long long* block_sums) {
  const uint64_t W = min(Wp ? *Wp : st->woff[st->nlevels], cap);
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanPerBlock;
  if (b0 >= W) return;
  uint64_t s = 0;
#pragma unroll
  for (int t = 0; t < kScanPerThread; ++t) {
    const uint64_t w = b0 + (uint64_t)t * kBlock + threadIdx.x;
    if (w < W) s += __popcll(bits[w]);
  }
  uint64_t tot;
  block_exclusive_scan(s, &tot);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_top(unsigned long long* block_sums, LevelState* st,
                                                   const uint64_t* Wp, uint64_t cap,
                                                   unsigned long long* total_out) {
  __shared__ uint64_t s_wave[16];
  __shared__ uint64_t s_carry;
  const uint64_t W = min(Wp ? *Wp : st->woff[st->nlevels], cap);
  const uint64_t nb = (W + kScanPerBlock - 1) / kScanPerBlock;
  const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nb; base += 1024) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t v = (i < nb) ? block_sums[i] : 0;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint64_t y = __shfl_up(x, d);
      if (lane >= (unsigned)d) x += y;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    uint64_t wp = 0, tot = 0;
    for (unsigned w = 0; w < 16; ++w) {
      if (w < wave) wp += s_wave[w];
      tot += s_wave[w];
    }
    const uint64_t carry = s_carry;
    if (i < nb) block_sums[i] = carry + wp + x - v;
    __syncthreads();
    if (threadIdx.x == 0) s_carry = carry + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (st) st->rank_total = s_carry;
    if (total_out) *total_out = s_carry;
  }
}

__global__ __launch_bounds__(kBlock) void k_scan_down(const uint64_t* __restrict__ bits,
                                                      const LevelState* st, const uint64_t* Wp,
                                                      uint64_t cap,
                                                      const unsigned long long* block_sums,
                                                      uint64_t* __restrict__ rank_base) {
  const uint64_t W = min(Wp ? *Wp : st->woff[st->nlevels], cap);
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanPerBlock;
  if (b0 >= W) return;
  // Thread t owns words [b0 + t*8, b0 + t*8 + 8): contiguous so its prefix is local.
  const uint64_t w0 = b0 + (uint64_t)threadIdx.x * kScanPerThread;
  uint64_t v[kScanPerThread];
  uint64_t s = 0;
#pragma unroll
  for (int t = 0; t < kScanPerThread; ++t) {
    const uint64_t w = w0 + t;
    v[t] = (w < W) ? bits[w] : 0;
    s += __popcll(v[t]);
  }
  uint64_t tot;
  uint64_t run = block_sums[blockIdx.x] + block_exclusive_scan(s, &tot);
#pragma unroll
  for (int t = 0; t < kScanPerThread; ++t) {
    const uint64_t w = w0 + t;
    if (w < W) rank_base[w] = run;
    run += __popcll(v[t]);
  }
}

// p = rank_base[word] + popcount(word & below(bit)); fp_out[p] = fp_i; pos_out[p] = pos_i.
__global__ __launch_bounds__(kBlock) void k_place(uint64_t n, const uint64_t* __restrict__ settle,
                                                  const uint64_t* __restrict__ fp,
                                                  const uint64_t* __restrict__ pos, uint64_t pos_base,
                                                  const uint64_t* __restrict__ bits,
                                                  const uint64_t* __restrict__ rank_base,
                                                  uint64_t* __restrict__ fp_out,
                                                  uint64_t* __restrict__ pos_out, LevelState* st) {
  if (st->status) return;  // some key never settled: settle[] is not trustworthy
  const uint64_t W = st->woff[st->nlevels];
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint64_t gb = settle[i];
    const uint64_t w = gb >> 6;
    if (w >= W) {
      bad = true;
      continue;
    }
    const uint64_t word = bits[w];
    const uint64_t below = (1ull << (gb & 63)) - 1;
    const uint64_t p = rank_base[w] + __popcll(word & below);
    if (p < n && ((word >> (gb & 63)) & 1ull)) {
      fp_out[p] = fp[i];
      pos_out[p] = pos ? pos[i] : pos_base + i;
    } else {
      bad = true;
    }
  }
  if (bad) atomicOr(&st->status, kStRank);
}

// Batched MPHF.Lookup: FNV-1a -> Find -> p -> range check -> FNV-1 == fp[p] -> pos[p].
__global__ __launch_bounds__(kBlock) void k_lookup(const uint8_t* __restrict__ blob,
                                                   const uint64_t* __restrict__ offsets, uint64_t n,
                                                   const uint64_t* __restrict__ bits,
                                                   const uint64_t* __restrict__ rank_base,
                                                   const LevelState* __restrict__ st,
                                                   const uint64_t* __restrict__ fp,
                                                   const uint64_t* __restrict__ pos, uint64_t count,
                                                   uint64_t* __restrict__ result) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const unsigned nl = st->nlevels;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    uint64_t h1, h2;
    fnv_both(blob, offsets[i], offsets[i + 1], h1, h2);
    uint64_t out = ~0ull;
    if (count != 0) {
      for (unsigned L = 0; L < nl; ++L) {
        const uint64_t x = bb_index(level_seed(L), h1, st->words[L], st->magic[L]);
        const uint64_t gw = st->woff[L] + (x >> 6);
        const uint64_t word = bits[gw];
        if ((word >> (x & 63)) & 1ull) {
          const uint64_t p = rank_base[gw] + __popcll(word & ((1ull << (x & 63)) - 1));
          if (p < count && fp[p] == h2) out = pos[p];
          break;
        }
      }
    }
    result[i] = out;
  }
}

// ---- distributed-build kernels ---------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_dist_mark(int level, const uint64_t* __restrict__ keys,
                                                      uint64_t n, uint64_t words, uint64_t magic,
                                                      uint32_t* A, uint32_t* C) {
  const uint64_t seed = level_seed(level);
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    mark_bit(A, C, bb_index(seed, keys[j], words, magic));
}

__global__ __launch_bounds__(kBlock) void k_dist_hash_mark0(
    const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offsets, uint64_t n,
    uint64_t* __restrict__ kh, uint64_t* __restrict__ fp, uint64_t words, uint64_t magic,
    uint32_t* A, uint32_t* C, unsigned* status) {
  const uint64_t seed = level_seed(0);
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  bool zero = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    uint64_t h1, h2;
    fnv_both(blob, offsets[i], offsets[i + 1], h1, h2);
    kh[i] = h1;
    fp[i] = h2;
    zero |= (h1 == 0);
    mark_bit(A, C, bb_index(seed, h1, words, magic));
  }
  if (zero) atomicOr(status, kStKeyZero);
}

// Saturating per-position local count (0, 1, 2 = "two or more") as one byte per
// position, the lane RCCL sums across ranks (max 2*nranks <= 255).  Also clears A/C.
__global__ __launch_bounds__(kBlock) void k_dist_counts(uint32_t* A, uint32_t* C, uint64_t positions,
                                                        uint8_t* __restrict__ cnt) {
  const uint64_t nw = positions / 32;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
    const uint32_t a = A[w], c = C[w];
    A[w] = 0;
    C[w] = 0;
    uint32_t out[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int b = q * 4 + t;
        const uint32_t av = (a >> b) & 1u, cv = (c >> b) & 1u;
        v |= (av + cv) << (8 * t);
      }
      out[q] = v;
    }
    uint4* dst = reinterpret_cast<uint4*>(cnt + w * 32);
    dst[0] = make_uint4(out[0], out[1], out[2], out[3]);
    dst[1] = make_uint4(out[4], out[5], out[6], out[7]);
  }
}

// Final level bit = (global count == 1).  One u64 word (64 positions) per thread.
__global__ __launch_bounds__(kBlock) void k_dist_pack(const uint8_t* __restrict__ sum,
                                                      uint64_t positions, uint64_t* __restrict__ out) {
  const uint64_t nw = positions / 64;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
    const uint4* src = reinterpret_cast<const uint4*>(sum + w * 64);
    uint64_t word = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = src[q];
      const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t c = (d[r] >> (8 * t)) & 0xffu;
          if (c == 1u) word |= 1ull << (q * 16 + r * 4 + t);
        }
      }
    }
    out[w] = word;
  }
}

__global__ __launch_bounds__(kBlock) void k_dist_resolve(int level, const uint64_t* __restrict__ keys_in,
                                                         const uint32_t* __restrict__ idx_in,
                                                         uint64_t n, uint64_t words, uint64_t magic,
                                                         uint64_t woff, const uint64_t* __restrict__ bits,
                                                         uint64_t* __restrict__ keys_out,
                                                         uint32_t* __restrict__ idx_out,
                                                         unsigned long long* out_count,
                                                         uint64_t* __restrict__ settle) {
  __shared__ unsigned s_wcnt[kBlock / 64];
  __shared__ unsigned long long s_wbase[kBlock / 64];
  const uint64_t seed = level_seed(level);
  const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
  const uint64_t* A = bits + woff;
  constexpr uint64_t kTile = (uint64_t)kBlock * kResolveKPT;
  for (uint64_t t0 = (uint64_t)blockIdx.x * kTile; t0 < n; t0 += (uint64_t)gridDim.x * kTile) {
    bool r[kResolveKPT];
    uint64_t k[kResolveKPT];
    uint32_t id[kResolveKPT];
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      const uint64_t j = t0 + (uint64_t)q * kBlock + threadIdx.x;
      r[q] = false;
      k[q] = 0;
      id[q] = 0;
      if (j < n) {
        k[q] = keys_in[j];
        id[q] = idx_in ? idx_in[j] : (uint32_t)j;
        const uint64_t x = bb_index(seed, k[q], words, magic);
        r[q] = !((A[x >> 6] >> (x & 63)) & 1ull);
        if (!r[q]) settle[id[q]] = woff * 64 + x;
      }
    }
    uint64_t m[kResolveKPT];
    unsigned wc = 0;
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      m[q] = __ballot(r[q]);
      wc += __popcll(m[q]);
    }
    if (lane == 0) s_wcnt[wave] = wc;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned tot = 0;
      for (int w = 0; w < kBlock / 64; ++w) tot += s_wcnt[w];
      unsigned long long base = tot ? atomicAdd(out_count, (unsigned long long)tot) : 0;
      for (int w = 0; w < kBlock / 64; ++w) {
        s_wbase[w] = base;
        base += s_wcnt[w];
      }
    }
    __syncthreads();
    uint64_t o = s_wbase[wave];
#pragma unroll
    for (int q = 0; q < kResolveKPT; ++q) {
      if (r[q]) {
        const uint64_t slot = o + __popcll(m[q] & lanemask_lt());
        keys_out[slot] = k[q];
        idx_out[slot] = id[q];
      }
      o += __popcll(m[q]);
    }
  }
}

__device__ __forceinline__ uint64_t settle_rank(const uint64_t* bits, const uint64_t* rank_base,
                                                uint64_t gb) {
  const uint64_t w = gb >> 6;
  return rank_base[w] + __popcll(bits[w] & ((1ull << (gb & 63)) - 1));
}

__global__ __launch_bounds__(kBlock) void k_dist_count_owners(uint64_t n, const uint64_t* settle,
                                                              const uint64_t* bits,
                                                              const uint64_t* rank_base,
                                                              uint64_t per_rank, int nranks,
                                                              unsigned long long* counts) {
  __shared__ unsigned long long s_cnt[64];
  if (threadIdx.x < 64) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint64_t p = settle_rank(bits, rank_base, settle[i]);
    uint64_t o = p / per_rank;
    if (o >= (uint64_t)nranks) o = nranks - 1;
    atomicAdd(&s_cnt[o], 1ull);
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)nranks && s_cnt[threadIdx.x]) atomicAdd(&counts[threadIdx.x], s_cnt[threadIdx.x]);
}

__global__ __launch_bounds__(kBlock) void k_dist_place(uint64_t n, const uint64_t* __restrict__ settle,
                                                       const uint64_t* __restrict__ fp,
                                                       const uint64_t* __restrict__ pos,
                                                       uint64_t pos_base, const uint64_t* bits,
                                                       const uint64_t* rank_base, uint64_t per_rank,
                                                       int nranks, unsigned long long* fill,
                                                       const unsigned long long* off,
                                                       uint64_t* __restrict__ triples) {
  __shared__ unsigned long long s_cnt[64], s_base[64];
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kBlock; b0 < n; b0 += stride) {
    if (threadIdx.x < 64) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = b0 + threadIdx.x;
    uint64_t p = 0, o = 0, local = 0;
    const bool act = i < n;
    if (act) {
      p = settle_rank(bits, rank_base, settle[i]);
      o = p / per_rank;
      if (o >= (uint64_t)nranks) o = nranks - 1;
      local = atomicAdd(&s_cnt[o], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nranks)
      s_base[threadIdx.x] = s_cnt[threadIdx.x] ? atomicAdd(&fill[threadIdx.x], s_cnt[threadIdx.x]) : 0;
    __syncthreads();
    if (act) {
      uint64_t* t = triples + 3 * (off[o] + s_base[o] + local);
      t[0] = p;
      t[1] = fp[i];
      t[2] = pos ? pos[i] : pos_base + i;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_dist_unpack(const uint64_t* __restrict__ triples,
                                                        uint64_t count, uint64_t lo, uint64_t out_n,
                                                        uint64_t* __restrict__ fp_out,
                                                        uint64_t* __restrict__ pos_out,
                                                        unsigned* status) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
    const uint64_t p = triples[3 * i];
    if (p >= lo && p - lo < out_n) {
      fp_out[p - lo] = triples[3 * i + 1];
      pos_out[p - lo] = triples[3 * i + 2];
    } else {
      bad = true;
    }
  }
  if (bad) atomicOr(status, kStRank);
}

}  // namespace

// ================================ launchers =======================================
int default_grid(uint64_t work, int block) {
  uint64_t g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_init_state(LevelState* st, uint64_t n, uint64_t, hipStream_t s) {
  k_init_state<<<1, 256, 0, s>>>(st, n);
}

void launch_hash_mark0(const uint8_t* blob, const uint64_t* offsets, uint64_t n, uint64_t* kh,
                       uint64_t* fp, uint64_t* bits, uint64_t* C, uint64_t words0, LevelState* st,
                       int grid, hipStream_t s) {
  k_hash_mark0<<<grid, kBlock, 0, s>>>(blob, offsets, n, kh, fp, reinterpret_cast<uint32_t*>(bits),
                                       reinterpret_cast<uint32_t*>(C), words0, level_magic(words0), st);
}

void launch_resolve(int level, const uint64_t* keys_in, const uint32_t* idx_in, const uint64_t* C,
                    uint64_t* keys_out, uint32_t* idx_out, uint64_t seg_cap, uint64_t* settle,
                    LevelState* st, unsigned long long gate, int grid, hipStream_t s) {
  const uint32_t* C32 = reinterpret_cast<const uint32_t*>(C);
  grid = ((grid + kNSeg - 1) / kNSeg) * kNSeg;
  if (level == 0)
    k_resolve<true><<<grid, kBlock, 0, s>>>(0, keys_in, nullptr, C32, keys_out, idx_out, seg_cap, settle,
                                            st, gate);
  else
    k_resolve<false><<<grid, kBlock, 0, s>>>(level, keys_in, idx_in, C32, keys_out, idx_out, seg_cap,
                                             settle, st, gate);
}

void launch_finalize(int level, uint64_t* bits, uint64_t* C, uint64_t cap_words, LevelState* st,
                     unsigned long long gate, int grid, hipStream_t s) {
  k_finalize<<<grid, kBlock, 0, s>>>(level, bits, C, cap_words, st, gate);
}

void launch_mark(int level, const uint64_t* keys, uint64_t seg_cap, uint64_t* bits, uint64_t* C,
                 LevelState* st, unsigned long long gate, int grid, hipStream_t s) {
  grid = ((grid + kNSeg - 1) / kNSeg) * kNSeg;
  k_mark<<<grid, kBlock, 0, s>>>(level, keys, seg_cap, bits, reinterpret_cast<uint32_t*>(C), st, gate);
}

void launch_tail(int big_launched, uint64_t* bits, uint64_t cap_words, uint64_t* C, uint64_t* keys0,
                 uint32_t* idx0, uint64_t* keys1, uint32_t* idx1, uint64_t seg_cap, uint64_t* settle,
                 LevelState* st, hipStream_t s) {
  k_tail<<<1, kTailThreads, 0, s>>>(big_launched, bits, cap_words, reinterpret_cast<uint32_t*>(C), keys0,
                                    idx0, keys1, idx1, seg_cap, settle, st);
}

void launch_rank_scan(const uint64_t* bits, uint64_t cap_words, uint64_t* rank_base,
                      unsigned long long* block_sums, uint64_t max_blocks, LevelState* st,
                      hipStream_t s) {
  uint64_t nb = (cap_words + kScanPerBlock - 1) / kScanPerBlock;
  if (nb > max_blocks) nb = max_blocks;
  if (nb < 1) nb = 1;
  k_scan_reduce<<<(unsigned)nb, kBlock, 0, s>>>(bits, st, nullptr, cap_words, block_sums);
  k_scan_top<<<1, 1024, 0, s>>>(block_sums, st, nullptr, cap_words, nullptr);
  k_scan_down<<<(unsigned)nb, kBlock, 0, s>>>(bits, st, nullptr, cap_words, block_sums, rank_base);
}

void launch_words_scan(const uint64_t* bits, uint64_t words, uint64_t* rank_base,
                       unsigned long long* block_sums, unsigned long long* total, hipStream_t s) {
  // `total` doubles as the word count input: callers store W there first.
  uint64_t nb = (words + kScanPerBlock - 1) / kScanPerBlock;
  if (nb < 1) nb = 1;
  const uint64_t* Wp = reinterpret_cast<const uint64_t*>(total);
  k_scan_reduce<<<(unsigned)nb, kBlock, 0, s>>>(bits, nullptr, Wp, words, block_sums);
  k_scan_top<<<1, 1024, 0, s>>>(block_sums, nullptr, Wp, words, total + 1);
  k_scan_down<<<(unsigned)nb, kBlock, 0, s>>>(bits, nullptr, Wp, words, block_sums, rank_base);
}

void launch_place(uint64_t n, const uint64_t* settle, const uint64_t* fp, const uint64_t* pos,
                  uint64_t pos_base, const uint64_t* bits, const uint64_t* rank_base,
                  uint64_t* fp_out, uint64_t* pos_out, LevelState* st, int grid, hipStream_t s) {
  k_place<<<grid, kBlock, 0, s>>>(n, settle, fp, pos, pos_base, bits, rank_base, fp_out, pos_out, st);
}

void launch_lookup(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const uint64_t* bits,
                   const uint64_t* rank_base, const LevelState* st, const uint64_t* fp,
                   const uint64_t* pos, uint64_t count, uint64_t* result, int grid, hipStream_t s) {
  k_lookup<<<grid, kBlock, 0, s>>>(blob, offsets, n, bits, rank_base, st, fp, pos, count, result);
}

void launch_dist_mark(int level, const uint64_t* keys, uint64_t n_local, uint64_t words, uint32_t* A,
                      uint32_t* C, int grid, hipStream_t s) {
  k_dist_mark<<<grid, kBlock, 0, s>>>(level, keys, n_local, words, level_magic(words), A, C);
}

void launch_dist_hash_mark0(const uint8_t* blob, const uint64_t* offsets, uint64_t n, uint64_t* kh,
                            uint64_t* fp, uint64_t words0, uint32_t* A, uint32_t* C, unsigned* status,
                            int grid, hipStream_t s) {
  k_dist_hash_mark0<<<grid, kBlock, 0, s>>>(blob, offsets, n, kh, fp, words0, level_magic(words0), A, C,
                                            status);
}

void launch_dist_counts(const uint32_t* A, const uint32_t* C, uint64_t positions, uint8_t* cnt, int grid,
                        hipStream_t s) {
  k_dist_counts<<<grid, kBlock, 0, s>>>(const_cast<uint32_t*>(A), const_cast<uint32_t*>(C), positions, cnt);
}

void launch_dist_pack(const uint8_t* sum, uint64_t positions, uint64_t* words_out, int grid, hipStream_t s) {
  k_dist_pack<<<grid, kBlock, 0, s>>>(sum, positions, words_out);
}

void launch_dist_resolve(int level, const uint64_t* keys_in, const uint32_t* idx_in, uint64_t n_local,
                         uint64_t words, uint64_t woff, const uint64_t* bits, uint64_t* keys_out,
                         uint32_t* idx_out, unsigned long long* out_count, uint64_t* settle, int grid,
                         hipStream_t s) {
  k_dist_resolve<<<grid, kBlock, 0, s>>>(level, keys_in, idx_in, n_local, words, level_magic(words), woff,
                                         bits, keys_out, idx_out, out_count, settle);
}

void launch_dist_count_owners(uint64_t n, const uint64_t* settle, const uint64_t* bits,
                              const uint64_t* rank_base, uint64_t per_rank, int nranks,
                              unsigned long long* counts, int grid, hipStream_t s) {
  k_dist_count_owners<<<grid, kBlock, 0, s>>>(n, settle, bits, rank_base, per_rank, nranks, counts);
}

void launch_dist_place(uint64_t n, const uint64_t* settle, const uint64_t* fp, const uint64_t* pos,
                       uint64_t pos_base, const uint64_t* bits, const uint64_t* rank_base,
                       uint64_t per_rank, int nranks, unsigned long long* bucket_fill,
                       const unsigned long long* bucket_off, uint64_t* triples, unsigned*, int grid,
                       hipStream_t s) {
  k_dist_place<<<grid, kBlock, 0, s>>>(n, settle, fp, pos, pos_base, bits, rank_base, per_rank, nranks,
                                       bucket_fill, bucket_off, triples);
}

void launch_dist_unpack(const uint64_t* triples, uint64_t count, uint64_t lo, uint64_t out_n,
                        uint64_t* fp_out, uint64_t* pos_out, unsigned* status, int grid, hipStream_t s) {
  k_dist_unpack<<<grid, kBlock, 0, s>>>(triples, count, lo, out_n, fp_out, pos_out, status);
}

}  // namespace s3imph
