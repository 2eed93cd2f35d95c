// s3imph_kernels.hip — hand-written gfx950 kernels for the MPHF build.
//
// The single-GPU build lives in s3imph_binned.hip.  This file holds:
//   k_init_state  per-build level bookkeeping.
//   k_scan_*      word-level rank prefix over all levels (ranks[L] + in-level popcount,
//                 SURVEY App. A.3) — used by the batched lookup and the multi-GPU build.
//   k_lookup      MPHF.Lookup (pkg/format/mphf.go:275-302), batched.
//   k_dist_*      the multi-GPU (RCCL) level build: per-level count exchange and the
//                 output exchange (s3imph_build.hip, build_dist).
//
// No MFMA anywhere: this is 64-bit integer hashing and bit-vector work.  Every
// level bit vector depends only on the SET of keys active at that level, so the
// atomic-OR construction is bit-exact whatever the schedule.
#include <hip/hip_runtime.h>

#include "s3imph_device.h"
#include "s3imph_internal.h"

namespace s3imph {

namespace {

constexpr int kBlock = 256;

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

constexpr int kResolveKPT = 4;  // keys per thread per block tile in k_dist_resolve

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
