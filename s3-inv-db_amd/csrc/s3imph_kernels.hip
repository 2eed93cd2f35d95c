// s3imph_kernels.hip — hand-written gfx950 kernels for the MPHF build.
//
// The single-GPU build lives in s3imph_binned.hip.  This file holds:
//   k_init_state  per-build level bookkeeping.
//   k_scan_*      word-level rank prefix over all levels (ranks[L] + in-level popcount,
//                 SURVEY App. A.3) — used by the batched lookup.
//   k_lookup      MPHF.Lookup (pkg/format/mphf.go:275-302), batched.
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
// Also samples kSkewSamples evenly spaced key lengths (when offsets are given): a set
// whose longest sampled key exceeds twice the mean + 16 B is hashed length-sorted
// (st->skew), since a wave runs as long as its longest key.
constexpr int kSkewSamples = 1024;  // 4 per thread, all loads in flight together
__global__ void k_init_state(LevelState* st, uint64_t n, uint64_t out_cap, const uint64_t* offsets) {
  __shared__ unsigned long long s_max[kBlock / 64], s_sum[kBlock / 64];
  unsigned long long* p = reinterpret_cast<unsigned long long*>(st);
  for (size_t i = threadIdx.x; i < sizeof(LevelState) / 8; i += blockDim.x) p[i] = 0;
  unsigned long long mx = 0, sm = 0;
  if (offsets && n) {
    unsigned long long a[kSkewSamples / kBlock], b[kSkewSamples / kBlock];
#pragma unroll
    for (int u = 0; u < kSkewSamples / kBlock; ++u) {
      const uint64_t i = (uint64_t)(threadIdx.x + u * kBlock) * n / kSkewSamples;
      a[u] = offsets[i];
      b[u] = offsets[i + 1];
    }
#pragma unroll
    for (int u = 0; u < kSkewSamples / kBlock; ++u) {
      mx = max(mx, b[u] - a[u]);
      sm += b[u] - a[u];
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mx = max(mx, (unsigned long long)__shfl_xor(mx, d));
    sm += __shfl_xor(sm, d);
  }
  if (lane_id() == 0) {
    s_max[threadIdx.x >> 6] = mx;
    s_sum[threadIdx.x >> 6] = sm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t w = level_words(n);
    st->n[0] = n;
    st->words[0] = w;
    st->woff[0] = 0;
    st->woff[1] = w;
    st->magic[0] = level_magic(w);
    st->out_cap = out_cap;
    unsigned long long gm = 0, gs = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
      gm = max(gm, s_max[k]);
      gs += s_sum[k];
    }
    st->skew = offsets && n && gm * kSkewSamples > 2 * gs + 16ull * kSkewSamples;
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
    if (w < W) {  // rank directory: (word, rank before it) side by side, one 16-byte read per probe
      rank_base[2 * w] = v[t];
      rank_base[2 * w + 1] = run;
    }
    run += __popcll(v[t]);
  }
}

// Batched MPHF.Lookup: FNV-1a -> Find -> p -> range check -> FNV-1 == fp[p] -> pos[p].
// Each thread takes two keys at a time (i and i + kBlock, so a wave's offsets stay
// coalesced) and walks their level probes side by side: each probe is one 16-byte read
// of the (word, rank) directory, and the two keys' dependent reads are in flight together.
__device__ __forceinline__ bool probe(const ulonglong2* __restrict__ dir, const LevelState* __restrict__ st,
                                      unsigned L, uint64_t h1, uint64_t& p) {
  const uint64_t x = bb_index(level_seed(L), h1, st->words[L], st->magic[L]);
  const ulonglong2 e = dir[st->woff[L] + (x >> 6)];
  if (!((e.x >> (x & 63)) & 1ull)) return false;
  p = e.y + __popcll(e.x & ((1ull << (x & 63)) - 1));
  return true;
}

__global__ __launch_bounds__(kBlock) void k_lookup(const uint8_t* __restrict__ blob,
                                                   const uint64_t* __restrict__ offsets, uint64_t n,
                                                   const uint64_t* __restrict__ bits,
                                                   const uint64_t* __restrict__ rank_base,
                                                   const LevelState* __restrict__ st,
                                                   const uint64_t* __restrict__ fp,
                                                   const uint64_t* __restrict__ pos, uint64_t count,
                                                   uint64_t* __restrict__ result) {
  const ulonglong2* dir = reinterpret_cast<const ulonglong2*>(rank_base);  // (word, rank) per level word
  const uint64_t stride = 2ull * gridDim.x * kBlock;
  const unsigned nl = st->nlevels;
  for (uint64_t i0 = 2ull * blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += stride) {
    const uint64_t i1 = i0 + kBlock;
    const bool v1 = i1 < n;
    uint64_t a1, a2, b1 = 0, b2 = 0;
    fnv_both_pf(blob, offsets[i0], offsets[i0 + 1], a1, a2);
    if (v1) fnv_both_pf(blob, offsets[i1], offsets[i1 + 1], b1, b2);
    uint64_t pa = ~0ull, pb = ~0ull;
    bool da = count == 0, db = count == 0 || !v1;  // done: found, or nothing to look in
    for (unsigned L = 0; L < nl && !(da && db); ++L) {
      uint64_t qa = 0, qb = 0;
      const bool fa = !da && probe(dir, st, L, a1, qa);
      const bool fb = !db && probe(dir, st, L, b1, qb);
      if (fa) {
        pa = qa;
        da = true;
      }
      if (fb) {
        pb = qb;
        db = true;
      }
    }
    const bool ha = pa < count, hb = pb < count;
    const uint64_t fa = ha ? fp[pa] : 0, fb = hb ? fp[pb] : 0;
    const uint64_t oa = ha && fa == a2 ? pos[pa] : ~0ull;
    const uint64_t ob = hb && fb == b2 ? pos[pb] : ~0ull;
    result[i0] = oa;
    if (v1) result[i1] = ob;
  }
}

// u32 <-> u64 conversion of a staged host array (offsets in, identity positions out):
// one element per thread per grid stride (HBM-bound; a few µs per 10M elements).
__global__ __launch_bounds__(256) void k_widen32(const uint32_t* __restrict__ in, uint64_t* __restrict__ out,
                                                 uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}
__global__ __launch_bounds__(256) void k_narrow32(const uint64_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    out[i] = (uint32_t)in[i];
}

// Key lengths (u16, the host's narrowest form of the offsets: 2 B per key over PCIe instead
// of 4 or 8) back to offsets: offsets[0] = 0, offsets[i + 1] = offsets[i] + len[i].  Three
// passes over 16384-key blocks: block sums, one-block scan of the sums, block-local scans.
constexpr int kLsT = 1024, kLsPer = 16;
constexpr uint64_t kLsBlock = (uint64_t)kLsT * kLsPer;
__device__ __forceinline__ uint64_t ls_block_exscan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t s_w[kLsT / 64];
  const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
  for (int w = 0; w < kLsT / 64; ++w) {
    if ((unsigned)w < wave) pre += s_w[w];
    tot += s_w[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}
// a thread's 16 consecutive lengths (two 16-byte loads when the block is whole)
__device__ __forceinline__ void ls_load(const uint16_t* __restrict__ len, uint64_t n, uint64_t i0, unsigned (&v)[kLsPer]) {
  if (i0 + kLsPer <= n) {
    const uint4 a = *reinterpret_cast<const uint4*>(len + i0), b = *reinterpret_cast<const uint4*>(len + i0 + 8);
    const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[2 * q] = w[q] & 0xffffu;
      v[2 * q + 1] = w[q] >> 16;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kLsPer; ++q) v[q] = i0 + q < n ? len[i0 + q] : 0u;
  }
}
__global__ __launch_bounds__(kLsT) void k_len_sums(const uint16_t* __restrict__ len, uint64_t n,
                                                   uint64_t* __restrict__ sums) {
  unsigned v[kLsPer];
  ls_load(len, n, blockIdx.x * kLsBlock + (uint64_t)threadIdx.x * kLsPer, v);
  uint64_t t = 0;
#pragma unroll
  for (int q = 0; q < kLsPer; ++q) t += v[q];
  uint64_t tot;
  (void)ls_block_exscan(t, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kLsT) void k_len_scan_sums(uint64_t* __restrict__ sums, uint64_t nb) {
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nb; b0 += kLsT) {
    const uint64_t i = b0 + threadIdx.x;
    const uint64_t v = i < nb ? sums[i] : 0;
    uint64_t tot;
    const uint64_t ex = ls_block_exscan(v, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
}
__global__ __launch_bounds__(kLsT) void k_len_offsets(const uint16_t* __restrict__ len, uint64_t n,
                                                      const uint64_t* __restrict__ sums, uint64_t* __restrict__ out) {
  unsigned v[kLsPer];
  const uint64_t i0 = blockIdx.x * kLsBlock + (uint64_t)threadIdx.x * kLsPer;
  ls_load(len, n, i0, v);
  uint64_t t = 0;
#pragma unroll
  for (int q = 0; q < kLsPer; ++q) t += v[q];
  uint64_t tot;
  uint64_t o = sums[blockIdx.x] + ls_block_exscan(t, &tot);
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
  for (int q = 0; q < kLsPer; ++q) {
    o += v[q];
    if (i0 + q < n) out[i0 + q + 1] = o;
  }
}

// FNV-1a hash of every key (mphf.go:349-369), nothing else: the error path's recount of
// the ORIGINAL key hashes (the level-0 pipeline keeps them only in its own layouts).
__global__ __launch_bounds__(kBlock) void k_key_hash(const uint8_t* __restrict__ blob,
                                                     const uint64_t* __restrict__ offsets, uint64_t n,
                                                     uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    uint64_t a, b;
    fnv_both_pf(blob, offsets[i], offsets[i + 1], a, b);
    out[i] = a;
  }
}

}  // namespace

// ================================ launchers =======================================
int default_grid(uint64_t work, int block) {
  uint64_t g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_init_state(LevelState* st, uint64_t n, uint64_t out_cap, hipStream_t s, const uint64_t* offsets) {
  k_init_state<<<1, kBlock, 0, s>>>(st, n, out_cap, offsets);
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

void launch_lookup(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const uint64_t* bits,
                   const uint64_t* rank_base, const LevelState* st, const uint64_t* fp,
                   const uint64_t* pos, uint64_t count, uint64_t* result, int grid, hipStream_t s) {
  k_lookup<<<grid, kBlock, 0, s>>>(blob, offsets, n, bits, rank_base, st, fp, pos, count, result);
}

void launch_widen32(const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
  if (n) k_widen32<<<(unsigned)std::min<uint64_t>(8192, (n + 255) / 256), 256, 0, s>>>(in, out, n);
}
void launch_narrow32(const uint64_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (n) k_narrow32<<<(unsigned)std::min<uint64_t>(8192, (n + 255) / 256), 256, 0, s>>>(in, out, n);
}

uint64_t len16_scratch_words(uint64_t n) { return (n + kLsBlock - 1) / kLsBlock; }
void launch_len16_offsets(const uint16_t* len, uint64_t n, uint64_t* sums, uint64_t* out, hipStream_t s) {
  const uint64_t nb = len16_scratch_words(n);
  if (!nb) return;
  k_len_sums<<<(unsigned)nb, kLsT, 0, s>>>(len, n, sums);
  k_len_scan_sums<<<1, kLsT, 0, s>>>(sums, nb);
  k_len_offsets<<<(unsigned)nb, kLsT, 0, s>>>(len, n, sums, out);
}

void launch_key_hashes(const uint8_t* blob, const uint64_t* offsets, uint64_t n, uint64_t* out, hipStream_t s) {
  if (n) k_key_hash<<<(unsigned)std::min<uint64_t>(4096, (n + kBlock - 1) / kBlock), kBlock, 0, s>>>(blob, offsets, n, out);
}

}  // namespace s3imph
