// s3imph_finalize.hip — the rest of IndexBuilder.Finalize on the GPU:
// the arrays the reference writes beside the MPHF, computed from the same sorted prefix
// blob the MPHF build reads.
//
// Reference (/root/reference/pkg/extsort/indexbuild.go, pkg/format/depthindex.go):
//   depth.u32                 row.Depth per prefix in Add order (indexbuild.go:185); the
//                             aggregator's Depth is the number of '/' in the prefix
//                             (aggregator.go:44-60) — used when the caller passes none;
//   subtree_end.u64           the ancestor stack of indexbuild.go:154-248: a prefix's node
//                             is closed by the first later prefix it is not a byte prefix
//                             of (every entry under it on the stack is a prefix of it, so
//                             nothing closes it earlier) and its subtree ends just before;
//                             Finalize closes the rest at N - 1 (:393-395, written :474-487);
//   max_depth_in_subtree.u32  the deepest depth of that range (closeTopNode propagates the
//                             maximum to the parent, :241-245; written :489-503);
//   depth_offsets.u64,        DepthIndexBuilder.Build (depthindex.go:32-96): positions
//   depth_positions.u64       grouped by depth, ascending inside a depth, maxDepth+2 offsets.
//
// GPU formulation.  Keys are byte-sorted, so the prefixes that extend key i form the run
// right after it: subtree_end(i) = the first t >= i with lcp(t, t+1) < len(i), where
// lcp(t, t+1) is the longest common prefix of neighbours (lcp(N-1, N) := -1).  One pass
// computes depth, len and lcp per key (two-level block minima / depth maxima beside it);
// a second answers each key's "first lcp below my length" and the depth maximum over the
// run by walking the block hierarchy; the depth index is a stable radix sort of the
// positions by depth (rocPRIM, bits = bit width of maxDepth) plus a boundary pass.  All
// integer work, HBM-bound: ΣL·2 + 32 B per key for the pass over the keys.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "s3imph_ctx.h"
#include "s3imph_device.h"

namespace s3imph {

int write_finalize_files(const std::string& dir, const uint32_t* depth, const uint64_t* subtree_end,
                         const uint32_t* max_depth_sub, const uint64_t* depth_offsets, uint64_t n_offsets,
                         const uint64_t* depth_positions, uint64_t n, std::string* msg);
s3imph_ctx* default_ctx(int device, std::string* msg);

namespace {

constexpr int kFB = 1024;   // keys per block (one block-minimum of lcp / maximum of depth)
constexpr int kFS = 1024;   // blocks per superblock

// 8 key bytes from blob address a (any alignment): two aligned words and a byte funnel.
// The blob is readable up to end8 = round_up(offsets[n], 8).
__device__ __forceinline__ uint64_t load8(const uint8_t* blob, uint64_t a, uint64_t end8) {
  const uint64_t al = a & ~7ull;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(blob + al);
  const uint64_t lo = w[0];
  const uint64_t hi = (a & 7) && al + 8 < end8 ? w[1] : 0;
  return (a & 7) ? funnel_bytes(lo, hi, (unsigned)(a & 7)) : lo;
}

// exact per-byte zero test: high bit of each byte of the result set iff that byte of x is 0
__device__ __forceinline__ uint64_t zero_bytes(uint64_t x) {
  constexpr uint64_t k7f = 0x7f7f7f7f7f7f7f7full;
  const uint64_t t = (x & k7f) + k7f;
  return ~(t | x | k7f);
}

// Pass 1: per key depth ('/' count, or the caller's), lcp with the next key; block
// minima of lcp (int32; -1 marks the last key) and maxima of depth; the global maxDepth.
__global__ __launch_bounds__(kFB) void k_fin_keys(const uint8_t* __restrict__ blob,
                                                  const uint64_t* __restrict__ offsets,
                                                  const uint32_t* __restrict__ depths_in, uint64_t n,
                                                  uint32_t* __restrict__ depth, int32_t* __restrict__ lcp,
                                                  int32_t* __restrict__ bmin, uint32_t* __restrict__ bmax,
                                                  unsigned* __restrict__ maxd) {
  __shared__ int32_t s_min[kFB / 64];
  __shared__ uint32_t s_max[kFB / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kFB + threadIdx.x;
  const uint64_t end8 = (offsets[n] + 7) & ~7ull;
  int32_t l = 0x7fffffff;  // neutral for the block minimum
  uint32_t d = 0;
  if (i < n) {
    const uint64_t b0 = offsets[i], b1 = offsets[i + 1], len = b1 - b0;
    if (depths_in) {
      d = depths_in[i];
    } else {
      for (uint64_t k = 0; k < len; k += 8) {
        uint64_t z = zero_bytes(load8(blob, b0 + k, end8) ^ 0x2f2f2f2f2f2f2f2full);  // '/' bytes
        if (len - k < 8) z &= (1ull << (8 * (len - k))) - 1;
        d += (uint32_t)__popcll(z & 0x8080808080808080ull);
      }
    }
    depth[i] = d;
    if (i + 1 < n) {
      const uint64_t c0 = b1, m = min(len, offsets[i + 2] - c0);
      uint64_t k = 0;
      for (; k < m; k += 8) {
        const uint64_t x = load8(blob, b0 + k, end8) ^ load8(blob, c0 + k, end8);
        if (x) {
          k += (uint64_t)(__builtin_ctzll(x) >> 3);
          break;
        }
      }
      l = (int32_t)min(k, m);
    } else {
      l = -1;
    }
    lcp[i] = l;
  }
  int32_t mn = l;
  uint32_t mx = d;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = min(mn, __shfl_xor(mn, o));
    mx = max(mx, __shfl_xor(mx, o));
  }
  if (lane_id() == 0) {
    s_min[threadIdx.x >> 6] = mn;
    s_max[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kFB / 64; ++w) {
      mn = min(mn, s_min[w]);
      mx = max(mx, s_max[w]);
    }
    mn = min(mn, s_min[0]);
    mx = max(mx, s_max[0]);
    bmin[blockIdx.x] = mn;
    bmax[blockIdx.x] = mx;
    atomicMax(maxd, mx);
  }
}

// Pass 1, LDS-staged (byte-aligned blobs, the default): a workgroup walks its contiguous
// key range in rounds of up to 2 kFinT keys whose bytes (<= kFinBB) come in with coalesced
// 16-byte loads and are staged in LDS, as the level-0 hash does; each lane then counts its
// keys' '/' bytes and compares each key with its successor from LDS words.  The round's
// last key meets its successor (the next round's first key) through global loads.
constexpr int kFinT = 256;
constexpr int kFinBB = 32 << 10;
constexpr int kFinGrid = 4096;

// 8 bytes at byte offset o of the LDS window (16 readable bytes past its end)
__device__ __forceinline__ uint64_t lds8(const uint64_t* sw, unsigned o) {
  const unsigned s8 = o & 7u;
  const uint64_t lo = sw[o >> 3];
  return s8 ? funnel_bytes(lo, sw[(o >> 3) + 1], s8) : lo;
}

__global__ __launch_bounds__(kFinT) void k_fin_keys_lds(const uint8_t* __restrict__ blob,
                                                        const uint64_t* __restrict__ offsets,
                                                        const uint32_t* __restrict__ depths_in, uint64_t n,
                                                        uint32_t* __restrict__ depth, int32_t* __restrict__ lcp) {
  constexpr int G = 2 * kFinT;
  constexpr int KW = (kFinBB / 16 + kFinT - 1) / kFinT;
  __shared__ uint64_t sw[kFinBB / 8 + 4];
  __shared__ unsigned s_cnt[kFinT / 64];
  const unsigned tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  uint64_t g = (uint64_t)blockIdx.x * per;
  const uint64_t gend = min(n, g + per);
  const uint64_t end8 = (offsets[n] + 7) & ~7ull;
  // the round at r0: key bounds and its window chunks in registers (issued one round ahead)
  uint64_t kb0[2], kb1[2], wlo = 0, wend = 0;
  bool kin[2];
  uint4 wr[KW];
  auto prefetch = [&](uint64_t r0) {
    const uint64_t last = min(gend, r0 + G);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t i = r0 + tid + (unsigned)h * kFinT;
      kin[h] = i < last;
      kb0[h] = kin[h] ? offsets[i] : 0;
      kb1[h] = kin[h] ? offsets[i + 1] : 0;
    }
    wlo = uniform64(offsets[r0] & ~15ull);
    wend = uniform64(min((offsets[last] + 15) & ~15ull, wlo + (uint64_t)kFinBB));
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {
      const uint64_t a = wlo + 16ull * (tid + (unsigned)kk * kFinT);
      wr[kk] = make_uint4(0, 0, 0, 0);
      if (a < wend) {
        if (a + 16 <= end8) {
          wr[kk] = *reinterpret_cast<const uint4*>(blob + a);
        } else {
          const uint2 hh = *reinterpret_cast<const uint2*>(blob + a);
          wr[kk].x = hh.x;
          wr[kk].y = hh.y;
        }
      }
    }
  };
  if (g < gend) prefetch(g);
  while (g < gend) {
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {
      const unsigned c = tid + (unsigned)kk * kFinT;
      if (wlo + 16ull * c < wend) {
        sw[2 * c] = (uint64_t)wr[kk].x | ((uint64_t)wr[kk].y << 32);
        sw[2 * c + 1] = (uint64_t)wr[kk].z | ((uint64_t)wr[kk].w << 32);
      }
    }
    if (tid < 4) sw[(wend - wlo) / 8 + tid] = 0;  // read slack past the window
    // keys whose bytes all lie in the window: a prefix of the round (offsets ascend)
    bool fits[2];
    unsigned mine = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      fits[h] = kin[h] && kb1[h] - wlo <= (uint64_t)(wend - wlo);
      mine += (unsigned)__popcll(__ballot(fits[h]));
    }
    if (lane == 0) s_cnt[wave] = mine;
    __syncthreads();
    unsigned m = 0;
#pragma unroll
    for (int w = 0; w < kFinT / 64; ++w) m += s_cnt[w];
    if (m == 0) m = 1;  // a first key longer than the window: taken from global memory
    const uint64_t r0 = g, rwlo = wlo, rwend = wend;
    const uint64_t t0[2] = {kb0[0], kb0[1]}, t1[2] = {kb1[0], kb1[1]};
    g += m;
    if (g < gend) prefetch(g);  // the next round's loads land while this one is compared
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned idx = tid + (unsigned)h * kFinT;
      const uint64_t i = r0 + idx;
      if (idx < m && i < n) {
        const uint64_t b0 = t0[h], b1 = t1[h], len = b1 - b0;
        const bool in_w = fits[h];
        auto key8 = [&](uint64_t k8) -> uint64_t {  // 8 bytes of key i from byte k8
          return in_w ? lds8(sw, (unsigned)(b0 - rwlo + k8)) : load8(blob, b0 + k8, end8);
        };
        uint32_t d = 0;
        if (depths_in) {
          d = depths_in[i];
        } else {
          for (uint64_t k8 = 0; k8 < len; k8 += 8) {
            uint64_t z = zero_bytes(key8(k8) ^ 0x2f2f2f2f2f2f2f2full);
            if (len - k8 < 8) z &= (1ull << (8 * (len - k8))) - 1;
            d += (uint32_t)__popcll(z & 0x8080808080808080ull);
          }
        }
        depth[i] = d;
        int32_t l = -1;
        if (i + 1 < n) {
          // the successor: in the window when it is one of this round's keys that fit
          const uint64_t c0 = b1, c1 = offsets[i + 2], mm = min(len, c1 - c0);
          const bool nin = in_w && idx + 1 < m && c1 - rwlo <= (uint64_t)(rwend - rwlo);
          uint64_t k8 = 0;
          for (; k8 < mm; k8 += 8) {
            const uint64_t y = nin ? lds8(sw, (unsigned)(c0 - rwlo + k8)) : load8(blob, c0 + k8, end8);
            const uint64_t x = key8(k8) ^ y;
            if (x) {
              k8 += (uint64_t)(__builtin_ctzll(x) >> 3);
              break;
            }
          }
          l = (int32_t)min(k8, mm);
        }
        lcp[i] = l;
      }
    }
    __syncthreads();  // the window is reused by the next round
  }
}

// Block minima of lcp / maxima of depth from the arrays pass 1 wrote: one 1024-key block
// per 256-thread workgroup, four keys per lane in 16-byte loads (a 1024-thread workgroup per
// block was latency-bound: 1.13 ms on C3).  The global maxDepth is taken per superblock.
constexpr int kFBT = kFB / 4;
__global__ __launch_bounds__(kFBT) void k_fin_blocks(const uint32_t* __restrict__ depth,
                                                     const int32_t* __restrict__ lcp, uint64_t n,
                                                     int32_t* __restrict__ bmin, uint32_t* __restrict__ bmax) {
  __shared__ int32_t s_min[kFBT / 64];
  __shared__ uint32_t s_max[kFBT / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kFB + 4ull * threadIdx.x;
  int32_t mn = 0x7fffffff;
  uint32_t mx = 0;
  if (i + 4 <= n && ((uintptr_t)depth & 15) == 0) {  // lcp is our scratch (aligned); depth the caller's
    const int4 l4 = *reinterpret_cast<const int4*>(lcp + i);
    const uint4 d4 = *reinterpret_cast<const uint4*>(depth + i);
    mn = min(min(l4.x, l4.y), min(l4.z, l4.w));
    mx = max(max(d4.x, d4.y), max(d4.z, d4.w));
  } else {
    const uint64_t qe = i + 4 < n ? i + 4 : n;  // this lane's four keys only
    for (uint64_t q = i; q < qe; ++q) {
      mn = min(mn, lcp[q]);
      mx = max(mx, depth[q]);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = min(mn, __shfl_xor(mn, o));
    mx = max(mx, __shfl_xor(mx, o));
  }
  if (lane_id() == 0) {
    s_min[threadIdx.x >> 6] = mn;
    s_max[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < kFBT / 64; ++w) {
      mn = min(mn, s_min[w]);
      mx = max(mx, s_max[w]);
    }
    bmin[blockIdx.x] = mn;
    bmax[blockIdx.x] = mx;
  }
}

// Pass 1b: superblock minima / maxima over the block arrays (one block per superblock).
__global__ __launch_bounds__(kFS) void k_fin_super(const int32_t* __restrict__ bmin, const uint32_t* __restrict__ bmax,
                                                   uint64_t nb, int32_t* __restrict__ smin,
                                                   uint32_t* __restrict__ smax, unsigned* __restrict__ maxd) {
  __shared__ int32_t s_min[kFS / 64];
  __shared__ uint32_t s_max[kFS / 64];
  const uint64_t b = (uint64_t)blockIdx.x * kFS + threadIdx.x;
  int32_t mn = b < nb ? bmin[b] : 0x7fffffff;
  uint32_t mx = b < nb ? bmax[b] : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = min(mn, __shfl_xor(mn, o));
    mx = max(mx, __shfl_xor(mx, o));
  }
  if (lane_id() == 0) {
    s_min[threadIdx.x >> 6] = mn;
    s_max[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < kFS / 64; ++w) {
      mn = min(mn, s_min[w]);
      mx = max(mx, s_max[w]);
    }
    smin[blockIdx.x] = mn;
    smax[blockIdx.x] = mx;
    if (maxd) atomicMax(maxd, mx);  // one atomic per superblock
  }
}

// Pass 2: subtree_end(i) = first t >= i with lcp[t] < len(i) (exists: lcp[n-1] = -1),
// found element -> block -> superblock -> back down; then max depth over [i, t] by the
// same hierarchy.  Leaves (most keys) stop at t = i after one load.
__global__ __launch_bounds__(256) void k_fin_subtree(const uint64_t* __restrict__ offsets, uint64_t n,
                                                     const uint32_t* __restrict__ depth,
                                                     const int32_t* __restrict__ lcp,
                                                     const int32_t* __restrict__ bmin,
                                                     const uint32_t* __restrict__ bmax,
                                                     const int32_t* __restrict__ smin,
                                                     const uint32_t* __restrict__ smax, uint64_t nb, uint64_t nsb,
                                                     uint64_t* __restrict__ subtree_end,
                                                     uint32_t* __restrict__ max_depth_sub) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t L = (int64_t)(offsets[i + 1] - offsets[i]);
  auto scan = [&](uint64_t lo, uint64_t hi) -> uint64_t {  // first t in [lo, hi) with lcp < L, or hi
    for (uint64_t t = lo; t < hi; ++t)
      if ((int64_t)lcp[t] < L) return t;
    return hi;
  };
  const uint64_t b = i / kFB;
  uint64_t t = scan(i, min(n, (b + 1) * kFB));
  if (t == min(n, (b + 1) * kFB)) {
    const uint64_t sb = b / kFS;
    uint64_t bb = b + 1;
    const uint64_t bend = min(nb, (sb + 1) * kFS);
    while (bb < bend && (int64_t)bmin[bb] >= L) ++bb;
    if (bb == bend) {
      uint64_t s = sb + 1;
      while (s < nsb && (int64_t)smin[s] >= L) ++s;
      bb = s * kFS;  // s < nsb: lcp[n-1] = -1 lies in the last superblock
      while ((int64_t)bmin[bb] >= L) ++bb;
    }
    t = scan(bb * kFB, min(n, (bb + 1) * kFB));
  }
  subtree_end[i] = t;
  // max depth over [i, t]
  uint32_t mx = 0;
  const uint64_t bt = t / kFB;
  if (bt == b) {
    for (uint64_t q = i; q <= t; ++q) mx = max(mx, depth[q]);
  } else {
    for (uint64_t q = i; q < (b + 1) * kFB; ++q) mx = max(mx, depth[q]);
    uint64_t bb = b + 1;
    while (bb < bt) {
      if (bb % kFS == 0 && bb + kFS <= bt) {  // a whole superblock
        mx = max(mx, smax[bb / kFS]);
        bb += kFS;
      } else {
        mx = max(mx, bmax[bb]);
        ++bb;
      }
    }
    for (uint64_t q = bt * kFB; q <= t; ++q) mx = max(mx, depth[q]);
  }
  max_depth_sub[i] = mx;
}

// depth_offsets from the depth-sorted keys: offset of depth d = first sorted index whose
// depth is >= d; entries up to maxDepth + 1 (= n).
__global__ __launch_bounds__(256) void k_fin_doff(const uint32_t* __restrict__ sdepth, uint64_t n, uint32_t maxd,
                                                  uint64_t* __restrict__ doff) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t prev = i ? (int64_t)sdepth[i - 1] : -1;
  for (int64_t d = prev + 1; d <= (int64_t)sdepth[i]; ++d) doff[d] = i;
  if (i == n - 1)
    for (uint64_t d = (uint64_t)sdepth[i] + 1; d <= (uint64_t)maxd + 1; ++d) doff[d] = n;
}

}  // namespace

// Scratch of the finalize pass, kept in the context and grown as needed.
struct FinScratch {
  int32_t* lcp = nullptr;
  uint32_t* sdepth = nullptr;
  int32_t* bmin = nullptr;
  uint32_t* bmax = nullptr;
  int32_t* smin = nullptr;
  uint32_t* smax = nullptr;
  unsigned* maxd = nullptr;
  void* tmp = nullptr;
  size_t tmp_cap = 0;
  uint64_t cap = 0;
  void release() {
    dfree(lcp);
    dfree(sdepth);
    dfree(bmin);
    dfree(bmax);
    dfree(smin);
    dfree(smax);
    dfree(maxd);
    dfree(tmp);
    tmp_cap = 0;
    cap = 0;
  }
};

void fin_scratch_free(s3imph_ctx* c) {
  if (c->fin) {
    c->fin->release();
    delete c->fin;
    c->fin = nullptr;
  }
}

// The five arrays for n keys already in HBM (blob readable to round_up(offsets[n], 8)).
// Returns S3IMPH_ERR_INVALID with *max_depth set when doff_cap < maxDepth + 2.
int finalize_device(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths, uint64_t n,
                    uint32_t* depth, uint64_t* subtree_end, uint32_t* max_depth_sub, uint64_t* depth_positions,
                    uint64_t* depth_offsets, uint64_t doff_cap, uint32_t* max_depth, hipStream_t s, std::string* msg) {
  *max_depth = 0;
  if (n == 0) {
    if (doff_cap < 2) {
      *msg = "finalize: depth_offsets needs 2 entries";
      return S3IMPH_ERR_INVALID;
    }
    const uint64_t z[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(depth_offsets, z, sizeof z, hipMemcpyHostToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    return S3IMPH_OK;
  }
  if (n > 0xffffffffull) {
    *msg = "finalize: more than 2^32-1 keys on one GPU";
    return S3IMPH_ERR_INVALID;
  }
  if (!c->fin) c->fin = new FinScratch();
  FinScratch& f = *c->fin;
  const uint64_t nb = (n + kFB - 1) / kFB, nsb = (nb + kFS - 1) / kFS;
  if (n > f.cap) {
    f.release();
    dalloc(f.lcp, n);
    dalloc(f.sdepth, n);
    dalloc(f.bmin, nb);
    dalloc(f.bmax, nb);
    dalloc(f.smin, nsb);
    dalloc(f.smax, nsb);
    dalloc(f.maxd, 1);
    f.cap = n;
  }
  HIPCHECK(hipMemsetAsync(f.maxd, 0, sizeof(unsigned), s));
  const bool staged = ((uintptr_t)blob & 15) == 0;
  if (staged) {
    k_fin_keys_lds<<<(unsigned)std::min<uint64_t>(kFinGrid, (n + 2 * kFinT - 1) / (2 * kFinT)), kFinT, 0, s>>>(
        blob, offsets, depths, n, depth, f.lcp);
    k_fin_blocks<<<(unsigned)nb, kFBT, 0, s>>>(depth, f.lcp, n, f.bmin, f.bmax);
  } else {  // a caller's unaligned blob: per-lane unaligned loads
    k_fin_keys<<<(unsigned)nb, kFB, 0, s>>>(blob, offsets, depths, n, depth, f.lcp, f.bmin, f.bmax, f.maxd);
  }
  k_fin_super<<<(unsigned)nsb, kFS, 0, s>>>(f.bmin, f.bmax, nb, f.smin, f.smax, staged ? f.maxd : nullptr);
  k_fin_subtree<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(offsets, n, depth, f.lcp, f.bmin, f.bmax, f.smin, f.smax,
                                                           nb, nsb, subtree_end, max_depth_sub);
  HIPCHECK(hipGetLastError());
  unsigned md = 0;
  HIPCHECK(hipMemcpyAsync(&md, f.maxd, sizeof md, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  *max_depth = md;
  if (doff_cap < (uint64_t)md + 2) {
    *msg = "finalize: depth_offsets needs " + std::to_string((uint64_t)md + 2) + " entries";
    return S3IMPH_ERR_INVALID;
  }
  // depth index: positions stably sorted by depth (keys = depth, values = 0..n-1)
  unsigned bits = 1;
  while (bits < 32 && (md >> bits)) ++bits;
  rocprim::counting_iterator<uint64_t> iota(0);
  size_t need = 0;
  HIPCHECK(rocprim::radix_sort_pairs(nullptr, need, depth, f.sdepth, iota, depth_positions, n, 0, bits, s));
  if (need > f.tmp_cap) {
    dfree(f.tmp);
    HIPCHECK(hipMalloc(&f.tmp, need));
    f.tmp_cap = need;
  }
  HIPCHECK(rocprim::radix_sort_pairs(f.tmp, need, depth, f.sdepth, iota, depth_positions, n, 0, bits, s));
  k_fin_doff<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(f.sdepth, n, md, depth_offsets);
  HIPCHECK(hipGetLastError());
  return S3IMPH_OK;
}

// Host-memory finalize: H2D of the prefix blob (and depths), the device pass, D2H, and the
// five files in out_dir with the reference's S3ID framing.
int finalize_from_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths, uint64_t n,
                       const std::string& dir, std::string* msg) {
  std::vector<uint32_t> depth(n), maxds(n);
  std::vector<uint64_t> send(n), dpos(n), doff;
  if (n) {
    s3imph_ctx* c = default_ctx(device, msg);
    if (!c) return S3IMPH_ERR_HIP;
    std::lock_guard<std::mutex> lk(c->mu);
    try {
      HIPCHECK(hipSetDevice(c->device));
      hipStream_t s = c->own_stream;
      const uint64_t b0 = offsets[0], nbytes = offsets[n] - b0;
      uint8_t* d_blob = nullptr;
      uint64_t *d_offs = nullptr, *d_send = nullptr, *d_dpos = nullptr, *d_doff = nullptr;
      uint32_t *d_depth = nullptr, *d_maxds = nullptr, *d_din = nullptr;
      struct Guard {
        std::vector<void*> p;
        ~Guard() {
          for (void* q : p)
            if (q) (void)hipFree(q);
        }
      } g;
      dalloc(d_blob, ((nbytes + 7) & ~7ull) + 16);
      g.p.push_back(d_blob);
      dalloc(d_offs, n + 1);
      g.p.push_back(d_offs);
      dalloc(d_send, n);
      g.p.push_back(d_send);
      dalloc(d_dpos, n);
      g.p.push_back(d_dpos);
      dalloc(d_depth, n);
      g.p.push_back(d_depth);
      dalloc(d_maxds, n);
      g.p.push_back(d_maxds);
      if (depths) {
        dalloc(d_din, n);
        g.p.push_back(d_din);
        HIPCHECK(hipMemcpy(d_din, depths, n * 4, hipMemcpyHostToDevice));
      }
      HIPCHECK(hipMemcpy(d_blob, blob + b0, nbytes, hipMemcpyHostToDevice));
      staged_copy(c, true, d_offs, offsets, (n + 1) * 8, b0);
      uint64_t cap = 64;
      uint32_t md = 0;
      for (int attempt = 0; attempt < 2; ++attempt) {
        dalloc(d_doff, cap);
        g.p.push_back(d_doff);
        int rc = finalize_device(c, d_blob, d_offs, d_din, n, d_depth, d_send, d_maxds, d_dpos, d_doff, cap, &md, s,
                                 msg);
        if (rc == S3IMPH_OK) break;
        if (rc != S3IMPH_ERR_INVALID || attempt) return rc;
        cap = (uint64_t)md + 2;
        g.p.back() = nullptr;
        dfree(d_doff);
      }
      doff.resize((uint64_t)md + 2);
      HIPCHECK(hipStreamSynchronize(s));
      HIPCHECK(hipMemcpy(doff.data(), d_doff, doff.size() * 8, hipMemcpyDeviceToHost));
      staged_copy(c, false, depth.data(), d_depth, n * 4);
      staged_copy(c, false, maxds.data(), d_maxds, n * 4);
      staged_copy(c, false, send.data(), d_send, n * 8);
      staged_copy(c, false, dpos.data(), d_dpos, n * 8);
    } catch (const Fail& e) {
      *msg = e.msg;
      return e.code;
    }
  } else {
    doff = {0, 0};  // writeEmpty-like: maxDepth 0 -> offsets [0, 0]
  }
  return write_finalize_files(dir, depth.data(), send.data(), maxds.data(), doff.data(), doff.size(), dpos.data(), n,
                              msg);
}

}  // namespace s3imph

using namespace s3imph;

extern "C" {

int s3imph_finalize_index_host(int device, const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths,
                               uint64_t n, const char* out_dir, char* err, size_t errlen) {
  if (!out_dir || (n && (!blob || !offsets))) return S3IMPH_ERR_INVALID;
  std::string msg;
  try {
    const int rc = finalize_from_host(device, blob, offsets, depths, n, out_dir, &msg);
    if (rc != S3IMPH_OK) set_err(err, errlen, msg);
    return rc;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "finalize index: out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
}

int s3imph_finalize_index_device(s3imph_ctx* c, const uint8_t* d_blob, const uint64_t* d_offsets,
                                 const uint32_t* d_depths, uint64_t n, uint32_t* d_depth, uint64_t* d_subtree_end,
                                 uint32_t* d_max_depth_in_subtree, uint64_t* d_depth_positions,
                                 uint64_t* d_depth_offsets, uint64_t offsets_cap, uint32_t* max_depth, void* stream) {
  if (!c || !max_depth || !d_depth_offsets ||
      (n && (!d_blob || !d_offsets || !d_depth || !d_subtree_end || !d_max_depth_in_subtree || !d_depth_positions)))
    return S3IMPH_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  std::string msg;
  try {
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->own_stream;
    int rc = finalize_device(c, d_blob, d_offsets, d_depths, n, d_depth, d_subtree_end, d_max_depth_in_subtree,
                             d_depth_positions, d_depth_offsets, offsets_cap, max_depth, s, &msg);
    if (rc == S3IMPH_OK) HIPCHECK(hipStreamSynchronize(s));
    c->last_msg = msg;
    return rc;
  } catch (const Fail& f) {
    c->last_msg = f.msg;
    return f.code;
  }
}

}  // extern "C"
