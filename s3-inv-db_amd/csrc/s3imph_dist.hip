// s3imph_dist.hip — kernels of the multi-GPU build (one process per GPU, RCCL over xGMI).
//
// Decomposition: position-range ownership.  At a distributed level L (global key count
// n_L, words_L = ceil(2 n_L / 64)) rank r owns the level's words
// [r*dS, min((r+1)*dS, words_L)), dS = ceil(words_L / P).  Every rank routes its
// active records (k, f, p) to the owner of their level-L position (k_route: one
// all-to-all of 24-byte records per level), and each owner runs the single-GPU tile
// pipeline (s3imph_binned.hip) over its own position range.  Its settled keys get
// consecutive LOCAL output slots, so each (level, rank) pair is one contiguous segment
// of mph_fp / mph_pos whose global start is a prefix sum over (level, rank) counts:
// the same p = ranks[L] + popcount(A_L[0:x)) a single GPU computes.
// Collided records stay on their owner and are routed again at the next level.  Once a
// level is small the remaining records are all-gathered and every rank finishes the
// build identically (the tail levels' outputs are written by rank 0).
//
// Reference work replaced: bbhash.New levels + computeHashPositionsReverseMap + the
// scatter (pkg/format/mphf_streaming.go:141,176-204); hashing as in Add (:73,80).
#include <hip/hip_runtime.h>

#include "s3imph_device.h"
#include "s3imph_internal.h"

#include <algorithm>

namespace s3imph {

namespace {

constexpr int kRT = 1024;               // route block
constexpr int kRK = 2;                  // records per thread per round
constexpr int kRRound = kRT * kRK;

// Route this rank's records of level `level` to their owners.  kSrc 2: level 0 from the
// hash kernel's key-order kh / fp arrays (a skewed set, or a retried route; the pair-round
// hash routes level 0 itself otherwise); 1: the collided records list[0..n[level]).  Each
// round of kRRound records is counting-sorted by owner in LDS; one atomic per (round, owner) reserves its run in the owner's send region
// [d*cap, (d+1)*cap), and the runs are written out coalesced.  Records this rank owns
// itself skip the exchange: they go straight to `self_dst` (the level's input list,
// capacity self_cap), counted in scnt[rank] like any owner's.  A region overflow sets
// kStRouteOverflow (the host re-routes with larger regions; bytes are unaffected).
template <int kSrc>
__global__ __launch_bounds__(kRT) void k_route(int level, const uint64_t* __restrict__ ikh, const uint64_t* __restrict__ ifp,
                                               const uint64_t* __restrict__ ipos, uint64_t pos_base,
                                               uint64_t n_keys, const Rec* __restrict__ ilist,
                                               Rec* __restrict__ send, uint64_t cap,
                                               unsigned long long* __restrict__ scnt, LevelState* st, int P,
                                               int rank, Rec* __restrict__ self_dst, uint64_t self_cap,
                                               const unsigned long long* __restrict__ mat_prev, int only_skew) {
  __shared__ Rec stage[kRRound];
  __shared__ unsigned char sdst[kRRound];
  __shared__ unsigned cnt[kMaxRanks], start[kMaxRanks];
  __shared__ Rec* base[kMaxRanks];
  __shared__ unsigned s_over;
  __shared__ uint64_t s_rb;
  if (only_skew && !st->skew) return;  // the fused hash kernel routed this set
  const unsigned tid = threadIdx.x;
  if (tid == 0) s_over = 0;
  if (tid < 64) {  // records received for earlier key chunks sit before this rank's own ones
    uint64_t v = mat_prev && tid < (unsigned)P && (int)tid != rank ? mat_prev[(uint64_t)tid * (P + 1) + rank] : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (tid == 0) s_rb = v;
  }
  __syncthreads();
  if (s_rb > self_cap) {
    if (tid == 0) atomicOr(&st->status, kStRouteOverflow);
    return;
  }
  self_dst += s_rb;
  self_cap -= s_rb;
  const uint64_t n = kSrc != 1 ? n_keys : st->n[level];
  const uint64_t words = st->words[level], magic = st->magic[level];
  const uint64_t S = st->dS[level], mS = st->dmagic[level];
  const uint64_t seed = level_seed(level);
  for (uint64_t r0 = (uint64_t)blockIdx.x * kRRound; r0 < n; r0 += (uint64_t)gridDim.x * kRRound) {
    if (tid < kMaxRanks) cnt[tid] = 0;
    __syncthreads();
    Rec rec[kRK];
    unsigned d[kRK], rk[kRK];
#pragma unroll
    for (int q = 0; q < kRK; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kRT + tid;
      d[q] = rk[q] = 0;
      if (i < n) {
        if (kSrc == 2) {
          rec[q] = Rec{ikh[i], ifp[i], ipos ? ipos[i] : pos_base + i};
        } else {
          rec[q] = ilist[i];
        }
        const uint64_t x = bb_index(seed, rec[q].k, words, magic);
        d[q] = owner_of(x >> 6, S, mS);
        if (d[q] >= (unsigned)P) d[q] = P - 1;  // unreachable: x < 64 words <= 64 P S
        rk[q] = atomicAdd(&cnt[d[q]], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {  // one wave: owner-run starts and the per-owner reservations
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
        const bool self = (int)tid == rank;
        if (at + c > (self ? self_cap : cap)) s_over = 1;
        base[tid] = (self ? self_dst : send + (uint64_t)tid * cap) + at;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kRK; ++q) {
      const uint64_t i = r0 + (uint64_t)q * kRT + tid;
      if (i < n) {
        const unsigned slot = start[d[q]] + rk[q];
        stage[slot] = rec[q];
        sdst[slot] = (unsigned char)d[q];
      }
    }
    __syncthreads();
    const unsigned m = (unsigned)min<uint64_t>(kRRound, n - r0);
    if (!s_over) {
      for (unsigned j = tid; j < m; j += kRT) {
        const unsigned o = sdst[j];
        base[o][j - start[o]] = stage[j];
      }
    }
    __syncthreads();
  }
  if (tid == 0 && s_over) atomicOr(&st->status, kStRouteOverflow);
}

// Size distributed level L on the device from its global key count (*gcount, the
// all-reduced redo counts of level L-1, or n for level 0) and this rank's word range.
__device__ void dist_setup(LevelState* st, int L, const unsigned long long* gcount, uint64_t n_value, int rank,
                           int P) {
  const uint64_t n = gcount ? *gcount : n_value;
  const uint64_t w = level_words(n);
  const uint64_t S = (w + P - 1) / P;
  const uint64_t lo = min<uint64_t>((uint64_t)rank * S, w);
  st->gn[L] = n;
  st->words[L] = w;
  st->magic[L] = level_magic(w);
  st->woff[L] = L ? st->woff[L - 1] + st->words[L - 1] : 0;
  st->woff[L + 1] = st->woff[L] + w;
  st->preset[L] = 1;
  st->wlo[L] = lo;
  st->rw[L] = min<uint64_t>(S, w - lo);
  st->dS[L] = S ? S : 1;
  st->dmagic[L] = level_magic(S ? S : 1);
  st->nlevels = L + 1;
  st->n[L + 1] = 0;                     // this level's collided records (tile atomics)
  st->lvl_base[L + 1] = st->lvl_base[L];  // overwritten by the last tile, if any
}
__global__ void k_dist_setup(LevelState* st, int L, const unsigned long long* gcount, uint64_t n_value, int rank,
                             int P) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  dist_setup(st, L, gcount, n_value, rank, P);
}
// A bitmap level's start in one launch: its setup (setup: from the gathered count), the whole
// level's range (k_bm_range), and its size against the host's bound wmax (k_bm_check)
__global__ void k_bm_level_begin(LevelState* st, int L, bool setup, const unsigned long long* gcount, int rank, int P,
                                 uint64_t wmax) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (setup) dist_setup(st, L, gcount, 0, rank, P);
  st->wlo[L] = 0;
  st->rw[L] = st->words[L];
  if (st->words[L] > wmax) atomicOr(&st->status, kStBitmapBound);
}

__global__ void k_set_u64(unsigned long long* p, uint64_t v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *p = v;
}

// Multi-GPU replicated tail: level L is the first level every rank runs on all records;
// its predecessor's global count gates the single-GPU kernels ("was a big level").
__global__ void k_dist_replicate(LevelState* st, int L, uint64_t n_all, uint64_t skip_from) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  st->n[L - 1] = st->gn[L - 1];
  st->n[L] = n_all;
  st->out_skip_from = skip_from;
}

// Route overflow flag -> scnt[P] (gathered with the counts), then clear it for a retry.
__global__ void k_route_flag(LevelState* st, unsigned long long* scnt, int P) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  scnt[P] = (st->status & kStRouteOverflow) ? 1ull : 0ull;
  st->status &= ~kStRouteOverflow;
}

// Fixed-size exchange regions (routed levels >= 1): the tail [min(scnt[t], C), C) of every
// region — send region t, or this rank's own region in the level's input list — is
// filled with k = 0 records, which the reservation scatter skips (no key hashes to 0:
// level 0 rejects it), so every region can be sent whole and the receivers need no
// counts on the host.
__global__ __launch_bounds__(256) void k_route_pad(Rec* __restrict__ send, uint64_t C,
                                                   const unsigned long long* __restrict__ scnt, int rank,
                                                   Rec* __restrict__ self_region) {
  const int t = blockIdx.y;
  Rec* reg = t == rank ? self_region : send + (uint64_t)t * C;
  const uint64_t c0 = min<uint64_t>(scnt[t], C);
  for (uint64_t i = c0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < C; i += (uint64_t)gridDim.x * 256)
    reg[i] = Rec{0, 0, 0};
}

}  // namespace

void launch_route_flag(LevelState* st, unsigned long long* scnt, int P, hipStream_t s) {
  k_route_flag<<<1, 64, 0, s>>>(st, scnt, P);
}

void launch_route0_arrays(const uint64_t* kh, const uint64_t* fp, const uint64_t* pos, uint64_t pos_base, uint64_t n,
                          Rec* send, uint64_t cap, unsigned long long* scnt, LevelState* st, int P, int rank,
                          Rec* self_dst, uint64_t self_cap, hipStream_t s) {
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n + kRRound - 1) / kRRound, 2048));
  k_route<2><<<grid, kRT, 0, s>>>(0, kh, fp, pos, pos_base, n, nullptr, send, cap, scnt, st, P, rank,
                                   self_dst, self_cap, nullptr, 0);
}

void launch_route0_arrays(const uint64_t* kh, const uint64_t* fp, uint64_t n, const Route0& rt, LevelState* st,
                          bool only_skew, hipStream_t s) {
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n + kRRound - 1) / kRRound, 2048));
  k_route<2><<<grid, kRT, 0, s>>>(0, kh, fp, rt.pos, rt.pos_base, n, nullptr, rt.send, rt.cap, rt.scnt,
                                   st, rt.P, rt.rank, rt.self_dst, rt.self_cap, rt.mat_prev, only_skew ? 1 : 0);
}

void launch_route(int level, const Rec* list, uint64_t n_pred, Rec* send, uint64_t cap, unsigned long long* scnt,
                  LevelState* st, int P, int rank, Rec* self_dst, uint64_t self_cap, hipStream_t s) {
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((n_pred + kRRound - 1) / kRRound + 8, 2048));
  k_route<1><<<grid, kRT, 0, s>>>(level, nullptr, nullptr, nullptr, 0, 0, list, send, cap, scnt, st,
                                   P, rank, self_dst, self_cap, nullptr, 0);
}

void launch_route_pad(Rec* send, uint64_t C, const unsigned long long* scnt, int P, int rank, Rec* self_region,
                      hipStream_t s) {
  const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((C / 8 + 255) / 256, 256));
  k_route_pad<<<dim3(gx, (unsigned)P), 256, 0, s>>>(send, C, scnt, rank, self_region);
}

void launch_dist_setup(LevelState* st, int L, const unsigned long long* gcount, uint64_t n_value, int rank, int P,
                       hipStream_t s) {
  k_dist_setup<<<1, 64, 0, s>>>(st, L, gcount, n_value, rank, P);
}

void launch_set_u64(unsigned long long* p, uint64_t v, hipStream_t s) { k_set_u64<<<1, 64, 0, s>>>(p, v); }

void launch_bm_level_begin(LevelState* st, int L, bool setup, const unsigned long long* gcount, int rank, int P,
                           uint64_t wmax, hipStream_t s) {
  k_bm_level_begin<<<1, 64, 0, s>>>(st, L, setup, gcount, rank, P, wmax);
}

void launch_dist_replicate(LevelState* st, int L, uint64_t n_all, uint64_t skip_from, hipStream_t s) {
  k_dist_replicate<<<1, 64, 0, s>>>(st, L, n_all, skip_from);
}

}  // namespace s3imph
