// s3imph_device.h — device helpers shared by every kernel file: the FNV hashes of
// pkg/format/mphf.go:341-369, the restated relab/bbhash position function
//  and wave-level utilities.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "bbhash_spec.h"

namespace s3imph {

// Integer min / max.  HIP's mixed-type overloads (unsigned long against unsigned long long,
// a 64-bit value against an int literal) promote both operands to double: v_cvt_f64 /
// v_min_f64 / v_trunc in the ISA, and inexact past 2^53.  Inside namespace s3imph these
// hide them; mixed signedness does not compile (say which conversion is meant).
template <class A, class B>
__host__ __device__ __forceinline__ typename std::common_type<A, B>::type min(A a, B b) {
  static_assert(std::is_integral<A>::value && std::is_integral<B>::value, "integer min");
  static_assert(std::is_signed<A>::value == std::is_signed<B>::value, "min of mixed signedness");
  using T = typename std::common_type<A, B>::type;
  return (T)a < (T)b ? (T)a : (T)b;
}
template <class A, class B>
__host__ __device__ __forceinline__ typename std::common_type<A, B>::type max(A a, B b) {
  static_assert(std::is_integral<A>::value && std::is_integral<B>::value, "integer max");
  static_assert(std::is_signed<A>::value == std::is_signed<B>::value, "max of mixed signedness");
  using T = typename std::common_type<A, B>::type;
  return (T)a < (T)b ? (T)b : (T)a;
}

// Key bytes are read once, in whole 16-B units of consecutive lanes: the level-0 hash loads
// them with the non-temporal hint (S3IMPH_NT_LOADS, default on), so the 6.4 GB byte stream
// leaves L2 first and the block's region write runs stay in it until completed (C3 hash
// 2.73 -> 2.55 ms, step 6.65 -> 6.49 ms, profiles/r5_hash/nt_loads_ab_r5ae.txt).  Measured
// and dropped: the hint on the 20-B record loads of the scatters and tile kernels (15-30 %
// slower, nt_loads_all_ab_r5ad.txt; in k_scatter_p0 alone, with the 4-B load first, still
// 1.09 -> 1.37 ms, nt_rec_scatter_ab_r5af.txt) and on k_hash_skew's 64-B chunk loads
// (S3IMPH_NT_SKEW, C5 hash 1.63 -> 2.34 ms: a chunk is half a line that neighbouring keys'
// chunks share).
#ifndef S3IMPH_NT_LOADS
#define S3IMPH_NT_LOADS 1
#endif
// fnv_window two stream words per loop iteration: measured neutral to slightly slower (C3 hash
// 2.53-2.61 vs 2.56-2.64 ms, 4 alternating builds each, profiles/r6_hash/fnv_unroll2_ab_r6h.txt:
// the loop control it saves issues beside the multiply chain anyway); off
#ifndef S3IMPH_FNV_UNROLL2
#define S3IMPH_FNV_UNROLL2 0
#endif
#ifndef S3IMPH_NT_SKEW
#define S3IMPH_NT_SKEW 0
#endif
// k_hash0_pair's two keys per lane as ONE word loop (fnv_window_pair): each key zero-prefixed
// to whole 8-byte words, no tail loops; A/B switch (S3IMPH_FNV_PAIR=1 at compile time)
#ifndef S3IMPH_FNV_PAIR
#define S3IMPH_FNV_PAIR 0
#endif
// Stores of whole runs that this build does not read back soon: the tile kernels' staged
// fp_out / pos_out runs and the unfused hash's key-order kh / fp, with the non-temporal hint
// (S3IMPH_NT_OUT, default on: C2 0.777 -> 0.765 ms, C3 6.45 -> 6.43 ms,
// profiles/r5_levels/nt_out_ab_r5ai.txt).
#ifndef S3IMPH_NT_OUT
#define S3IMPH_NT_OUT 1
#endif
template <class T>
static __device__ __forceinline__ void st_stream(T* p, T v) {
#if S3IMPH_NT_OUT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
static __device__ __forceinline__ uint4 ld_stream16(const void* p) {
#if S3IMPH_NT_LOADS
  const u32x4v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}

static __device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

// The XCD (accelerator complex die) this wave runs on: each has its own L2, so a producer and
// a consumer on the same XCD exchange data through that L2 without an L2 write-back.
static __device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}

// A wave-uniform 64-bit value moved to scalar registers.
static __device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

static __device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
}

// Position of `key` in a level of 64*words bits: keyHash % (64*words), computed as
// 64*((h>>6) mod words) + (h & 63) with a Barrett step (q < 2^58, one correction).
static __device__ __forceinline__ uint64_t bb_index(uint64_t seed, uint64_t key, uint64_t words,
                                             uint64_t magic) {
  uint64_t h = key_mix(seed, key);
  uint64_t q = h >> 6;
  uint64_t qe = __umul64hi(q, magic);
  uint64_t r = q - qe * words;
  if (r >= words) r -= words;
  return (r << 6) | (h & 63);
}

// bb_index for a level of at least 2^19 words (level_magic < 2^45, P0's level 0): the same
// Barrett quotient, its high half built from three 32x32 products whose 64-bit sum cannot
// overflow (q < 2^58), and qe * words from qe < 2^39 and words < 2^32 (the compiler's
// general 64x64 forms spent ~10 more VALU per key, half of them moves).
static __device__ __forceinline__ uint64_t bb_index_big(uint64_t seed, uint64_t key, uint64_t words,
                                                      uint64_t magic) {
  const uint64_t h = key_mix(seed, key);
  const uint64_t q = h >> 6;
  const uint32_t ql = (uint32_t)q, qh = (uint32_t)(q >> 32);
  const uint32_t ml = (uint32_t)magic, mh = (uint32_t)(magic >> 32);
  uint64_t sum = (uint64_t)qh * ml + __umulhi(ql, ml);
  sum += (uint64_t)ql * mh;
  const uint64_t qe = (uint64_t)qh * mh + (sum >> 32);
  const uint32_t wl = (uint32_t)words;
  const uint64_t prod = (uint64_t)(uint32_t)qe * wl + ((uint64_t)((uint32_t)(qe >> 32) * wl) << 32);
  uint64_t r = q - prod;
  if (r >= words) r -= words;
  return (r << 6) | (h & 63);
}

// bb_index with the level-independent half of key_mix already applied (mk = mix64(key)),
// for code that revisits the same key at several levels.
static __device__ __forceinline__ uint64_t bb_index_mk(uint64_t seed, uint64_t mk, uint64_t words,
                                                     uint64_t magic) {
  uint64_t h = mix64((seed ^ mk) * kHashM);
  uint64_t q = h >> 6;
  uint64_t qe = __umul64hi(q, magic);
  uint64_t r = q - qe * words;
  if (r >= words) r -= words;
  return (r << 6) | (h & 63);
}

// Owner rank of level word w in the multi-GPU build: w / S by a Barrett step (w < 2^32,
// one correction; mS = level_magic(S)).
static __device__ __forceinline__ unsigned owner_of(uint64_t w, uint64_t S, uint64_t mS) {
  uint64_t d = __umul64hi(w, mS);
  if (w - d * S >= S) ++d;
  return (unsigned)d;
}

// ---- FNV-64 multiply by the prime P = 2^40 + 435, on 32-bit halves -----------------
// x * P mod 2^64 with x = lo + 2^32 hi:
//   lo' = lo * 435 (low word),  hi' = mulhi(lo, 435) + hi * 435 + (lo << 8)   (mod 2^32).
// hi * 435 + (lo << 8) is one v_mul_lo_u32 and one v_lshl_add_u32, and rides into
// v_mad_u64_u32 (lo * 435) as its addend's high word, so the multiply costs 3 VALU ops
// (the compiler's own lowering of a 64-bit multiply takes 5).  tools/ubench_fnv.hip
// prices the FNV-1a + FNV-1 byte step at 36 SIMD-cycles per wave (45 compiler-lowered;
// 40 with the top byte of hi * 435 taken by an SDWA 24-bit multiply).
constexpr uint32_t kFnvPLow = 435u;
static_assert(kFnvPrime == (1ull << 40) + kFnvPLow, "fnv_mulP decomposes the FNV-64 prime as 2^40 + 435");
static __device__ __forceinline__ void fnv_mulP(uint32_t& lo, uint32_t& hi) {
  const uint32_t x = (lo << 8) + hi * kFnvPLow;
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(lo), "s"(kFnvPLow), "v"((uint64_t)x << 32));
  lo = (uint32_t)r;
  hi = (uint32_t)(r >> 32);
}

// One FNV-1a step and one FNV-1 step on byte c
static __device__ __forceinline__ void fnv_step_w(uint32_t& alo, uint32_t& ahi, uint32_t& blo, uint32_t& bhi,
                                                  uint32_t c) {
  alo ^= c;  // FNV-1a (hashBytes): h ^= b; h *= P
  fnv_mulP(alo, ahi);
  fnv_mulP(blo, bhi);  // FNV-1 (computeFingerprintBytes): h *= P; h ^= b
  blo ^= c;
}

// x ^ (byte B of w): one v_xor_b32 with an SDWA byte select (the compiler's own lowering
// spends a shift on bytes 1 and 2).
template <int B>
static __device__ __forceinline__ uint32_t xor_byte(uint32_t x, uint32_t w) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(r) : "v"(w), "v"(x));
  else if constexpr (B == 1)
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(r) : "v"(w), "v"(x));
  else if constexpr (B == 2)
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(r) : "v"(w), "v"(x));
  else
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
        : "=v"(r) : "v"(w), "v"(x));
  return r;
}

// FNV-1a + FNV-1 steps on byte B of w: 8 VALU ops (xor, 3 for the multiply, per hash).
template <int B>
static __device__ __forceinline__ void fnv_step_b(uint32_t& alo, uint32_t& ahi, uint32_t& blo, uint32_t& bhi,
                                                  uint32_t w) {
  alo = xor_byte<B>(alo, w);
  fnv_mulP(alo, ahi);
  fnv_mulP(blo, bhi);
  blo = xor_byte<B>(blo, w);
}

// The four bytes of w in stream order.
static __device__ __forceinline__ void fnv_4b(uint32_t& alo, uint32_t& ahi, uint32_t& blo, uint32_t& bhi,
                                              uint32_t w) {
  fnv_step_b<0>(alo, ahi, blo, bhi, w);
  fnv_step_b<1>(alo, ahi, blo, bhi, w);
  fnv_step_b<2>(alo, ahi, blo, bhi, w);
  fnv_step_b<3>(alo, ahi, blo, bhi, w);
}

// The first `rem` (< 8) bytes of the stream words r0, r1.
static __device__ __forceinline__ void fnv_tail_b(uint32_t& alo, uint32_t& ahi, uint32_t& blo, uint32_t& bhi,
                                                  uint32_t r0, uint32_t r1, unsigned rem) {
  if (rem > 0) fnv_step_b<0>(alo, ahi, blo, bhi, r0);
  if (rem > 1) fnv_step_b<1>(alo, ahi, blo, bhi, r0);
  if (rem > 2) fnv_step_b<2>(alo, ahi, blo, bhi, r0);
  if (rem > 3) fnv_step_b<3>(alo, ahi, blo, bhi, r0);
  if (rem > 4) fnv_step_b<0>(alo, ahi, blo, bhi, r1);
  if (rem > 5) fnv_step_b<1>(alo, ahi, blo, bhi, r1);
  if (rem > 6) fnv_step_b<2>(alo, ahi, blo, bhi, r1);
}

// FNV-1a + FNV-1 of a key of `len` bytes starting `o` bytes into a dword-addressed window
// (LDS): each 8-byte stream word is two v_alignbyte funnels of consecutive dwords, so the
// key's start needs no select between the word's halves.  Reads up to 12 bytes past the
// key's end.
static __device__ __forceinline__ void fnv_window(const uint32_t* win, unsigned o, unsigned len, uint64_t& ha,
                                                  uint64_t& hb) {
  uint32_t alo = (uint32_t)kFnvOffset, ahi = (uint32_t)(kFnvOffset >> 32), blo = alo, bhi = ahi;
  const uint32_t* w = win + (o >> 2);
  const unsigned sb = o & 3u;
  const unsigned nfull = len >> 3;
  // the next stream word's dwords are read one iteration ahead, so the LDS latency hides
  // behind the current word's 64 steps (reads stay within w[0 .. 2 nfull + 2], as the tail's)
  uint32_t cur = w[0], n1 = w[1], n2 = w[2];
  unsigned q = 0;
#if S3IMPH_FNV_UNROLL2
  // two stream words per iteration: half the loop control and no register rotation moves
  // (the 16 bytes' dwords w[2q+3 .. 2q+6] requested ahead, within w[0 .. 2 nfull + 2])
  for (; q + 2 <= nfull; q += 2) {
    const uint32_t m1 = w[2 * q + 3], m2 = w[2 * q + 4], m3 = w[2 * q + 5], m4 = w[2 * q + 6];
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb));
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n2, n1, sb));
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(m1, n2, sb));
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(m2, m1, sb));
    cur = m2;
    n1 = m3;
    n2 = m4;
  }
#endif
  for (; q < nfull; ++q) {
    const uint32_t m1 = w[2 * q + 3], m2 = w[2 * q + 4];
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb));
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n2, n1, sb));
    cur = n2;
    n1 = m1;
    n2 = m2;
  }
  const unsigned rem = len & 7u;
  if (rem)
    fnv_tail_b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb), __builtin_amdgcn_alignbyte(n2, n1, sb),
               rem);
  ha = (uint64_t)alo | ((uint64_t)ahi << 32);
  hb = (uint64_t)blo | ((uint64_t)bhi << 32);
}

// ---- two keys as one word loop (S3IMPH_FNV_PAIR) ------------------------------------
// A key of len bytes hashed as pad = (-len) mod 8 zero bytes and then its bytes: both FNV
// forms map a zero byte to h * P, so starting from offset_basis * P^-pad the pad steps
// arrive at offset_basis exactly, and the key is whole 8-byte words.  The window must hold
// >= 8 readable bytes before every key (the bytes before a key's start are masked to zero).
__host__ __device__ constexpr uint64_t fnv_prime_inverse() {
  uint64_t x = kFnvPrime;  // P odd: x = P is right to 3 bits; each Newton step doubles them
  for (int i = 0; i < 5; ++i) x *= 2 - kFnvPrime * x;
  return x;
}
static_assert(kFnvPrime * fnv_prime_inverse() == 1, "P^-1 mod 2^64");
__host__ __device__ constexpr uint64_t fnv_prefixed_basis(unsigned pad) {
  uint64_t h = kFnvOffset;
  for (unsigned i = 0; i < pad; ++i) h *= fnv_prime_inverse();
  return h;
}
// Keys A (len lA at byte oA of win) and B (if hasB) of one lane: the lane runs ceil(lA/8) +
// ceil(lB/8) words in one loop, switching state after A's last word, so a wave whose lanes
// pair a short key with a long one runs to the largest SUM of word counts instead of the
// largest A plus the largest B plus two byte-step tails.  init[pad] = fnv_prefixed_basis(pad).
static __device__ __forceinline__ void fnv_mask_first(unsigned pad, uint32_t& mlo, uint32_t& mhi) {
  mlo = pad >= 4 ? 0u : ~0u << (8 * pad);
  mhi = pad <= 4 ? ~0u : ~0u << (8 * (pad - 4));
}
static __device__ __forceinline__ void fnv_window_pair(const uint32_t* win, unsigned oA, unsigned lA, unsigned oB,
                                                       unsigned lB, bool hasB, const uint64_t* init, uint64_t& haA,
                                                       uint64_t& hbA, uint64_t& haB, uint64_t& hbB) {
  const unsigned padA = (8u - (lA & 7u)) & 7u, padB = (8u - (lB & 7u)) & 7u;
  const unsigned WA = (lA + padA) >> 3, W = WA + (hasB ? (lB + padB) >> 3 : 0u);
  uint64_t h0 = init[padA];
  uint32_t alo = (uint32_t)h0, ahi = (uint32_t)(h0 >> 32), blo = alo, bhi = ahi;
  uint32_t mlo, mhi;
  fnv_mask_first(padA, mlo, mhi);
  unsigned s0 = oA - padA;
  if (WA == 0) {  // an empty A: its hashes are offset_basis; B from the start
    haA = hbA = kFnvOffset;
    h0 = init[padB];
    alo = blo = (uint32_t)h0;
    ahi = bhi = (uint32_t)(h0 >> 32);
    fnv_mask_first(padB, mlo, mhi);
    s0 = oB - padB;
  }
  const uint32_t* w = win + (s0 >> 2);
  unsigned sb = s0 & 3u;
  uint32_t cur = w[0], n1 = w[1], n2 = w[2];
  for (unsigned q = 0; q < W; ++q) {
    const uint32_t m1 = w[3], m2 = w[4];
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb) & mlo);
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n2, n1, sb) & mhi);
    mlo = mhi = ~0u;
    cur = n2;
    n1 = m1;
    n2 = m2;
    w += 2;
    if (q + 1 == WA) {  // A done: B's state, first-word mask and words
      haA = (uint64_t)alo | ((uint64_t)ahi << 32);
      hbA = (uint64_t)blo | ((uint64_t)bhi << 32);
      h0 = init[padB];
      alo = blo = (uint32_t)h0;
      ahi = bhi = (uint32_t)(h0 >> 32);
      fnv_mask_first(padB, mlo, mhi);
      const unsigned s1 = oB - padB;
      w = win + (s1 >> 2);
      sb = s1 & 3u;
      cur = w[0];
      n1 = w[1];
      n2 = w[2];
    }
  }
  haB = (uint64_t)alo | ((uint64_t)ahi << 32);
  hbB = (uint64_t)blo | ((uint64_t)bhi << 32);
}

// fnv_window continuing a running state (alo:ahi FNV-1a, blo:bhi FNV-1): the bytes of a
// key that arrive chunk by chunk.
static __device__ __forceinline__ void fnv_window_cont(const uint32_t* win, unsigned o, unsigned len, uint32_t& alo,
                                                       uint32_t& ahi, uint32_t& blo, uint32_t& bhi) {
  const uint32_t* w = win + (o >> 2);
  const unsigned sb = o & 3u;
  const unsigned nfull = len >> 3;
  uint32_t cur = w[0], n1 = w[1], n2 = w[2];  // one stream word ahead, as fnv_window
  for (unsigned q = 0; q < nfull; ++q) {
    const uint32_t m1 = w[2 * q + 3], m2 = w[2 * q + 4];
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb));
    fnv_4b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n2, n1, sb));
    cur = n2;
    n1 = m1;
    n2 = m2;
  }
  const unsigned rem = len & 7u;
  if (rem)
    fnv_tail_b(alo, ahi, blo, bhi, __builtin_amdgcn_alignbyte(n1, cur, sb), __builtin_amdgcn_alignbyte(n2, n1, sb),
               rem);
}

// FNV-1a and FNV-1 over the 8 bytes of v, little-endian order.
static __device__ __forceinline__ void fnv_8(uint64_t& a, uint64_t& b, uint64_t v) {
  uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
  fnv_4b(alo, ahi, blo, bhi, (uint32_t)v);
  fnv_4b(alo, ahi, blo, bhi, (uint32_t)(v >> 32));
  a = (uint64_t)alo | ((uint64_t)ahi << 32);
  b = (uint64_t)blo | ((uint64_t)bhi << 32);
}

// FNV-1a and FNV-1 over the first rem (< 8) bytes of v.
static __device__ __forceinline__ void fnv_tail8(uint64_t& a, uint64_t& b, uint64_t v, unsigned rem) {
  uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
  fnv_tail_b(alo, ahi, blo, bhi, (uint32_t)v, (uint32_t)(v >> 32), rem);
  a = (uint64_t)alo | ((uint64_t)ahi << 32);
  b = (uint64_t)blo | ((uint64_t)bhi << 32);
}

// Bytes [s, s + 8) of the 16-byte little-endian concatenation lo:hi (s in 0..7), from
// 32-bit byte funnels (v_alignbyte_b32): the key stream word of a key that starts s bytes
// into aligned word `lo`.
static __device__ __forceinline__ uint64_t funnel_bytes(uint64_t lo, uint64_t hi, unsigned s) {
  const uint32_t c0 = (uint32_t)lo, c1 = (uint32_t)(lo >> 32), n0 = (uint32_t)hi, n1 = (uint32_t)(hi >> 32);
  const bool up = s >= 4;
  const uint32_t x0 = up ? c1 : c0, x1 = up ? n0 : c1, x2 = up ? n1 : n0;
  const unsigned sb = s & 3u;
  const uint32_t r0 = __builtin_amdgcn_alignbyte(x1, x0, sb);
  const uint32_t r1 = __builtin_amdgcn_alignbyte(x2, x1, sb);
  return (uint64_t)r0 | ((uint64_t)r1 << 32);
}

// FNV-1a + FNV-1 of blob[b0, b1) with the aligned-word loads software-pipelined two
// words ahead: word q+2 is requested while word q is hashed, so a lane's dependent
// load latency overlaps its own multiply chain.  Never reads past the key's last
// aligned word.
static __device__ __forceinline__ void fnv_both_pf(const uint8_t* __restrict__ blob, uint64_t b0, uint64_t b1,
                                                   uint64_t& ha, uint64_t& hb) {
  uint64_t a = kFnvOffset, b = kFnvOffset;
  if (b1 > b0) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(blob + (b0 & ~7ull));
    const uint64_t nw = ((b1 - 1) >> 3) - (b0 >> 3) + 1;  // aligned words overlapping the key
    const unsigned sh = (unsigned)(b0 & 7) * 8;
    const uint64_t len = b1 - b0;
    const uint64_t nfull = len >> 3;
    uint64_t cur = w[0];
    uint64_t nxt = nw > 1 ? w[1] : 0;
    for (uint64_t q = 0; q < nfull; ++q) {
      const uint64_t nn = (q + 2 < nw) ? w[q + 2] : 0;
      const uint64_t v = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
      fnv_8(a, b, v);
      cur = nxt;
      nxt = nn;
    }
    const unsigned rem = (unsigned)(len & 7);
    if (rem) {
      const uint64_t v = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
      fnv_tail8(a, b, v, rem);
    }
  }
  ha = a;
  hb = b;
}

// FNV-1a + FNV-1 of blob[b0, b1) from 16-byte aligned loads (half the load
// instructions of the 8-byte variants), software-pipelined one chunk ahead.  Stream
// chunk c = bytes [b0 + 16c, b0 + 16c + 16) = the 128-bit funnel of aligned chunks
// C[c], C[c+1] by (b0 & 15) bytes.  Reads stay inside the 16-byte chunks overlapping
// the key, and the last one is read as 8 bytes when the key ends in its low half, so
// nothing past the key's last aligned 8-byte word is touched.
struct U128 {
  uint64_t lo, hi;
};
static __device__ __forceinline__ U128 ld_chunk(const uint8_t* p, bool full) {
  U128 r;
  if (full) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    r.lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
    r.hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  } else {
    r.lo = *reinterpret_cast<const uint64_t*>(p);
    r.hi = 0;
  }
  return r;
}
static __device__ __forceinline__ void fnv_both_16(const uint8_t* __restrict__ blob, uint64_t b0, uint64_t b1,
                                                   uint64_t& ha, uint64_t& hb) {
  uint64_t a = kFnvOffset, b = kFnvOffset;
  if (b1 > b0) {
    const uint64_t c0 = b0 & ~15ull;
    const uint8_t* base = blob + c0;
    const uint64_t nc = ((b1 - 1) >> 4) - (b0 >> 4) + 1;  // 16-byte chunks overlapping the key
    const bool last_full = ((b1 - 1) & 8) != 0;            // key ends in the last chunk's high half
    const unsigned d = (unsigned)(b0 & 15) * 8;             // funnel shift in bits, 0..120
    const uint64_t len = b1 - b0;
    const uint64_t nfull = len >> 4;                        // whole 16-byte stream chunks
    U128 cur = ld_chunk(base, nc > 1 || last_full);
    U128 nxt = nc > 1 ? ld_chunk(base + 16, nc > 2 || last_full) : U128{0, 0};
    auto funnel = [&](const U128& x, const U128& y, uint64_t& lo, uint64_t& hi) {
      if (d == 0) {
        lo = x.lo;
        hi = x.hi;
      } else if (d < 64) {
        lo = (x.lo >> d) | (x.hi << (64 - d));
        hi = (x.hi >> d) | (y.lo << (64 - d));
      } else if (d == 64) {
        lo = x.hi;
        hi = y.lo;
      } else {
        lo = (x.hi >> (d - 64)) | (y.lo << (128 - d));
        hi = (y.lo >> (d - 64)) | (y.hi << (128 - d));
      }
    };
    for (uint64_t c = 0; c < nfull; ++c) {
      const U128 nn = c + 2 < nc ? ld_chunk(base + 16 * (c + 2), c + 3 < nc || last_full) : U128{0, 0};
      uint64_t lo, hi;
      funnel(cur, nxt, lo, hi);
      fnv_8(a, b, lo);
      fnv_8(a, b, hi);
      cur = nxt;
      nxt = nn;
    }
    const unsigned rem = (unsigned)(len & 15);
    if (rem) {
      uint64_t lo, hi;
      funnel(cur, nxt, lo, hi);
      uint64_t v = lo;
      if (rem >= 8) {
        fnv_8(a, b, lo);
        v = hi;
      }
      fnv_tail8(a, b, v, rem & 7);
    }
  }
  ha = a;
  hb = b;
}



}  // namespace s3imph
