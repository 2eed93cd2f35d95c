// bbhash_spec.h — constants of the BBHash build the reference delegates to
// github.com/relab/bbhash v0.0.0-20250331135148-7358f69256fb (go.mod:10), called as
// bbhash.New(hashes, bbhash.Gamma(2.0), bbhash.WithReverseMap()) at
// pkg/format/mphf_streaming.go:141, and of the FNV hashes at pkg/format/mphf.go:341-369.
//
// relab/bbhash is not vendored; the constants restate its public algorithm
// (toggles T1-T8).  The oracle keeps an independent copy
// (oracle/bbhash_oracle_spec.h); tests/test_spec_agreement.py checks they agree.
#pragma once

#include <stdint.h>

namespace s3imph {

// Go hash/fnv 64-bit parameters (FNV-1a for keys, FNV-1 for fingerprints).
constexpr uint64_t kFnvOffset = 14695981039346656037ull;
constexpr uint64_t kFnvPrime = 1099511628211ull;  // 2^40 + 0x1b3

// T1: fasthash mix and multiplier.
constexpr uint64_t kMixMul = 0x2127599bf4325c37ull;
constexpr uint64_t kHashM = 0x880355f21e6d1965ull;

// gamma = 2.0 (mphf_streaming.go:141): level bit count = 2n, words = ceil(2n/64) (T3).
constexpr uint64_t kGammaNum = 2;

// T6: level budget before the build is declared unresolvable (duplicate key hashes).
constexpr int kMaxLevels = 64;

// T4/T8: mph.bin = [u64 partitions = 1][u64 levels]{[u64 words][words]}.
constexpr uint64_t kPartitions = 1;

// S3ID columnar framing (pkg/format/format.go:6-32).
constexpr uint32_t kS3idMagic = 0x53334944u;
constexpr uint32_t kS3idVersion = 1u;
constexpr uint32_t kS3idHeaderSize = 20u;

#if defined(__HIPCC__)
#define S3IMPH_HD __host__ __device__ __forceinline__
#else
#define S3IMPH_HD inline
#endif

S3IMPH_HD uint64_t level_words(uint64_t n) { return (kGammaNum * n + 63) / 64; }

S3IMPH_HD uint64_t mix64(uint64_t h) {
  h ^= h >> 23;
  h *= kMixMul;
  h ^= h >> 47;
  return h;
}

// T7: levels are numbered from 0.
S3IMPH_HD uint64_t level_seed(uint64_t level) { return mix64(level) * kHashM; }

S3IMPH_HD uint64_t key_mix(uint64_t seed, uint64_t key) { return mix64((seed ^ mix64(key)) * kHashM); }

// Barrett reciprocal for the per-level reduction: magic = floor((2^64-1)/words).
S3IMPH_HD uint64_t level_magic(uint64_t words) { return words ? ~0ull / words : 0; }

}  // namespace s3imph
