// s3imph_internal.h — shared declarations between the kernels, the build
// orchestration and the host-side mirror of StreamingMPHFBuilder.  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "bbhash_spec.h"

namespace s3imph {

// Redo (next-level) key lists are split into kNSeg segments: block b of a big-level
// kernel reads input segment (b % kNSeg) and appends to the same output segment, so
// compaction counters are sharded 64 ways and one atomic covers a whole block tile.
constexpr int kNSeg = 64;

// Device-resident per-build level bookkeeping.  Written only by kernels (and the
// init kernel); the host copies it back once, after the build.
struct LevelState {
  unsigned long long n[kMaxLevels + 2];      // active keys entering level L
  unsigned long long words[kMaxLevels + 2];  // u64 words of level L's bit vector
  unsigned long long woff[kMaxLevels + 2];   // first word of level L in the concatenated bits
  unsigned long long magic[kMaxLevels + 2];  // Barrett reciprocal of words[L]
  unsigned long long rank_total;             // popcount over all levels (== N on success)
  unsigned int nlevels;
  unsigned int status;                       // kSt* flags
  unsigned int tail_first;                   // first level run by the single-workgroup tail
  unsigned int pad;
  unsigned long long seg[kMaxLevels + 2][kNSeg];  // per-segment active keys of level L >= 1
};

// Device status flags.
constexpr unsigned kStKeyZero = 1u;       // some FNV-1a key hash == 0
constexpr unsigned kStTooManyLevels = 2u;  // level budget exhausted (duplicates)
constexpr unsigned kStOverflow = 4u;       // workspace capacity exceeded
constexpr unsigned kStRank = 8u;           // a position landed outside [0, N)

// Levels whose active-key count is at most this run inside one workgroup with
// LDS-resident bit vectors (k_tail); larger levels run as full-grid kernels.
constexpr unsigned long long kTailKeys = 65536;
constexpr int kTailThreads = 1024;
constexpr int kTailLdsWords32 = 2 * 2 * ((kGammaNum * kTailKeys + 63) / 64);  // A and C, u32 words

struct KernelArgs;  // fwd

// ---- launchers (s3imph_kernels.hip) -------------------------------------------
void launch_init_state(LevelState* st, uint64_t n, uint64_t key_base, hipStream_t s);
void launch_hash_mark0(const uint8_t* blob, const uint64_t* offsets, uint64_t n, uint64_t* kh,
                       uint64_t* fp, uint64_t* bits, uint64_t* C, uint64_t words0, LevelState* st,
                       int grid, hipStream_t s);
void launch_resolve(int level, const uint64_t* keys_in, const uint32_t* idx_in, const uint64_t* C,
                    uint64_t* keys_out, uint32_t* idx_out, uint64_t seg_cap, uint64_t* settle,
                    LevelState* st, unsigned long long gate, int grid, hipStream_t s);
void launch_finalize(int level, uint64_t* bits, uint64_t* C, uint64_t cap_words, LevelState* st,
                     unsigned long long gate, int grid, hipStream_t s);
void launch_mark(int level, const uint64_t* keys, uint64_t seg_cap, uint64_t* bits, uint64_t* C,
                 LevelState* st, unsigned long long gate, int grid, hipStream_t s);
void launch_tail(int big_launched, uint64_t* bits, uint64_t cap_words, uint64_t* C, uint64_t* keys0,
                 uint32_t* idx0, uint64_t* keys1, uint32_t* idx1, uint64_t seg_cap, uint64_t* settle,
                 LevelState* st, hipStream_t s);
void launch_rank_scan(const uint64_t* bits, uint64_t cap_words, uint64_t* rank_base,
                      unsigned long long* block_sums, uint64_t max_blocks, LevelState* st,
                      hipStream_t s);
void launch_place(uint64_t n, const uint64_t* settle, const uint64_t* fp, const uint64_t* pos,
                  uint64_t pos_base, const uint64_t* bits, const uint64_t* rank_base,
                  uint64_t* fp_out, uint64_t* pos_out, LevelState* st, int grid, hipStream_t s);
void launch_lookup(const uint8_t* blob, const uint64_t* offsets, uint64_t n, const uint64_t* bits,
                   const uint64_t* rank_base, const LevelState* st, const uint64_t* fp,
                   const uint64_t* pos, uint64_t count, uint64_t* result, int grid, hipStream_t s);

// Distributed (per-level count exchange) kernels.
void launch_dist_mark(int level, const uint64_t* keys, uint64_t n_local, uint64_t words,
                      uint32_t* A, uint32_t* C, int grid, hipStream_t s);
void launch_dist_hash_mark0(const uint8_t* blob, const uint64_t* offsets, uint64_t n,
                            uint64_t* kh, uint64_t* fp, uint64_t words0, uint32_t* A, uint32_t* C,
                            unsigned* status, int grid, hipStream_t s);
void launch_dist_counts(const uint32_t* A, const uint32_t* C, uint64_t positions, uint8_t* cnt,
                        int grid, hipStream_t s);
void launch_dist_pack(const uint8_t* sum, uint64_t positions, uint64_t* words_out, int grid,
                      hipStream_t s);
void launch_dist_resolve(int level, const uint64_t* keys_in, const uint32_t* idx_in, uint64_t n_local,
                         uint64_t words, uint64_t woff, const uint64_t* bits, uint64_t* keys_out,
                         uint32_t* idx_out, unsigned long long* out_count, uint64_t* settle,
                         int grid, hipStream_t s);
void launch_dist_place(uint64_t n, const uint64_t* settle, const uint64_t* fp, const uint64_t* pos,
                       uint64_t pos_base, const uint64_t* bits, const uint64_t* rank_base,
                       uint64_t per_rank, int nranks, unsigned long long* bucket_fill,
                       const unsigned long long* bucket_off, uint64_t* triples, unsigned* status,
                       int grid, hipStream_t s);
void launch_dist_count_owners(uint64_t n, const uint64_t* settle, const uint64_t* bits,
                              const uint64_t* rank_base, uint64_t per_rank, int nranks,
                              unsigned long long* counts, int grid, hipStream_t s);
void launch_dist_unpack(const uint64_t* triples, uint64_t count, uint64_t lo, uint64_t out_n,
                        uint64_t* fp_out, uint64_t* pos_out, unsigned* status, int grid,
                        hipStream_t s);
void launch_words_scan(const uint64_t* bits, uint64_t words, uint64_t* rank_base,
                       unsigned long long* block_sums, unsigned long long* total, hipStream_t s);

int default_grid(uint64_t work, int block);

// ---- host helpers (s3imph_host.cpp) -------------------------------------------
void set_err(char* err, size_t errlen, const std::string& msg);
int write_index_files(const std::string& dir, const uint8_t* mph_bin, uint64_t mph_len,
                      const uint64_t* fp, const uint64_t* pos, uint64_t n, const uint8_t* blob,
                      const uint64_t* offsets, std::string* msg);

}  // namespace s3imph
