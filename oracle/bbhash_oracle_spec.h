/*
 * bbhash_oracle_spec.h — every constant and toggle of the restated relab/bbhash
 * algorithm, kept in ONE place so that pinning a toggle
 * against upstream bytes is a one-line change.  TEST INFRASTRUCTURE ONLY.
 *
 * The product path keeps its own copy (s3-inv-db_amd/csrc/bbhash_spec.h) on
 * purpose: the two are written independently and a test asserts they agree.
 *
 * Toggle status (relab/bbhash v0.0.0-20250331135148-7358f69256fb, not vendored):
 *   T1 hash constants/structure  : fasthash mix, m = 0x880355f21e6d1965          (restated)
 *   T2 position reduction        : true 64-bit modulo by 64*words                (restated)
 *   T3 words formula             : ceil(gamma*n/64), gamma = 2 -> ceil(n/32)      (restated)
 *   T4 MarshalBinary framing     : [u64 partitions][u64 levels]{[u64 words][..]} (restated)
 *   T5 reverse map serialized?   : no                                             (restated)
 *   T6 max levels                : ORC_MAX_LEVELS                                 (restated)
 *   T7 level numbering           : from 0                                         (restated)
 *   T8 partitions                : 1 (no Partitions() option at mphf_streaming.go:141)
 */
#ifndef BBHASH_ORACLE_SPEC_H
#define BBHASH_ORACLE_SPEC_H

#define ORC_FNV_OFFSET64 0xcbf29ce484222325ULL /* 14695981039346656037 */
#define ORC_FNV_PRIME64 0x00000100000001b3ULL  /* 1099511628211 */

#define ORC_HASH_M 0x880355f21e6d1965ULL
#define ORC_MIX_MUL 0x2127599bf4325c37ULL

#define ORC_GAMMA_NUM 2ULL /* gamma = 2.0 (mphf_streaming.go:141) */
#define ORC_GAMMA_DEN 1ULL
#define ORC_MIN_WORDS 1ULL

#define ORC_MAX_LEVELS 64u
#define ORC_MARSHAL_PARTITION_HDR 1

#define ORC_OK 0
#define ORC_ERR_TOO_MANY_LEVELS 3
#define ORC_ERR_KEY_ZERO 4
#define ORC_ERR_FORMAT 9
#define ORC_ERR_INTERNAL 10

#endif
