/*
 * s3imph.h — C ABI of libs3imph.so, the MI355X-native MPHF (BBHash, gamma = 2.0)
 * builder for s3-inv-db indexes.
 *
 * This ABI is the drop-in boundary for the reference's MPHF stage,
 * format.StreamingMPHFBuilder (/root/reference/pkg/format/mphf_streaming.go).
 * The reference has no FFI layer of its own (pure Go, README.md:12); its caller
 * holds the concrete type at pkg/extsort/indexbuild.go:39 and constructs it at :81.
 * Each entry point below names the reference interface it replaces (file:line).
 * INTEGRATION.md shows the cgo binding a maintainer would add.
 *
 * Conventions
 *   - Plain pointers and sizes only; no C++ exceptions cross this boundary.
 *   - Every function returns an s3imph_status (0 = OK) unless stated otherwise;
 *     when `err`/`errlen` are given, a NUL-terminated message is written there,
 *     worded like the reference's Go errors ("build MPHF: ...").
 *   - Every call selects its own HIP device (cgo may call from any OS thread).
 *   - Keys are byte strings laid out as prefix_blob.bin + prefix_offsets.u64:
 *     key i = blob[offsets[i] .. offsets[i+1]), offsets has n+1 entries.
 *   - Outputs are byte-identical to the reference's mph.bin / mph_fp.u64 /
 *     mph_pos.u64 under the restated relab/bbhash spec ("parity").
 */
#ifndef S3IMPH_H
#define S3IMPH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define S3IMPH_ABI_VERSION 1

typedef enum s3imph_status {
    S3IMPH_OK = 0,
    S3IMPH_ERR_INVALID = 1,          /* bad argument / misuse */
    S3IMPH_ERR_DUP_KEY_HASH = 2,     /* duplicate FNV-1a key hashes: bbhash.New cannot place them (mphf_streaming.go:141-144) */
    S3IMPH_ERR_TOO_MANY_LEVELS = 3,  /* level budget exhausted (relab/bbhash maxLevel analogue) */
    S3IMPH_ERR_KEY_HASH_ZERO = 4,    /* a key hashes to 0: "MPHF Key(%d) returned 0" (mphf_streaming.go:248-252) */
    S3IMPH_ERR_HIP = 5,
    S3IMPH_ERR_RCCL = 6,
    S3IMPH_ERR_IO = 7,
    S3IMPH_ERR_NOMEM = 8,
    S3IMPH_ERR_FORMAT = 9,
    S3IMPH_ERR_INTERNAL = 10,
    S3IMPH_ERR_STATE = 11            /* e.g. Add after Build, use after Close */
} s3imph_status;

int s3imph_abi_version(void);
const char *s3imph_status_string(int status);

/* ------------------------------------------------------------------------
 * 1. StreamingMPHFBuilder mirror (pkg/format/mphf_streaming.go:29-232).
 *    Same method set: New(tempDir) / Add(prefix, pos) / Count() / Build(outDir) / Close().
 * ------------------------------------------------------------------------ */
typedef struct s3imph_builder s3imph_builder;

/* NewStreamingMPHFBuilder(tempDir) — mphf_streaming.go:48-64.
 * temp_dir must name an existing directory (or be NULL/""), as os.CreateTemp requires.
 * Keys are staged in host memory instead of a temp file. */
int s3imph_builder_new(const char *temp_dir, int device, s3imph_builder **out, char *err, size_t errlen);

/* Add(prefix, pos) — mphf_streaming.go:68-97. Copies the bytes. */
int s3imph_builder_add(s3imph_builder *b, const uint8_t *prefix, uint64_t len, uint64_t pos,
                       char *err, size_t errlen);

/* Batched Add (n keys in blob/offsets layout; pos may be NULL => pos_i = Count()+i).
 * Same effect as n calls of Add; exists to amortise the per-call FFI cost. */
int s3imph_builder_add_batch(s3imph_builder *b, const uint8_t *blob, const uint64_t *offsets,
                             const uint64_t *pos, uint64_t n, char *err, size_t errlen);

/* Capacity hint (no reference counterpart; the reference's IndexBuilder sizes its own
 * arrays from NewIndexBuilderWithCapacity, indexbuild.go:72-127): the device copy of the keys
 * is allocated once for n_keys keys of n_bytes key bytes, so Add never grows it.  Optional;
 * exceeding it is allowed (the buffers then grow).  A device allocation failure is not an
 * error: the build then runs from the host copy. */
int s3imph_builder_reserve(s3imph_builder *b, uint64_t n_keys, uint64_t n_bytes, char *err, size_t errlen);

/* Count() — mphf_streaming.go:100-102. */
uint64_t s3imph_builder_count(const s3imph_builder *b);

/* Build(outDir) — mphf_streaming.go:122-232: builds on the GPU and writes mph.bin,
 * mph_fp.u64, mph_pos.u64, prefix_blob.bin, prefix_offsets.u64 into out_dir.
 * Count()==0 writes the empty set (writeEmpty, :506-541). On failure mph.bin is removed (:159-168). */
int s3imph_builder_build(s3imph_builder *b, const char *out_dir, char *err, size_t errlen);

/* Build on several GPUs (s3imph_build_host_multi's num_gpus / devices / flags); the
 * default is the one device given to s3imph_builder_new.  No reference counterpart (the
 * reference builds on one CPU thread, mphf_streaming.go:141). */
int s3imph_builder_set_gpus(s3imph_builder *b, int num_gpus, const int *devices, unsigned flags);

/* Close() — mphf_streaming.go:105-114. Frees everything; b is invalid afterwards. */
int s3imph_builder_close(s3imph_builder *b);

/* ------------------------------------------------------------------------
 * 2. One-shot host-memory build: replaces bbhash.New + MarshalBinary +
 *    computeHashPositionsReverseMap + the scatter loop (mphf_streaming.go:141-204).
 * ------------------------------------------------------------------------ */

/* fp_out/pos_out: caller-allocated n entries each. *mph_bin is allocated by the
 * library (free with s3imph_free); n == 0 gives *mph_bin = NULL, *mph_len = 0.
 * pos may be NULL => pos_i = i (the production caller, indexbuild.go:160-175). */
int s3imph_build_host(int device, const uint8_t *blob, const uint64_t *offsets, const uint64_t *pos,
                      uint64_t n, uint64_t *fp_out, uint64_t *pos_out, uint8_t **mph_bin,
                      uint64_t *mph_len, char *err, size_t errlen);

/* The same build with mph.bin marshalled into the caller's buffer (mph_cap bytes, at least
 * s3imph_mph_bin_bound(n); *mph_len gets its size), which a pipeline reuses across calls as it
 * reuses fp_out / pos_out: no library allocation, no fresh pages to fault in. */
int s3imph_build_host_into(int device, const uint8_t *blob, const uint64_t *offsets, const uint64_t *pos,
                           uint64_t n, uint64_t *fp_out, uint64_t *pos_out, uint8_t *mph_out, uint64_t mph_cap,
                           uint64_t *mph_len, char *err, size_t errlen);
/* An upper bound on mph.bin's size for n keys (0 for n == 0). */
uint64_t s3imph_mph_bin_bound(uint64_t n);

void s3imph_free(void *p);

/* Free the device workspaces the host-memory builds keep between calls (the default context
 * of every device, the cached per-rank contexts of s3imph_build_host_multi); the next build
 * allocates again.  Call when no build is running (a pipeline between index builds, or
 * before handing HBM to something else).  A build that runs out of HBM does the same for the
 * caches it is not using (those no other thread is building on) and retries once before
 * returning S3IMPH_ERR_NOMEM (s3imph_build_host[_into|_multi], s3imph_builder_build,
 * s3imph_build_device, s3imph_ctx_reserve). */
int s3imph_release_workspaces(void);

/* Multi-GPU host-memory build for ONE calling process (the reference's caller is one
 * process: indexbuild.go:506-518 -> Build).  num_gpus host threads, one per GPU, each
 * run the sharded rank build of section 4 on a contiguous key shard of about equal key
 * bytes; collectives are RCCL communicators made in-process (ncclCommInitAll, xGMI) or,
 * when `devices` repeat or S3IMPH_MULTI_HOST_TRANSPORT is set, in-process host copies.
 * Each rank writes its output segments straight to their global offsets in fp_out /
 * pos_out; mph.bin comes from rank 0 (identical on every rank).  devices may be NULL
 * (GPUs 0 .. num_gpus-1).  num_gpus == 1 without S3IMPH_MULTI_FORCE_SHARDED is
 * s3imph_build_host.  Outputs equal s3imph_build_host's byte for byte. */
#define S3IMPH_MULTI_FORCE_SHARDED 1u   /* the sharded (multi-GPU) build even for one GPU */
#define S3IMPH_MULTI_HOST_TRANSPORT 2u  /* host-copy collectives instead of RCCL */
#define S3IMPH_MULTI_BITMAP 4u          /* the bitmap decomposition (s3imph_ctx_set_dist_mode) */
int s3imph_build_host_multi(int num_gpus, const int *devices, unsigned flags, const uint8_t *blob,
                            const uint64_t *offsets, const uint64_t *pos, uint64_t n, uint64_t *fp_out,
                            uint64_t *pos_out, uint8_t **mph_bin, uint64_t *mph_len, char *err, size_t errlen);

/* Emit the 5 files of the MPHF stage with the reference's framing:
 * mph.bin raw (mphf_streaming.go:152-169), mph_fp.u64 / mph_pos.u64 as S3ID
 * u64 arrays (writeArraysParallel :546-596; ArrayWriter writer.go:19-46,79-96,113-140;
 * header format.go:6-32), prefix_blob.bin + prefix_offsets.u64 with the N+1 sentinel
 * (BlobWriter writer.go:148-237). n == 0 reproduces writeEmpty (:506-541). */
int s3imph_write_index_files(const char *out_dir, const uint8_t *mph_bin, uint64_t mph_len,
                             const uint64_t *fp, const uint64_t *pos, uint64_t n,
                             const uint8_t *blob, const uint64_t *offsets, char *err, size_t errlen);

/* ------------------------------------------------------------------------
 * 3. Device-resident build (inputs already in HBM; what bench.py times).
 * ------------------------------------------------------------------------ */
typedef struct s3imph_ctx s3imph_ctx;

typedef struct s3imph_build_info {
    int32_t status;            /* s3imph_status of the build */
    uint32_t num_levels;       /* BBHash levels */
    uint64_t total_words;      /* u64 words over all level bit vectors */
    uint64_t mph_bin_len;      /* bytes of the marshalled mph.bin */
    uint64_t big_levels;       /* levels run as full-grid kernels (rest: single-workgroup tail) */
    uint64_t n_keys;           /* keys in the whole build (all ranks) */
} s3imph_build_info;

int s3imph_ctx_create(int device, s3imph_ctx **out, char *err, size_t errlen);
int s3imph_ctx_destroy(s3imph_ctx *ctx);

/* Pre-size the workspace for up to max_keys keys on this GPU (optional: builds
 * grow it on demand, but a reserved workspace keeps allocation out of timed runs). */
int s3imph_ctx_reserve(s3imph_ctx *ctx, uint64_t max_keys, uint64_t max_global_keys);

/* Enqueue the whole build on `stream` (a hipStream_t; NULL = the ctx's own stream,
 * a blocking stream, i.e. ordered after work queued on the legacy NULL stream) and
 * wait for it.  d_blob must be readable up to offsets[n] rounded up to 8 bytes.
 * d_pos may be NULL (identity).  d_fp_out / d_pos_out: n entries each.
 * The level bit vectors stay on the device until s3imph_ctx_mph_bin(). */
int s3imph_build_device(s3imph_ctx *ctx, const uint8_t *d_blob, const uint64_t *d_offsets,
                        const uint64_t *d_pos, uint64_t n, uint64_t *d_fp_out, uint64_t *d_pos_out,
                        void *stream, s3imph_build_info *info);

/* Marshal the last build's level bit vectors into mph.bin bytes (D2H + framing). */
int s3imph_ctx_mph_bin(s3imph_ctx *ctx, uint8_t *out, uint64_t cap, uint64_t *len);

/* Per-stage device times of the last build (ms), recorded with HIP events on the
 * build stream when profiling is on (on = 1: every stage; on = 2: only the level-0
 * hash / route stage, two events per build).  names: comma-separated stage names. */
int s3imph_ctx_set_profiling(s3imph_ctx *ctx, int on);
int s3imph_ctx_stage_times(s3imph_ctx *ctx, float *ms, int cap, int *count, char *names, size_t names_len);

/* ------------------------------------------------------------------------
 * 4. Multi-GPU build: one process per GPU, RCCL over xGMI.  No reference
 *    counterpart (the reference builds in one process, mphf_streaming.go:141);
 *    the outputs are byte-identical to the single-GPU build.
 *
 *    Keys are sharded in contiguous index ranges.  At each large BBHash level
 *    rank r owns a contiguous range of the level's bit positions: every rank
 *    routes its active records to the owners (one all-to-all), each owner
 *    resolves collisions and ranks for its range, and its settled keys fill
 *    consecutive local output slots.  Small levels run replicated on every rank
 *    (outputs written by rank 0).  A rank's outputs are therefore a few
 *    contiguous segments of mph_fp / mph_pos (s3imph_dist_segments), which the
 *    caller writes at their global offsets (e.g. pwrite into the column files).
 * ------------------------------------------------------------------------ */

/* Rank 0 creates the 128-byte RCCL unique id; the host broadcasts it.
 * s3imph_ctx_create_dist is collective: every rank calls it with the same id.  At
 * nranks > 1 it also splits a second communicator off the first (ncclCommSplit, kept only
 * if every rank got one): the bitmap decomposition's output exchange runs on it, on its own
 * stream, beside the next levels' collectives. */
int s3imph_dist_unique_id(uint8_t id_out[128]);

int s3imph_ctx_create_dist(int device, const uint8_t id[128], int rank, int nranks,
                           s3imph_ctx **out, char *err, size_t errlen);

/* Host-callback collectives (test transport: several ranks may share one GPU).
 * allgather: recv (nranks * bytes) = every rank's send, in rank order.
 * alltoallv: send_bytes[q] bytes at send + send_off[q] go to rank q; the bytes from
 *            rank q land at recv + recv_off[q] (recv_bytes[q]).  Host pointers.
 * Each returns 0 on success. */
typedef struct s3imph_host_comm {
    void *user;
    int (*allgather)(void *user, const void *send, void *recv, uint64_t bytes);
    int (*alltoallv)(void *user, const void *send, const uint64_t *send_off, const uint64_t *send_bytes,
                     void *recv, const uint64_t *recv_off, const uint64_t *recv_bytes);
} s3imph_host_comm;

int s3imph_ctx_create_dist_host(int device, const s3imph_host_comm *comm, int rank, int nranks,
                                s3imph_ctx **out, char *err, size_t errlen);

/* Decomposition of the sharded levels (every rank of a build must choose the same; the
 * default comes from S3IMPH_DIST_MODE=route|bitmap, else route):
 *   S3IMPH_DIST_ROUTE  — position-range ownership: each level's 24-byte records are routed
 *                        to the rank owning their position range (one all-to-all per level);
 *   S3IMPH_DIST_BITMAP — the per-level collision bitmap reduced over RCCL: count lanes
 *                        (min(local count, 2), one byte per position) reduce-scattered, the
 *                        final bits all-gathered, each rank settles its own keys; one
 *                        all-to-all of the settled (p, fp, pos) at the end.  A level larger
 *                        than its host-side bound reruns the build on ROUTE.
 * Both give byte-identical outputs.  No reference counterpart (bbhash.New runs on one
 * thread, mphf_streaming.go:141).  S3IMPH_DIST_STRICT or-ed into BITMAP: no fallback — a
 * level past its size bound fails the build (S3IMPH_ERR_INTERNAL) instead of rerunning on
 * ROUTE (a benchmark of the bitmap decomposition uses it so it never times the other one); a
 * capacity miss (a reservation-slot overflow, a settle-fed level without its buffers) reruns
 * the bitmap decomposition once in its conservative form in either mode.  With one rank,
 * ROUTE is the single-GPU build (nothing to route). */
#define S3IMPH_DIST_ROUTE 0
#define S3IMPH_DIST_BITMAP 1
#define S3IMPH_DIST_STRICT 0x100
int s3imph_ctx_set_dist_mode(s3imph_ctx *ctx, int mode);

/* This rank holds keys [key_base, key_base + n_local) of the global set (the
 * shard's blob/offsets/pos, offsets relative to d_blob; d_pos NULL => pos_i =
 * key_base + i).  On return *out_n local outputs are in d_fp_out / d_pos_out
 * (capacity out_cap entries, at least s3imph_dist_out_cap()).  mph.bin is
 * identical on every rank. */
int s3imph_build_device_dist(s3imph_ctx *ctx, const uint8_t *d_blob, const uint64_t *d_offsets,
                             const uint64_t *d_pos, uint64_t n_local, uint64_t key_base,
                             uint64_t *d_fp_out, uint64_t *d_pos_out, uint64_t out_cap,
                             uint64_t *out_n, void *stream, s3imph_build_info *info);

/* The last build's output segments of this rank: seg[3i] = first global position p,
 * seg[3i+1] = count, seg[3i+2] = offset in d_fp_out / d_pos_out.  *count = segments. */
int s3imph_dist_segments(s3imph_ctx *ctx, uint64_t *seg, uint64_t cap, uint64_t *count);

/* Output capacity (entries) one rank needs for a build of n_global keys. */
uint64_t s3imph_dist_out_cap(s3imph_ctx *ctx, uint64_t n_global);

/* Message of the last failed device-resident build on ctx ("" if none). */
const char *s3imph_ctx_last_error(s3imph_ctx *ctx);

/* ------------------------------------------------------------------------
 * 5. Batched lookup on the device: MPHF.Lookup (pkg/format/mphf.go:275-302)
 *    over the last build's levels, for n query keys; result[i] = pos or
 *    UINT64_MAX when not found.  Self-verifies a build (VerifyMPHF, :372-393).
 * ------------------------------------------------------------------------ */
/* OpenMPHF (pkg/format/mphf.go:186-247): load a marshalled mph.bin (any builder's, e.g.
 * an index on disk) into ctx in place of its last build, so that s3imph_lookup_device
 * answers MPHF.Lookup against it.  S3IMPH_ERR_FORMAT (message: s3imph_ctx_last_error)
 * on a malformed file; len == 0 is the empty MPHF (writeEmpty's 0-byte mph.bin). */
int s3imph_ctx_load_mph_bin(s3imph_ctx *ctx, const uint8_t *mph_bin, uint64_t len);

int s3imph_lookup_device(s3imph_ctx *ctx, const uint8_t *d_blob, const uint64_t *d_offsets, uint64_t n,
                         const uint64_t *d_fp, const uint64_t *d_pos, uint64_t count,
                         uint64_t *d_result, void *stream);

/* ------------------------------------------------------------------------
 * 5b. The rest of IndexBuilder.Finalize (pkg/extsort/indexbuild.go:393-415,
 *     474-503; pkg/format/depthindex.go:32-96), from the same sorted prefix blob:
 *       depth.u32                 per prefix: row.Depth (indexbuild.go:185), or when
 *                                 depths == NULL the aggregator's '/' count
 *                                 (aggregator.go:44-60);
 *       subtree_end.u64           last position of the prefix's subtree (the ancestor
 *                                 stack, indexbuild.go:154-248);
 *       max_depth_in_subtree.u32  deepest depth in that subtree;
 *       depth_offsets.u64         maxDepth + 2 offsets into depth_positions;
 *       depth_positions.u64       positions grouped by depth, ascending in a depth.
 *     Positions are the Add order 0..n-1 (indexbuild.go:160).  The prefixes must be
 *     byte-sorted (the reference's Add order); the blob on the device is readable up to
 *     round_up(offsets[n], 8) as for the build.
 * ------------------------------------------------------------------------ */
/* Replaces DepthIndexBuilder.Build + writeSubtreeArrays + the depth.u32 writer: computes
 * on `device` and writes the five files into out_dir (S3ID framing, format.go:25-32). */
int s3imph_finalize_index_host(int device, const uint8_t *blob, const uint64_t *offsets,
                               const uint32_t *depths, uint64_t n, const char *out_dir, char *err,
                               size_t errlen);
/* Device form: all arrays in HBM (depths nullable).  depth_offsets holds offsets_cap
 * entries; *max_depth receives maxDepth, and S3IMPH_ERR_INVALID comes back (outputs other
 * than depth undefined) when offsets_cap < maxDepth + 2.  Synchronous on `stream`. */
int s3imph_finalize_index_device(s3imph_ctx *ctx, const uint8_t *d_blob, const uint64_t *d_offsets,
                                 const uint32_t *d_depths, uint64_t n, uint32_t *d_depth,
                                 uint64_t *d_subtree_end, uint32_t *d_max_depth_in_subtree,
                                 uint64_t *d_depth_positions, uint64_t *d_depth_offsets,
                                 uint64_t offsets_cap, uint32_t *max_depth, void *stream);

/* ------------------------------------------------------------------------
 * 5b. manifest.json (optional part): size + SHA-256 of every index file.
 *     Replaces format.WriteManifest / VerifyManifest (pkg/format/manifest.go:33-138), which
 *     IndexBuilder.Finalize calls after the other files (indexbuild.go:429-432).  The JSON
 *     text is Go's json.MarshalIndent output (map keys sorted; created_at RFC 3339 UTC).
 *     Host-only; files are hashed in parallel, with the x86 SHA extensions when present.
 * ------------------------------------------------------------------------ */
/* WriteManifest(dir, nodeCount, maxDepth): absent index files are skipped; error text
 * "write manifest: ..." as IndexBuilder wraps it. */
int s3imph_write_manifest(const char *out_dir, uint64_t node_count, uint32_t max_depth, char *err,
                          size_t errlen);
/* ReadManifest + VerifyManifest: S3IMPH_ERR_FORMAT on a size or checksum mismatch
 * ("file %s: checksum mismatch"), S3IMPH_ERR_IO when a listed file is missing. */
int s3imph_verify_manifest(const char *dir, char *err, size_t errlen);
/* checksumFile (manifest.go:140-155): lowercase hex SHA-256 of a file into hex_out (65 B,
 * NUL-terminated); portable != 0 forces the portable compression loop (tests). */
int s3imph_sha256_file(const char *path, int portable, char hex_out[65], char *err, size_t errlen);

/* ------------------------------------------------------------------------
 * 6. Deterministic synthetic prefix sets (bench/test support, not on the path).
 *    kind: 0 = s3-like, lengths uniform in [max(10, avg/2), 3avg/2],
 *              distinct and byte-sorted;
 *          1 = lengths log-uniform in [1, 1024] (C5), each raised to the base-64 digit
 *              count of its index where that is longer (4 bytes hold 16.7M keys), so
 *              keys stay distinct; not byte-sorted.
 *    Key 0 = "" when lo == 0 (the root prefix).  Generate keys
 *    [lo, lo+n) of the global sequence: call once with blob == NULL to get the
 *    byte count, then again to fill.  offsets are relative to the shard start.
 * ------------------------------------------------------------------------ */
int s3imph_gen_keys(int kind, uint64_t seed, uint32_t avg_len, uint64_t lo, uint64_t n,
                    uint8_t *blob, uint64_t *offsets, uint64_t *total_bytes);

/* ------------------------------------------------------------------------
 * 7. Developer knobs (not on the path; no reference counterpart).
 *    The library reads its A/B geometry knobs, test-only fallbacks and fault-injection hooks
 *    (S3IMPH_P0, S3IMPH_L20, S3IMPH_FAULT_DUP_REC, S3IMPH_HASH_ONLY, S3IMPH_DIST_SWITCH, ...;
 *    DESIGN.md section 5) from the environment ONLY after s3imph_dev_knobs(1), so a stray
 *    variable in an embedding process cannot change a production build.  The documented user
 *    settings S3IMPH_DIST_MODE, S3IMPH_PINNED_KEEP and S3IMPH_DEBUG are read regardless.
 *    Knobs are sampled when a context is created (some on first use): call this first.
 * ------------------------------------------------------------------------ */
int s3imph_dev_knobs(int on);

#ifdef __cplusplus
}
#endif

#endif /* S3IMPH_H */
