// s3imph_multi.hip — multi-GPU builds behind the host-memory boundary.
//
// The reference's caller is ONE process: IndexBuilder.FinalizeWithContext -> buildMPHF
// -> StreamingMPHFBuilder.Build (/root/reference/pkg/extsort/indexbuild.go:506-518,
// pkg/format/mphf_streaming.go:122-232).  s3imph_build_host_multi (and the builder mirror
// with s3imph_builder_set_gpus) gives that single caller every GPU of the node: one host
// thread per GPU runs the rank build of s3imph_build_device_dist (position-range
// ownership, s3imph_dist.hip) on a contiguous key shard, balanced by key BYTES (SURVEY
// §8e: C5's lengths are skewed).  Collectives: RCCL communicators made in-process with
// ncclCommInitAll (xGMI between the GPUs), or — when ranks share a device, or on request
// — an in-process host-copy transport (ThreadComm).  Each rank copies its output segments
// straight to their global offsets in the caller's fp_out / pos_out; rank 0 marshals
// mph.bin (identical on every rank).  Outputs are byte-identical to the single-GPU build.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "s3imph_ctx.h"

namespace s3imph {

namespace {

// ------------------------------------------------------------ in-process transport ----
// P host threads, one per rank, meet at a generation barrier; every collective moves the
// device bytes through host buffers.  A rank that fails aborts the hub, so its peers
// leave their barrier with an error instead of waiting forever.
struct ThreadHub {
  int P = 1;
  // serial (S3IMPH_HOST_SERIAL, a measurement mode): the ranks' device work never overlaps —
  // a rank holds `token` from the end of one collective to the point the next one has synced
  // its stream, so each kernel of a rank runs alone on the shared GPU and its trace duration
  // is that rank's device time (the P = 8 geometry on one GPU)
  bool serial = false;
  std::mutex token;
  std::vector<char> held;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<std::vector<uint8_t>> slot;  // per rank
  std::vector<std::vector<uint64_t>> soff, sbytes;
  // every rank on one device: the gathers and all-to-alls copy device to device, each rank
  // from its peers' published send buffers (dptr), instead of through host memory
  bool same_dev = false;
  std::vector<const uint8_t*> dptr;

  explicit ThreadHub(int p) : P(p), held(p, 0), slot(p), soff(p), sbytes(p), dptr(p, nullptr) {}
  void seg_begin(int r) {  // this rank's device work starts
    if (!serial || held[r]) return;
    token.lock();
    held[r] = 1;
  }
  void seg_end(int r) {  // ... and has completed (its stream synchronised)
    if (!serial || !held[r]) return;
    held[r] = 0;
    token.unlock();
  }
  void reset() {
    std::lock_guard<std::mutex> lk(mu);
    arrived = 0;
    aborted = false;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
  // the host staging of the collectives (sized by the largest exchange so far) back to the OS
  void free_buffers() {
    for (auto& v : slot) std::vector<uint8_t>().swap(v);
    for (auto& v : soff) std::vector<uint64_t>().swap(v);
    for (auto& v : sbytes) std::vector<uint64_t>().swap(v);
  }
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw Fail{S3IMPH_ERR_RCCL, "build MPHF: a peer rank failed"};
    const uint64_t g = gen;
    if (++arrived == P) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    if (gen == g) throw Fail{S3IMPH_ERR_RCCL, "build MPHF: a peer rank failed"};
  }
};

struct ThreadComm final : Comm {
  ThreadHub* hub = nullptr;
  void d2h(void* h, const void* d, uint64_t bytes, hipStream_t s) {
    if (bytes) HIPCHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
  }
  void h2d(void* d, const void* h, uint64_t bytes, hipStream_t s) {
    if (bytes) HIPCHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
  }
  void d2d(void* d, const void* src, uint64_t bytes, hipStream_t s) {
    if (bytes) HIPCHECK(hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, s));
  }
  void allgather(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    if (hub->same_dev) {
      hub->dptr[rank] = static_cast<const uint8_t*>(d_send);
      HIPCHECK(hipStreamSynchronize(s));  // the send buffer is complete
      hub->seg_end(rank);
      hub->barrier();
      for (int r = 0; r < nranks; ++r) d2d(static_cast<uint8_t*>(d_recv) + (uint64_t)r * bytes, hub->dptr[r], bytes, s);
      HIPCHECK(hipStreamSynchronize(s));
      hub->barrier();  // every rank has read the peers' buffers before they change
      hub->seg_begin(rank);
      return;
    }
    auto& mine = hub->slot[rank];
    mine.resize(bytes + 1);
    d2h(mine.data(), d_send, bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->seg_end(rank);
    hub->barrier();
    for (int r = 0; r < nranks; ++r) h2d(static_cast<uint8_t*>(d_recv) + (uint64_t)r * bytes, hub->slot[r].data(), bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->barrier();  // every rank has read the slots before they are reused
    hub->seg_begin(rank);
  }
  void reduce_scatter_u8(const void* d_send, void* d_recv, uint64_t bytes, hipStream_t s) override {
    auto& mine = hub->slot[rank];
    mine.resize(bytes * nranks + 1);
    d2h(mine.data(), d_send, bytes * nranks, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->seg_end(rank);
    hub->barrier();
    std::vector<uint8_t> sum(bytes + 1, 0);
    for (int r = 0; r < nranks; ++r) {
      const uint8_t* q = hub->slot[r].data() + (uint64_t)rank * bytes;
      for (uint64_t i = 0; i < bytes; ++i) sum[i] = (uint8_t)(sum[i] + q[i]);
    }
    h2d(d_recv, sum.data(), bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->barrier();
    hub->seg_begin(rank);
  }
  void allreduce_u64(const unsigned long long* d_in, unsigned long long* d_out, uint64_t count,
                     hipStream_t s) override {
    const uint64_t bytes = 8 * count;
    auto& mine = hub->slot[rank];
    mine.resize(bytes + 1);
    d2h(mine.data(), d_in, bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->seg_end(rank);
    hub->barrier();
    std::vector<unsigned long long> sum(count, 0);
    for (int r = 0; r < nranks; ++r)
      for (uint64_t i = 0; i < count; ++i) {
        unsigned long long v;
        std::memcpy(&v, hub->slot[r].data() + 8 * i, 8);
        sum[i] += v;
      }
    h2d(d_out, sum.data(), bytes, s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->barrier();
    hub->seg_begin(rank);
  }
  void alltoallv(const void* d_send, const uint64_t* soff, const uint64_t* sbytes, void* d_recv,
                 const uint64_t* roff, const uint64_t* rbytes, hipStream_t s) override {
    if (hub->same_dev) {
      hub->dptr[rank] = static_cast<const uint8_t*>(d_send);
      hub->soff[rank].assign(soff, soff + nranks);
      hub->sbytes[rank].assign(sbytes, sbytes + nranks);
      HIPCHECK(hipStreamSynchronize(s));
      hub->seg_end(rank);
      hub->barrier();
      for (int q = 0; q < nranks; ++q) {
        if (hub->sbytes[q][rank] != rbytes[q]) throw Fail{S3IMPH_ERR_INTERNAL, "alltoallv: size mismatch"};
        d2d(static_cast<uint8_t*>(d_recv) + roff[q], hub->dptr[q] + hub->soff[q][rank], rbytes[q], s);
      }
      HIPCHECK(hipStreamSynchronize(s));
      hub->barrier();
      hub->seg_begin(rank);
      return;
    }
    // this rank's send regions, packed back to back in its slot
    auto& mine = hub->slot[rank];
    auto& po = hub->soff[rank];
    auto& pb = hub->sbytes[rank];
    po.assign(nranks, 0);
    pb.assign(sbytes, sbytes + nranks);
    uint64_t tot = 0;
    for (int q = 0; q < nranks; ++q) {
      po[q] = tot;
      tot += sbytes[q];
    }
    mine.resize(tot + 1);
    for (int q = 0; q < nranks; ++q)
      d2h(mine.data() + po[q], static_cast<const uint8_t*>(d_send) + soff[q], sbytes[q], s);
    HIPCHECK(hipStreamSynchronize(s));
    hub->seg_end(rank);
    hub->barrier();
    for (int q = 0; q < nranks; ++q) {
      if (hub->sbytes[q][rank] != rbytes[q]) throw Fail{S3IMPH_ERR_INTERNAL, "alltoallv: size mismatch"};
      h2d(static_cast<uint8_t*>(d_recv) + roff[q], hub->slot[q].data() + hub->soff[q][rank], rbytes[q], s);
    }
    HIPCHECK(hipStreamSynchronize(s));
    hub->barrier();
    hub->seg_begin(rank);
  }
};

// A set of per-rank contexts for one device list and transport, reused across builds
// (workspaces, RCCL communicators and pinned stagers persist).
struct MultiCtx {
  std::vector<int> devs;
  bool host_transport = false;
  std::vector<s3imph_ctx*> ctx;
  std::unique_ptr<ThreadHub> hub;
  std::mutex mu;
  std::mutex abort_mu;
  bool aborted = false;  // a rank failed alone: the transport was torn down, the set is dropped
  bool released = false;  // its contexts were freed (release_sets): a caller takes a fresh set
  // Unblock every rank: the host hub wakes its barrier waiters with an error; RCCL
  // communicators are aborted (their pending kernels exit, so peers blocked in a stream
  // sync return) and cannot be reused.
  void abort_all() {
    std::lock_guard<std::mutex> lk(abort_mu);
    if (aborted) return;
    aborted = true;
    if (hub) hub->abort();
    for (s3imph_ctx* c : ctx) {
      if (c->d.comm) c->d.comm->abort();
      if (c->d.xcomm) c->d.xcomm->abort();
    }
  }
};

std::mutex g_multi_mu;
std::map<std::tuple<std::vector<int>, bool, uint64_t>, std::unique_ptr<MultiCtx>> g_multi;
std::vector<std::unique_ptr<MultiCtx>> g_retired;  // aborted sets (see build_from_host_multi)

// Free the contexts (workspaces, communicators) of sets already taken out of g_multi, once no
// build holds them, and the host transport's staging; the emptied shells (a few words each)
// stay allocated (g_retired) for callers that still hold a pointer and will see `released`.
void release_sets(std::vector<std::unique_ptr<MultiCtx>> sets) {
  for (auto& mc : sets) {
    {
      std::lock_guard<std::mutex> lk(mc->mu);
      for (s3imph_ctx* c : mc->ctx) s3imph_ctx_destroy(c);
      mc->ctx.clear();
      std::vector<s3imph_ctx*>().swap(mc->ctx);
      if (mc->hub) mc->hub->free_buffers();
      mc->released = true;
    }
    std::lock_guard<std::mutex> glk(g_multi_mu);
    g_retired.push_back(std::move(mc));
  }
}

// The cached set for (devs, transport, S3IMPH_DIST_SWITCH); another cached set over the same
// devices (a different switch: tests) is released first, so sets never pile up in HBM.
MultiCtx* multi_ctx(const std::vector<int>& devs, bool host_transport, std::string* msg) {
  uint64_t sw = kDistSwitchKeysDefault;  // contexts read S3IMPH_DIST_SWITCH when made
  if (const char* e = dev_env("S3IMPH_DIST_SWITCH")) sw = std::strtoull(e, nullptr, 10);
  auto key = std::make_tuple(devs, host_transport, sw);
  {
    std::vector<std::unique_ptr<MultiCtx>> stale;
    {
      std::lock_guard<std::mutex> lk(g_multi_mu);
      auto it = g_multi.find(key);
      if (it != g_multi.end()) return it->second.get();
      for (auto jt = g_multi.begin(); jt != g_multi.end();) {
        if (std::get<0>(jt->first) == devs && std::get<1>(jt->first) == host_transport) {
          stale.push_back(std::move(jt->second));
          jt = g_multi.erase(jt);
        } else {
          ++jt;
        }
      }
    }
    release_sets(std::move(stale));
  }
  std::lock_guard<std::mutex> lk(g_multi_mu);
  auto it = g_multi.find(key);  // (another caller may have made it meanwhile)
  if (it != g_multi.end()) return it->second.get();
  auto mc = std::make_unique<MultiCtx>();
  mc->devs = devs;
  mc->host_transport = host_transport;
  const int P = (int)devs.size();
  std::vector<Comm*> comms(P, nullptr);
  if (host_transport) {
    mc->hub = std::make_unique<ThreadHub>(P);
    mc->hub->same_dev = std::all_of(devs.begin(), devs.end(), [&](int d) { return d == devs[0]; });
    for (int r = 0; r < P; ++r) {
      ThreadComm* tc = new ThreadComm();
      tc->hub = mc->hub.get();
      comms[r] = tc;
    }
  } else {
    std::vector<ncclComm_t> nc(P);
    const ncclResult_t rr = ncclCommInitAll(nc.data(), P, devs.data());
    if (rr != ncclSuccess) {
      *msg = std::string("ncclCommInitAll: ") + ncclGetErrorString(rr);
      return nullptr;
    }
    for (int r = 0; r < P; ++r) {
      RcclComm* rc = new RcclComm();
      rc->comm = nc[r];
      comms[r] = rc;
    }
  }
  for (int r = 0; r < P; ++r) {
    comms[r]->rank = r;
    comms[r]->nranks = P;
    s3imph_ctx* c = make_dist_ctx(devs[r], comms[r], r, P, msg);
    if (!c) {
      for (int q = r + 1; q < P; ++q) delete comms[q];
      for (s3imph_ctx* x : mc->ctx) s3imph_ctx_destroy(x);
      return nullptr;
    }
    mc->ctx.push_back(c);
  }
  MultiCtx* out = mc.get();
  g_multi[key] = std::move(mc);
  return out;
}

// Contiguous key shards [cuts[r], cuts[r+1]) holding about equal key bytes.
std::vector<uint64_t> byte_cuts(const uint64_t* offsets, uint64_t n, int P) {
  std::vector<uint64_t> cuts(P + 1, 0);
  const uint64_t b0 = offsets[0], tot = offsets[n] - b0;
  cuts[P] = n;
  for (int r = 1; r < P; ++r) {
    const uint64_t target = b0 + (uint64_t)((__uint128_t)tot * (uint64_t)r / (uint64_t)P);
    cuts[r] = (uint64_t)(std::lower_bound(offsets, offsets + n, target) - offsets);
    cuts[r] = std::max(cuts[r], cuts[r - 1]);
  }
  return cuts;
}

// One rank: stage its shard, build, copy its output segments to their global offsets.
int rank_build(s3imph_ctx* c, const uint8_t* blob, const uint64_t* offsets, const uint64_t* pos, uint64_t n,
               uint64_t lo, uint64_t hi, uint64_t* fp_out, uint64_t* pos_out, std::vector<uint8_t>* mph,
               std::string* msg) {
  std::lock_guard<std::mutex> lk(c->mu);
  HIPCHECK(hipSetDevice(c->device));
  const uint64_t nl = hi - lo, b0 = offsets[lo], nbytes = offsets[hi] - b0;
  const uint64_t cap = dist_out_cap(c, n);
  const uint64_t bcap = ((nbytes + 7) & ~7ull) + 8;
  if (bcap > c->s_blob_cap) {
    c->s_blob_cap = 0;
    dalloc(c->s_blob, bcap);
    c->s_blob_cap = bcap;
  }
  const uint64_t need = std::max(cap, nl + 1);
  if (need > c->s_cap) {  // s_cap keys: s_offsets holds s_cap + 1 words (as build_from_host's)
    c->s_cap = 0;
    dalloc(c->s_offsets, need + 1);
    dalloc(c->s_fp, need);
    dalloc(c->s_posout, need);
    c->s_cap = need;
  }
  if (pos) ensure_s_pos(c, need);
  hipStream_t s = c->own_stream;
  HIPCHECK(hipStreamSynchronize(s));
  staged_copy(c, true, c->s_blob, blob + b0, nbytes);
  staged_copy(c, true, c->s_offsets, offsets + lo, (nl + 1) * 8, b0);
  if (pos) staged_copy(c, true, c->s_pos, pos + lo, nl * 8);
  uint64_t out_n = 0;
  s3imph_build_info info{};
  c->last_msg.clear();
  int rc = build_dist(c, c->s_blob, c->s_offsets, pos ? c->s_pos : nullptr, nl, lo, c->s_fp, c->s_posout, cap, &out_n,
                      s, &info, msg);
  if (rc != S3IMPH_OK) return rc;
  for (size_t i = 0; i + 2 < c->d.seg.size(); i += 3) {
    const uint64_t p = c->d.seg[i], cnt = c->d.seg[i + 1], off = c->d.seg[i + 2];
    if (p + cnt > n || off + cnt > out_n) {
      *msg = "build MPHF: output segment outside the arrays";
      return S3IMPH_ERR_INTERNAL;
    }
    staged_copy(c, false, fp_out + p, c->s_fp + off, cnt * 8);
    staged_copy(c, false, pos_out + p, c->s_posout + off, cnt * 8);
  }
  if (c->d.rank == 0) {
    mph->resize(info.mph_bin_len);
    uint64_t len = 0;
    rc = marshal_locked(c, mph->data(), mph->size(), &len, msg);
  }
  return rc;
}

}  // namespace

s3imph_ctx* make_dist_ctx(int device, Comm* comm, int rank, int nranks, std::string* msg) {
  s3imph_ctx* c = nullptr;
  char err[256] = {0};
  if (s3imph_ctx_create(device, &c, err, sizeof err) != S3IMPH_OK) {
    *msg = err;
    delete comm;
    return nullptr;
  }
  c->dist = true;
  c->d.comm = comm;
  c->d.rank = rank;
  c->d.nranks = nranks;
  return c;
}

int build_from_host_multi(const std::vector<int>& devs, unsigned flags, const uint8_t* blob, const uint64_t* offsets,
                          const uint64_t* pos, uint64_t n, uint64_t* fp_out, uint64_t* pos_out,
                          std::vector<uint8_t>* mph, std::string* msg) {
  const int P = (int)devs.size();
  if (P < 1 || P > kMaxRanks) {
    *msg = "build MPHF: num_gpus must be 1.." + std::to_string(kMaxRanks);
    return S3IMPH_ERR_INVALID;
  }
  bool repeated = false;
  for (int a = 0; a < P; ++a)
    for (int b = a + 1; b < P; ++b) repeated |= devs[a] == devs[b];
  if (P == 1 && !(flags & S3IMPH_MULTI_FORCE_SHARDED))
    return build_from_host(devs[0], blob, offsets, pos, n, fp_out, pos_out, mph, msg);
  mph->clear();
  if (n == 0) return S3IMPH_OK;
  try {
    MultiCtx* mc = nullptr;
    std::unique_lock<std::mutex> lk;
    for (;;) {  // a set released between the lookup and its lock: take a fresh one
      mc = multi_ctx(devs, repeated || (flags & S3IMPH_MULTI_HOST_TRANSPORT), msg);
      if (!mc) return S3IMPH_ERR_RCCL;
      lk = std::unique_lock<std::mutex>(mc->mu);
      if (!mc->released) break;
      lk.unlock();
    }
    if (mc->aborted) {
      *msg = "build MPHF: the multi-GPU set was torn down by a failed build; call again";
      return S3IMPH_ERR_RCCL;
    }
    if (mc->hub) {
      mc->hub->reset();
      mc->hub->serial = dev_env("S3IMPH_HOST_SERIAL") != nullptr;
    }
    {
      const char* em = std::getenv("S3IMPH_DIST_MODE");
      const bool bitmap = (flags & S3IMPH_MULTI_BITMAP) || (em && std::strcmp(em, "bitmap") == 0);
      for (s3imph_ctx* c : mc->ctx) c->d.mode = bitmap ? kDistBitmap : kDistRoute;
    }
    const std::vector<uint64_t> cuts = byte_cuts(offsets, n, P);
    // argument checks every rank would make alone, made here so that all ranks fail together
    for (int r = 0; r < P; ++r)
      if (cuts[r + 1] - cuts[r] > 0xffffffffull) {
        *msg = "build MPHF: more than 2^32-1 keys on one rank";
        return S3IMPH_ERR_INVALID;
      }
    std::vector<int> rcs(P, S3IMPH_OK);
    std::vector<std::string> msgs(P);
    auto work = [&](int r) {
      try {
        if (mc->hub) mc->hub->seg_begin(r);
        rcs[r] = rank_build(mc->ctx[r], blob, offsets, pos, n, cuts[r], cuts[r + 1], fp_out, pos_out, mph, &msgs[r]);
      } catch (const Fail& f) {
        rcs[r] = f.code;
        msgs[r] = f.msg;
      } catch (const std::bad_alloc&) {
        rcs[r] = S3IMPH_ERR_NOMEM;
        msgs[r] = "out of host memory";
      }
      if (mc->hub) mc->hub->seg_end(r);
      // Key-set failures (duplicate or zero key hashes, too many levels) are decided from
      // all-reduced counts, so every rank returns them at the same point.  Anything else
      // (HIP / RCCL errors, allocation failures, internal checks) may leave the peers inside
      // a collective: tear the transport down so that they return too.
      const int rc = rcs[r];
      if (rc != S3IMPH_OK && rc != S3IMPH_ERR_DUP_KEY_HASH && rc != S3IMPH_ERR_KEY_HASH_ZERO &&
          rc != S3IMPH_ERR_TOO_MANY_LEVELS)
        mc->abort_all();
    };
    std::vector<std::thread> th;
    for (int r = 1; r < P; ++r) th.emplace_back(work, r);
    work(0);
    for (auto& t : th) t.join();
    if (mc->aborted) {
      // the communicators are gone: retire this set (the next build makes a fresh one).  It
      // stays allocated, empty and marked aborted, for any caller already waiting on its mutex.
      for (s3imph_ctx* c : mc->ctx) {
        (void)hipSetDevice(c->device);
        (void)hipDeviceSynchronize();
      }
      for (s3imph_ctx* c : mc->ctx) s3imph_ctx_destroy(c);
      mc->ctx.clear();
      if (mc->hub) mc->hub->free_buffers();
      std::lock_guard<std::mutex> glk(g_multi_mu);
      for (auto it = g_multi.begin(); it != g_multi.end(); ++it)
        if (it->second.get() == mc) {
          g_retired.push_back(std::move(it->second));
          g_multi.erase(it);
          break;
        }
    }
    // every rank takes the same branches (decisions use global counts), so a build error
    // shows on every rank; report the first rank's, or the first transport failure
    for (int r = 0; r < P; ++r)
      if (rcs[r] != S3IMPH_OK) {
        *msg = msgs[r];
        return rcs[r];
      }
    return S3IMPH_OK;
  } catch (const Fail& f) {
    *msg = f.msg;
    return f.code;
  }
}

// every cached multi-GPU set that no build holds, except `keep` (a build that ran out of HBM
// drops them before its one retry); returns how many were freed
int release_idle_multi_sets(const void* keep) {
  std::vector<std::unique_ptr<MultiCtx>> idle;
  {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    for (auto it = g_multi.begin(); it != g_multi.end();) {
      MultiCtx* mc = it->second.get();
      if (mc != keep && mc->mu.try_lock()) {  // (out of g_multi now: no new caller can take it)
        mc->mu.unlock();
        idle.push_back(std::move(it->second));
        it = g_multi.erase(it);
      } else {
        ++it;
      }
    }
  }
  const int n = (int)idle.size();
  release_sets(std::move(idle));
  return n;
}

// every cached multi-GPU set (s3imph_release_workspaces)
void release_multi_sets() {
  std::vector<std::unique_ptr<MultiCtx>> all;
  {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    for (auto& kv : g_multi) all.push_back(std::move(kv.second));
    g_multi.clear();
  }
  release_sets(std::move(all));
}

}  // namespace s3imph

extern "C" int s3imph_build_host_multi(int num_gpus, const int* devices, unsigned flags, const uint8_t* blob,
                                       const uint64_t* offsets, const uint64_t* pos, uint64_t n, uint64_t* fp_out,
                                       uint64_t* pos_out, uint8_t** mph_bin, uint64_t* mph_len, char* err,
                                       size_t errlen) {
  using namespace s3imph;
  if (!mph_bin || !mph_len || num_gpus < 1 || (n && (!blob || !offsets || !fp_out || !pos_out))) {
    set_err(err, errlen, "invalid argument");
    return S3IMPH_ERR_INVALID;
  }
  *mph_bin = nullptr;
  *mph_len = 0;
  std::vector<int> devs(num_gpus);
  for (int r = 0; r < num_gpus; ++r) devs[r] = devices ? devices[r] : r;
  std::vector<uint8_t> mph;
  std::string msg;
  int rc;
  try {
    rc = build_from_host_multi(devs, flags, blob, offsets, pos, n, fp_out, pos_out, &mph, &msg);
    // out of HBM (the failed set is retired already): free the other cached workspaces, once more
    if (rc == S3IMPH_ERR_NOMEM && reclaim_cached(nullptr)) {
      msg.clear();
      rc = build_from_host_multi(devs, flags, blob, offsets, pos, n, fp_out, pos_out, &mph, &msg);
    }
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of host memory");
    return S3IMPH_ERR_NOMEM;
  }
  if (rc != S3IMPH_OK) {
    set_err(err, errlen, msg);
    return rc;
  }
  if (!mph.empty()) {
    *mph_bin = static_cast<uint8_t*>(std::malloc(mph.size()));
    if (!*mph_bin) return S3IMPH_ERR_NOMEM;
    std::memcpy(*mph_bin, mph.data(), mph.size());
    *mph_len = mph.size();
  }
  return S3IMPH_OK;
}
