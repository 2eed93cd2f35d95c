"""World-size-2 gloo test (CPU) of the multi-GPU decomposition used by
s3imph_build_device_dist (s3-inv-db_amd/csrc/s3imph_build.hip, build_dist):

  per level: each rank marks its own keys into full-size local A/C bit vectors ->
  one saturating count byte per position (0, 1, 2+) -> cross-rank SUM (RCCL
  reduce-scatter on the GPU; gloo all-reduce here) -> final bit = (sum == 1), padded
  to 64*P positions and sliced per rank -> each rank settles keys whose bit is set,
  the rest form its next-level set; level sizes from the summed redo counts.
  After the levels: (p, fp, pos) go to the rank owning p's range (ShardPlan.out_*).

The per-rank arithmetic is a numpy restatement of the kernels; the cross-rank
exchange is real torch.distributed traffic.  The result must equal the oracle's
single-process build byte for byte, whatever the number of ranks.
"""
import os
import socket

import numpy as np
import pytest

import oracle as O

M64 = (1 << 64) - 1


def _mix(h):
    h = h ^ (h >> np.uint64(23))
    h = h * np.uint64(O.MIX_MUL)
    return h ^ (h >> np.uint64(47))


def _positions(level, keys, words):
    with np.errstate(over="ignore"):
        seed = _mix(np.uint64(level)) * np.uint64(O.HASH_M)
        h = _mix((seed ^ _mix(keys.astype(np.uint64))) * np.uint64(O.HASH_M))
    return (h % np.uint64(64 * words)).astype(np.uint64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, blob, offs, result_q):
    import torch
    import torch.distributed as dist
    import sys
    for p in (os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"),
              os.path.join(os.path.dirname(__file__), "..", "oracle")):
        sys.path.insert(0, p)
    import oracle as Orc
    from s3imph import ShardPlan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_global = len(offs) - 1
    plan = ShardPlan(rank, world, n_global)
    lo, hi = plan.lo, plan.hi
    kh, fp = Orc.lib().hash_keys(blob, offs)
    kh, fp = kh[lo:hi], fp[lo:hi]
    idx = np.arange(hi - lo, dtype=np.int64)
    settle = np.zeros(hi - lo, np.uint64)
    nL, woff, levels = n_global, 0, []
    keys = kh.copy()
    level = 0
    while True:
        words = (2 * nL + 63) // 64
        pos_pad = -(-64 * words // (64 * world)) * (64 * world)
        x = _positions(level, keys, words).astype(np.int64)
        cnt = np.bincount(x, minlength=pos_pad).astype(np.int64)
        lanes = torch.from_numpy(np.minimum(cnt, 2).astype(np.uint8))   # k_dist_counts
        dist.all_reduce(lanes)                                           # RCCL reduce-scatter (+ slice)
        total = lanes.numpy().astype(np.int64)
        S = pos_pad // world
        mine = (total[rank * S:(rank + 1) * S] == 1)                     # k_dist_pack on the slice
        gathered = [torch.zeros(S, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(mine.astype(np.uint8)))  # ncclAllGather
        final = np.concatenate([g.numpy() for g in gathered]).astype(bool)[: 64 * words]
        ok = final[x]                                                    # k_dist_resolve
        settle[idx[ok]] = np.uint64(woff * 64) + x[ok].astype(np.uint64)
        keys, idx = keys[~ok], idx[~ok]
        nxt = torch.tensor([len(keys)], dtype=torch.int64)
        dist.all_reduce(nxt)
        bits = np.packbits(final, bitorder="little").view(np.uint64)
        levels.append(bits)
        woff += words
        level += 1
        if int(nxt.item()) == 0:
            break
        nL = int(nxt.item())
    allbits = np.concatenate(levels)
    pc = np.array([bin(int(w)).count("1") for w in allbits], np.uint64)
    rank_base = np.concatenate([[0], np.cumsum(pc)[:-1]]).astype(np.uint64)
    w = (settle >> np.uint64(6)).astype(np.int64)
    below = (np.uint64(1) << (settle & np.uint64(63))) - np.uint64(1)
    p = rank_base[w] + np.array([bin(int(v)).count("1") for v in (allbits[w] & below)], np.uint64)
    # owner exchange (ncclSend/Recv of (p, fp, pos) triples)
    per = plan.out_per_rank
    owner = np.minimum(p // np.uint64(per), world - 1).astype(np.int64)
    send = [torch.from_numpy(np.stack([p[owner == q], fp[owner == q],
                                       (np.arange(lo, hi, dtype=np.uint64))[owner == q]]).view(np.int64).copy())
            for q in range(world)]
    counts = torch.tensor([s.shape[1] for s in send], dtype=torch.int64)
    allc = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, counts)
    recv = [torch.zeros((3, int(allc[q][rank])), dtype=torch.int64) for q in range(world)]
    reqs = []
    for q in range(world):
        if q == rank:
            recv[q] = send[q]
            continue
        reqs.append(dist.isend(send[q], q))
        reqs.append(dist.irecv(recv[q], q))
    for r in reqs:
        r.wait()
    trip = np.concatenate([r.numpy().view(np.uint64) for r in recv], axis=1)
    fp_slice = np.zeros(plan.out_n, np.uint64)
    pos_slice = np.zeros(plan.out_n, np.uint64)
    rel = (trip[0] - np.uint64(plan.out_lo)).astype(np.int64)
    fp_slice[rel] = trip[1]
    pos_slice[rel] = trip[2]
    mph = np.uint64(1).tobytes() + np.uint64(len(levels)).tobytes() + b"".join(
        np.uint64(len(b)).tobytes() + b.tobytes() for b in levels)
    result_q.put((rank, plan.out_lo, fp_slice, pos_slice, mph))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_levels_match_single_process(world, oracle_lib):
    import torch.multiprocessing as mp
    import s3imph

    n = 40000
    blob, offs = s3imph.gen_keys(0, 5, 24, 0, n)
    blob = blob[: int(offs[-1])]
    st, fp, po, mph = oracle_lib.build(blob, offs)
    assert st == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, blob, offs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    got_fp = np.concatenate([r[2] for r in res])
    got_pos = np.concatenate([r[3] for r in res])
    assert all(r[4] == mph for r in res)
    assert np.array_equal(got_fp, fp)
    assert np.array_equal(got_pos, po)
