"""World-size 2/3 gloo test (CPU) of the multi-GPU decomposition used by
s3imph_build_device_dist (s3-inv-db_amd/csrc/s3imph_dist.hip, s3imph_build.hip:
dist_attempt):

  level L (global n_L keys, words_L = ceil(2 n_L / 64)): rank r owns words
  [r*S, min((r+1)*S, words_L)), S = ceil(words_L / P).  Every rank routes its active
  records (k, f, pos) to the owner of their level-L position (all-to-all); the owner
  marks A/C over its range, settles keys at positions hit exactly once, numbers them
  in position order into consecutive LOCAL output slots, and keeps the collided ones
  for the next level.  While n_L * (1 - e^-1/2) > switch the next level is routed
  again; then every rank all-gathers the remaining records and finishes the build
  identically, rank 0 writing those outputs.  Each (level, rank) is one output segment
  whose global start is a prefix sum over (level, rank) settled counts.

The second decomposition (s3-inv-db_amd/csrc/s3imph_bitmap.hip, s3imph_build.hip:
dist_attempt_bitmap — the north_star's per-level collision-bitmap reduction):

  every rank keeps its key shard; at level L it computes the count lane
  min(local count, 2) of every global position, the lanes are summed over the ranks
  (RCCL reduce-scatter of u8; here an all-reduce whose slice each rank keeps), the
  slice owner sets final bit = (sum == 1) — or (mode "planes", the default on the GPU)
  the 2-bit (A, C) planes go to the slice owners by an all-to-all and are merged with
  (A, C) + (a, c) = (A | a, C | c | (A & a)), final bit = A & ~C — the final bits are
  all-gathered, and every
  rank settles its own records (bit set at x: placed at lvl_base + popcount(A[0:x)));
  the next level's global size is n_L - popcount(A_L).  Below the switch the remaining
  records are replicated as above; at the end one all-to-all moves the settled
  (p, fp, pos) triples to the owner of p's output slice [r*ceil(N/P), ...).

The per-rank arithmetic is a numpy restatement of the kernels; the cross-rank
exchange is real torch.distributed traffic.  The assembled result must equal the
oracle's single-process build byte for byte, whatever the number of ranks.
"""
import math
import os
import socket

import numpy as np
import pytest

import oracle as O

Q = 1.0 - math.exp(-0.5)


def _mix(h):
    h = h ^ (h >> np.uint64(23))
    h = h * np.uint64(O.MIX_MUL)
    return h ^ (h >> np.uint64(47))


def _positions(level, keys, words):
    with np.errstate(over="ignore"):
        seed = _mix(np.uint64(level)) * np.uint64(O.HASH_M)
        h = _mix((seed ^ _mix(keys.astype(np.uint64))) * np.uint64(O.HASH_M))
    return (h % np.uint64(64 * words)).astype(np.int64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _settle(level, k, f, p, words, plo, prange):
    """One owner's level over positions [plo, plo + prange): A/C marking, final bits,
    in-range ranks.  Returns (bits of the range, settled (f, p) in rank order, redo)."""
    x = _positions(level, k, words) - plo
    assert ((x >= 0) & (x < prange)).all()
    cnt = np.bincount(x, minlength=prange)
    final = cnt == 1
    ok = final[x]
    order = np.argsort(x[ok], kind="stable")
    return final, (f[ok][order], p[ok][order]), (k[~ok], f[~ok], p[~ok])


def _rank_main(rank, world, port, blob, offs, switch, result_q):
    import torch
    import torch.distributed as dist
    import sys
    for d in (os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"),
              os.path.join(os.path.dirname(__file__), "..", "oracle")):
        sys.path.insert(0, d)
    import oracle as Orc
    from s3imph import ShardPlan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_global = len(offs) - 1
    plan = ShardPlan(rank, world, n_global)
    kh, fp = Orc.lib().hash_keys(blob, offs)
    k, f = kh[plan.lo:plan.hi], fp[plan.lo:plan.hi]
    p = np.arange(plan.lo, plan.hi, dtype=np.uint64)
    out_f, out_p, segs_local, level_bits = [], [], [], []
    local_base = 0
    nL, level = n_global, 0
    while True:
        words = (2 * nL + 63) // 64
        S = -(-words // world)
        lo, hi = min(rank * S, words), min((rank + 1) * S, words)
        # route: records to the owner of their position (k_route + all-to-all)
        owner = _positions(level, k, words) // 64 // S
        send = [np.stack([k[owner == q], f[owner == q], p[owner == q]]) for q in range(world)]
        counts = torch.tensor([s.shape[1] for s in send], dtype=torch.int64)
        allc = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, counts)
        recv = [None] * world
        reqs = []
        for q in range(world):
            if q == rank:
                recv[q] = torch.from_numpy(send[q].view(np.int64).copy())
                continue
            recv[q] = torch.zeros((3, int(allc[q][rank])), dtype=torch.int64)
            reqs.append(dist.isend(torch.from_numpy(send[q].view(np.int64).copy()), q))
            reqs.append(dist.irecv(recv[q], q))
        for r in reqs:
            r.wait()
        mine = np.concatenate([r.numpy().view(np.uint64) for r in recv], axis=1)
        final, (sf, sp), (k, f, p) = _settle(level, mine[0], mine[1], mine[2], words, 64 * lo, 64 * (hi - lo))
        segs_local.append((level, len(sf), local_base))
        out_f.append(sf)
        out_p.append(sp)
        local_base += len(sf)
        level_bits.append((words, S, final))
        nxt = torch.tensor([len(k)], dtype=torch.int64)
        dist.all_reduce(nxt)
        if nL * Q <= switch:
            break
        nL = int(nxt.item())
        level += 1
    Ls = level + 1
    # replicated tail: all-gather the remaining records, every rank runs them
    cnts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cnts, torch.tensor([len(k)], dtype=torch.int64))
    maxc = max(int(c.item()) for c in cnts)
    pad = np.zeros((3, maxc), np.uint64)
    pad[:, :len(k)] = np.stack([k, f, p])
    gat = [torch.zeros((3, maxc), dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gat, torch.from_numpy(pad.view(np.int64).copy()))
    allr = np.concatenate([g.numpy().view(np.uint64)[:, :int(c.item())] for g, c in zip(gat, cnts)], axis=1)
    k, f, p = allr
    rep_f, rep_p, tail_bits = [], [], []
    L = Ls
    while len(k):
        words = (2 * len(k) + 63) // 64
        final, (sf, sp), (k, f, p) = _settle(L, k, f, p, words, 0, 64 * words)
        rep_f.append(sf)
        rep_p.append(sp)
        tail_bits.append(final)
        L += 1
    # output segments: prefix sums over (level, rank) settled counts
    mycounts = torch.tensor([c for _, c, _ in segs_local], dtype=torch.int64)
    allcounts = [torch.zeros(Ls, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allcounts, mycounts)
    C = np.stack([a.numpy() for a in allcounts])  # [rank, level]
    segs, G = [], 0
    for lvl in range(Ls):
        segs.append((G + int(C[:rank, lvl].sum()), int(C[rank, lvl]), segs_local[lvl][2]))
        G += int(C[:, lvl].sum())
    lf = np.concatenate(out_f) if out_f else np.zeros(0, np.uint64)
    lp = np.concatenate(out_p) if out_p else np.zeros(0, np.uint64)
    if rank == 0 and rep_f:
        rf, rp = np.concatenate(rep_f), np.concatenate(rep_p)
        segs.append((G, len(rf), len(lf)))
        lf, lp = np.concatenate([lf, rf]), np.concatenate([lp, rp])
    # level bit vectors: all-gather of each rank's word range, then the tail levels
    bits_levels = []
    for words, S, final in level_bits:
        pad = np.zeros(64 * S, bool)
        pad[:len(final)] = final
        g = [torch.zeros(64 * S, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(g, torch.from_numpy(pad.astype(np.uint8)))
        full = np.concatenate([x.numpy() for x in g]).astype(bool)[:64 * words]
        bits_levels.append(np.packbits(full, bitorder="little").view(np.uint64))
    for final in tail_bits:
        bits_levels.append(np.packbits(final, bitorder="little").view(np.uint64))
    mph = np.uint64(1).tobytes() + np.uint64(len(bits_levels)).tobytes() + b"".join(
        np.uint64(len(b)).tobytes() + b.tobytes() for b in bits_levels)
    result_q.put((rank, lf, lp, [s for s in segs if s[1]], mph, Ls))
    dist.barrier()
    dist.destroy_process_group()


def _bitmap_rank_main(rank, world, port, blob, offs, switch, result_q, planes=False):
    import torch
    import torch.distributed as dist
    import sys
    for d in (os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"),
              os.path.join(os.path.dirname(__file__), "..", "oracle")):
        sys.path.insert(0, d)
    import oracle as Orc
    from s3imph import ShardPlan

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = len(offs) - 1
    plan = ShardPlan(rank, world, N)
    kh, fp = Orc.lib().hash_keys(blob, offs)
    k, f = kh[plan.lo:plan.hi], fp[plan.lo:plan.hi]
    p = np.arange(plan.lo, plan.hi, dtype=np.uint64)
    out = []  # settled (p, fp, pos) of this rank's keys
    bits_levels = []
    nL, level, base = N, 0, 0
    while True:
        words = (2 * nL + 63) // 64
        S = -(-words // world)
        x = _positions(level, k, words)
        cnt = np.bincount(x, minlength=64 * S * world)
        if planes:
            # the 2-bit (A, C) planes by output slice ([A words | C words] per slice) go to the
            # slice owners (all-to-all); the owner merges (A, C) + (a, c) = (A|a, C|c|(A&a))
            A = np.packbits(cnt >= 1, bitorder="little").view(np.uint64).reshape(world, S)
            C = np.packbits(cnt >= 2, bitorder="little").view(np.uint64).reshape(world, S)
            send = torch.from_numpy(np.concatenate([A, C], axis=1).reshape(-1).view(np.int64).copy())
            recv = torch.zeros(2 * S * world, dtype=torch.int64)
            dist.all_to_all_single(recv, send)
            rv = recv.numpy().view(np.uint64).reshape(world, 2, S)
            Am = np.zeros(S, np.uint64)
            Cm = np.zeros(S, np.uint64)
            for q in range(world):
                Cm |= rv[q, 1] | (Am & rv[q, 0])
                Am |= rv[q, 0]
            mine = np.unpackbits((Am & ~Cm).view(np.uint8), bitorder="little").astype(bool)
        else:
            t = torch.from_numpy(np.minimum(cnt, 2).astype(np.int32))
            dist.all_reduce(t)  # the reduce-scatter's sums; this rank decides its slice only
            mine = t.numpy()[64 * S * rank:64 * S * (rank + 1)] == 1
        g = [torch.zeros(64 * S, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(g, torch.from_numpy(mine.astype(np.uint8)))
        final = np.concatenate([a.numpy() for a in g]).astype(bool)
        bits_levels.append(np.packbits(final[:64 * words], bitorder="little").view(np.uint64))
        prefix = np.concatenate([[0], np.cumsum(final)])
        ok = final[x]
        out.append(np.stack([base + prefix[x[ok]].astype(np.uint64), f[ok], p[ok]]))
        k, f, p = k[~ok], f[~ok], p[~ok]
        pop = int(final.sum())
        base += pop
        nL -= pop  # known to every rank: no collective for the next level's size
        level += 1
        if nL <= switch:  # the production code compares its bound of n_{L+1}
            break
    # replicated tail (every rank runs it; outputs numbered from base)
    cnts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cnts, torch.tensor([len(k)], dtype=torch.int64))
    maxc = max(int(c.item()) for c in cnts)
    pad = np.zeros((3, maxc), np.uint64)
    pad[:, :len(k)] = np.stack([k, f, p])
    gat = [torch.zeros((3, maxc), dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gat, torch.from_numpy(pad.view(np.int64).copy()))
    k, f, p = np.concatenate([g.numpy().view(np.uint64)[:, :int(c.item())] for g, c in zip(gat, cnts)], axis=1)
    tail = []
    L = level
    while len(k):
        words = (2 * len(k) + 63) // 64
        final, (sf, sp), (k, f, p) = _settle(L, k, f, p, words, 0, 64 * words)
        tail.append(np.stack([base + np.arange(len(sf), dtype=np.uint64), sf, sp]))
        base += len(sf)
        bits_levels.append(np.packbits(final, bitorder="little").view(np.uint64))
        L += 1
    assert base == N
    # settled triples -> the owner of p's slice (all-to-all); the tail is on every rank
    sl = -(-N // world)
    trip = np.concatenate(out, axis=1) if out else np.zeros((3, 0), np.uint64)
    owner = (trip[0] // np.uint64(sl)).astype(np.int64)
    send = [trip[:, owner == q] for q in range(world)]
    allc = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, torch.tensor([s.shape[1] for s in send], dtype=torch.int64))
    recv, reqs = [None] * world, []
    for q in range(world):
        if q == rank:
            recv[q] = torch.from_numpy(send[q].view(np.int64).copy())
            continue
        recv[q] = torch.zeros((3, int(allc[q][rank])), dtype=torch.int64)
        reqs.append(dist.isend(torch.from_numpy(send[q].view(np.int64).copy()), q))
        reqs.append(dist.irecv(recv[q], q))
    for r in reqs:
        r.wait()
    lo, hi = min(rank * sl, N), min((rank + 1) * sl, N)
    lf = np.zeros(hi - lo, np.uint64)
    lp = np.zeros(hi - lo, np.uint64)
    filled = np.zeros(hi - lo, bool)
    for r in recv + [torch.from_numpy(t.view(np.int64)) for t in tail]:
        a = r.numpy().view(np.uint64)
        m = (a[0] >= lo) & (a[0] < hi)
        idx = (a[0][m] - np.uint64(lo)).astype(np.int64)
        lf[idx], lp[idx] = a[1][m], a[2][m]
        filled[idx] = True
    assert filled.all()
    mph = np.uint64(1).tobytes() + np.uint64(len(bits_levels)).tobytes() + b"".join(
        np.uint64(len(b)).tobytes() + b.tobytes() for b in bits_levels)
    result_q.put((rank, lf, lp, [(lo, hi - lo, 0)] if hi > lo else [], mph, level))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["route", "bitmap", "planes"])
@pytest.mark.parametrize("world,switch", [(2, 5000), (3, 5000), (3, 10 ** 9)])
def test_position_range_ownership_matches_single_process(world, switch, mode, oracle_lib):
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
    target = _rank_main if mode == "route" else _bitmap_rank_main
    extra = (True,) if mode == "planes" else ()
    procs = [ctx.Process(target=target, args=(r, world, port, blob, offs, switch, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    assert all(r[4] == mph for r in res)
    if switch < n:
        assert res[0][5] >= 2  # several sharded levels before the replicated tail
    got_fp, got_pos = s3imph.assemble_dist([(r[1], r[2], r[3]) for r in res], n)
    assert np.array_equal(got_fp, fp)
    assert np.array_equal(got_pos, po)
