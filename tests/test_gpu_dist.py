"""Multi-GPU build (s3imph_build_device_dist) on the GPU, bit-exact against the oracle,
for both decompositions of the sharded levels (route and bitmap, s3imph.h).

Several ranks share the box's one GPU through the host-callback transport
(tests/dist_worker.py: torch.distributed/gloo collectives on host copies); every
kernel, the position-range routing, the output segments and the replicated tail are
the production path.  The RCCL transport itself runs at nranks = 1 (an RCCL
communicator cannot hold two ranks on one GPU).  S3IMPH_DIST_SWITCH lowers the
replicated-tail threshold so that small sets still route several levels.
"""
import socket

import numpy as np
import pytest

import oracle as O
from conftest import from_dev, to_dev

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shards(blob, offs, cuts, pos=None):
    """Contiguous key shards [cuts[r], cuts[r+1]) as (blob, rebased offsets, pos, key_base)."""
    out = []
    for r in range(len(cuts) - 1):
        a, b = cuts[r], cuts[r + 1]
        o = offs[a:b + 1].astype(np.uint64)
        sb = blob[int(o[0]):int(o[-1])]
        out.append((sb.copy(), (o - o[0]).copy(), None if pos is None else pos[a:b].copy(), a))
    return out


def _run(world, shards, n, switch, mode="route"):
    import torch.multiprocessing as mp
    import dist_worker
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=dist_worker.rank_main, args=(r, world, port, shards[r], n, switch, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "exception", r[2]
    res.sort(key=lambda r: r[0])
    return res


def _check(res, n, fp, po, mph):
    import s3imph
    for r in res:
        assert r[1] == "ok", r
        assert r[5] == mph, f"rank {r[0]}: mph.bin differs"
    got_fp, got_po = s3imph.assemble_dist([(r[2], r[3], r[4]) for r in res], n)
    assert np.array_equal(got_fp, fp)
    assert np.array_equal(got_po, po)


@pytest.mark.parametrize("mode", ["route", "bitmap"])
@pytest.mark.parametrize("world,n,switch", [(2, 200_000, 20_000), (3, 120_000, 10_000), (2, 300_000, 2 << 20)])
def test_dist_host_comm_matches_oracle(world, n, switch, mode, oracle_lib):
    """Both decompositions of the sharded levels (route: records to position owners;
    bitmap: count lanes reduce-scattered, final bits all-gathered) bit-exact."""
    import s3imph
    blob, offs = s3imph.gen_keys(0, 7, 32, 0, n)
    blob = blob[: int(offs[-1])]
    st, fp, po, mph = oracle_lib.build(blob, offs)
    assert st == 0
    cuts = [n * r // world for r in range(world + 1)]
    res = _run(world, _shards(blob, offs, cuts), n, switch, mode)
    assert res[0][1] == "ok", res[0]
    assert res[0][6]["big_levels"] >= (3 if switch < 50_000 else 1)
    _check(res, n, fp, po, mph)


@pytest.mark.parametrize("mode", ["route", "bitmap"])
def test_dist_unbalanced_shards_custom_pos(oracle_lib, mode):
    import s3imph
    n, world = 90_000, 3
    blob, offs = s3imph.gen_keys(1, 3, 0, 0, n)  # ragged lengths 5-1024 B
    blob = blob[: int(offs[-1])]
    pos = (np.random.default_rng(1).permutation(n).astype(np.uint64) + np.uint64(7_000_000))
    st, fp, po, mph = oracle_lib.build(blob, offs, pos)
    assert st == 0
    cuts = [0, 5_000, 70_000, n]
    res = _run(world, _shards(blob, offs, cuts, pos), n, 8_000, mode)
    _check(res, n, fp, po, mph)


def test_dist_chunked_level0_unbalanced(oracle_lib):
    """N / P >= 8M keys: level 0 runs chunked on every rank (the decision is global), here
    with one rank holding 16M keys and the other 1M (chunks of 4M and 250k), custom
    positions, two processes over gloo on the one GPU: bit-exact."""
    import s3imph
    n, world = 17_000_000, 2
    blob, offs = s3imph.gen_keys(0, 13, 16, 0, n)
    blob = blob[: int(offs[-1])]
    pos = (np.random.default_rng(3).permutation(n).astype(np.uint64) + np.uint64(11))
    st, fp, po, mph = oracle_lib.build_mt(blob, offs, pos, threads=16)
    assert st == 0
    res = _run(world, _shards(blob, offs, [0, 16_000_000, n], pos), n, 1 << 21)
    _check(res, n, fp, po, mph)


@pytest.mark.parametrize("mode", ["route", "bitmap"])
def test_dist_tiny_set_and_empty_rank(oracle_lib, mode):
    """5 keys on 3 ranks (one rank holds none; most ranks own no level positions)."""
    keys = [b"", b"a/", b"data/", b"data/2024/", b"root/"]
    blob, offs = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(blob, offs)
    res = _run(3, _shards(blob, offs, [0, 2, 2, 5]), 5, 1 << 20, mode)
    _check(res, 5, fp, po, mph)


@pytest.mark.parametrize("mode", ["route", "bitmap"])
def test_dist_duplicate_across_ranks_fails_everywhere(mode):
    keys = [b"x/%05d/" % i for i in range(3000)]
    keys[2500] = keys[10]  # the duplicate lives on the other rank
    blob, offs = O.keys_to_blob(keys)
    res = _run(2, _shards(blob, offs, [0, 1500, 3000]), 3000, 1 << 20, mode)
    import s3imph
    for r in res:
        assert r[1] == "error" and r[2] == s3imph.ERR_DUP_KEY_HASH, r


@pytest.mark.parametrize("mode", ["route", "bitmap"])
def test_dist_duplicated_record_is_an_internal_fault(mode, monkeypatch):
    """A record duplicated inside the sharded build (S3IMPH_FAULT_DUP_REC: the gathered
    replicated level's record 0 copied over record 1) stops it on leftovers with one key
    hash; the ranks count that value among their ORIGINAL key hashes, sum the counts, find
    it once, and every rank reports ERR_INTERNAL (not the caller's duplicate keys)."""
    monkeypatch.setenv("S3IMPH_FAULT_DUP_REC", "1")
    keys = [b"x/%05d/" % i for i in range(3000)]
    blob, offs = O.keys_to_blob(keys)
    res = _run(2, _shards(blob, offs, [0, 1500, 3000]), 3000, 1 << 20, mode)
    import s3imph
    for r in res:
        assert r[1] == "error" and r[2] == s3imph.ERR_INTERNAL and "duplicated" in r[3], r


@pytest.mark.parametrize("mode", ["route", "route_self", "bitmap"])
def test_dist_rccl_single_rank_routes_levels(oracle_lib, monkeypatch, mode):
    """The RCCL transport (nranks = 1 on this box) through several sharded levels: route
    (one rank: nothing to route, the single-GPU level 0 and ping-ponged levels), route_self
    (S3IMPH_DIST_ROUTE_SELF: the fused level-0 route, the padded fixed-region routes of levels
    >= 1 and their all-to-alls, as with P > 1) and bitmap (ncclReduceScatter of the count
    lanes, ncclAllGather of the final bits, the output all-to-all)."""
    import torch
    import s3imph
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "20000")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    if mode == "route_self":
        monkeypatch.setenv("S3IMPH_DIST_ROUTE_SELF", "1")
    d = s3imph.DistBuilder(0, s3imph.dist_unique_id(), 0, 1)
    d.set_mode(s3imph.DIST_BITMAP if mode == "bitmap" else s3imph.DIST_ROUTE)
    n = 300_000
    blob, offs = s3imph.gen_keys(0, 11, 32, 0, n)
    st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
    cap = d.out_cap(n)
    d_fp = torch.zeros(cap, dtype=torch.int64, device="cuda")
    d_po = torch.zeros(cap, dtype=torch.int64, device="cuda")
    out_n, segs, info = d.build_shard(to_dev(blob), to_dev(offs), n, 0, d_fp, d_po, cap)
    assert out_n == n and info["big_levels"] >= 3
    got_fp, got_po = s3imph.assemble_dist([(from_dev(d_fp), from_dev(d_po), segs)], n)
    assert d.mph_bin() == mph
    assert np.array_equal(got_fp, fp) and np.array_equal(got_po, po)
    # lookups on the distributed context use the same level bit vectors
    res = torch.zeros(n, dtype=torch.int64, device="cuda")
    d.lookup(to_dev(blob), to_dev(offs), n, to_dev(got_fp), to_dev(got_po), n, res)
    assert torch.equal(res, torch.arange(n, dtype=torch.int64, device="cuda"))
    d.close()
