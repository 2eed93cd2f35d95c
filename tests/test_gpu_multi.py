"""Multi-GPU builds behind the host-memory boundary (s3imph_build_host_multi and the
builder's set_gpus): one calling process, one host thread per rank.

The box has one GPU, so the ranks of the thread-per-rank logic share it through the
in-process host-copy transport (devices = [0] * P); the RCCL path runs with one rank
made by ncclCommInitAll.  S3IMPH_DIST_SWITCH lowers the replicated-tail threshold so
that small sets still route several levels between ranks.  Every result is compared
byte for byte with the oracle (mph.bin, mph_fp, mph_pos).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s3():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import s3imph
    return s3imph


def _expect(oracle_lib, blob, offs, pos=None):
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, pos, threads=16)
    assert st == 0
    return fp, po, mph


def test_one_rank_routed_build_is_the_single_gpu_build(s3, oracle_lib, monkeypatch, capfd):
    """A one-rank sharded build in the routed mode has nothing to route: it runs the single-GPU
    pipeline (P0 level 0 for sets past 2048 tiles), outputs at their global positions."""
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 53))
    blob, offs = s3.gen_keys(0, 14, 24, 0, 18_000_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, num_gpus=1, flags=s3.MULTI_FORCE_SHARDED)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert "attempt 0: status 0x0" in err, err[-2000:]  # build_single's debug line


def test_one_gpu_default_is_the_single_gpu_build(s3, oracle_lib):
    blob, offs = s3.gen_keys(0, 5, 32, 0, 300_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, num_gpus=1)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


def test_one_gpu_sharded_over_rccl(s3, oracle_lib, monkeypatch):
    """num_gpus = 1 forced onto the sharded path: an in-process RCCL communicator
    (ncclCommInitAll) carries every collective of the routed levels (S3IMPH_DIST_ROUTE_SELF:
    one rank routes like P > 1; without it a one-rank routed build is the single-GPU build)."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "20001")  # a fresh set (reads S3IMPH_DIST_ROUTE_SELF)
    monkeypatch.setenv("S3IMPH_DIST_ROUTE_SELF", "1")
    blob, offs = s3.gen_keys(0, 6, 40, 0, 400_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    for _ in range(2):  # the second build reuses the cached contexts and communicator
        g = s3.build_host(blob, offs, num_gpus=1, flags=s3.MULTI_FORCE_SHARDED)
        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


@pytest.mark.parametrize("bitmap", [False, True])
@pytest.mark.parametrize("ranks,kind,avg,n", [(2, 0, 32, 300_000), (3, 1, 0, 400_000), (4, 0, 64, 500_000),
                                              (8, 0, 24, 2_000_000)])
def test_thread_per_rank_shared_gpu(s3, oracle_lib, monkeypatch, ranks, kind, avg, n, bitmap):
    """2-8 ranks in one process on the one GPU (host-copy transport), shards balanced by
    key bytes, skewed lengths on one case, both decompositions (route / bitmap; the
    bitmap build may not fall back, S3IMPH_DIST_STRICT): bit-exact."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15000")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    blob, offs = s3.gen_keys(kind, 8, avg, 0, n)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, devices=[0] * ranks, flags=s3.MULTI_BITMAP if bitmap else 0)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


@pytest.mark.parametrize("bitmap", [False, True])
def test_thread_per_rank_serialised_device_work(s3, oracle_lib, monkeypatch, bitmap):
    """S3IMPH_HOST_SERIAL (the measurement mode of tools/p8_geometry.py): the host transport
    hands the GPU to one rank at a time between collectives; 4 ranks, both decompositions,
    bit-exact, twice (the token is released at the end of every build)."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15001")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_HOST_SERIAL", "1")
    blob, offs = s3.gen_keys(0, 14, 24, 0, 1_200_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    for _ in range(2):
        g = s3.build_host(blob, offs, devices=[0] * 4, flags=s3.MULTI_BITMAP if bitmap else 0)
        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


def test_release_workspaces_then_build_again(s3, oracle_lib, monkeypatch):
    """s3imph_release_workspaces frees the cached default contexts and multi-GPU sets; the next
    builds (single, 3 ranks, and a Lookup-free rebuild on the same default context) allocate
    again and stay bit-exact."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15002")
    blob, offs = s3.gen_keys(0, 15, 24, 0, 700_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    for devices in (None, [0, 0, 0]):
        g = s3.build_host(blob, offs, devices=devices, flags=s3.MULTI_BITMAP if devices else 0)
        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
        s3.release_workspaces()
        g = s3.build_host(blob, offs, devices=devices, flags=s3.MULTI_BITMAP if devices else 0)
        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    s3.release_workspaces()


def test_thread_per_rank_64_ranks_bitmap(s3, oracle_lib, monkeypatch):
    """kMaxRanks = 64 ranks (the API's limit) on the bitmap decomposition: 64 output
    slices counted by the settle (the last slice's count included), the (A, C) plane
    all-to-all over 64 ranks; bit-exact."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15000")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    blob, offs = s3.gen_keys(0, 12, 24, 0, 640_000)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, devices=[0] * 64, flags=s3.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


@pytest.mark.parametrize("switch,n", [(20_000, 1_500_000), (2 << 20, 4_000_000)])
def test_one_gpu_sharded_bitmap_over_rccl(s3, oracle_lib, monkeypatch, switch, n):
    """The bitmap decomposition on an in-process RCCL communicator (one rank):
    ncclReduceScatter of the count lanes and ncclAllGather of the final bits per level;
    a tiny replicated tail (switch 20k) and a 1.5M-record one (the default 2M switch: the
    tail's scatter / tile kernels run beside the held settled triples)."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str(switch))
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    blob, offs = s3.gen_keys(0, 16, 40, 0, n)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    for _ in range(2):
        g = s3.build_host(blob, offs, num_gpus=1, flags=s3.MULTI_FORCE_SHARDED | s3.MULTI_BITMAP)
        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


@pytest.mark.parametrize("ranks,kind,avg,n", [(1, 0, 24, 17_500_000), (2, 0, 24, 20_000_000),
                                              (3, 1, 0, 18_000_000), (1, 0, 16, 40_000_000)])
def test_bitmap_level0_through_p0_tiles(s3, oracle_lib, monkeypatch, capfd, ranks, kind, avg, n):
    """The bitmap decomposition's level 0 through the P0 super-tiles (tiles of 2^(14 + lg P)
    positions, a rank's ~8k records each, from 256 of them; 40M at one rank: 4883 tiles, more
    than the reservation scatter's 4096): fused hash partition (skewed lengths:
    k_hash_skew + the partition pass), super-tile scatter into R20 slots, then the bitmap
    mark / settle over R20 records.  One rank over RCCL, 2-3 over the host transport;
    every rank reports the P0 level 0 (S3IMPH_DEBUG); bit-exact (S3IMPH_DIST_STRICT)."""
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str(2_000_000 + 7 * ranks))  # fresh contexts read S3IMPH_DEBUG
    blob, offs = s3.gen_keys(kind, 31, avg, 0, n)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    if ranks == 1:
        g = s3.build_host(blob, offs, num_gpus=1, flags=s3.MULTI_FORCE_SHARDED | s3.MULTI_BITMAP)
    else:
        g = s3.build_host(blob, offs, devices=[0] * ranks, flags=s3.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("level 0 through P0 super-tiles") == ranks, err[-2000:]


@pytest.mark.parametrize("ranks", [1, 2])
def test_bitmap_capacity_miss_reruns_conservatively(s3, oracle_lib, monkeypatch, capfd, ranks):
    """under S3IMPH_DIST_STRICT only a size-bound miss fails the bitmap build.  A
    capacity miss (a reservation-slot overflow, or a settle-fed level without its P0 buffers:
    injected after level 0 by S3IMPH_FAULT_BM_OVERFLOW) reruns the bitmap decomposition once in
    its conservative form (no settle-fed levels, no list levels through P0): bit-exact, and
    every rank reports the rerun."""
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_FAULT_BM_OVERFLOW", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str(2_000_000 + 29 * ranks))  # fresh contexts read S3IMPH_DEBUG
    n = 18_000_000
    blob, offs = s3.gen_keys(0, 37, 20, 0, n)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    if ranks == 1:
        g = s3.build_host(blob, offs, num_gpus=1, flags=s3.MULTI_FORCE_SHARDED | s3.MULTI_BITMAP)
    else:
        g = s3.build_host(blob, offs, devices=[0] * ranks, flags=s3.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("a capacity miss, rerunning conservatively") == ranks, err[-2000:]


@pytest.mark.parametrize("ranks", [2, 3])
def test_thread_per_rank_chunked_level0_exchange(s3, oracle_lib, monkeypatch, capfd, ranks):
    """Shards of >= 8M keys take the chunked level 0 (s3imph_build.hip route0_chunked):
    four key chunks, each hashed and routed on the build stream while the previous one's
    records cross on the exchange stream; own records land between chunks' received
    ones.  Bit-exact with the oracle (10-12M keys per rank, host-copy transport), and
    every rank reports the chunked exchange on its first attempt (S3IMPH_DEBUG)."""
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str(3_000_000 + ranks))  # fresh contexts read S3IMPH_DEBUG
    n = 10_000_000 * ranks + 2_000_000
    blob, offs = s3.gen_keys(0, 21, 24, 0, n)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, devices=[0] * ranks)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("level 0 exchanged in 4 chunks") == ranks, err[-2000:]


def test_thread_per_rank_custom_positions_offset_blob(s3, oracle_lib, monkeypatch):
    """A blob starting at a non-zero offsets[0] with custom positions, 3 ranks."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15000")
    n = 250_000
    blob, offs = s3.gen_keys(0, 9, 24, 0, n)
    blob = blob[: int(offs[-1])]
    pos = np.random.default_rng(2).permutation(n).astype(np.uint64) + np.uint64(10**9)
    fp, po, mph = _expect(oracle_lib, blob, offs, pos)
    shifted = np.concatenate([np.frombuffer(b"abcde", np.uint8), blob])
    g = s3.build_host(shifted, offs + np.uint64(5), pos, devices=[0, 0, 0])
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)


def test_thread_per_rank_tiny_and_duplicate_sets(s3, oracle_lib):
    keys = [b"", b"a/", b"data/", b"data/2024/", b"root/"]
    blob, offs = O.keys_to_blob(keys)
    fp, po, mph = _expect(oracle_lib, blob, offs)
    g = s3.build_host(blob, offs, devices=[0, 0, 0, 0])
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    dup = [b"x/%05d/" % i for i in range(3000)]
    dup[2500] = dup[10]  # the duplicate lands on another rank's shard
    b2, o2 = O.keys_to_blob(dup)
    with pytest.raises(s3.MPHFError) as e:
        s3.build_host(b2, o2, devices=[0, 0])
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    # the cached rank contexts stay usable after the error
    g = s3.build_host(blob, offs, devices=[0, 0, 0, 0])
    assert g[2] == mph


def test_builder_on_several_gpus_writes_identical_files(s3, oracle_lib, tmp_path, monkeypatch):
    """StreamingMPHFBuilder mirror with set_gpus: Add x N -> Build(outDir) on 3 ranks ->
    the 5 files equal the oracle's."""
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", "15000")
    blob, offs = s3.gen_keys(0, 4, 32, 0, 120_000)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    b.set_gpus(3, [0, 0, 0])
    for i, k in enumerate(keys):
        b.add(k, i)
    out = tmp_path / "idx"
    out.mkdir()
    b.build(str(out))
    b.close()
    kb, ko = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(kb, ko)
    want = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(po),
            "prefix_blob.bin": kb.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(ko)}
    for name, data in want.items():
        assert (out / name).read_bytes() == data, name


def _bitmap_subprocess(env: dict, cases) -> None:
    """Bitmap-decomposition builds of `cases` (ranks, kind, avg, n) on the thread-per-rank
    transport, in a fresh process with `env` set (the library reads its knobs once per
    process): bit-exact vs the oracle, twice each (the second build reuses the contexts)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (
        "import sys; sys.path[:0]=[%r, %r]\n"
        "import numpy as np, torch, s3imph, oracle as O\n"
        "for ranks, kind, avg, n in %r:\n"
        "    blob, offs = s3imph.gen_keys(kind, 8, avg, 0, n)\n"
        "    st, fp, po, mph = O.lib().build_mt(blob[: offs[-1]], offs, None, threads=16)\n"
        "    for _ in range(2):\n"
        "        g = s3imph.build_host(blob, offs, devices=[0] * ranks, flags=s3imph.MULTI_BITMAP)\n"
        "        assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po), (ranks, n)\n"
        "print('ok')\n"
    ) % (os.path.join(here, "..", "s3-inv-db_amd"), os.path.join(here, "..", "oracle"), list(cases))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280,
                       env={**os.environ, "S3IMPH_DEV": "1", "S3IMPH_DIST_STRICT": "1", **env})
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_bitmap_output_exchange_by_level_group(s3, oracle_lib):
    """The bitmap build's output exchange by level group: levels 0 and 1 leave as
    soon as they are settled and land in their slices through per-group merges, the rest at
    the end.  On the build's stream (the host transports' default), on the exchange stream
    (S3IMPH_XCH_STREAM=1: the order RCCL runs them in, events included), and as one exchange at
    the end (S3IMPH_XCH_LEVELS=0); 2, 3 and 8 ranks, skewed lengths on one case, sets with one,
    two and several sharded levels (S3IMPH_DIST_SWITCH): bit-exact."""
    cases = [(2, 0, 32, 3_000_000), (3, 1, 0, 2_000_000), (8, 0, 24, 6_000_000)]
    _bitmap_subprocess({"S3IMPH_DIST_SWITCH": "20000"}, cases)
    _bitmap_subprocess({"S3IMPH_DIST_SWITCH": "20000", "S3IMPH_XCH_STREAM": "1"}, cases)
    _bitmap_subprocess({"S3IMPH_DIST_SWITCH": "20000", "S3IMPH_XCH_LEVELS": "0"}, cases[:2])
    # one and two sharded levels: the last group alone, level 0 then the rest
    _bitmap_subprocess({"S3IMPH_DIST_SWITCH": "2500000", "S3IMPH_XCH_STREAM": "1"}, [(2, 0, 32, 3_000_000)])
    _bitmap_subprocess({"S3IMPH_DIST_SWITCH": "800000", "S3IMPH_XCH_STREAM": "1"}, [(2, 0, 32, 3_000_000)])
