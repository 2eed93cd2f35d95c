"""BASELINE.json's large configurations on the GPU (run with -m gpu on an MI355X).

C4 (configs[3]: 1B prefixes, avg key 32 B, quoted on 8 GPUs) runs here at FULL size on
one GPU (about 150 GB of HBM): the product's outputs are checked through
size-independent properties (mph_pos is a permutation of [0, N); every key looks itself
up through the batched Lookup, which also checks its fingerprint, mphf.go:275-302), and
one GPU's share of C4 (125M keys) is compared byte for byte with the oracle.

C3 (configs[2]: 100M prefixes, avg key 64 B — the bench headline) is compared byte for
byte with the oracle at its exact geometry (level 0 on 2^18-position split tiles of 16
sub-tiles, level 1 on host-chosen ts x 2^14 tiles).

C5 (configs[4]: skewed key lengths 1-1024 B, 200M keys, quoted on 8 GPUs) runs at FULL
size on one GPU (~30 GB of key bytes) with the C4-style properties; one GPU's share
(25M keys) is compared byte for byte with the oracle; and 2M keys run as 4 and 8 ranks on
the box's one GPU through the host-callback transport (tests/dist_worker.py), with the
replicated-tail threshold lowered so that at least 3 levels are routed between ranks:
mph.bin on every rank and the assembled mph_fp / mph_pos equal the oracle's.

The reference's acceptance check is VerifyMPHF over every key (mphf.go:372-393): the
property tests run exactly that through the batched GPU Lookup.
"""
import numpy as np
import pytest

from test_gpu_dist import _check, _run, _shards

pytestmark = pytest.mark.gpu


def _dev(a: np.ndarray):
    """numpy -> cuda tensor without a host copy (these arrays are tens of GB)."""
    import torch
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(a).to("cuda")


@pytest.fixture(autouse=True)
def _release_cached_workspaces():
    """These builds take most of the HBM: free what earlier host builds keep cached (the default
    contexts, the multi-GPU sets of up to 8 ranks) before and after each."""
    import s3imph
    s3imph.release_workspaces()
    yield
    s3imph.release_workspaces()


def _properties(n, d_blob, d_offs, min_big_levels):
    """Size-independent checks of one full build: mph_pos is a permutation of [0, N), and
    every member looks itself up (VerifyMPHF, mphf.go:372-393)."""
    import torch
    import s3imph
    d_fp = torch.empty(n, dtype=torch.int64, device="cuda")
    d_po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = s3imph.DeviceBuilder(0)
    try:
        info = ctx.build(d_blob, d_offs, n, d_fp, d_po)
        assert info["n_keys"] == n and info["big_levels"] >= min_big_levels
        assert len(ctx.mph_bin()) == info["mph_bin_len"]
        assert int(d_po.min()) == 0 and int(d_po.max()) == n - 1
        seen = torch.zeros(n, dtype=torch.uint8, device="cuda")
        seen[d_po] = 1
        assert int(seen.sum(dtype=torch.int64)) == n
        del seen
        res = torch.empty(n, dtype=torch.int64, device="cuda")
        ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)
        step = 1 << 27
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            want = torch.arange(lo, hi, dtype=torch.int64, device="cuda")
            assert torch.equal(res[lo:hi], want), lo
    finally:
        ctx.close()


def _bit_exact(oracle_lib, kind, avg, n):
    import torch
    import s3imph
    blob, offs = s3imph.gen_keys(kind, 42, avg, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    d_fp = torch.empty(n, dtype=torch.int64, device="cuda")
    d_po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = s3imph.DeviceBuilder(0)
    try:
        info = ctx.build(_dev(blob), _dev(offs), n, d_fp, d_po)
        assert ctx.mph_bin() == mph
        assert np.array_equal(d_fp.cpu().numpy().view(np.uint64), fp)
        assert np.array_equal(d_po.cpu().numpy().view(np.uint64), po)
        return info
    finally:
        ctx.close()


def test_c3_100m_bit_exact(oracle_lib):
    """The bench headline's exact workload (100M keys, avg 64 B, seed 42) against the
    oracle: mph.bin, mph_fp and mph_pos byte for byte."""
    info = _bit_exact(oracle_lib, 0, 64, 100_000_000)
    assert info["big_levels"] >= 5


def test_c3_bitmap_one_rank_bit_exact(oracle_lib, monkeypatch, capfd):
    """The north_star decomposition (per-level collision bitmap) on the bench headline's
    workload at one rank (RCCL, nranks = 1): level 0 through the P0 super-tiles into 2^14
    tiles, level 1 (39M records: 4.8k tiles, more than the reservation scatter takes) through
    its own super-tile pass, the in-tile positions (u16) read by the marks, staged settles;
    mph.bin, mph_fp and mph_pos byte for byte against the oracle, no fallback
    (S3IMPH_DIST_STRICT)."""
    import s3imph
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 11))  # a fresh context (reads S3IMPH_DEBUG)
    n = 100_000_000
    blob, offs = s3imph.gen_keys(0, 42, 64, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    g = s3imph.build_host(blob, offs, num_gpus=1, flags=s3imph.MULTI_FORCE_SHARDED | s3imph.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert "level 0 through P0 super-tiles" in err and "level 1 through P0 super-tiles" in err, err[-3000:]
    assert "partitioned by the previous settle" in err, err[-3000:]  # level 0's settle fed level 1's regions


def test_bitmap_2_ranks_settle_fed_level1_bit_exact(oracle_lib, monkeypatch, capfd):
    """Two ranks x 88M keys (176M globally: level 1's 69M records take 4.2k tiles of 2^15, past the
    reservation scatter's 4096) through the host transport: each rank's level-0 settle
    partitions its collided records into level 1's super-tile regions (NextPart), level 1 goes
    straight to the super-tile scatter; bit-exact against the oracle (S3IMPH_DIST_STRICT)."""
    import s3imph
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 17))
    n = 176_000_000
    blob, offs = s3imph.gen_keys(0, 91, 16, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    g = s3imph.build_host(blob, offs, devices=[0] * 2, flags=s3imph.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("partitioned by the previous settle") == 2, err[-3000:]


def test_bitmap_8_ranks_past_p0_single_limit_bit_exact(oracle_lib, monkeypatch, capfd):
    """the bitmap decomposition at 8 ranks x 40M keys (320M globally, past the
    268M that P0's 2^14 tiles covered) through the host transport on one GPU: every rank's
    level 0 goes through P0 with tiles scaled to the rank count (2^16 positions, a rank's
    ~4k records each); bit-exact against the oracle, no fallback (S3IMPH_DIST_STRICT)."""
    import s3imph
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 13))
    n = 320_000_000
    blob, offs = s3imph.gen_keys(0, 77, 16, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    g = s3imph.build_host(blob, offs, devices=[0] * 8, flags=s3imph.MULTI_BITMAP)
    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("level 0 through P0 super-tiles") == 8 and "tiles of 2^16" in err, err[-3000:]


def test_c5_one_gpu_share_bit_exact(oracle_lib):
    """One GPU's share of C5 (keys [0, 25M) of the 200M skewed sequence) against the oracle."""
    _bit_exact(oracle_lib, 1, 0, 25_000_000)


def test_c5_200m_single_gpu_properties():
    """C5 at full size (200M keys, 1-1024 B log-uniform, ~30 GB) on one GPU."""
    import s3imph
    n = 200_000_000
    blob, offs = s3imph.gen_keys(1, 42, 0, 0, n)
    key_bytes = int(offs[-1])
    assert 28e9 < key_bytes < 31e9  # mean ~148 B (~29.5 GB)
    d_blob = _dev(blob)
    del blob
    d_offs = _dev(offs)
    del offs
    _properties(n, d_blob, d_offs, 5)


def test_c4_1b_keys_single_gpu_properties():
    import torch
    import s3imph
    n = 1_000_000_000
    blob, offs = s3imph.gen_keys(0, 42, 32, 0, n)
    key_bytes = int(offs[-1])
    assert 31e9 < key_bytes < 33e9  # avg 32 B, as SURVEY §8d records for C4
    d_blob = _dev(blob)
    del blob
    d_offs = _dev(offs)
    del offs
    d_fp = torch.empty(n, dtype=torch.int64, device="cuda")
    d_po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = s3imph.DeviceBuilder(0)
    try:
        info = ctx.build(d_blob, d_offs, n, d_fp, d_po)
        assert info["n_keys"] == n and info["big_levels"] >= 5
        assert len(ctx.mph_bin()) == info["mph_bin_len"]
        # mph_pos is a permutation of [0, N): every value in range, every slot hit once
        assert int(d_po.min()) == 0 and int(d_po.max()) == n - 1
        seen = torch.zeros(n, dtype=torch.uint8, device="cuda")
        seen[d_po] = 1
        assert int(seen.sum(dtype=torch.int64)) == n
        del seen
        # every member looks itself up (hash -> levels -> fingerprint check -> pos)
        res = torch.empty(n, dtype=torch.int64, device="cuda")
        ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)
        step = 1 << 27
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            want = torch.arange(lo, hi, dtype=torch.int64, device="cuda")
            assert torch.equal(res[lo:hi], want), lo
    finally:
        ctx.close()


def test_c4_one_gpu_share_bit_exact(oracle_lib):
    """One GPU's share of C4 (keys [0, 125M) of the 1B sequence) against the oracle."""
    import torch
    import s3imph
    n = 125_000_000
    blob, offs = s3imph.gen_keys(0, 42, 32, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    d_fp = torch.empty(n, dtype=torch.int64, device="cuda")
    d_po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = s3imph.DeviceBuilder(0)
    try:
        ctx.build(_dev(blob), _dev(offs), n, d_fp, d_po)
        assert ctx.mph_bin() == mph
        assert np.array_equal(d_fp.cpu().numpy().view(np.uint64), fp)
        assert np.array_equal(d_po.cpu().numpy().view(np.uint64), po)
    finally:
        ctx.close()


@pytest.mark.parametrize("world", [4, 8])
def test_c5_skewed_multi_rank_bit_exact(world, oracle_lib):
    """C5's generator (log-uniform 1-1024 B) sharded over `world` ranks on one GPU; the
    replicated tail starts below 20k keys, so levels 0-4 are routed between ranks."""
    import s3imph
    n = 2_000_000
    blob, offs = s3imph.gen_keys(1, 42, 0, 0, n)
    blob = blob[: int(offs[-1])]
    lens = np.diff(offs.astype(np.int64))
    assert lens[1:].min() == 5 and lens.max() == 1024
    st, fp, po, mph = oracle_lib.build_mt(blob, offs, threads=16)
    assert st == 0
    # shards balanced by key BYTES (C5's lengths are skewed)
    cum = offs.astype(np.float64)
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * r / world)) for r in range(1, world)] + [n]
    res = _run(world, _shards(blob, offs, cuts), n, 20_000)
    assert res[0][6]["big_levels"] >= 3
    _check(res, n, fp, po, mph)
