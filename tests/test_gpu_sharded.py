"""The 8-GPU configurations at their sharded shape, as 8 ranks on this box's one GPU (run with
-m gpu on an MI355X), and the bitmap decomposition at its tile bound.

BASELINE.md §3 asks for 1/2/4/8-GPU outputs byte-identical for C4 and C5.  Here every rank is
a host thread of s3imph_build_host_multi on device 0 (the in-process transport: device-to-
device copies), running the north_star's per-level collision-bitmap decomposition with no
fallback (S3IMPH_DIST_STRICT) — the same rank code RCCL drives on an 8-GPU node:

- C5 (configs[4]): 8 ranks x 25M skewed keys (200M global, 1-1024 B log-uniform), mph.bin,
  mph_fp and mph_pos byte for byte against the oracle;
- C4 (configs[3]): 8 ranks x 125M keys (1B global, avg 32 B; level 0 in 30 518 tiles of 2^16,
  93 % of kBmMaxTiles) against the single-GPU build of the same 1B keys, byte for byte (the
  single-GPU build itself is checked by properties in test_gpu_scale.py and bit-exact against
  the oracle at 125M);
- the P0 tile bound: one rank at exactly kBmMaxTiles = 32 768 level-0 tiles of 2^16 positions
  (N = 2^30 keys: 2^31 positions) equals the single-GPU build; one key more misses the bound:
  an error under strict mode; otherwise the routed fallback, which at one rank is the single-GPU
  build, refuses the set cleanly (no single GPU takes level 0 past 2^31 positions; two or more
  ranks split them).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _release_cached_workspaces():
    """These builds take most of the HBM: free what earlier builds keep cached before and after."""
    import torch
    import s3imph
    s3imph.release_workspaces()
    torch.cuda.empty_cache()
    yield
    s3imph.release_workspaces()
    torch.cuda.empty_cache()


def _single_gpu(blob, offs):
    """(mph.bin, mph_fp, mph_pos) of the single-GPU device build (host copies)."""
    import torch
    import s3imph
    n = len(offs) - 1
    d_blob = torch.from_numpy(blob).to("cuda")
    d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda")
    d_fp = torch.empty(n, dtype=torch.int64, device="cuda")
    d_po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = s3imph.DeviceBuilder(0)
    try:
        ctx.build(d_blob, d_offs, n, d_fp, d_po)
        mph = ctx.mph_bin()
        fp = d_fp.cpu().numpy().view(np.uint64)
        po = d_po.cpu().numpy().view(np.uint64)
    finally:
        ctx.close()
        del d_blob, d_offs, d_fp, d_po
        torch.cuda.empty_cache()
    return mph, fp, po


def test_c5_8_ranks_x_25m_skewed_bit_exact(oracle_lib, monkeypatch, capfd):
    import s3imph
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 41))  # a fresh set (reads S3IMPH_DEBUG)
    n = 200_000_000
    blob, offs = s3imph.gen_keys(1, 42, 0, 0, n)
    st, fp, po, mph = oracle_lib.build_mt(blob[: int(offs[-1])], offs, threads=16)
    assert st == 0
    g = s3imph.build_host(blob, offs, devices=[0] * 8, flags=s3imph.MULTI_BITMAP)
    assert g[2] == mph
    assert np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("level 0 through P0 super-tiles") == 8, err[-3000:]


def test_c4_8_ranks_x_125m_equals_single_gpu(monkeypatch, capfd):
    import s3imph
    n = 1_000_000_000
    blob, offs = s3imph.gen_keys(0, 42, 32, 0, n)
    mph, fp, po = _single_gpu(blob, offs)
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 43))
    out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))
    g = s3imph.build_host(blob, offs, devices=[0] * 8, flags=s3imph.MULTI_BITMAP, out=out)
    assert g[2] == mph
    assert np.array_equal(g[0], fp) and np.array_equal(g[1], po)
    err = capfd.readouterr().err
    assert err.count("level 0 through P0 super-tiles (30518 tiles of 2^16)") == 8, err[-3000:]


def test_bitmap_level0_at_and_past_the_p0_tile_bound(monkeypatch, capfd):
    import s3imph
    n = 1 << 30  # 2^25 words = 2^31 positions = 32 768 tiles of 2^16
    blob, offs = s3imph.gen_keys(0, 5, 16, 0, n + 1)
    monkeypatch.setenv("S3IMPH_DEBUG", "1")
    monkeypatch.setenv("S3IMPH_DIST_STRICT", "1")
    monkeypatch.setenv("S3IMPH_DIST_SWITCH", str((2 << 20) + 47))
    at = offs[: n + 1]
    mph, fp, po = _single_gpu(blob, at)
    out = (np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64))
    g = s3imph.build_host(blob, at, num_gpus=1, flags=s3imph.MULTI_FORCE_SHARDED | s3imph.MULTI_BITMAP, out=out)
    assert g[2] == mph
    assert np.array_equal(g[0][:n], fp) and np.array_equal(g[1][:n], po)
    err = capfd.readouterr().err
    assert "level 0 through P0 super-tiles (32768 tiles of 2^16)" in err, err[-3000:]
    del fp, po
    # one key more: 2^31 + 64 positions, past every bitmap level-0 form
    with pytest.raises(s3imph.MPHFError) as e:
        s3imph.build_host(blob, offs, num_gpus=1, flags=s3imph.MULTI_FORCE_SHARDED | s3imph.MULTI_BITMAP, out=out)
    assert "size bounds" in str(e.value)
    # without strict mode the build falls back to routing, which at one rank is the single-GPU
    # build — and no single GPU takes level 0 past 2^31 positions: a clear error, not a fault
    monkeypatch.delenv("S3IMPH_DIST_STRICT")
    with pytest.raises(s3imph.MPHFError) as e:
        s3imph.build_host(blob, offs, num_gpus=1, flags=s3imph.MULTI_FORCE_SHARDED | s3imph.MULTI_BITMAP, out=out)
    assert e.value.status == s3imph.ERR_INVALID and "more than 2^30 keys on one GPU" in str(e.value)
