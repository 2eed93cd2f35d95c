"""IndexBuilder.Finalize's depth / subtree / depth-index arrays on the GPU
(s3imph_finalize_index_device / _host) against the oracle (oracle/finalize_oracle.c, the
reference's stack algorithm and DepthIndexBuilder.Build restated and pinned to the
reference's own tests in tests/test_finalize_oracle.py).  Bit-exact arrays; files
byte-identical to the reference framing."""
import json
import os

import numpy as np
import pytest

import finalize_queries as Q
import oracle as O
from conftest import GOLDEN, to_dev

pytestmark = pytest.mark.gpu

CASES = json.load(open(os.path.join(GOLDEN, "finalize", "cases.json")))
FILES = {"depth.u32": ("depth", 4), "subtree_end.u64": ("subtree_end", 8),
         "max_depth_in_subtree.u32": ("max_depth_in_subtree", 4), "depth_offsets.u64": ("depth_offsets", 8),
         "depth_positions.u64": ("depth_positions", 8)}


@pytest.fixture(scope="module")
def s3():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import s3imph
    return s3imph


@pytest.fixture(scope="module")
def ctx(s3):
    c = s3imph_ctx = s3.DeviceBuilder(0)
    yield s3imph_ctx
    c.close()


def _device(ctx, blob, offs, depths=None):
    import torch
    d_depths = None if depths is None else torch.from_numpy(np.asarray(depths, np.uint32).view(np.int32)).cuda()
    r = ctx.finalize_index(to_dev(blob, pad8=True), to_dev(offs), len(offs) - 1, d_depths)
    torch.cuda.synchronize()
    out = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in r.items()}
    for k in ("depth", "max_depth_in_subtree"):
        out[k] = out[k].view(np.uint32)
    for k in ("subtree_end", "depth_positions", "depth_offsets"):
        out[k] = out[k].view(np.uint64)
    return out


def _same(got, want):
    for k in ("depth", "subtree_end", "max_depth_in_subtree", "depth_offsets", "depth_positions"):
        assert np.array_equal(np.asarray(got[k]), np.asarray(want[k])), k
    assert got["max_depth"] == want["max_depth"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_reference_cases(s3, ctx, oracle_lib, case, tmp_path):
    keys = case["keys"]
    blob, offs = O.keys_to_blob([k.encode() for k in keys])
    depths = case.get("depths")
    got = _device(ctx, blob, offs, depths)
    _same(got, oracle_lib.finalize(blob, offs, None if depths is None else np.array(depths, np.uint32)))
    Q.check_case(case, got, keys)
    s3.finalize_index_host(blob, offs, str(tmp_path), None if depths is None else np.array(depths, np.uint32))
    for name, (k, w) in FILES.items():
        data = s3.read_array(str(tmp_path / name), w)
        assert np.array_equal(data, got[k]), name


def _prefix_set(seed, n_objects, fanout, max_depth, closed):
    rng = np.random.default_rng(seed)
    s = {""} if closed else set()
    for _ in range(n_objects):
        d = int(rng.integers(1, max_depth + 1))
        parts = ["%x" % int(rng.integers(0, fanout)) for _ in range(d)]
        if closed:
            for j in range(1, d + 1):
                s.add("/".join(parts[:j]) + "/")
        else:
            s.add("/".join(parts) + "/")
    return sorted(k.encode() for k in s)


@pytest.mark.parametrize("closed", [True, False])
@pytest.mark.parametrize("seed,n_obj,fan,depth", [(1, 2000, 4, 5), (2, 200_000, 16, 9), (3, 400_000, 64, 4)])
def test_random_trees(ctx, oracle_lib, seed, n_obj, fan, depth, closed):
    keys = _prefix_set(seed, n_obj, fan, depth, closed)
    blob, offs = O.keys_to_blob(keys)
    _same(_device(ctx, blob, offs), oracle_lib.finalize(blob, offs))


def test_wide_subtrees_cross_superblocks(ctx, oracle_lib):
    """Internal nodes whose runs span several 1024-key blocks and 1M-key superblocks (the
    hierarchical search), keys of every alignment, plus a root."""
    keys = [b""]
    for top in range(3):
        keys.append(b"t%d/" % top)
        for i in range(700_000 + 123_457 * top):
            keys.append(b"t%d/%07x/" % (top, i))
    keys.sort()
    blob, offs = O.keys_to_blob(keys)
    _same(_device(ctx, blob, offs), oracle_lib.finalize(blob, offs))


def test_c2_synthetic_and_custom_depths(s3, ctx, oracle_lib):
    """C2's 10M synthetic prefixes (not ancestor-closed, one root), then the same keys with
    caller-given depths (row.Depth) instead of the '/' count."""
    blob, offs = s3.gen_keys(0, 42, 32, 0, 10_000_000)
    blob = blob[: int(offs[-1])]
    _same(_device(ctx, blob, offs), oracle_lib.finalize(blob, offs))
    depths = (np.arange(len(offs) - 1, dtype=np.uint64) * 2654435761 % 23).astype(np.uint32)
    _same(_device(ctx, blob, offs, depths), oracle_lib.finalize(blob, offs, depths))


@pytest.mark.parametrize("n_obj", [3000, 300_000])
def test_unaligned_caller_depths(s3, ctx, oracle_lib, n_obj):
    """Caller depths (row.Depth) handed over as a view at a 4-byte offset: the block pass
    takes its per-lane fallback for every lane, and each lane must cover its own four keys
    only (subtrees crossing 1024-key blocks, the maximum depth below each node)."""
    import torch
    keys = _prefix_set(7, n_obj, 8, 7, True)
    blob, offs = O.keys_to_blob(keys)
    n = len(keys)
    depths = np.array([k.count(b"/") for k in keys], np.uint32)
    buf = torch.zeros(n + 4, dtype=torch.int32, device="cuda")
    buf[1:n + 1] = torch.from_numpy(depths.view(np.int32)).cuda()
    view = buf[1:n + 1]
    assert view.data_ptr() % 16 == 4
    r = ctx.finalize_index(to_dev(blob, pad8=True), to_dev(offs), n, view)
    torch.cuda.synchronize()
    got = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in r.items()}
    for k in ("depth", "max_depth_in_subtree"):
        got[k] = got[k].view(np.uint32)
    for k in ("subtree_end", "depth_positions", "depth_offsets"):
        got[k] = got[k].view(np.uint64)
    _same(got, oracle_lib.finalize(blob, offs, depths))


def test_empty_and_single(s3, ctx, oracle_lib, tmp_path):
    blob, offs = O.keys_to_blob([])
    s3.finalize_index_host(blob, offs, str(tmp_path))
    assert (tmp_path / "depth_offsets.u64").read_bytes() == O.s3id_u64_array([0, 0])
    assert (tmp_path / "depth.u32").read_bytes() == O.s3id_u32_array([])
    blob, offs = O.keys_to_blob([b"only/"])
    _same(_device(ctx, blob, offs), oracle_lib.finalize(blob, offs))
