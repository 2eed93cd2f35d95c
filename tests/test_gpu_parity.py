"""Parity of the HIP build against the CPU oracle (run on an MI355X with -m gpu).

Bit-exact bar: mph.bin bytes, mph_fp.u64 and mph_pos.u64 equal the oracle's for the
same input (integer path — no tolerance).  Small/medium sets compare everything;
BASELINE's full sizes are checked through size-independent properties (positions
form a permutation, every member looks itself up, determinism across runs).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import keysets
import oracle as O
from conftest import GOLDEN, from_dev, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s3():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import s3imph
    return s3imph


@pytest.fixture(scope="module")
def ctx(s3):
    c = s3.DeviceBuilder(0)
    yield c
    c.close()


def _device_build(s3, ctx, blob, offs, pos=None):
    import torch
    n = len(offs) - 1
    d_blob = to_dev(np.ascontiguousarray(blob, np.uint8), pad8=True)
    d_offs = to_dev(offs)
    d_pos = to_dev(pos) if pos is not None else None
    d_fp = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    d_po = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    info = ctx.build(d_blob, d_offs, n, d_fp, d_po, d_pos=d_pos)
    torch.cuda.synchronize()
    return from_dev(d_fp)[:n], from_dev(d_po)[:n], ctx.mph_bin(), info


def _check_vs_oracle(oracle_lib, s3, ctx, keys, pos=None):
    blob, offs = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(blob, offs, pos)
    assert st == 0
    gfp, gpo, gmph, info = _device_build(s3, ctx, blob, offs, pos)
    assert gmph == mph
    assert np.array_equal(gfp, fp)
    assert np.array_equal(gpo, po)
    return info


def _fixture_files():
    return sorted(p for p in os.listdir(GOLDEN) if p.endswith(".json") and p != "fnv_kat.json")


@pytest.mark.parametrize("fname", _fixture_files())
def test_golden_fixture(s3, ctx, fname):
    """Device build reproduces each committed fixture (the reference's own test key sets)."""
    with open(os.path.join(GOLDEN, fname)) as f:
        fx = json.load(f)
    name = fx["name"]
    if "keys" in fx:
        ks = fx["keys"]
    else:
        ks = {"memory_test_10000": keysets.memory_test_prefixes,
              "wide_single_level_100k": keysets.wide_single_level_prefixes,
              "realistic_100k": lambda: keysets.realistic_prefixes(100000)}[name]()
    keys = [k.encode() for k in ks]
    blob, offs = O.keys_to_blob(keys)
    gfp, gpo, gmph, _ = _device_build(s3, ctx, blob, offs)
    got = {"mph.bin": gmph, "mph_fp.u64": O.s3id_u64_array(gfp), "mph_pos.u64": O.s3id_u64_array(gpo)}
    for k, v in got.items():
        assert hashlib.sha256(v).hexdigest() == fx["files_sha256"][k], (name, k)


def test_builder_writes_identical_files(s3, oracle_lib, tmp_path):
    """StreamingMPHFBuilder mirror: Add x N -> Build(outDir) -> the 5 files equal the oracle's."""
    keys = [k.encode() for k in keysets.wide_single_level_prefixes(20000)]
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    for i, k in enumerate(keys):
        b.add(k, i)
    assert b.count() == len(keys)
    out = tmp_path / "idx"
    out.mkdir()
    b.build(str(out))
    b.close()
    blob, offs = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(blob, offs)
    want = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(po),
            "prefix_blob.bin": blob.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(offs)}
    for name, data in want.items():
        assert (out / name).read_bytes() == data, name


def test_builder_feed_many_chunks(s3, oracle_lib, tmp_path):
    """f3 + f2: Add copies the keys once into pooled pinned chunks (256 KiB doubling to
    64 MiB) that DMA to the GPU while the caller is still adding (2.5M keys, ~80 MB of blob:
    past the feed's first 16 MiB device buffers, so they grow), in batches of 100k with
    custom positions, then single Adds; Build writes mph_fp / mph_pos as their chunks come
    back and the prefix files from the host chunks beside them.  The 5 files equal the
    oracle's."""
    n = 2_500_000
    blob, offs = s3.gen_keys(0, 21, 32, 0, n)
    blob = blob[: int(offs[-1])]
    pos = np.random.default_rng(5).permutation(n).astype(np.uint64) + np.uint64(7)
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    tail = n - 10
    for lo in range(0, tail, 100_000):
        hi = min(lo + 100_000, tail)
        b.add_batch(blob, offs[lo:hi + 1], pos[lo:hi])
    for i in range(tail, n):
        b.add(bytes(blob[offs[i]:offs[i + 1]]), int(pos[i]))
    assert b.count() == n
    out = tmp_path / "idx"
    out.mkdir()
    b.build(str(out))
    b.close()
    st, fp, po, mph = oracle_lib.build_mt(blob, offs, pos, threads=16)
    assert st == 0
    want = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(po),
            "prefix_blob.bin": blob.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(offs)}
    for name, data in want.items():
        assert (out / name).read_bytes() == data, name


@pytest.mark.parametrize("hint", ["exact", "short", "none"])
def test_builder_reserve_hint(s3, oracle_lib, tmp_path, hint):
    """The capacity hint (s3imph_builder_reserve): exact (device arrays allocated once), too
    short (they grow past it), none; batches with identity positions (pos NULL ->
    Count()+i) between single Adds.  The 5 files equal the oracle's."""
    n = 1_200_000
    blob, offs = s3.gen_keys(0, 23, 40, 0, n)
    blob = blob[: int(offs[-1])]
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    if hint == "exact":
        b.reserve(n, int(offs[-1]))
    elif hint == "short":
        b.reserve(n // 10, int(offs[-1]) // 10)
    i = 0
    for lo, hi in ((0, 3), (3, 500_003), (500_003, 500_010), (500_010, n)):
        if hi - lo < 10:
            for k in range(lo, hi):
                b.add(bytes(blob[offs[k]:offs[k + 1]]), k)
        else:
            b.add_batch(blob, offs[lo:hi + 1])
        i = hi
    assert b.count() == n == i
    out = tmp_path / "idx"
    out.mkdir()
    b.build(str(out))
    b.close()
    st, fp, po, mph = oracle_lib.build_mt(blob, offs, threads=16)
    assert st == 0
    want = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(po),
            "prefix_blob.bin": blob.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(offs)}
    for name, data in want.items():
        assert (out / name).read_bytes() == data, name


def test_builder_feed_duplicate_keys_error(s3, tmp_path):
    """A duplicate key fed through the device feed fails Build with the duplicate-hash
    status; no half-written success is reported."""
    keys = [b"p/%06d/" % i for i in range(50_000)]
    keys[40_000] = keys[123]
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    for i, k in enumerate(keys):
        b.add(k, i)
    out = tmp_path / "idx"
    out.mkdir()
    with pytest.raises(s3.MPHFError) as e:
        b.build(str(out))
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    # the reference's Build fails in bbhash.New before it writes any file
    # (mphf_streaming.go:141-144): out_dir stays empty
    assert list(out.iterdir()) == []
    b.close()


def test_build_host_roundtrip_lookup(s3, oracle_lib):
    """build_host + the oracle's Lookup restatement: every member -> its pos (VerifyMPHF)."""
    keys = [k.encode() for k in keysets.mphf_test_sets()["mphf_no_false_pos"]]
    blob, offs = O.keys_to_blob(keys)
    fp, po, mph = s3.build_host(blob, offs)
    st, m = oracle_lib.unmarshal(mph)
    assert st == 0
    for i, k in enumerate(keys):
        assert oracle_lib.lookup(m, fp, po, k) == i
    for k in keysets.NON_MEMBERS:
        assert oracle_lib.lookup(m, fp, po, k.encode()) is None


def test_build_host_staged_chunks_offset_blob_custom_pos(s3, oracle_lib):
    """s3imph_build_host moves pageable host data through the pinned chunk stager
    (8 MiB chunks over 8 workers): a multi-chunk set whose blob starts at a non-zero
    offsets[0] (rebased while staged) with custom positions, bit-exact vs the oracle."""
    n = 3_000_000
    blob, offs = s3.gen_keys(0, 23, 32, 0, n)
    blob = blob[: int(offs[-1])]
    pos = np.random.default_rng(9).permutation(n).astype(np.uint64) * np.uint64(5)
    st, fp, po, mph = oracle_lib.build(blob, offs, pos)
    assert st == 0
    shifted = np.concatenate([np.frombuffer(b"0123456789abc", np.uint8), blob])
    gfp, gpo, gmph = s3.build_host(shifted, offs + np.uint64(13), pos)
    assert gmph == mph
    assert np.array_equal(gfp, fp) and np.array_equal(gpo, po)


def test_build_host_offsets_as_u16_lengths(s3, oracle_lib):
    """build_host sends the offsets as u16 key lengths (device scan back to offsets): a set
    whose lengths span several 8 MiB staging chunks (4.2M keys: 8.4 MB of lengths, the
    scan's last block ragged), a non-zero offsets[0]."""
    n = 4_200_001
    blob, offs = s3.gen_keys(0, 5, 40, 0, n)
    blob = blob[: int(offs[-1])]
    st, fp, po, mph = oracle_lib.build(blob, offs)
    assert st == 0
    shifted = np.concatenate([np.frombuffer(b"0123456", np.uint8), blob])
    gfp, gpo, gmph = s3.build_host(shifted, offs + np.uint64(7))
    assert gmph == mph
    assert np.array_equal(gfp, fp) and np.array_equal(gpo, po)


def test_build_host_key_longer_than_u16(s3, oracle_lib):
    """A key of 65536 B or more cannot travel as a u16 length: build_host falls back to
    u32 offsets for the whole set, bit-exact."""
    rng = np.random.default_rng(12)
    keys = {rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in (65535, 65536, 70000)}
    while len(keys) < 50000:
        keys.add(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8).tobytes())
    keys = sorted(keys)
    blob, offs = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(blob, offs)
    assert st == 0
    gfp, gpo, gmph = s3.build_host(blob, offs)
    assert gmph == mph
    assert np.array_equal(gfp, fp) and np.array_equal(gpo, po)


def test_build_host_into_reused_buffers_piecewise_hash(s3, oracle_lib):
    """s3imph_build_host_into: outputs and mph.bin go to caller buffers reused across calls.
    Sets of every level-0 path — P0 (18M keys), the plain pair hash (2M), a skewed set
    (k_hash_skew), a blob at a non-zero offsets[0] with custom positions, a tiny set — each
    bit-exact vs the oracle, and equal to s3imph_build_host's malloc'd mph.bin.  (Every blob
    here is under 512 MiB, so with the default piece size it crosses PCIe as ONE piece; the
    piecewise hash is test_piecewise_hash_every_level0_path.)"""
    cap = 18_000_000
    out = (np.zeros(cap, np.uint64), np.zeros(cap, np.uint64))
    mph_buf = np.zeros(s3.mph_bin_bound(cap), np.uint8)
    cases = [(0, 29, 20, 18_000_000, False), (0, 30, 32, 2_000_000, False), (1, 31, 0, 1_500_000, False),
             (0, 32, 24, 900_000, True), (0, 33, 24, 5, False)]
    for kind, seed, avg, n, shifted in cases:
        blob, offs = s3.gen_keys(kind, seed, avg, 0, n)
        blob = blob[: int(offs[-1])]
        pos = np.random.default_rng(seed).permutation(n).astype(np.uint64) * np.uint64(3) if shifted else None
        st, fp, po, mph = oracle_lib.build_mt(blob, offs, pos, threads=16)
        assert st == 0
        if shifted:
            blob = np.concatenate([np.frombuffer(b"xyz", np.uint8), blob])
            offs = offs + np.uint64(3)
        ln = s3.build_host_into(blob, offs, out, mph_buf, pos)
        assert bytes(mph_buf[:ln]) == mph, (kind, n)
        assert np.array_equal(out[0][:n], fp) and np.array_equal(out[1][:n], po), (kind, n)
        g = s3.build_host(blob, offs, pos)
        assert g[2] == mph


@pytest.mark.parametrize("n", [1, 2, 3, 31, 32, 33, 63, 64, 65, 1000, 4097, 65535, 65536, 65537, 200000])
def test_sizes_around_boundaries(s3, oracle_lib, ctx, n):
    blob, offs = s3.gen_keys(0, 7, 24, 0, n)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(n)]
    _check_vs_oracle(oracle_lib, s3, ctx, keys)


def test_ragged_lengths_0_to_1024(s3, oracle_lib, ctx):
    rng = np.random.default_rng(5)
    keys = set()
    while len(keys) < 30000:
        L = int(rng.integers(0, 1025)) if rng.random() < 0.5 else int(rng.integers(0, 12))
        keys.add(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
    _check_vs_oracle(oracle_lib, s3, ctx, sorted(keys))


def test_very_long_keys_mixed(s3, oracle_lib, ctx):
    """A few 16-200 KiB keys among short ones (the sampled-skew path and the per-lane
    word chains at extreme lengths), and one key of exactly 2^16 bytes: bit-exact."""
    rng = np.random.default_rng(11)
    keys = set()
    for L in [65536] + [int(x) for x in rng.integers(16 << 10, 200 << 10, 40)]:
        keys.add(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
    while len(keys) < 20000:
        keys.add(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes())
    _check_vs_oracle(oracle_lib, s3, ctx, sorted(keys))


def test_unaligned_blob_offsets(s3, oracle_lib, ctx):
    """Keys starting at every byte phase, including a non-zero offsets[0]."""
    keys = [bytes([65 + (i % 26)] * (i % 19)) + b"%d/" % i for i in range(5000)]
    blob, offs = O.keys_to_blob(keys)
    shifted = np.concatenate([np.frombuffer(b"zzz", np.uint8), blob])
    st, fp, po, mph = oracle_lib.build(blob, offs)
    gfp, gpo, gmph, _ = _device_build(s3, ctx, shifted, offs + 3)
    assert gmph == mph and np.array_equal(gfp, fp) and np.array_equal(gpo, po)


def test_custom_positions(s3, oracle_lib, ctx):
    keys = [("p%06d/" % i).encode() for i in range(50000)]
    pos = np.random.default_rng(1).permutation(50000).astype(np.uint64) + np.uint64(10**12)
    _check_vs_oracle(oracle_lib, s3, ctx, keys, pos)


def test_empty_and_single(s3, ctx):
    fp, po, mph, info = _device_build(s3, ctx, np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert mph == b"" and len(fp) == 0 and info["num_levels"] == 0
    fp, po, mph, info = _device_build(s3, ctx, np.frombuffer(b"a/", np.uint8), np.array([0, 2], np.uint64))
    assert info["num_levels"] == 1 and po[0] == 0


def test_duplicate_keys_error(s3, ctx):
    keys = [b"a/", b"b/", b"a/", b"c/"]
    blob, offs = O.keys_to_blob(keys)
    with pytest.raises(s3.MPHFError) as e:
        _device_build(s3, ctx, blob, offs)
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    # the context stays usable after the error
    _device_build(s3, ctx, *O.keys_to_blob([b"x/", b"y/"]))


def test_duplicate_keys_error_builder(s3, tmp_path):
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    for k in ["a/", "b/", "a/"]:
        b.add(k, 0)
    with pytest.raises(s3.MPHFError) as e:
        b.build(str(tmp_path))
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    assert "build MPHF" in str(e.value)
    assert not (tmp_path / "mph.bin").exists()


def test_tiny_distinct_sets_are_never_reported_as_duplicates(s3, oracle_lib, ctx):
    """A build stops early when a level places no key, but only when every key left has a
    twin: 3000 two-key sets (about 1 in 64 collide at a level by chance) all build, equal
    to the oracle."""
    for i in range(3000):
        keys = [b"k%d/a" % i, b"k%d/bb" % i]
        blob, offs = O.keys_to_blob(keys)
        st, fp, po, mph = oracle_lib.build(blob, offs)
        gfp, gpo, gmph, info = _device_build(s3, ctx, blob, offs)
        assert gmph == mph and np.array_equal(gfp, fp) and np.array_equal(gpo, po), i


def test_duplicates_stop_the_build_early(s3, ctx):
    """Keys with duplicate hashes stop the build at the first level that places nothing
    (the host then finds the twins among the records left): a 1M-key set with 500
    duplicated keys fails with DUP_KEY_HASH, in about the time of a build."""
    import time
    n = 1_000_000
    blob, offs = s3.gen_keys(0, 21, 32, 0, n)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(n)]
    keys += keys[1000:1500]
    blob, offs = O.keys_to_blob(keys)
    t0 = time.perf_counter()
    with pytest.raises(s3.MPHFError) as e:
        _device_build(s3, ctx, blob, offs)
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    assert time.perf_counter() - t0 < 5.0


def test_duplicated_record_is_an_internal_fault(s3, monkeypatch):
    """A record duplicated inside the build (S3IMPH_FAULT_DUP_REC copies level 1's record 0
    over record 1, as a kernel race would) stops the build on two records with one key
    hash; every ORIGINAL key hash is distinct, so the error is ERR_INTERNAL naming the
    level, never the caller's ERR_DUP_KEY_HASH.  A context without the hook builds the
    same keys."""
    monkeypatch.setenv("S3IMPH_FAULT_DUP_REC", "1")
    blob, offs = s3.gen_keys(0, 5, 32, 0, 200_000)
    faulty = s3.DeviceBuilder(0)
    with pytest.raises(s3.MPHFError) as e:
        _device_build(s3, faulty, blob, offs)
    faulty.close()
    assert e.value.status == s3.ERR_INTERNAL, e.value
    assert "duplicated" in str(e.value) and "level" in str(e.value)
    monkeypatch.delenv("S3IMPH_FAULT_DUP_REC")
    clean = s3.DeviceBuilder(0)
    _device_build(s3, clean, blob, offs)
    clean.close()


def test_duplicate_group_overflowing_a_reservation_slot(s3, ctx):
    """150k copies of one key all land in one tile of every level: the small-level
    reservation slot overflows, the build reruns on the counted path, and the result is
    still the reference's duplicate error (mphf_streaming.go:143)."""
    keys = [b"p/%07d/" % i for i in range(50_000)] + [b"dup/"] * 150_000
    blob, offs = O.keys_to_blob(keys)
    with pytest.raises(s3.MPHFError) as e:
        _device_build(s3, ctx, blob, offs)
    assert e.value.status == s3.ERR_DUP_KEY_HASH
    _device_build(s3, ctx, *O.keys_to_blob([b"x/", b"y/"]))


def test_repeated_builds_same_context_bit_exact(s3, oracle_lib, ctx):
    """Builds of different inputs back to back in one context: every one bit-exact, so
    no level depends on workspace contents left by an earlier build."""
    for seed, n in [(3, 1_500_000), (4, 1_500_000), (5, 900_000), (3, 1_500_000)]:
        blob, offs = s3.gen_keys(0, seed, 32, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, _ = _device_build(s3, ctx, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp)
        assert np.array_equal(gpo, po)


@pytest.mark.parametrize("res_max", ["0", "100000000"])
def test_small_level_paths_bit_exact(s3, oracle_lib, res_max, monkeypatch):
    """Levels >= 1 on the counted path only (res_max 0) and on the reservation path for
    every level (res_max large): both bit-exact with the oracle."""
    monkeypatch.setenv("S3IMPH_RES_MAX", res_max)
    c = s3.DeviceBuilder(0)
    try:
        n = 2_000_000
        blob, offs = s3.gen_keys(0, 7, 32, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, info = _device_build(s3, c, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp)
        assert np.array_equal(gpo, po)
    finally:
        c.close()


@pytest.mark.parametrize("cfg", ["0", "1"])
def test_scatter_forms_bit_exact(s3, oracle_lib, cfg, monkeypatch):
    """The reservation scatter's other LDS forms (S3IMPH_SCAT_CFG 0: 4096 tile counters and
    4096-record rounds for every level; 1: counters sized to the level's tiles, 4096-record
    rounds) on a set whose levels take 1221 / 481 / 189 tiles: bit-exact with the oracle,
    like the default form (5120-record rounds) in test_c2_10m_bit_exact."""
    monkeypatch.setenv("S3IMPH_SCAT_CFG", cfg)
    c = s3.DeviceBuilder(0)
    try:
        n = 10_000_000
        blob, offs = s3.gen_keys(0, 42, 32, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, info = _device_build(s3, c, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp)
        assert np.array_equal(gpo, po)
    finally:
        c.close()


@pytest.mark.parametrize("cfg", ["0", "1"])
def test_skew_shapes_bit_exact(s3, oracle_lib, cfg, monkeypatch):
    """The skewed-length hash's other block / group shapes (S3IMPH_SKEW_CFG 0: two 512-thread
    blocks per CU with 2048-key groups; 1: 1024 threads with 4096-key groups) on a C5-style
    log-uniform 1-1024 B set: bit-exact with the oracle, like the default 768 / 5120 shape
    in test_c5_one_gpu_share_bit_exact."""
    monkeypatch.setenv("S3IMPH_SKEW_CFG", cfg)
    c = s3.DeviceBuilder(0)
    try:
        n = 3_000_000
        blob, offs = s3.gen_keys(1, 23, 0, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, info = _device_build(s3, c, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp)
        assert np.array_equal(gpo, po)
    finally:
        c.close()


@pytest.mark.parametrize("l20", ["0", "1"])
def test_list_record_formats_bit_exact(s3, oracle_lib, l20, monkeypatch):
    """List levels on the reservation path carry R20 records (k, f, key index) by default and
    Rec (k, f, p) with S3IMPH_L20=0: both byte-identical to the oracle on a 6M set whose
    levels 1-3 are reservation levels on the persistent 2^14-position tiles."""
    monkeypatch.setenv("S3IMPH_L20", l20)
    c = s3.DeviceBuilder(0)
    try:
        n = 6_000_000
        blob, offs = s3.gen_keys(0, 31, 40, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, info = _device_build(s3, c, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp)
        assert np.array_equal(gpo, po)
    finally:
        c.close()


def test_c2_10m_bit_exact(s3, oracle_lib, ctx):
    """BASELINE config 2: 10M synthetic prefixes, avg 32 B — full bit-exact comparison."""
    n = 10_000_000
    blob, offs = s3.gen_keys(0, 42, 32, 0, n)
    st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
    assert st == 0
    gfp, gpo, gmph, info = _device_build(s3, ctx, blob, offs)
    assert gmph == mph
    assert np.array_equal(gfp, fp)
    assert np.array_equal(gpo, po)
    assert info["big_levels"] >= 1


def test_determinism_and_device_lookup(s3, ctx):
    """Same input twice -> identical bytes; batched Lookup (mphf.go:275-302) finds every member
    at its pos and rejects non-members (mphf_test.go:182-217 at scale)."""
    import torch
    n = 1_000_000
    blob, offs = s3.gen_keys(0, 3, 40, 0, n)
    a = _device_build(s3, ctx, blob, offs)
    b = _device_build(s3, ctx, blob, offs)
    assert a[2] == b[2] and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    d_fp, d_po = to_dev(a[0]), to_dev(a[1])
    res = torch.zeros(n, dtype=torch.int64, device="cuda")
    ctx.lookup(to_dev(blob, pad8=True), to_dev(offs), n, d_fp, d_po, n, res)
    assert np.array_equal(from_dev(res), np.arange(n, dtype=np.uint64))
    # non-members: keys of a different seed/range
    qb, qo = s3.gen_keys(0, 4, 40, n + 10, 100000)
    res2 = torch.zeros(100000, dtype=torch.int64, device="cuda")
    ctx.lookup(to_dev(qb, pad8=True), to_dev(qo), 100000, d_fp, d_po, n, res2)
    assert (from_dev(res2) == np.uint64(2**64 - 1)).all()


def test_c3_100m_properties(s3, ctx):
    """BASELINE config 3 (100M keys, avg 64 B) at full size: size-independent properties —
    positions are a permutation of [0, N), and every key looks itself up."""
    import torch
    n = 100_000_000
    blob, offs = s3.gen_keys(0, 42, 64, 0, n)
    d_blob = to_dev(blob)
    d_offs = to_dev(offs)
    d_fp = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
    info = ctx.build(d_blob, d_offs, n, d_fp, d_po)
    assert info["n_keys"] == n
    # pos_out is a permutation of 0..N-1
    srt = torch.sort(d_po).values
    assert torch.equal(srt, torch.arange(n, dtype=torch.int64, device="cuda"))
    del srt
    res = torch.zeros(n, dtype=torch.int64, device="cuda")
    ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)
    assert torch.equal(res, torch.arange(n, dtype=torch.int64, device="cuda"))


@pytest.mark.parametrize("n,kind,avg", [(70_000, 0, 32), (1_000_000, 1, 0), (10_000_000, 0, 32)])
def test_level0_ragged_and_c2_custom_positions(s3, oracle_lib, ctx, n, kind, avg):
    """Level 0 on near-uniform and skewed (length-sorted hash) inputs, custom positions on
    the skewed one: bit-exact with the oracle."""
    blob, offs = s3.gen_keys(kind, 19, avg, 0, n)
    pos = None
    if n == 1_000_000:
        pos = np.random.default_rng(5).permutation(n).astype(np.uint64) * np.uint64(3)
    st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs, pos)
    assert st == 0
    gfp, gpo, gmph, info = _device_build(s3, ctx, blob, offs, pos)
    assert gmph == mph
    assert np.array_equal(gfp, fp)
    assert np.array_equal(gpo, po)


def test_big_tiles_bit_exact(s3, oracle_lib):
    """70M keys, short (avg 12 B): level 0 (8.5k tiles of 2^14 positions) through the P0
    super-tiles and the pipelined register tiles, level 1 on the split kernel.  Bit-exact
    with the oracle."""
    c = s3.DeviceBuilder(0)
    try:
        n = 70_000_000
        blob, offs = s3.gen_keys(0, 31, 12, 0, n)
        st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
        assert st == 0
        gfp, gpo, gmph, info = _device_build(s3, c, blob, offs)
        assert gmph == mph
        assert np.array_equal(gfp, fp) and np.array_equal(gpo, po)
    finally:
        c.close()


@pytest.mark.parametrize("n,unaligned", [(16_800_000, False), (20_000_000, True), (40_000_000, False)])
def test_p0_level0_bit_exact(s3, oracle_lib, n, unaligned):
    """Level 0 with more than 2048 tiles of 2^14 positions (P0, s3imph_internal.h): the
    records go to super-tile slots, then to their tiles' slots, then the pipelined register
    tiles (k_tile_p0).  Just past the threshold (2051 tiles), and an unaligned blob whose
    level-0 hash is k_hash_count0 (kh / fp, then the partition pass); 5 / 10 super-tiles
    (blocks per super-tile a multiple of the 8 XCD shards, ~768 in all).  Bit-exact, and the build's
    last attempt is P0's (no conservative rerun: its stage marks are P0's)."""
    c = s3.DeviceBuilder(0)
    try:
        blob, offs = s3.gen_keys(0, 19, 20, 0, n)
        blob = blob[: int(offs[-1])]
        st, fp, po, mph = oracle_lib.build_mt(blob, offs, threads=16)
        assert st == 0
        c.set_profiling(1)
        if unaligned:
            gfp, gpo, gmph, _ = _device_build(s3, c, np.concatenate([np.frombuffer(b"q", np.uint8), blob]), offs + 1)
        else:
            gfp, gpo, gmph, _ = _device_build(s3, c, blob, offs)
        assert gmph == mph and np.array_equal(gfp, fp) and np.array_equal(gpo, po)
        assert "scatter0_p0" in c.stage_times(), c.stage_times()
    finally:
        c.close()


def test_p0_allocation_failure_falls_back_and_recovers(s3, oracle_lib, monkeypatch):
    """P0's super-tile buffer is replaced when a bigger set needs more.  With the
    allocation failing (S3IMPH_FAULT_P0_NOMEM frees the old buffer, then fails), the build
    takes the split-kernel level 0 and is still bit-exact; the next, SMALLER build on the same
    context must not take the freed buffer as big enough: it reallocates and runs P0 again."""
    c = s3.DeviceBuilder(0)
    try:
        c.set_profiling(1)
        for n, fault in [(18_000_000, False), (21_000_000, True), (17_500_000, False)]:
            blob, offs = s3.gen_keys(0, 23, 20, 0, n)
            blob = blob[: int(offs[-1])]
            st, fp, po, mph = oracle_lib.build_mt(blob, offs, threads=16)
            assert st == 0
            if fault:
                monkeypatch.setenv("S3IMPH_FAULT_P0_NOMEM", "1")
            else:
                monkeypatch.delenv("S3IMPH_FAULT_P0_NOMEM", raising=False)
            gfp, gpo, gmph, _ = _device_build(s3, c, blob, offs)
            assert gmph == mph and np.array_equal(gfp, fp) and np.array_equal(gpo, po), (n, fault)
            assert ("scatter0_p0" in c.stage_times()) == (not fault), (n, fault, c.stage_times())
    finally:
        c.close()


def test_dev_knobs_ignored_without_opt_in(s3, oracle_lib, monkeypatch):
    """ADVICE / VERDICT r4: the release library reads no developer knob unless the caller opted
    in (s3imph_dev_knobs, include/s3imph.h section 7).  Without the opt-in a context made under
    S3IMPH_FAULT_DUP_REC builds normally (bit-exact); with it the same context setup faults."""
    monkeypatch.setenv("S3IMPH_FAULT_DUP_REC", "1")
    blob, offs = s3.gen_keys(0, 5, 32, 0, 200_000)
    st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
    s3.dev_knobs(False)
    try:
        c = s3.DeviceBuilder(0)
        gfp, gpo, gmph, _ = _device_build(s3, c, blob, offs)
        c.close()
        assert gmph == mph and np.array_equal(gfp, fp) and np.array_equal(gpo, po)
    finally:
        s3.dev_knobs(True)
    c = s3.DeviceBuilder(0)
    with pytest.raises(s3.MPHFError) as e:
        _device_build(s3, c, blob, offs)
    c.close()
    assert e.value.status == s3.ERR_INTERNAL


def test_p0_off_split_kernel_bit_exact(s3, oracle_lib):
    """S3IMPH_P0=0 (A/B knob): the same big level 0 on the split kernel instead: bit-exact."""
    _parity_subprocess({"S3IMPH_P0": "0"}, [(40_000_000, 0, 12)])


def test_big_tiles_counted_path(s3, oracle_lib):
    """2^16-position tiles fed by the counted scatter (histogram-scan ranges instead of
    reservation shards), 40M keys: the split big-tile kernel reads contiguous buckets."""
    _parity_subprocess({"S3IMPH_RES_MAX": "0", "S3IMPH_RES0": "0"}, [(40_000_000, 0, 12)])


@pytest.mark.parametrize("kind,avg", [(0, 32), (1, 0)])
def test_repeated_builds_identical(s3, oracle_lib, ctx, kind, avg):
    """Schedule-dependent races show up as a build that differs from the others: 12
    device builds of one 10M-key set (level 0 and levels 1..7 on the reservation path)
    each equal the oracle's outputs byte for byte."""
    import torch
    n = 10_000_000
    blob, offs = s3.gen_keys(kind, 3, avg, 0, n)
    st, fp, po, mph = oracle_lib.build(blob[: offs[-1]], offs)
    assert st == 0
    d_blob, d_offs = to_dev(blob), to_dev(offs)
    d_fp = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
    for r in range(12):
        d_fp.zero_()
        d_po.zero_()
        ctx.build(d_blob, d_offs, n, d_fp, d_po)
        assert ctx.mph_bin() == mph, r
        assert np.array_equal(from_dev(d_fp), fp), r
        assert np.array_equal(from_dev(d_po), po), r


def _parity_subprocess(env: dict, cases) -> None:
    """Build `cases` (n, kind, avg[, custom positions]) through s3imph.build_host in a fresh process with
    `env` set (the library reads its A/B knobs once per process): bit-exact vs the oracle."""
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0]=[%r, %r]\n"
        "import numpy as np, torch, s3imph, oracle as O\n"
        "for case in %r:\n"
        "    n, kind, avg = case[:3]\n"
        "    blob, offs = s3imph.gen_keys(kind, 3, avg, 0, n)\n"
        "    pos = np.random.default_rng(n).permutation(n).astype(np.uint64) * np.uint64(5) if case[3:] else None\n"
        "    st, fp, po, mph = O.lib().build_mt(blob[: offs[-1]], offs, pos, threads=16)\n"
        "    g = s3imph.build_host(blob, offs, pos)\n"
        "    assert g[2] == mph and np.array_equal(g[0], fp) and np.array_equal(g[1], po), n\n"
        "print('ok')\n"
    ) % (os.path.join(os.path.dirname(GOLDEN), "..", "s3-inv-db_amd"), os.path.join(os.path.dirname(GOLDEN), "..", "oracle"),
         list(cases))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280,
                       env={**os.environ, **env})
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def _parity_device_subprocess(env: dict, cases, builds: int = 2) -> None:
    """Build `cases` (n, kind, avg) device-resident (s3imph.DeviceBuilder: keys and outputs in
    HBM) `builds` times each in a fresh process with `env` set: bit-exact vs the oracle."""
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0]=[%r, %r]\n"
        "import numpy as np, torch, s3imph, oracle as O\n"
        "ctx = s3imph.DeviceBuilder(0)\n"
        "for n, kind, avg in %r:\n"
        "    blob, offs = s3imph.gen_keys(kind, 3, avg, 0, n)\n"
        "    st, fp, po, mph = O.lib().build_mt(blob[: offs[-1]], offs, None, threads=16)\n"
        "    d_blob = torch.from_numpy(blob).to('cuda')\n"
        "    d_offs = torch.from_numpy(offs.view(np.int64)).to('cuda')\n"
        "    for b in range(%d):\n"
        "        d_fp = torch.zeros(n, dtype=torch.int64, device='cuda')\n"
        "        d_po = torch.zeros(n, dtype=torch.int64, device='cuda')\n"
        "        ctx.build(d_blob, d_offs, n, d_fp, d_po)\n"
        "        assert ctx.mph_bin() == mph, (n, b)\n"
        "        assert np.array_equal(d_fp.cpu().numpy().view(np.uint64), fp), (n, b)\n"
        "        assert np.array_equal(d_po.cpu().numpy().view(np.uint64), po), (n, b)\n"
        "ctx.close()\n"
        "print('ok')\n"
    ) % (os.path.join(os.path.dirname(GOLDEN), "..", "s3-inv-db_amd"), os.path.join(os.path.dirname(GOLDEN), "..", "oracle"),
         list(cases), builds)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280,
                       env={**os.environ, **env})
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_p0_scatter_overlapped_on_hash_bit_exact(s3, oracle_lib):
    """Level 0's super-tile scatter overlapped on the hash (S3IMPH_P0_OV=1): the
    direct-form scatter runs beside k_hash0_pair on a second stream, taking each XCD's parts as
    their hash blocks publish them, the follow-up launch the rest; then the direct form alone
    (S3IMPH_P0_DIRECT=1).  Uniform sets at 509 / 191 / 1024-tile super-tiles (C3 100M and
    smaller) and a skewed set (the follow-up takes every part): bit-exact, two builds each."""
    cases = [(100_000_000, 0, 64), (30_000_000, 0, 16), (40_000_000, 1, 0)]
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_P0_OV": "1"}, cases)
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_P0_OV": "1", "S3IMPH_P0_TPS": "191"}, cases[:1], builds=1)
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_P0_OV": "1", "S3IMPH_P0_MAXS": "4"}, cases[1:2], builds=1)
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_P0_DIRECT": "1"}, cases[:2], builds=1)


def test_mid_levels_over_every_cu_bit_exact(s3, oracle_lib):
    """The mid-size levels on 256 workgroups (S3IMPH_MID_BIG=1: the levels of 440k-1.75M keys;
    =2: every level down to the tail; off by default): C2's 10M keys and a skewed
    4M set, bit-exact, two builds each (the second reuses the 256-workgroup scratch)."""
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_MID_BIG": "1"}, [(10_000_000, 0, 32), (4_000_000, 1, 0)])
    _parity_device_subprocess({"S3IMPH_DEV": "1", "S3IMPH_MID_BIG": "2"}, [(10_000_000, 0, 32)], builds=1)


def test_p0_many_super_tiles_bit_exact(s3, oracle_lib):
    """More than 32 super-tiles on the two-block-per-CU super-tile scatter (S3IMPH_P0_BIG=0,
    S3IMPH_P0_TPS=48: 45 / 51 super-tiles on 17.5M uniform / 20M skewed keys, 8 blocks of 512
    threads each), reading the fused hash's regions and k_hash_skew's; bit-exact."""
    _parity_subprocess({"S3IMPH_P0_TPS": "48", "S3IMPH_P0_BIG": "0"}, [(17_500_000, 0, 20), (20_000_000, 1, 0)])


def test_skew_partition_two_blocks_bit_exact(s3, oracle_lib):
    """k_hash_skew's partition form without result arrays, two 512-thread blocks per CU
    (S3IMPH_SKEW_CFG=3; off by default, profiles/r6_skew/): a 20M-key skewed set through
    P0's 512 region sets, bit-exact."""
    _parity_subprocess({"S3IMPH_SKEW_CFG": "3"}, [(20_000_000, 1, 0)])


def test_p0_super_tile_cap_bit_exact(s3, oracle_lib):
    """S3IMPH_P0_MAXS=8 (A/B knob; 64 by default): 60M short keys in 8 super-tiles of 916 tiles
    (the super-tile scatter's 1024-tile-counter form) instead of 15 of ~489: bit-exact."""
    _parity_subprocess({"S3IMPH_P0_MAXS": "8"}, [(60_000_000, 0, 12)])


def test_counted_path_every_level(s3, oracle_lib):
    """With the reservation scatter off (S3IMPH_RES_MAX=0, S3IMPH_RES0=0) every level runs
    count -> histogram scan -> counted scatter -> tile: bit-exact."""
    _parity_subprocess({"S3IMPH_RES_MAX": "0", "S3IMPH_RES0": "0"},
                       [(300_000, 0, 24), (2_500_000, 1, 0), (10_000_000, 0, 32)])


def test_reservation_overflow_reruns(s3, oracle_lib):
    """Reservation slots forced too small (level 0 forced onto the reservation path for
    sets whose shard fills are tiny, list-level slots at 1x the mean fill): the device
    flags the overflow, the build reruns on the counted path, outputs stay bit-exact."""
    _parity_subprocess({"S3IMPH_RES0": "2", "S3IMPH_RES_FILL": "1"},
                       [(3000, 0, 40), (300_000, 0, 24), (2_500_000, 1, 0)])


def test_piecewise_hash_every_level0_path(s3, oracle_lib):
    """the host build's blob crossing PCIe in many pieces (S3IMPH_PIECE_BITS=20: 1 MiB
    and up, at most 16 pieces), the level-0 hash of each piece launched as it lands (HashFeed),
    on every level-0 path below P0: the pair hash with caller positions (3M keys), the pair hash
    with identity positions (2M), the skewed hash (1.5M); plus P0's fused hash (18M).
    Bit-exact vs the oracle."""
    _parity_subprocess({"S3IMPH_PIECE_BITS": "20"},
                       [(3_000_000, 0, 24, True), (2_000_000, 0, 32), (1_500_000, 1, 0), (18_000_000, 0, 20)])


def test_p0f_fed_level1_bit_exact(s3, oracle_lib):
    """P0F (developer knob S3IMPH_P0F=1): level 1 of a 90M-key P0 build (4.4k 2^14
    tiles, past the reservation scatter's 4096) fed by level 0's tile kernel — a count pass
    over the slots' in-tile positions sizes level 1 first, level 0's tiles write level 1's
    records straight into its super-tile regions, level 1 runs the super-tile scatter and the
    register tiles; a skewed 90M set the same way: bit-exact vs the oracle."""
    _parity_subprocess({"S3IMPH_P0F": "1"}, [(90_000_000, 0, 24), (90_000_000, 1, 0)])
