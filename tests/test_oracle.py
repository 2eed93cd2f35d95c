"""The CPU oracle, pinned before it is trusted (runs without a GPU).

- FNV-1a / FNV-1 against published vectors (pkg/format/mphf.go:341-369 use Go hash/fnv).
- C restatement == independent pure-Python restatement (relab/bbhash).
- Committed golden fixtures (tests/golden/*.json) reproduce byte for byte.
- The reference's own MPHF tests (pkg/format/mphf_test.go) hold as round trips:
  every member looks up to its pos, listed non-members are rejected, the empty
  set looks up nothing.  mph.bin bytes are "vs restated spec" (parity unpinned
  against upstream relab/bbhash, which is not available offline).
"""
import glob
import json
import os
import random

import numpy as np
import pytest

import keysets
import oracle as O
from conftest import GOLDEN


def _kat():
    with open(os.path.join(GOLDEN, "fnv_kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("key", list(_kat()["fnv1a64"]))
def test_fnv1a_kat(oracle_lib, key):
    want = int(_kat()["fnv1a64"][key], 16)
    b = key.encode()
    assert O.py_fnv1a64(b) == want
    assert oracle_lib.fnv1a64(b) == want


@pytest.mark.parametrize("key", list(_kat()["fnv1_64"]))
def test_fnv1_kat(oracle_lib, key):
    want = int(_kat()["fnv1_64"][key], 16)
    b = key.encode()
    assert O.py_fnv1_64(b) == want
    assert oracle_lib.fnv1_64(b) == want


def test_fingerprint_determinism(oracle_lib):
    """mphf_test.go:251-264 (TestComputeFingerprint)."""
    assert oracle_lib.fnv1_64(b"test") == oracle_lib.fnv1_64(b"test")
    assert oracle_lib.fnv1_64(b"test") != oracle_lib.fnv1_64(b"other")


def _fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.json")))


def _fixture_keys(fx):
    if "keys" in fx:
        return fx["keys"]
    name = fx["name"]
    if name == "memory_test_10000":
        return keysets.memory_test_prefixes()
    if name == "wide_single_level_100k":
        return keysets.wide_single_level_prefixes()
    if name == "realistic_100k":
        return keysets.realistic_prefixes(100000)
    raise KeyError(name)


def _load(path):
    with open(path) as f:
        return json.load(f)


@pytest.mark.parametrize("path", [p for p in _fixtures() if not p.endswith("fnv_kat.json")],
                         ids=lambda p: os.path.basename(p))
def test_oracle_reproduces_golden(oracle_lib, path):
    import hashlib
    fx = _load(path)
    keys = [k.encode() for k in _fixture_keys(fx)]
    assert len(keys) == fx["n"]
    assert hashlib.sha256(b"".join(len(k).to_bytes(4, "little") + k for k in keys)).hexdigest() == fx["keys_sha256"]
    blob, offs = O.keys_to_blob(keys)
    st, fp, pos, mph = oracle_lib.build(blob, offs)
    assert st == O.ORC_OK
    files = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(pos),
             "prefix_blob.bin": blob.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(offs)}
    for name, data in files.items():
        assert hashlib.sha256(data).hexdigest() == fx["files_sha256"][name], name
    if "mph_bin_hex" in fx:
        assert mph.hex() == fx["mph_bin_hex"]
        assert [int(x) for x in fp] == fx["fp_out"]
        assert [int(x) for x in pos] == fx["pos_out"]


@pytest.mark.parametrize("name", list(keysets.mphf_test_sets()))
def test_reference_roundtrip_sets(oracle_lib, name):
    """mphf_test.go:31-180,219-249: every member looks up to its own position."""
    keys = [k.encode() for k in keysets.mphf_test_sets()[name]]
    blob, offs = O.keys_to_blob(keys)
    st, fp, pos, mph = oracle_lib.build(blob, offs)
    assert st == O.ORC_OK
    st, m = oracle_lib.unmarshal(mph)
    assert st == O.ORC_OK
    for i, k in enumerate(keys):
        assert oracle_lib.lookup(m, fp, pos, k) == i


def test_reference_no_false_positives(oracle_lib):
    """mphf_test.go:182-217 (TestMPHFNoFalsePositives)."""
    keys = [k.encode() for k in keysets.mphf_test_sets()["mphf_no_false_pos"]]
    blob, offs = O.keys_to_blob(keys)
    st, fp, pos, mph = oracle_lib.build(blob, offs)
    _, m = oracle_lib.unmarshal(mph)
    for k in keysets.NON_MEMBERS:
        assert oracle_lib.lookup(m, fp, pos, k.encode()) is None


def test_empty_build(oracle_lib):
    """mphf_test.go:7-29 and writeEmpty (mphf_streaming.go:506-541): 0-byte mph.bin."""
    st, fp, pos, mph = oracle_lib.build(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert st == O.ORC_OK and mph == b"" and len(fp) == 0
    assert O.s3id_u64_array(np.zeros(0, np.uint64)) == O.s3id_header(0)
    assert O.s3id_u64_array(np.zeros(1, np.uint64)) == O.s3id_header(1) + b"\0" * 8


def test_duplicates_fail(oracle_lib):
    """Duplicate key hashes can never be placed: bbhash.New errors (mphf_streaming.go:141-144)."""
    st, _ = oracle_lib.bbhash_new(np.array([5, 7, 7, 9], np.uint64))
    assert st == O.ORC_ERR_TOO_MANY_LEVELS


def test_c_vs_python_random_keysets(oracle_lib):
    rng = random.Random(1234)
    for trial in range(5):
        n = rng.choice([1, 2, 3, 31, 32, 33, 64, 65, 500, 2500])
        keys = list({bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) for _ in range(n)})
        blob, offs = O.keys_to_blob(keys)
        st, fp, pos, mph = oracle_lib.build(blob, offs)
        pfp, ppos, pmph = O.py_build(keys)
        assert st == 0 and mph == pmph
        assert list(map(int, fp)) == pfp and list(map(int, pos)) == ppos


@pytest.mark.parametrize("threads", [1, 3, 8, 16])
def test_build_mt_and_revmap_equal_build(oracle_lib, threads):
    """The big-config checkers: orc_build_mt (FNV and placement on several threads, used by
    every >= 10M-key GPU parity test) and orc_build_revmap (the reference-shaped reverse-map
    build, bench.py's CPU baseline) give orc_build's exact outputs, with identity and custom
    positions, around word / thread-split boundaries."""
    rng = random.Random(99 + threads)
    for n in [1, 2, 63, 64, 65, 1000, 4097, 120_000]:
        keys = [b"t/%d/%08x/" % (i, rng.getrandbits(32)) for i in range(n)]
        blob, offs = O.keys_to_blob(keys)
        pos = np.array([rng.getrandbits(63) for _ in range(n)], np.uint64)
        for pv in (None, pos):
            st, fp, po, mph = oracle_lib.build(blob, offs, pv)
            assert st == 0
            st2, fp2, po2, mph2 = oracle_lib.build_mt(blob, offs, pv, threads=threads)
            assert st2 == 0 and mph2 == mph and np.array_equal(fp2, fp) and np.array_equal(po2, po), (n, threads)
            st3, fp3, po3 = oracle_lib.build_revmap(blob, offs, pv)
            assert st3 == 0 and np.array_equal(fp3, fp) and np.array_equal(po3, po), n


def test_build_mt_and_revmap_equal_python_restatement(oracle_lib):
    """The same checkers against the independent pure-Python restatement (small sets)."""
    rng = random.Random(4321)
    for n in [1, 5, 33, 200, 1500]:
        keys = list({bytes(rng.randrange(256) for _ in range(rng.randrange(0, 24))) for _ in range(n)})
        blob, offs = O.keys_to_blob(keys)
        pfp, ppos, pmph = O.py_build(keys)
        st, fp, po, mph = oracle_lib.build_mt(blob, offs, threads=4)
        assert st == 0 and mph == pmph and list(map(int, fp)) == pfp and list(map(int, po)) == ppos
        st, fp, po = oracle_lib.build_revmap(blob, offs)
        assert st == 0 and list(map(int, fp)) == pfp and list(map(int, po)) == ppos


def test_build_mt_and_revmap_report_duplicates(oracle_lib):
    keys = [b"a/%d" % i for i in range(5000)] + [b"a/17"]
    blob, offs = O.keys_to_blob(keys)
    st = oracle_lib.build(blob, offs)[0]
    assert st != 0
    assert oracle_lib.build_mt(blob, offs, threads=8)[0] == st
    assert oracle_lib.build_revmap(blob, offs)[0] == st


def test_custom_pos_permutes_with_keys(oracle_lib):
    """Add(prefix, pos) accepts arbitrary pos (mphf_streaming.go:68); pos_out[p] = pos_i."""
    keys = [("k%d/" % i).encode() for i in range(300)]
    blob, offs = O.keys_to_blob(keys)
    posv = np.arange(1000, 1300, dtype=np.uint64)[::-1].copy()
    st, fp, pos, mph = oracle_lib.build(blob, offs, posv)
    st2, fp2, pos2, mph2 = oracle_lib.build(blob, offs)
    assert mph == mph2 and (fp == fp2).all()
    assert (pos == posv[pos2.astype(np.int64)]).all()


def test_level_structure_invariants(oracle_lib):
    keys = np.array(sorted({random.Random(7).getrandbits(64) | 1 for _ in range(20000)}), np.uint64)
    st, m = oracle_lib.bbhash_new(keys)
    assert st == 0
    total = 0
    n_active = len(keys)
    for lvl in range(m.num_levels):
        bits = m.level_bits(lvl)
        assert len(bits) == (2 * n_active + 63) // 64
        pc = int(sum(bin(int(w)).count("1") for w in bits))
        total += pc
        n_active -= pc
    assert total == len(keys) and n_active == 0
    finds = sorted(m.find(int(k)) for k in keys)
    assert finds == list(range(1, len(keys) + 1))


def test_barrett_reduction_identity():
    """The device reduction (bbhash_spec.h / s3imph_kernels.hip bb_index) equals h % (64*words)."""
    rng = random.Random(99)
    M64 = (1 << 64) - 1
    for words in [1, 2, 3, 7, 63, 64, 65, 1000, 3125, (1 << 20) + 1, (1 << 31) - 1, (1 << 32) - 1]:
        magic = M64 // words
        for _ in range(300):
            h = rng.getrandbits(64)
            q = h >> 6
            qe = (q * magic) >> 64
            r = q - qe * words
            assert 0 <= r < 2 * words
            if r >= words:
                r -= words
            assert (r << 6) | (h & 63) == h % (64 * words)
