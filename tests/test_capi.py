"""The C-ABI library loads, exports exactly what include/s3imph.h declares, and its
host-only entry points (file framing, builder bookkeeping, generator) behave like the
reference's writers — all without a GPU (no compute calls here)."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

import oracle as O
import s3imph
from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "s3imph.h")).read()
    return set(re.findall(r"^(?:int|void|uint64_t|const char)\s*\*?\s*(s3imph_[a-z0-9_]+)\(", src, re.M))


def test_header_and_binding_agree():
    assert _declared() == set(s3imph.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(s3imph.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name


def test_abi_version_and_status_strings():
    assert s3imph.LIB.s3imph_abi_version() == 1
    for code in range(12):
        assert s3imph.status_string(code)


def test_write_index_files_matches_reference_framing(tmp_path, oracle_lib):
    """Framing of the 5 files == format.go/writer.go restated in the oracle (S3ID header,
    LE u64 payload, N+1 offsets with the sentinel)."""
    keys = [b"", b"a/", b"a/b/", b"b/", b"c/"]
    blob, offs = O.keys_to_blob(keys)
    st, fp, pos, mph = oracle_lib.build(blob, offs)
    s3imph.write_index_files(str(tmp_path), mph, fp, pos, blob, offs)
    want = {"mph.bin": mph, "mph_fp.u64": O.s3id_u64_array(fp), "mph_pos.u64": O.s3id_u64_array(pos),
            "prefix_blob.bin": blob.tobytes(), "prefix_offsets.u64": O.s3id_u64_array(offs)}
    for name, data in want.items():
        assert (tmp_path / name).read_bytes() == data, name


def test_write_files_split_over_writer_threads(tmp_path):
    """Files of 32 MiB and more are written by several threads, each pwrite()-ing its
    own range: large arrays (6M values, 48 MB) and a large blob (70 MB, not a multiple of
    the split) still come out byte-identical to the reference framing."""
    rng = np.random.default_rng(3)
    n = 6_000_000
    fp = rng.integers(0, 2**63, n, dtype=np.uint64)
    pos = rng.permutation(n).astype(np.uint64)
    blob = rng.integers(0, 256, 70_000_003, dtype=np.uint8)
    offs = np.linspace(0, len(blob), n + 1).astype(np.uint64)
    offs[-1] = len(blob)
    s3imph.write_index_files(str(tmp_path), b"xyz", fp, pos, blob, offs)
    assert (tmp_path / "mph_fp.u64").read_bytes() == O.s3id_u64_array(fp)
    assert (tmp_path / "mph_pos.u64").read_bytes() == O.s3id_u64_array(pos)
    assert (tmp_path / "prefix_blob.bin").read_bytes() == blob.tobytes()
    assert (tmp_path / "prefix_offsets.u64").read_bytes() == O.s3id_u64_array(offs)


def test_write_empty_matches_writeEmpty(tmp_path):
    """mphf_streaming.go:506-541: 0-byte mph.bin, count-0 arrays, offsets = [0] (count 1), empty blob."""
    s3imph.write_index_files(str(tmp_path), b"", np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                             np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert (tmp_path / "mph.bin").read_bytes() == b""
    assert (tmp_path / "mph_fp.u64").read_bytes() == O.s3id_header(0)
    assert (tmp_path / "mph_pos.u64").read_bytes() == O.s3id_header(0)
    assert (tmp_path / "prefix_blob.bin").read_bytes() == b""
    assert (tmp_path / "prefix_offsets.u64").read_bytes() == O.s3id_header(1) + b"\0" * 8


def test_write_files_rebases_offsets(tmp_path):
    blob = np.frombuffer(b"XXXXab/cd/", np.uint8).copy()
    offs = np.array([4, 7, 10], np.uint64)
    s3imph.write_index_files(str(tmp_path), b"\1", np.array([1, 2], np.uint64), np.array([0, 1], np.uint64),
                             blob, offs)
    assert (tmp_path / "prefix_blob.bin").read_bytes() == b"ab/cd/"
    assert (tmp_path / "prefix_offsets.u64").read_bytes() == O.s3id_u64_array([0, 3, 6])


def test_write_files_missing_dir_is_io_error(tmp_path):
    with pytest.raises(s3imph.MPHFError) as e:
        s3imph.write_index_files(str(tmp_path / "nope"), b"", np.zeros(0, np.uint64), np.zeros(0, np.uint64),
                                 np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert e.value.status == s3imph.ERR_IO


def test_builder_bookkeeping_without_gpu(tmp_path):
    b = s3imph.StreamingMPHFBuilder(str(tmp_path))
    assert b.count() == 0
    b.add("a/", 0)
    b.add(b"b/", 1)
    blob, offs = O.keys_to_blob([b"c/", b"d/"])
    b.add_batch(blob, offs)
    assert b.count() == 4
    b.close()


def test_builder_bad_temp_dir(tmp_path):
    with pytest.raises(s3imph.MPHFError) as e:
        s3imph.StreamingMPHFBuilder(str(tmp_path / "missing"))
    assert e.value.status == s3imph.ERR_IO


def test_builder_empty_build_needs_no_gpu(tmp_path):
    """Count()==0 -> writeEmpty; no device work at all."""
    b = s3imph.StreamingMPHFBuilder(str(tmp_path))
    b.build(str(tmp_path))
    assert (tmp_path / "mph.bin").read_bytes() == b""
    assert (tmp_path / "prefix_offsets.u64").read_bytes() == O.s3id_header(1) + b"\0" * 8
    with pytest.raises(s3imph.MPHFError) as e:
        b.add("x/", 0)
    assert e.value.status == s3imph.ERR_STATE


def test_generator_sorted_distinct_and_shardable():
    blob, offs = s3imph.gen_keys(0, 42, 32, 0, 50000)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(50000)]
    assert keys[0] == b""
    assert keys == sorted(keys) and len(set(keys)) == len(keys)
    lens = np.diff(offs.astype(np.int64))[1:]
    assert lens.min() >= 16 and lens.max() <= 48 and abs(lens.mean() - 32) < 0.5
    b2, o2 = s3imph.gen_keys(0, 42, 32, 12345, 100)
    for i in range(100):
        assert bytes(b2[o2[i]:o2[i + 1]]) == keys[12345 + i]
    # C5's kind 1: lengths log-uniform on [1, 1024] (raised to the 5-byte head a distinct
    # sorted key needs), byte-sorted, distinct, reproducible by shard
    b3, o3 = s3imph.gen_keys(1, 42, 0, 0, 20000)
    l3 = np.diff(o3.astype(np.int64))[1:]
    assert l3.min() == 5 and l3.max() == 1024 and 130 < l3.mean() < 170
    assert (l3 == 5).mean() > 0.2  # the log-uniform mass below 5 bytes lands on the head width
    k3 = [bytes(b3[o3[i]:o3[i + 1]]) for i in range(20000)]
    assert k3 == sorted(k3) and len(set(k3)) == 20000
    b4, o4 = s3imph.gen_keys(1, 42, 0, 777, 50)
    assert [bytes(b4[o4[i]:o4[i + 1]]) for i in range(50)] == k3[777:827]
    # around the switch from 5- to 7-byte heads (j = 63 * 64^4) and at 200M (C5's size)
    for lo in (63 * 64 ** 4 - 40, 200_000_000 - 100):
        b5, o5 = s3imph.gen_keys(1, 42, 0, lo, 80)
        k5 = [bytes(b5[o5[i]:o5[i + 1]]) for i in range(80)]
        assert k5 == sorted(k5) and len(set(k5)) == 80
    assert hashlib.sha256(blob[: offs[-1]].tobytes()).hexdigest() == \
        hashlib.sha256(s3imph.gen_keys(0, 42, 32, 0, 50000)[0][: offs[-1]].tobytes()).hexdigest()


def test_shard_plan_covers_everything():
    for n in [0, 1, 7, 100, 10**6 + 3]:
        for p in [1, 2, 3, 8]:
            plans = [s3imph.ShardPlan(r, p, n) for r in range(p)]
            assert sum(x.n_local for x in plans) == n
            assert all(plans[r].hi == plans[r + 1].lo for r in range(p - 1))


def test_builder_add_batch_empty_null_pointers(tmp_path):
    """An empty batch may pass NULL blob/offsets (a cgo caller's nil slices): a no-op."""
    b = s3imph.StreamingMPHFBuilder(str(tmp_path))
    err = ctypes.create_string_buffer(64)
    assert s3imph.LIB.s3imph_builder_add_batch(b._h, None, None, None, 0, err, 64) == s3imph.OK
    assert b.count() == 0
    assert s3imph.LIB.s3imph_builder_add_batch(b._h, None, None, None, 3, err, 64) == s3imph.ERR_INVALID
    b.close()


def test_read_u64_array_checks_the_s3id_header(tmp_path):
    """OpenArray (reader.go:81-119) restated in the binding: header checked, payload LE u64."""
    p = tmp_path / "a.u64"
    p.write_bytes(O.s3id_u64_array([5, 6, 2**64 - 1]))
    assert list(s3imph.read_u64_array(str(p))) == [5, 6, 2**64 - 1]
    for bad in (O.s3id_header(3, 4) + b"\0" * 12, O.s3id_header(4) + b"\0" * 24, b"\0" * 28):
        p.write_bytes(bad)
        with pytest.raises(s3imph.MPHFError) as e:
            s3imph.read_u64_array(str(p))
        assert e.value.status == s3imph.ERR_FORMAT
