"""OpenMPHF / Lookup / VerifyMPHF on the GPU over index files on disk (pkg/format/mphf.go
:186-302, :372-393): the device loads a marshalled mph.bin — the ORACLE's, written with
the oracle's own framing, as well as the product builder's — and answers Lookup for
members (their pos) and non-members (not found), as the reference's mphf_test.go checks."""
import numpy as np
import pytest

import keysets
import oracle as O

pytestmark = pytest.mark.gpu
NOT_FOUND = np.uint64(2**64 - 1)


@pytest.fixture(scope="module")
def s3():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import s3imph
    return s3imph


def _write_oracle_index(oracle_lib, d, keys, pos=None):
    blob, offs = O.keys_to_blob(keys)
    st, fp, po, mph = oracle_lib.build(blob, offs, pos)
    assert st == 0
    (d / "mph.bin").write_bytes(mph)
    (d / "mph_fp.u64").write_bytes(O.s3id_u64_array(fp))
    (d / "mph_pos.u64").write_bytes(O.s3id_u64_array(po))
    (d / "prefix_blob.bin").write_bytes(blob.tobytes())
    (d / "prefix_offsets.u64").write_bytes(O.s3id_u64_array(offs))


@pytest.mark.parametrize("name", ["mphf_simple", "mphf_large_1000", "mphf_unicode", "mphf_no_false_pos"])
def test_oracle_index_looks_up_on_gpu(s3, oracle_lib, tmp_path, name):
    keys = [k.encode() for k in keysets.mphf_test_sets()[name]]
    _write_oracle_index(oracle_lib, tmp_path, keys)
    m = s3.MPHF(str(tmp_path))
    m.verify()
    assert (m.lookup(keys) == np.arange(len(keys), dtype=np.uint64)).all()
    others = [k.encode() for k in keysets.NON_MEMBERS if k.encode() not in keys]
    assert (m.lookup(others) == NOT_FOUND).all()
    m.close()


def test_oracle_index_1m_custom_positions(s3, oracle_lib, tmp_path):
    blob, offs = s3.gen_keys(0, 12, 40, 0, 1_000_000)
    keys = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(1_000_000)]
    pos = np.random.default_rng(3).permutation(len(keys)).astype(np.uint64)
    _write_oracle_index(oracle_lib, tmp_path, keys, pos)
    m = s3.MPHF(str(tmp_path))
    assert np.array_equal(m.lookup_blob(blob[: int(offs[-1])], offs), pos)
    qb, qo = s3.gen_keys(0, 13, 40, 2_000_000, 50_000)  # other keys: not members
    assert (m.lookup_blob(qb, qo) == NOT_FOUND).all()
    m.close()


def test_builder_index_verifies(s3, tmp_path):
    keys = [("t/%06d/" % i).encode() for i in range(30_000)]
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    for i, k in enumerate(keys):
        b.add(k, i)
    b.build(str(tmp_path))
    b.close()
    m = s3.MPHF(str(tmp_path))
    m.verify()
    m.close()


def test_empty_and_malformed(s3, tmp_path):
    b = s3.StreamingMPHFBuilder(str(tmp_path))
    b.build(str(tmp_path))  # writeEmpty: 0-byte mph.bin
    b.close()
    m = s3.MPHF(str(tmp_path))
    assert m.count == 0 and (m.lookup([b"a/", b""]) == NOT_FOUND).all()
    m.close()
    ctx = s3.DeviceBuilder(0)
    good = O.lib().build(*O.keys_to_blob([b"a/", b"b/", b"c/"]))[3]
    import struct
    zero_word_level = struct.pack("<QQQQQ", 1, 2, 1, 0b111, 0)  # level 1 claims 0 words
    zero_first = struct.pack("<QQQQQ", 1, 2, 0, 1, 0b111)       # level 0 claims 0 words
    for bad in (good[:-1], good + b"\0", b"\2" + good[1:], good[:8], zero_word_level, zero_first):
        with pytest.raises(s3.MPHFError) as e:
            ctx.load_mph_bin(bad)
        assert e.value.status == s3.ERR_FORMAT
    ctx.load_mph_bin(good)
    ctx.close()
