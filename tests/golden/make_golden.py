"""Generate the committed parity fixtures in tests/golden/*.json.

Run from the repo root:  python tests/golden/make_golden.py

The expected outputs come from the CPU oracle (oracle/bbhash_oracle.c, cross-checked
against the independent pure-Python restatement in oracle/oracle.py on every set
small enough for it).  relab/bbhash itself is not available offline, so mph.bin
bytes are "vs restated spec"; the FNV values are pinned to published vectors
(tests/golden/fnv_kat.json) and the framing to the reference's writer code.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import keysets  # noqa: E402
import oracle as O  # noqa: E402

FULL_DUMP_MAX = 1000  # sets up to this size store mph.bin / fp / pos in full


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def files_for(keys: list[bytes], pos=None) -> dict[str, bytes]:
    """The 5 files StreamingMPHFBuilder.Build writes, framed by the oracle-side encoder."""
    lib = O.lib()
    blob, offs = O.keys_to_blob(keys)
    st, fp, pout, mph = lib.build(blob, offs, None if pos is None else np.asarray(pos, np.uint64))
    assert st == 0, st
    return {
        "mph.bin": mph,
        "mph_fp.u64": O.s3id_u64_array(fp),
        "mph_pos.u64": O.s3id_u64_array(pout),
        "prefix_blob.bin": blob.tobytes(),
        "prefix_offsets.u64": O.s3id_u64_array(offs),
    }, fp, pout


def fixture(name: str, keys_str: list[str], cross_check_py: bool) -> dict:
    keys = [k.encode() for k in keys_str]
    files, fp, pout = files_for(keys)
    if cross_check_py:
        pfp, ppos, pmph = O.py_build(keys)
        assert pmph == files["mph.bin"], name
        assert list(map(int, fp)) == pfp and list(map(int, pout)) == ppos, name
    st, m = O.lib().unmarshal(files["mph.bin"]) if keys else (0, None)
    fx = {
        "name": name,
        "n": len(keys),
        "sum_len": sum(len(k) for k in keys),
        "keys_sha256": sha(b"".join(len(k).to_bytes(4, "little") + k for k in keys)),
        "num_levels": m.num_levels if m else 0,
        "files_sha256": {k: sha(v) for k, v in files.items()},
        "files_len": {k: len(v) for k, v in files.items()},
        "cross_checked_with_python": cross_check_py,
    }
    if len(keys) <= FULL_DUMP_MAX:
        fx["keys"] = keys_str
        fx["mph_bin_hex"] = files["mph.bin"].hex()
        fx["fp_out"] = [int(x) for x in fp]
        fx["pos_out"] = [int(x) for x in pout]
    return fx


def main() -> None:
    O.build_oracle()
    out = {}
    for name, ks in keysets.mphf_test_sets().items():
        out[name] = fixture(name, ks, True)
    out["extsort_index_rows"] = fixture("extsort_index_rows", keysets.extsort_index_rows(), True)
    out["memory_test_10000"] = fixture("memory_test_10000", keysets.memory_test_prefixes(), True)
    out["wide_single_level_100k"] = fixture("wide_single_level_100k", keysets.wide_single_level_prefixes(), False)
    out["realistic_100k"] = fixture("realistic_100k", keysets.realistic_prefixes(100000), False)
    out["empty"] = fixture("empty", [], True)
    for name, fx in out.items():
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(fx, f, indent=1, ensure_ascii=False)
            f.write("\n")
        print(f"{name:28s} n={fx['n']:7d} levels={fx['num_levels']:2d} mph.bin={fx['files_len']['mph.bin']}")


if __name__ == "__main__":
    main()
