"""The finalize oracle (oracle/finalize_oracle.c, IndexBuilder's stack algorithm and
DepthIndexBuilder.Build restated) pinned to the reference's own finalize-path tests
(tests/golden/finalize/cases.json, transcribed by make_cases.py there), and checked
against the separately written pure-Python restatement on random prefix sets."""
import json
import os

import numpy as np
import pytest

import finalize_queries as Q
import oracle as O

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "finalize", "cases.json")))


def _as_lists(arr):
    return {k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in arr.items()}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_finalize_tests(case, oracle_lib):
    keys = case["keys"]
    blob, offs = O.keys_to_blob([k.encode() for k in keys])
    depths = np.array(case["depths"], np.uint32) if "depths" in case else None
    arr = oracle_lib.finalize(blob, offs, depths)
    if depths is not None:  # the '/' count agrees with the rows' Depth on these sets
        assert arr["depth"].tolist() == oracle_lib.finalize(blob, offs)["depth"].tolist()
    Q.check_case(case, arr, keys)


def _random_prefix_set(rng, n_objects, fanout, max_depth, closed=True):
    objs = []
    for _ in range(n_objects):
        d = int(rng.integers(1, max_depth + 1))
        objs.append("/".join("s%d" % rng.integers(0, fanout) for _ in range(d)) + "/f.txt")
    if closed:
        s = {""}
        for o in objs:
            for i, c in enumerate(o):
                if c == "/":
                    s.add(o[: i + 1])
    else:  # not ancestor-closed: only the objects' own directories
        s = {o[: o.rindex("/") + 1] for o in objs}
    return sorted((k.encode() for k in s))


@pytest.mark.parametrize("closed", [True, False])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_matches_python_restatement(oracle_lib, seed, closed):
    rng = np.random.default_rng(seed)
    keys = _random_prefix_set(rng, 300, 3 + seed, 6, closed)
    blob, offs = O.keys_to_blob(keys)
    got = _as_lists(oracle_lib.finalize(blob, offs))
    want = O.py_finalize(keys)
    for k in ("depth", "subtree_end", "max_depth_in_subtree", "depth_offsets", "depth_positions", "max_depth"):
        assert got[k] == want[k], k


def test_oracle_empty_and_single(oracle_lib):
    blob, offs = O.keys_to_blob([])
    arr = oracle_lib.finalize(blob, offs)
    assert arr["depth_offsets"].tolist() == [0, 0] and arr["max_depth"] == 0
    blob, offs = O.keys_to_blob([b"x/y/"])
    arr = _as_lists(oracle_lib.finalize(blob, offs))
    assert arr["depth"] == [2] and arr["subtree_end"] == [0] and arr["depth_offsets"] == [0, 0, 0, 1]
