"""Reader-side queries over the finalize arrays, restated from the reference so the tests
can check the arrays the way its own tests do:
  GetPositionsInSubtree  pkg/format/depthindex.go:191-259 (two binary searches)
  DescendantsAtDepth     pkg/indexread/index.go:206-228
  DescendantsUpToDepth   pkg/indexread/index.go:239-270"""
import bisect


def positions_at_depth(arr, d):
    if d > arr["max_depth"]:
        return []
    o = arr["depth_offsets"]
    return [int(x) for x in arr["depth_positions"][int(o[d]):int(o[d + 1])]]


def positions_in_subtree(arr, d, start, end):
    ps = positions_at_depth(arr, d)
    lo = bisect.bisect_left(ps, start)
    hi = bisect.bisect_right(ps, end, lo)
    return ps[lo:hi]


def descendants_at_depth(arr, pos, rel):
    target = int(arr["depth"][pos]) + rel
    if rel < 0 or target > arr["max_depth"]:
        return None
    return positions_in_subtree(arr, target, pos, int(arr["subtree_end"][pos]))


def descendants_up_to_depth(arr, pos, max_rel):
    base = int(arr["depth"][pos])
    msd = int(arr["max_depth_in_subtree"][pos])
    if max_rel < 0 or min(msd - base, max_rel) <= 0:
        return None
    out = []
    d = base + 1
    while d <= base + max_rel and d <= msd:
        out.append(positions_in_subtree(arr, d, pos, int(arr["subtree_end"][pos])))
        d += 1
    return out


def check_case(case, arr, keys):
    """Asserts every expectation a tests/golden/finalize/cases.json entry carries against arr."""
    idx = {k: i for i, k in enumerate(keys)}
    for d, want in case.get("positions_at_depth", {}).items():
        assert positions_at_depth(arr, int(d)) == want, (case["name"], d)
    if "max_depth" in case:
        assert arr["max_depth"] == case["max_depth"]
    for p, (lo, hi) in case.get("subtree_ranges", {}).items():
        assert (int(p), int(arr["subtree_end"][int(p)])) == (lo, hi), (case["name"], p)
    for d, lo, hi, want in case.get("positions_in_subtree", []):
        assert positions_in_subtree(arr, d, lo, hi) == want, (case["name"], d, lo, hi)
    for key, rel, names, count in case.get("descendants_at_depth", []):
        got = descendants_at_depth(arr, idx[key], rel)
        assert len(got) == count, (case["name"], key, rel)
        if names is not None:
            assert [keys[p] for p in got] == names, (case["name"], key, rel)
    for key, max_rel, sizes in case.get("descendants_up_to_depth", []):
        got = descendants_up_to_depth(arr, idx[key], max_rel)
        assert [len(g) for g in got] == sizes, (case["name"], key, max_rel)
