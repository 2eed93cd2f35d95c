"""Writes tests/golden/finalize/cases.json: the reference's own finalize-path test inputs
and the results its tests assert, transcribed (no values computed by this repo).

Sources (/root/reference):
  pkg/format/depthindex_test.go:31-97    TestDepthIndexBuilderSimple  (positions per depth)
  pkg/format/depthindex_test.go:99-170   TestDepthIndexSubtreeQuery   (subtree ranges in the
                                         comments, GetPositionsInSubtree results)
  pkg/extsort/extsort_test.go:255-333    TestIndexBuilder             (rows with Depth; data/2024/
                                         has 2 descendants at relative depth 1)
  pkg/indexread/index_test.go:87-164     TestDescendantsAtDepth       (object keys -> prefixes)
  pkg/indexread/index_test.go:166-211    TestDescendantsUpToDepth
Object keys become prefixes as Aggregator.AddObject does (aggregator.go:44-60): "" plus
every '/'-terminated prefix, depth = its '/' count."""
import json
import os


def prefixes_of(objects):
    s = {""}
    for key in objects:
        for i, c in enumerate(key):
            if c == "/":
                s.add(key[: i + 1])
    return sorted(s, key=lambda x: x.encode())


cases = [
    {"name": "depthindex_simple", "keys": ["", "a/", "a/x/", "a/y/", "b/", "b/z/"],
     "depths": [0, 1, 2, 2, 1, 2],
     "positions_at_depth": {"0": [0], "1": [1, 4], "2": [2, 3, 5], "3": []}, "max_depth": 2,
     "subtree_ranges": {"0": [0, 5], "1": [1, 3], "2": [2, 2], "3": [3, 3], "4": [4, 5], "5": [5, 5]},
     "positions_in_subtree": [[2, 1, 3, [2, 3]], [2, 4, 5, [5]], [1, 0, 5, [1, 4]]]},
    {"name": "extsort_index_builder",
     "keys": ["", "data/", "data/2024/", "data/2024/01/", "data/2024/02/", "logs/"],
     "depths": [0, 1, 2, 3, 3, 1],
     "descendants_at_depth": [["data/2024/", 1, None, 2]]},
    {"name": "index_descendants_at_depth",
     "keys": prefixes_of(["a/x/file.txt", "a/y/file.txt", "a/z/file.txt", "b/m/file.txt"]),
     "descendants_at_depth": [["", 1, ["a/", "b/"], 2], ["", 2, None, 4],
                              ["a/", 1, ["a/x/", "a/y/", "a/z/"], 3]]},
    {"name": "index_descendants_up_to_depth",
     "keys": prefixes_of(["a/b/c/file.txt", "a/b/d/file.txt", "a/e/file.txt"]),
     "descendants_up_to_depth": [["", 3, [1, 2, 2]]]},
]
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cases.json")
with open(out, "w") as f:
    json.dump(cases, f, indent=1)
print(out)
