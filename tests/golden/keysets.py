"""Key sets for the parity fixtures, restating the reference's own test/bench inputs.

Each generator cites the reference file:line whose input it reproduces (Go
`fmt.Sprintf` semantics restated in Python; no RNG-based Go generators are used,
since Go's math/rand streams cannot be reproduced offline — SURVEY.md §8d).
"""
from __future__ import annotations


def mphf_test_sets() -> dict[str, list[str]]:
    """pkg/format/mphf_test.go key sets (Lookup round-trip tests)."""
    return {
        "mphf_simple": ["", "a/", "a/b/", "b/", "c/"],                 # :35
        "mphf_verify_lookup": ["", "x/", "y/", "z/"],                  # :83
        "mphf_verify": ["", "foo/", "bar/", "baz/"],                   # :118
        "mphf_no_false_pos": ["alpha/", "beta/", "gamma/"],            # :186
        "mphf_unicode": ["", "日本語/", "한국어/", "emoji/🎉/"],          # :223
        "mphf_large_1000": [prefix_from_int(i) for i in range(1000)],  # :143-146
    }


# mphf_test.go:202-209 — strings that must NOT be found in the "mphf_no_false_pos" set.
NON_MEMBERS = ["delta/", "epsilon/", "alpha", "/alpha", "ALPHA/", ""]


def prefix_from_int(i: int) -> str:
    """pkg/format/mphf_test.go:267-279 (prefixFromInt)."""
    result = ""
    while i > 0:
        result = chr(ord("a") + i % 26) + "/" + result
        i //= 26
    return result or "root/"


def extsort_index_rows() -> list[str]:
    """pkg/extsort/extsort_test.go:266-273 (TestIndexBuilder sorted rows)."""
    return ["", "data/", "data/2024/", "data/2024/01/", "data/2024/02/", "logs/"]


def memory_test_prefixes(n: int = 10000) -> list[str]:
    """pkg/extsort/memory_test.go:79-84: fmt.Sprintf("data/%05d/", i)."""
    return ["data/%05d/" % i for i in range(n)]


def wide_single_level_prefixes(num_objects: int = 100000) -> list[str]:
    """benchutil.GenerateKeys(n, "wide_single_level") (pkg/benchutil/generator.go:326-332)
    fed through Aggregator.AddObject prefix extraction (pkg/extsort/aggregator.go:44-61:
    the root "" plus every '/'-terminated prefix), de-duplicated and byte-sorted
    (SortPrefixRows, pkg/extsort/types.go:160-164).  100000 objects -> 100002 prefixes."""
    seen = {""}
    for i in range(num_objects):
        key = "root/child%07d/file.txt" % i
        for j, ch in enumerate(key):
            if ch == "/":
                seen.add(key[: j + 1])
    return sorted(seen, key=lambda s: s.encode())


def realistic_prefixes(n: int) -> list[str]:
    """pkg/format/mphf_bench_test.go:11-27 (generateRealisticPrefixes); distinct for n <= 1e6."""
    out = []
    for i in range(n):
        depth = 1 + (i % 5)
        out.append("".join("seg%d/" % ((i * 7 + d * 13) % 1000000) for d in range(depth)))
    return out
