"""One line per bench.py JSON line of an A/B run (tools/gpu.sh ab / lib): ms per step and stages.

    python tools/ab_summary.py OUT PREFIX V1 V2 ...
reads OUT/PREFIX_v1.log, OUT/PREFIX_v2.log, ... for `ab` (V* are the env settings, listed
as labels), or OUT/PREFIX_V1.log ... for `lib` (V* = old, new); prints every line and the
median ms per variant.
"""
import json
import os
import statistics
import sys

out, prefix, labels = sys.argv[1], sys.argv[2], sys.argv[3:]
for i, lab in enumerate(labels, 1):
    path = os.path.join(out, f"{prefix}_v{i}.log" if prefix == "ab" else f"{prefix}_{lab}.log")
    ms = []
    if not os.path.exists(path):
        print(f"[{lab}] missing {path}")
        continue
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
            ms.append(d["ms_per_step"])
            print(f"[{lab}] {d['ms_per_step']:.4f} {d.get('stages_ms')}")
    if ms:
        print(f"[{lab}] median {statistics.median(ms):.4f} ms over {len(ms)}")
