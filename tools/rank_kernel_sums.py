"""Per-rank kernel time of the last build in a rocprofv3 kernel trace of tools/p8_geometry.py.

Each rank is a host thread launching on its own stream; with S3IMPH_HOST_SERIAL the ranks'
kernels never overlap, so a kernel's traced duration is its time alone on the GPU.  A rank's
builds start at its k_init_state launches: the last one opens the last build.
    python tools/rank_kernel_sums.py run_kernel_trace.csv [top]
"""
import collections
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
by_thread = collections.defaultdict(list)
for x in rows:
    by_thread[x["Thread_Id"]].append(x)


def name(x):
    return x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]


ranks = []
for tid, rs in by_thread.items():
    starts = [i for i, x in enumerate(rs) if "k_init_state" in x["Kernel_Name"]]
    if not starts:
        continue
    seg = rs[starts[-1]:]
    tot = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in seg) / 1e6
    per = collections.Counter()
    for x in seg:
        per[name(x)] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    ranks.append((tot, tid, len(seg), span, per))
ranks.sort(reverse=True)
for tot, tid, k, span, per in ranks:
    print(f"thread {tid}: {k} kernels, device time {tot:.3f} ms (first-to-last span {span:.1f} ms)")
if ranks:
    tot, tid, k, span, per = ranks[0]
    print(f"max over ranks: {tot:.3f} ms; mean {sum(r[0] for r in ranks) / len(ranks):.3f} ms over {len(ranks)} ranks")
    print(f"slowest rank ({tid}) by kernel:")
    for nm, ms in per.most_common(top):
        print(f"  {nm:24s} {ms:8.3f} ms")
