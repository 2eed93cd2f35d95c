"""Per-rank kernel time of the last build in a rocprofv3 kernel trace of tools/p8_geometry.py.

Each rank is a host thread (a new one per build) launching on its own stream; with
S3IMPH_HOST_SERIAL the ranks' kernels never overlap, so a kernel's traced duration is its time
alone on the GPU.  The last build starts at the earliest of the last P k_init_state launches (one per rank and
build; rank 0 runs on the calling thread, the same thread in every build).
The host transport's copies (the runtime's copyBuffer / fillBuffer blits: host <-> device
staging standing in for xGMI) are reported apart, not as device time.
    python tools/rank_kernel_sums.py run_kernel_trace.csv [P] [top]
"""
import collections
import csv
import sys

path = sys.argv[1]
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
by_thread = collections.defaultdict(list)
for x in rows:
    by_thread[x["Thread_Id"]].append(x)


def name(x):
    return x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]


def is_copy(x):
    return "rocclr" in x["Kernel_Name"]


inits = [x for x in rows if "k_init_state" in x["Kernel_Name"]]
t1 = min(int(x["Start_Timestamp"]) for x in inits[-P:])
last = sorted({x["Thread_Id"] for x in inits[-P:]})
ranks = []
for tid in last:
    seg = [x for x in by_thread[tid] if int(x["Start_Timestamp"]) >= t1]
    dev = [x for x in seg if not is_copy(x)]
    cp = [x for x in seg if is_copy(x)]
    tot = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in dev) / 1e6
    ctot = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in cp) / 1e6
    per = collections.Counter()
    for x in dev:
        per[name(x)] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    ranks.append((tot, tid, len(dev), span, per, ctot))
ranks.sort(reverse=True)
for tot, tid, k, span, per, ctot in ranks:
    print(f"thread {tid}: {k} kernels, device time {tot:.3f} ms; host-transport copies {ctot:.1f} ms "
          f"(first-to-last span {span:.1f} ms)")
if ranks:
    tot, tid, k, span, per, ctot = ranks[0]
    print(f"max over ranks: {tot:.3f} ms; mean {sum(r[0] for r in ranks) / len(ranks):.3f} ms over {len(ranks)} ranks")
    print(f"slowest rank ({tid}) by kernel:")
    for nm, ms in per.most_common(top):
        print(f"  {nm:24s} {ms:8.3f} ms")
