"""Per-launch kernel durations of one rank's last build in a p8_geometry trace (the launch order of
one rank, for comparing levels), plus each kernel's time on every rank.
    python tools/rank_kernel_table.py run_kernel_trace.csv [P] [kernel-substring]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
pick = sys.argv[3] if len(sys.argv) > 3 else None
inits = [x for x in rows if "k_init_state" in x["Kernel_Name"]]
t1 = min(int(x["Start_Timestamp"]) for x in inits[-P:])
tids = sorted({x["Thread_Id"] for x in inits[-P:]})


def name(x):
    return x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]


def dur(x):
    return (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3


per = collections.defaultdict(list)
for tid in tids:
    for x in rows:
        if x["Thread_Id"] == tid and int(x["Start_Timestamp"]) >= t1 and "rocclr" not in x["Kernel_Name"]:
            per[tid].append((name(x), dur(x)))
if pick:
    for tid in tids:
        print(tid, " ".join(f"{d:7.1f}" for n, d in per[tid] if pick in n))
else:
    tid = tids[0]
    for n, d in per[tid]:
        print(f"{d:9.1f} us  {n}")
