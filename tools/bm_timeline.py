"""Per-kernel timeline of the last complete build in a rocprofv3 kernel trace (debug aid).
python tools/bm_timeline.py gpurun_out/TAG/prof_c3"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_hash0" in r["Kernel_Name"] or "k_count0" in r["Kernel_Name"]]
seg = rows[idx[-2]:idx[-1]]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("s3imph::(anonymous namespace)::", "").replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if d >= float(sys.argv[2] if len(sys.argv) > 2 else 0):
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}  {n[:60]}")
