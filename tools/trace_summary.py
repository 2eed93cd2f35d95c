"""Print the kernel timeline of the last build in a rocprofv3 kernel-trace CSV."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
thresh = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if "k_init_state" in x["Kernel_Name"]]
seg = r[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
for x in seg:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    nm = x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
    if (e - s) / 1e3 > thresh:
        print(f"{nm:16s} start={(s - t0) / 1e3:8.1f} dur={(e - s) / 1e3:7.1f} "
              f"grid={int(x['Grid_Size_X']) // int(x['Workgroup_Size_X']):>6d} lds={x['LDS_Block_Size']}")
print("total", (int(seg[-1]["End_Timestamp"]) - t0) / 1e3, "us, kernels", len(seg))
