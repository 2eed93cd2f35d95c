"""Counters of one kernel from rocprofv3 --pmc CSVs: python tools/pmc_kernel.py CSV... -k NAME [-i DISPATCH_INDEX]
Prints each counter of the chosen dispatch (default: the last dispatch of a kernel whose
name contains NAME) and derived rates (VALU busy, effective clock)."""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv", nargs="+")
ap.add_argument("-k", "--kernel", required=True)
ap.add_argument("-i", "--index", type=int, default=-1)
a = ap.parse_args()
vals = {}
for path in a.csv:
    per = defaultdict(dict)
    dur = {}
    for r in csv.DictReader(open(path)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if not per:
        continue
    ds = sorted(per)
    d = ds[a.index]
    vals.update(per[d])
    vals["dur_us"] = dur[d]
for k in sorted(vals):
    print(f"{k:24s} {vals[k]:.6g}")
if "SQ_WAVE_CYCLES" in vals and "SQ_ACTIVE_INST_VALU" in vals:
    # SQ_* cycle counters are quad-cycles summed over waves (MI355X_MICROARCH.md)
    print("valu/wave_cycles          %.3f" % (vals["SQ_ACTIVE_INST_VALU"] / vals["SQ_WAVE_CYCLES"]))
    print("wait_any/wave_cycles      %.3f" % (vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]))
    print("wait_inst/wave_cycles     %.3f" % (vals["SQ_WAIT_INST_ANY"] / vals["SQ_WAVE_CYCLES"]))
if "GRBM_GUI_ACTIVE" in vals:
    print("clock_GHz (GUI/8/dur)     %.3f" % (vals["GRBM_GUI_ACTIVE"] / 8 / (vals["dur_us"] * 1e3)))
if "SQ_BUSY_CYCLES" in vals and "SQ_ACTIVE_INST_VALU" in vals:
    print("valu_inst_per_busy_simd   %.3f" % (vals["SQ_ACTIVE_INST_VALU"] * 4 / (vals["SQ_BUSY_CYCLES"] * 4 * 32)))
