"""Per-dispatch HBM traffic of the last build from rocprofv3 FETCH_SIZE / WRITE_SIZE runs.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming read, so the
corrected read bytes are 2 x FETCH_SIZE for streaming kernels (an upper bound for
others); WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import csv
import json
import sys


def load(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    inits = [i for i, r in enumerate(rows) if "k_init_state" in r["Kernel_Name"]]
    return rows[inits[-1]:]


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = []
    for f, w in zip(fetch, write):
        name = f["Kernel_Name"].split("(")[0].split("::")[-1]
        dur = (int(f["End_Timestamp"]) - int(f["Start_Timestamp"])) / 1e3
        fk, wk = float(f["Counter_Value"]), float(w["Counter_Value"])
        out.append({"kernel": name, "grid": int(f["Grid_Size"]), "fetch_kib": fk, "write_kib": wk,
                    "read_bytes_corrected": 2 * fk * 1024, "write_bytes": wk * 1024, "dur_us_profiled": dur})
    for o in out:
        if o["fetch_kib"] + o["write_kib"] > 1024:
            print(f"{o['kernel']:16s} grid={o['grid']:>8d} read(2xFETCH)={o['read_bytes_corrected']/1e6:8.1f} MB "
                  f"write={o['write_bytes']/1e6:8.1f} MB")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
