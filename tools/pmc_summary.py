"""Per-dispatch HBM traffic of the last build from rocprofv3 FETCH_SIZE / WRITE_SIZE runs.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming read, so the
corrected read bytes are 2 x FETCH_SIZE for streaming kernels; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Calibrated per access shape (`tools/ubench_fetch.hip`,
`profiles/r4_fetch_cal/`): 64-byte runs read in scrambled order count in full (x 1), so
k_hash_skew's per-key 64-B chunk reads take READ_FACTOR 1.
"""
import csv
import json
import sys


READ_FACTOR = {"k_hash_skew": 1.0}  # default 2.0 (streaming)


def kname(full: str) -> str:
    """'void ns::(anonymous namespace)::k_tile_reg<512, 20, 2, false>(int, ...)' -> 'k_tile_reg'."""
    s = full.replace("(anonymous namespace)::", "")
    s = s.split("(")[0].split("<")[0].split("::")[-1]
    return s.split(" ")[-1]


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
        name = kname(f["Kernel_Name"])
        dur = (int(f["End_Timestamp"]) - int(f["Start_Timestamp"])) / 1e3
        fk, wk = float(f["Counter_Value"]), float(w["Counter_Value"])
        out.append({"kernel": name, "grid": int(f["Grid_Size"]), "fetch_kib": fk, "write_kib": wk,
                    "read_bytes_corrected": READ_FACTOR.get(name, 2.0) * fk * 1024, "write_bytes": wk * 1024,
                    "read_factor": READ_FACTOR.get(name, 2.0), "dur_us_profiled": dur})
    for o in out:
        if o["fetch_kib"] + o["write_kib"] > 1024:
            print(f"{o['kernel']:16s} grid={o['grid']:>8d} read({o['read_factor']:.0f}xFETCH)={o['read_bytes_corrected']/1e6:8.1f} MB "
                  f"write={o['write_bytes']/1e6:8.1f} MB")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)
    if len(sys.argv) > 5:  # merge the level-0 stages into bench.py's traffic file: CONFIG PATH
        cfg, path = sys.argv[4], sys.argv[5]
        try:
            tr = json.load(open(path))
        except (OSError, ValueError):
            tr = {}
        first = {}
        for o in out:
            first.setdefault(o["kernel"], o)
        ent = tr.setdefault(cfg, {})
        scatter0 = "k_scatter_res" if "k_scatter_res" in first and "k_hscan" not in first else "k_scatter"
        tile0 = next((o["kernel"] for o in out if o["kernel"] in ("k_tile_reg", "k_tile_p0", "k_tile_split", "k_tile")), "k_tile_reg")
        # the level-0 hash that did the work (the others are no-op launches for this set's skew)
        hash0 = max((k for k in ("k_hash0_pair", "k_hash_skew", "k_hash_count0") if k in first),
                    key=lambda k: first[k]["read_bytes_corrected"] + first[k]["write_bytes"], default="k_hash0_pair")
        stages = (("hash_count0", hash0), ("scatter0", scatter0), ("tile0", tile0))
        if "k_scatter_p0" in first:  # P0 level 0: the fused hash partition, super-tile scatter, tiles
            stages = (("hash_part0", hash0), ("scatter0_p0", "k_scatter_p0"), ("tile0_p0", "k_tile_p0"))
        for stage, kern in stages:
            if kern in first:
                o = first[kern]
                ent[stage] = {"kernel": kern, "n_gpus": 1,
                              "hbm_bytes_per_launch": int(o["read_bytes_corrected"] + o["write_bytes"]),
                              "read_bytes": int(o["read_bytes_corrected"]), "write_bytes": int(o["write_bytes"])}
        # the whole build: every dispatch of the last build summed (bench.py's pipeline_traffic)
        per = {}
        for o in out:
            e = per.setdefault(o["kernel"], [0, 0])
            e[0] += int(o["read_bytes_corrected"])
            e[1] += int(o["write_bytes"])
        rd = sum(v[0] for v in per.values())
        wr = sum(v[1] for v in per.values())
        ent["_pipeline"] = {"n_gpus": 1, "hbm_bytes_per_build": rd + wr, "read_bytes": rd, "write_bytes": wr,
                            "dispatches": len(out),
                            "by_kernel": {k: {"read_bytes": v[0], "write_bytes": v[1]} for k, v in sorted(per.items())}}
        json.dump(tr, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
