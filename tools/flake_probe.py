"""Repeat device builds of one key set and compare every run with the oracle: a
nondeterministic (schedule-dependent) mismatch shows up as a run that differs.
  python tools/flake_probe.py [runs] [n]
Prints, per mismatching run, which output differs and where."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path[:0] = [os.path.join(ROOT, "s3-inv-db_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
import s3imph  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    for kind, seed, avg in [(0, 3, 32), (1, 3, 0)]:
        blob, offs = s3imph.gen_keys(kind, seed, avg, 0, n)
        st, fp, po, mph = O.lib().build(blob[: offs[-1]], offs)
        assert st == 0
        ctx = s3imph.DeviceBuilder(0)
        d_blob = torch.from_numpy(blob).cuda()
        d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
        d_fp = torch.zeros(n, dtype=torch.int64, device="cuda")
        d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
        bad = 0
        for r in range(runs):
            d_fp.zero_()
            d_po.zero_()
            info = ctx.build(d_blob, d_offs, n, d_fp, d_po)
            g_fp = d_fp.cpu().numpy().view(np.uint64)
            g_po = d_po.cpu().numpy().view(np.uint64)
            g_mph = ctx.mph_bin()
            ok_m, ok_f, ok_p = g_mph == mph, np.array_equal(g_fp, fp), np.array_equal(g_po, po)
            if not (ok_m and ok_f and ok_p):
                bad += 1
                mf = np.nonzero(g_fp != fp)[0]
                mp = np.nonzero(g_po != po)[0]
                print(f"kind {kind} run {r}: mph {'ok' if ok_m else 'DIFF'} ({len(g_mph)} vs {len(mph)} B), "
                      f"fp diffs {len(mf)} first {mf[:8].tolist()}, pos diffs {len(mp)} first {mp[:8].tolist()}, "
                      f"levels {info.get('num_levels')}", flush=True)
                if not ok_m:
                    a = np.frombuffer(g_mph, np.uint8)
                    b = np.frombuffer(mph, np.uint8)
                    m = min(len(a), len(b))
                    d = np.nonzero(a[:m] != b[:m])[0]
                    print(f"   mph byte diffs {len(d)} first {d[:8].tolist()}", flush=True)
        print(f"kind {kind}: {bad} of {runs} runs differ", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
