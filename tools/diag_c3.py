"""Diagnostic: 100M-key build vs the oracle (which output differs, where)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "s3-inv-db_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import s3imph, oracle as O
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
avg = int(sys.argv[2]) if len(sys.argv) > 2 else 64
blob, offs = s3imph.gen_keys(0, 42, avg, 0, n)
ctx = s3imph.DeviceBuilder(0)
d_blob = torch.from_numpy(blob).cuda(); d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
d_fp = torch.zeros(n, dtype=torch.int64, device="cuda"); d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
info = ctx.build(d_blob, d_offs, n, d_fp, d_po); print("info", info, flush=True)
res = torch.zeros(n, dtype=torch.int64, device="cuda")
ctx.lookup(d_blob, d_offs, n, d_fp, d_po, n, res)
bad = (res != torch.arange(n, device="cuda")).nonzero().flatten()
print("lookup mismatches", bad.numel(), bad[:10].tolist(), res[bad[:10]].tolist(), flush=True)
mph = ctx.mph_bin(); gfp = d_fp.cpu().numpy().view(np.uint64); gpo = d_po.cpu().numpy().view(np.uint64)
t = time.time(); st, fp, po, omph = O.lib().build(blob[: int(offs[-1])], offs); print("oracle", st, time.time() - t, flush=True)
print("mph equal", mph == omph, len(mph), len(omph))
if mph != omph:
    a = np.frombuffer(mph, np.uint64); b = np.frombuffer(omph, np.uint64); m = min(len(a), len(b))
    d = np.nonzero(a[:m] != b[:m])[0]; print("mph first diffs (u64 idx)", d[:10], a[d[:5]], b[d[:5]])
    print("levels", a[1], b[1])
dfp = np.nonzero(gfp != fp)[0]; dpo = np.nonzero(gpo != po)[0]
print("fp diffs", len(dfp), dfp[:10]); print("pos diffs", len(dpo), dpo[:10], gpo[dpo[:5]], po[dpo[:5]])
