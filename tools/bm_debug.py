"""Bitmap decomposition at N = 1 (RCCL, one rank) over a few sizes / switches, with the
library's debug report (S3IMPH_DEBUG): which stage flags what.
  python tools/bm_debug.py"""
import os
import sys
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, os, numpy as np, torch
sys.path[:0] = [%r, %r]
import s3imph, oracle as O
n, switch = int(sys.argv[1]), int(sys.argv[2])
blob, offs = s3imph.gen_keys(0, 42, 32, 0, n)
d = s3imph.DistBuilder(0, s3imph.dist_unique_id(), 0, 1)
d.set_mode(s3imph.DIST_BITMAP)
cap = d.out_cap(n)
fp = torch.zeros(cap, dtype=torch.int64, device="cuda"); po = torch.zeros(cap, dtype=torch.int64, device="cuda")
db = torch.from_numpy(blob).cuda(); do = torch.from_numpy(offs.view(np.int64)).cuda()
try:
    out_n, segs, info = d.build_shard(db, do, n, 0, fp, po, cap)
    st, ofp, opo, mph = O.lib().build_mt(blob[:offs[-1]], offs, threads=16)
    gf, gp = s3imph.assemble_dist([(fp.cpu().numpy().view(np.uint64), po.cpu().numpy().view(np.uint64), segs)], n)
    print("OK", n, switch, d.mph_bin() == mph, np.array_equal(gf, ofp), np.array_equal(gp, opo), info["big_levels"])
except s3imph.MPHFError as e:
    print("FAIL", n, switch, e)
''' % (os.path.join(ROOT, "s3-inv-db_amd"), os.path.join(ROOT, "oracle"))
for n, sw in [(1_500_000, 20000), (1_500_000, 2 << 20), (10_000_000, 20000), (10_000_000, 2 << 20), (4_000_000, 2 << 20)]:
    env = dict(os.environ, S3IMPH_DIST_SWITCH=str(sw), S3IMPH_DEBUG="1", S3IMPH_DIST_STRICT="1")
    r = subprocess.run([sys.executable, "-c", code, str(n), str(sw)], env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout.strip())
    print("\n".join(l for l in r.stderr.splitlines() if "bitmap" in l or " n:" in l or "attempt" in l)[-3000:])
    sys.stdout.flush()
