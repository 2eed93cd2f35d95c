"""Per-phase timestamps of the tile / reservation-scatter kernels of one C2 build
(S3IMPH_DEBUG=1 makes the library record them and print the summary to stderr)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "s3-inv-db_amd")]
os.environ["S3IMPH_DEBUG"] = "1"
import numpy as np, torch
import s3imph
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
avg = int(sys.argv[2]) if len(sys.argv) > 2 else 32
blob, offs = s3imph.gen_keys(0, 42, avg, 0, n)
ctx = s3imph.DeviceBuilder(0)
d_blob = torch.from_numpy(blob).cuda(); d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
d_fp = torch.zeros(n, dtype=torch.int64, device="cuda"); d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
for _ in range(3):
    info = ctx.build(d_blob, d_offs, n, d_fp, d_po)
print("info", info, flush=True)
