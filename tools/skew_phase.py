"""One C5 build with S3IMPH_DEBUG=1: k_hash_skew's per-wave phase clock (total / hashing /
waiting for chunk loads / rest) from the library's debug report.
  python tools/skew_phase.py [n]"""
import os
import sys

os.environ["S3IMPH_DEBUG"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"))
import s3imph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
blob, offs = s3imph.gen_keys(1, 42, 0, 0, n)
d_blob = torch.from_numpy(blob).to("cuda")
d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda")
fp = torch.empty(n, dtype=torch.int64, device="cuda")
po = torch.empty(n, dtype=torch.int64, device="cuda")
ctx = s3imph.DeviceBuilder(0)
for _ in range(2):
    ctx.build(d_blob, d_offs, n, fp, po)
torch.cuda.synchronize()
print("ok", n)
