"""Level-0 hash kernel alone (S3IMPH_HASH_ONLY=1: the build returns after the hash), C3's
byte volume from the C3 generator; run under rocprofv3 --kernel-trace for kernel times.
  python tools/hash_only.py [config] [reps]"""
import os
import sys

os.environ["S3IMPH_HASH_ONLY"] = "1"
os.environ["S3IMPH_DEV"] = "1"  # the library reads developer knobs only after the opt-in
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import s3imph  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = cfg["keys_per_gpu"]
blob, offs = s3imph.gen_keys(cfg["kind"], 42, cfg["avg"], 0, n)
d_blob = torch.from_numpy(blob).to("cuda")
d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda")
fp = torch.empty(n, dtype=torch.int64, device="cuda")
po = torch.empty(n, dtype=torch.int64, device="cuda")
ctx = s3imph.DeviceBuilder(0)
for _ in range(reps):
    try:
        ctx.build(d_blob, d_offs, n, fp, po)
    except s3imph.MPHFError:
        pass
torch.cuda.synchronize()
print("ok", n)
