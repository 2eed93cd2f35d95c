"""Finalize arrays alone on a bench config (default C3), for rocprofv3 kernel timing.
  python tools/fin_probe.py [config] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import s3imph  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = cfg["keys_per_gpu"]
blob, offs = s3imph.gen_keys(cfg["kind"], 42, cfg["avg"], 0, n)
d_blob = torch.from_numpy(blob).to("cuda")
d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda")
ctx = s3imph.DeviceBuilder(0)
for _ in range(reps):
    r = ctx.finalize_index(d_blob, d_offs, n)
torch.cuda.synchronize()
print("ok", n, r["max_depth"])
