"""Build C3 (100M keys, avg 64 B) once on cuda:0 with S3IMPH_DEBUG set; prints the
device level state of each attempt (stderr) and the outcome."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "s3-inv-db_amd"))
os.environ["S3IMPH_DEBUG"] = "1"
import torch  # noqa: E402
import s3imph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
avg = int(sys.argv[2]) if len(sys.argv) > 2 else 64
blob, offs = s3imph.gen_keys(0, 42, avg, 0, n)
d_blob = torch.from_numpy(blob).cuda()
d_offs = torch.from_numpy(offs.view("int64")).cuda()
d_fp = torch.zeros(n, dtype=torch.int64, device="cuda")
d_po = torch.zeros(n, dtype=torch.int64, device="cuda")
ctx = s3imph.DeviceBuilder(0)
try:
    print(ctx.build(d_blob, d_offs, n, d_fp, d_po), flush=True)
except s3imph.MPHFError as e:
    print("ERROR", e, flush=True)
