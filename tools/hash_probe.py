"""Level-0 hash probe: the same byte volume as C3 (100M keys, 64 B average) with fixed
64-byte keys and with uniform 32-96-byte keys, random bytes generated on the device.
Separates the lane-divergence cost (uneven lengths) from the memory-access cost.
  python tools/hash_probe.py [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "s3-inv-db_amd"))
import s3imph  # noqa: E402


def run(ctx, blob, offs, n, label, steps=5):
    fp = torch.empty(n, dtype=torch.int64, device="cuda")
    po = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.build(blob, offs, n, fp, po)
    ctx.set_profiling(True)
    acc = {}
    for _ in range(steps):
        ctx.build(blob, offs, n, fp, po)
        for k, v in ctx.stage_times().items():
            acc[k] = acc.get(k, 0.0) + v / steps
    ctx.set_profiling(False)
    print(label, {k: round(v, 3) for k, v in acc.items()}, flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    ctx = s3imph.DeviceBuilder(0)
    blob = torch.randint(0, 256, (n * 96 + 64,), dtype=torch.uint8, device="cuda", generator=g)
    offs = torch.arange(0, n + 1, dtype=torch.int64, device="cuda") * 64
    run(ctx, blob, offs, n, "fixed64  ")
    for lo, hi in [(56, 72), (48, 80), (32, 96)]:
        lens = torch.randint(lo, hi + 1, (n,), dtype=torch.int64, device="cuda", generator=g)
        offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
        torch.cumsum(lens, 0, out=offs[1:])
        del lens
        assert int(offs[-1]) <= blob.numel() - 8
        run(ctx, blob, offs, n, "unif%d-%d" % (lo, hi))
    ctx.close()


if __name__ == "__main__":
    main()
