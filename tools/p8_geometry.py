"""The 8-GPU bitmap geometry on ONE GPU: P ranks x K keys per rank (default
8 x 100M C3 keys: 800M globally, avg 64 B) built by s3imph_build_host_multi with the bitmap
decomposition, every rank a host thread on device 0, collectives through the in-process host
transport.  S3IMPH_HOST_SERIAL=1 (set here) runs the ranks' device work one rank at a time, so
under `rocprofv3 --kernel-trace` each kernel runs alone on the GPU and tools/rank_kernel_sums.py
sums one rank's kernel time — the device time that rank would spend on its own GPU (xGMI
transfers excluded: they are host copies here).  Prints the wall time of each build (not a
scaling number: the ranks share one GPU and serialise).
    python tools/p8_geometry.py [P] [keys_per_rank] [avg] [builds]
avg 0 selects the skewed generator (C5: lengths log-uniform on 1-1024 B).
"""
import os
import sys
import time

os.environ["S3IMPH_DEV"] = "1"          # the library reads developer knobs only after the opt-in
os.environ["S3IMPH_HOST_SERIAL"] = "1"
os.environ.setdefault("S3IMPH_DIST_STRICT", "1")  # no silent fallback to the routed build
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "s3-inv-db_amd"))
import numpy as np  # noqa: E402
import s3imph  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
AVG = int(sys.argv[3]) if len(sys.argv) > 3 else 64
B = int(sys.argv[4]) if len(sys.argv) > 4 else 2
n = P * K
t = time.perf_counter()
blob, offs = s3imph.gen_keys(1 if AVG == 0 else 0, 42, AVG, 0, n)
print(f"[p8] {P} ranks x {K} keys, avg {AVG} B: {n} keys, {int(offs[-1]) / 1e9:.1f} GB of key bytes "
      f"(generated in {time.perf_counter() - t:.1f} s)", file=sys.stderr, flush=True)
out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))
for b in range(B):
    t = time.perf_counter()
    fp, po, mph = s3imph.build_host(blob, offs, devices=[0] * P, flags=s3imph.MULTI_BITMAP, out=out)
    print(f"[p8] build {b}: {(time.perf_counter() - t) * 1e3:.1f} ms wall (serialised ranks, host transport), "
          f"mph.bin {len(mph)} B", file=sys.stderr, flush=True)
# a cheap property: every output slot written once (positions are a permutation of [0, n))
seen = np.zeros(n, np.uint8)
seen[po] = 1
print(f"[p8] mph_pos covers {int(seen.sum())} of {n} slots; mph.bin sha256 "
      f"{__import__('hashlib').sha256(mph).hexdigest()[:16]}", file=sys.stderr, flush=True)
assert int(seen.sum()) == n
