"""Phase split of the one-shot host-memory build (s3imph_build_host_into) on C2 (or [n] [avg]):
the library's phase line times every phase from entry to return (--phases: the line alone,
S3IMPH_HOST_PHASES, a developer knob; --debug: S3IMPH_DEBUG, with the kernels' profiling as well, which
slows the build); this prints the Python wall of the same calls beside it, so the table sums to the wall.
    python tools/host_phase.py [n] [avg] [--phases | --debug]"""
import os
import sys
import time

if "--debug" in sys.argv:
    sys.argv.remove("--debug")
    os.environ["S3IMPH_DEBUG"] = "1"
if "--phases" in sys.argv:
    sys.argv.remove("--phases")
    os.environ["S3IMPH_DEV"] = "1"
    os.environ["S3IMPH_HOST_PHASES"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "s3-inv-db_amd"))
import s3imph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
avg = int(sys.argv[2]) if len(sys.argv) > 2 else 32
blob, offs = s3imph.gen_keys(0, 42, avg, 0, n)
blob = blob[: int(offs[-1])].copy()
import numpy as np  # noqa: E402
out = (np.zeros(n, np.uint64), np.zeros(n, np.uint64))  # reused, as bench.py's host_e2e
mph_buf = np.zeros(s3imph.mph_bin_bound(n), np.uint8)
for i in range(6):
    t = time.perf_counter()
    s3imph.build_host_into(blob, offs, out, mph_buf)
    print(f"build_host_into {i}: {(time.perf_counter() - t) * 1e3:.2f} ms (python wall)", file=sys.stderr, flush=True)
t = time.perf_counter()
s3imph.build_host(blob, offs, out=out)
print(f"build_host (malloc'd mph.bin + bytes copy): {(time.perf_counter() - t) * 1e3:.2f} ms", file=sys.stderr,
      flush=True)
