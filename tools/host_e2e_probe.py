"""Time s3imph_build_host phases (S3IMPH_DEBUG prints entry / h2d / build / d2h / marshal)
and the Python wrapper around it on C2."""
import ctypes
import os
import sys
import time

os.environ.setdefault("S3IMPH_DEBUG", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "s3-inv-db_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import s3imph  # noqa: E402

blob, offs = s3imph.gen_keys(0, 42, 32, 0, 10_000_000)
n = len(offs) - 1
for i in range(4):
    t = time.perf_counter()
    fp = np.zeros(n, np.uint64)
    po = np.zeros(n, np.uint64)
    t1 = time.perf_counter()
    mp, ml = ctypes.c_void_p(), ctypes.c_uint64()
    err = ctypes.create_string_buffer(256)
    rc = s3imph.LIB.s3imph_build_host(0, s3imph._np_ptr(blob), s3imph._np_ptr(offs), None, n, s3imph._np_ptr(fp),
                                      s3imph._np_ptr(po), ctypes.byref(mp), ctypes.byref(ml), err, 256)
    t2 = time.perf_counter()
    mph = ctypes.string_at(mp.value, ml.value)
    s3imph.LIB.s3imph_free(mp)
    t3 = time.perf_counter()
    print(f"rc {rc} alloc {1e3 * (t1 - t):.2f} call {1e3 * (t2 - t1):.2f} copy-out {1e3 * (t3 - t2):.2f} ms", flush=True)
