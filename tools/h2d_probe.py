"""H2D of a C2-sized host buffer (360 MB) three ways: pageable hipMemcpy (the runtime's own
staging), hipHostRegister + hipMemcpy + hipHostUnregister per call, and an already pinned
buffer.   python tools/h2d_probe.py [MB]"""
import ctypes
import sys
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
MB = int(sys.argv[1]) if len(sys.argv) > 1 else 360
nb = MB << 20
host = np.ones(nb, np.uint8)
dev = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nb)) == 0
H2D = 1


def copy(src_ptr):
    assert hip.hipMemcpy(dev, ctypes.c_void_p(src_ptr), ctypes.c_size_t(nb), H2D) == 0
    assert hip.hipDeviceSynchronize() == 0


def timed(label, fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{label}: " + " ".join(f"{x:.2f}" for x in ts) + f" ms  (best {nb / min(ts) / 1e6:.1f} GB/s)", flush=True)


p = host.ctypes.data
timed("pageable hipMemcpy", lambda: copy(p))


def reg_copy():
    assert hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(nb), 0) == 0
    copy(p)
    assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0


timed("register + copy + unregister", reg_copy)


def reg_only():
    assert hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(nb), 0) == 0
    assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0


timed("register + unregister only", reg_only)
pin = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(pin), ctypes.c_size_t(nb), 0) == 0
ctypes.memmove(pin, p, nb)
timed("pinned hipMemcpy", lambda: copy(pin.value))
