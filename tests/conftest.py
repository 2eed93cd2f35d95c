"""Shared pytest setup: import paths, the `gpu` marker, and small helpers.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, C-ABI
load/export checks, gloo world_size-2 tests of the sharded-level decomposition.
`-m gpu` runs on an MI355X: parity of the HIP path against the oracle.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "s3-inv-db_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The tests drive the library's developer knobs (S3IMPH_* A/B geometry, fallbacks, fault
# hooks), which it reads only after the opt-in (include/s3imph.h section 7): set it before
# s3imph is imported here or in any subprocess a test starts.
os.environ["S3IMPH_DEV"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle as O
    O.build_oracle()
    return O.lib()


def to_dev(a: np.ndarray, pad8: bool = False):
    """numpy -> torch cuda tensor (u64 viewed as i64; u8 padded to 8 bytes when asked)."""
    import torch
    if a.dtype == np.uint8:
        if pad8:
            n = len(a)
            b = np.zeros(((n + 7) // 8) * 8 + 8, np.uint8)
            b[:n] = a
            a = b
        return torch.from_numpy(a.copy()).to("cuda")
    return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64).copy()).to("cuda")


def from_dev(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)
