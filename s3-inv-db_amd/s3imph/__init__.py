"""s3imph — Python binding of libs3imph.so, the MI355X-native MPHF builder.

Mirrors the reference's MPHF stage interface, ``format.StreamingMPHFBuilder``
(/root/reference/pkg/format/mphf_streaming.go:29-232):

    b = StreamingMPHFBuilder(temp_dir)       # NewStreamingMPHFBuilder (:48)
    b.add(prefix, pos)                       # Add (:68)
    b.count()                                # Count (:100)
    b.build(out_dir)                         # Build (:122) -> mph.bin, mph_fp.u64, mph_pos.u64,
                                             #                  prefix_blob.bin, prefix_offsets.u64
    b.close()                                # Close (:105)

plus the device-resident API that bench.py times (``DeviceBuilder``), the
multi-GPU rank API (``DistBuilder``) and the batched lookup.

Every compute call goes through the HIP library; there is no CPU fallback.
If libs3imph.so is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

try:  # One HIP runtime per process: let torch load its libamdhip64 first.
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libs3imph.so")

OK = 0
ERR_INVALID = 1
ERR_DUP_KEY_HASH = 2
ERR_TOO_MANY_LEVELS = 3
ERR_KEY_HASH_ZERO = 4
ERR_HIP = 5
ERR_RCCL = 6
ERR_IO = 7
ERR_NOMEM = 8
ERR_FORMAT = 9
ERR_INTERNAL = 10
ERR_STATE = 11

MULTI_FORCE_SHARDED = 1   # the sharded (multi-GPU) build even for one GPU
MULTI_HOST_TRANSPORT = 2  # in-process host-copy collectives instead of RCCL
MULTI_BITMAP = 4          # the bitmap decomposition of the sharded levels
DIST_ROUTE = 0            # sharded levels: records routed to their position-range owner
DIST_BITMAP = 1           # sharded levels: count-lane reduction of the collision bitmap
DIST_STRICT = 0x100       # or-ed into DIST_BITMAP: no fallback to routing (the build fails instead)

# Every entry point include/s3imph.h declares (checked by tests/test_capi.py).
EXPORTS = (
    "s3imph_abi_version", "s3imph_status_string",
    "s3imph_builder_new", "s3imph_builder_add", "s3imph_builder_add_batch", "s3imph_builder_count",
    "s3imph_builder_build", "s3imph_builder_close", "s3imph_builder_reserve",
    "s3imph_build_host", "s3imph_build_host_multi", "s3imph_builder_set_gpus", "s3imph_free",
    "s3imph_write_index_files",
    "s3imph_ctx_create", "s3imph_ctx_destroy", "s3imph_ctx_reserve", "s3imph_build_device",
    "s3imph_ctx_mph_bin", "s3imph_ctx_set_profiling", "s3imph_ctx_stage_times",
    "s3imph_dist_unique_id", "s3imph_ctx_create_dist", "s3imph_ctx_create_dist_host", "s3imph_build_device_dist",
    "s3imph_dist_segments", "s3imph_dist_out_cap", "s3imph_ctx_last_error", "s3imph_ctx_set_dist_mode",
    "s3imph_ctx_load_mph_bin", "s3imph_lookup_device", "s3imph_gen_keys",
    "s3imph_finalize_index_host", "s3imph_finalize_index_device",
    "s3imph_write_manifest", "s3imph_verify_manifest", "s3imph_sha256_file",
    "s3imph_dev_knobs", "s3imph_build_host_into", "s3imph_mph_bin_bound", "s3imph_release_workspaces",
)


class MPHFError(RuntimeError):
    """A non-OK s3imph_status; ``.status`` holds the code."""

    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(ctypes.c_uint64))


class HostComm(ctypes.Structure):
    """s3imph_host_comm: host-callback collectives (include/s3imph.h, section 4)."""
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


class BuildInfo(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32),
        ("num_levels", ctypes.c_uint32),
        ("total_words", ctypes.c_uint64),
        ("mph_bin_len", ctypes.c_uint64),
        ("big_levels", ctypes.c_uint64),
        ("n_keys", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libs3imph.so not built at {LIB_PATH}: run `make -C s3-inv-db_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    u64, i32, vp, cp, sz = ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
    P = ctypes.POINTER
    sig = {
        "s3imph_abi_version": (i32, []),
        "s3imph_status_string": (cp, [i32]),
        "s3imph_builder_new": (i32, [cp, i32, P(vp), cp, sz]),
        "s3imph_builder_add": (i32, [vp, cp, u64, u64, cp, sz]),
        "s3imph_builder_add_batch": (i32, [vp, vp, vp, vp, u64, cp, sz]),
        "s3imph_builder_count": (u64, [vp]),
        "s3imph_builder_reserve": (i32, [vp, u64, u64, cp, sz]),
        "s3imph_builder_build": (i32, [vp, cp, cp, sz]),
        "s3imph_builder_close": (i32, [vp]),
        "s3imph_build_host": (i32, [i32, vp, vp, vp, u64, vp, vp, P(vp), P(u64), cp, sz]),
        "s3imph_build_host_multi": (i32, [i32, vp, ctypes.c_uint, vp, vp, vp, u64, vp, vp, P(vp), P(u64), cp, sz]),
        "s3imph_builder_set_gpus": (i32, [vp, i32, vp, ctypes.c_uint]),
        "s3imph_free": (None, [vp]),
        "s3imph_write_index_files": (i32, [cp, vp, u64, vp, vp, u64, vp, vp, cp, sz]),
        "s3imph_ctx_create": (i32, [i32, P(vp), cp, sz]),
        "s3imph_ctx_destroy": (i32, [vp]),
        "s3imph_ctx_reserve": (i32, [vp, u64, u64]),
        "s3imph_build_device": (i32, [vp, vp, vp, vp, u64, vp, vp, vp, P(BuildInfo)]),
        "s3imph_ctx_mph_bin": (i32, [vp, vp, u64, P(u64)]),
        "s3imph_ctx_set_profiling": (i32, [vp, i32]),
        "s3imph_ctx_stage_times": (i32, [vp, P(ctypes.c_float), i32, P(i32), cp, sz]),
        "s3imph_dist_unique_id": (i32, [vp]),
        "s3imph_ctx_create_dist": (i32, [i32, vp, i32, i32, P(vp), cp, sz]),
        "s3imph_ctx_create_dist_host": (i32, [i32, P(HostComm), i32, i32, P(vp), cp, sz]),
        "s3imph_build_device_dist": (i32, [vp, vp, vp, vp, u64, u64, vp, vp, u64, P(u64), vp, P(BuildInfo)]),
        "s3imph_dist_segments": (i32, [vp, P(u64), u64, P(u64)]),
        "s3imph_dist_out_cap": (u64, [vp, u64]),
        "s3imph_ctx_set_dist_mode": (i32, [vp, i32]),
        "s3imph_ctx_last_error": (cp, [vp]),
        "s3imph_ctx_load_mph_bin": (i32, [vp, vp, u64]),
        "s3imph_lookup_device": (i32, [vp, vp, vp, u64, vp, vp, u64, vp, vp]),
        "s3imph_finalize_index_host": (i32, [i32, vp, vp, vp, u64, cp, cp, sz]),
        "s3imph_finalize_index_device": (i32, [vp, vp, vp, vp, u64, vp, vp, vp, vp, vp, u64,
                                               P(ctypes.c_uint32), vp]),
        "s3imph_gen_keys": (i32, [i32, u64, ctypes.c_uint32, u64, u64, vp, vp, P(u64)]),
        "s3imph_write_manifest": (i32, [cp, u64, ctypes.c_uint32, cp, sz]),
        "s3imph_verify_manifest": (i32, [cp, cp, sz]),
        "s3imph_sha256_file": (i32, [cp, i32, cp, cp, sz]),
        "s3imph_dev_knobs": (i32, [i32]),
        "s3imph_build_host_into": (i32, [i32, vp, vp, vp, u64, vp, vp, vp, u64, P(u64), cp, sz]),
        "s3imph_mph_bin_bound": (u64, [u64]),
        "s3imph_release_workspaces": (i32, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


LIB = _load()
# Developer knobs (A/B geometry, test fallbacks, fault hooks: include/s3imph.h section 7) are
# read by the library only after this opt-in; the tests and tools/gpu.sh set S3IMPH_DEV=1.
if os.environ.get("S3IMPH_DEV") == "1":
    LIB.s3imph_dev_knobs(1)


def dev_knobs(on: bool = True) -> None:
    """Let the library read its S3IMPH_* developer knobs (tests, A/B runs); not for builds
    that produce an index."""
    LIB.s3imph_dev_knobs(1 if on else 0)


def status_string(code: int) -> str:
    return LIB.s3imph_status_string(code).decode()


def _check(rc: int, err: ctypes.Array | None = None, what: str = ""):
    if rc != OK:
        msg = err.value.decode(errors="replace") if err is not None and err.value else status_string(rc)
        raise MPHFError(rc, f"{what}{': ' if what else ''}{msg}")


def _np_ptr(a: np.ndarray | None):
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def _dev_ptr(t) -> ctypes.c_void_p | None:
    """Device pointer of a torch tensor, an int address, or None."""
    if t is None:
        return None
    if isinstance(t, int):
        return ctypes.c_void_p(t)
    return ctypes.c_void_p(t.data_ptr())


def keys_to_blob(keys) -> tuple[np.ndarray, np.ndarray]:
    """Keys (bytes/str) -> (blob u8, offsets u64[N+1]): the prefix_blob.bin / prefix_offsets.u64 layout."""
    bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    offs = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(k) for k in bs], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bs), np.uint8).copy() if bs else np.zeros(0, np.uint8)
    return blob, offs


# ------------------------------------------------------------------- builder mirror --
class StreamingMPHFBuilder:
    """format.StreamingMPHFBuilder (mphf_streaming.go:29-232) backed by the GPU build."""

    def __init__(self, temp_dir: str | None = None, device: int = 0):
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        rc = LIB.s3imph_builder_new((temp_dir or "").encode(), device, ctypes.byref(h), err, 512)
        _check(rc, err, "create temp file" if rc == ERR_IO else "")
        self._h = h

    def add(self, prefix, pos: int) -> None:
        b = prefix.encode() if isinstance(prefix, str) else bytes(prefix)
        err = ctypes.create_string_buffer(256)
        _check(LIB.s3imph_builder_add(self._h, b, len(b), pos, err, 256), err)

    def add_batch(self, blob: np.ndarray, offsets: np.ndarray, pos: np.ndarray | None = None) -> None:
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        if pos is not None:
            pos = np.ascontiguousarray(pos, np.uint64)
        err = ctypes.create_string_buffer(256)
        _check(LIB.s3imph_builder_add_batch(self._h, _np_ptr(blob), _np_ptr(offsets), _np_ptr(pos),
                                            len(offsets) - 1, err, 256), err)

    def count(self) -> int:
        return LIB.s3imph_builder_count(self._h)

    def reserve(self, n_keys: int, n_bytes: int) -> None:
        """Capacity hint: the device copy of the keys is allocated once (s3imph_builder_reserve)."""
        err = ctypes.create_string_buffer(256)
        _check(LIB.s3imph_builder_reserve(self._h, n_keys, n_bytes, err, 256), err)

    def set_gpus(self, num_gpus: int, devices=None, flags: int = 0) -> None:
        """Build on `num_gpus` GPUs (s3imph_builder_set_gpus; see build_host)."""
        devs = None if devices is None else (ctypes.c_int * num_gpus)(*devices)
        _check(LIB.s3imph_builder_set_gpus(self._h, num_gpus, devs, flags), None, "set_gpus")

    def build(self, out_dir: str) -> None:
        err = ctypes.create_string_buffer(1024)
        _check(LIB.s3imph_builder_build(self._h, out_dir.encode(), err, 1024), err)

    def close(self) -> None:
        if self._h:
            LIB.s3imph_builder_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def release_workspaces() -> None:
    """Free the device workspaces cached by the host-memory builds (s3imph_release_workspaces)."""
    _check(LIB.s3imph_release_workspaces(), None, "release_workspaces")


def mph_bin_bound(n: int) -> int:
    """An upper bound on mph.bin's size for n keys (the buffer of build_host_into)."""
    return int(LIB.s3imph_mph_bin_bound(n))


def build_host_into(blob: np.ndarray, offsets: np.ndarray, out: tuple[np.ndarray, np.ndarray],
                    mph_buf: np.ndarray, pos: np.ndarray | None = None, device: int = 0) -> int:
    """s3imph_build_host_into: the one-shot host build into caller-owned, reusable outputs —
    fp / pos arrays (u64, N each) and mph_buf (u8, >= mph_bin_bound(N)); returns mph.bin's
    length (mph_buf[:len] holds it)."""
    blob = np.ascontiguousarray(blob, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    if pos is not None:
        pos = np.ascontiguousarray(pos, np.uint64)
    fp_out, pos_out = out
    for a in (fp_out, pos_out):
        if a.dtype != np.uint64 or len(a) < n or not a.flags.c_contiguous:
            raise ValueError("out arrays must be contiguous uint64 with at least N entries")
    if mph_buf.dtype != np.uint8 or not mph_buf.flags.c_contiguous:
        raise ValueError("mph_buf must be a contiguous uint8 array")
    ml = ctypes.c_uint64()
    err = ctypes.create_string_buffer(1024)
    rc = LIB.s3imph_build_host_into(device, _np_ptr(blob), _np_ptr(offsets), _np_ptr(pos), n, _np_ptr(fp_out),
                                    _np_ptr(pos_out), _np_ptr(mph_buf), len(mph_buf), ctypes.byref(ml), err, 1024)
    _check(rc, err)
    return int(ml.value)


def build_host(blob: np.ndarray, offsets: np.ndarray, pos: np.ndarray | None = None, device: int = 0,
               out: tuple[np.ndarray, np.ndarray] | None = None, num_gpus: int = 1, devices=None, flags: int = 0):
    """One-shot build from host memory: (fp_out u64[N], pos_out u64[N], mph_bin bytes).
    `out` may supply the two output arrays (u64, N each) to be filled in place.
    num_gpus > 1 (or `devices`, or `flags`) runs s3imph_build_host_multi: one host thread
    per GPU, RCCL between them (or in-process host copies when devices repeat or flags
    has MULTI_HOST_TRANSPORT)."""
    blob = np.ascontiguousarray(blob, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    if pos is not None:
        pos = np.ascontiguousarray(pos, np.uint64)
    if out is not None:
        fp_out, pos_out = out
        if fp_out.dtype != np.uint64 or pos_out.dtype != np.uint64 or len(fp_out) < n or len(pos_out) < n \
                or not fp_out.flags.c_contiguous or not pos_out.flags.c_contiguous:
            raise ValueError("out arrays must be contiguous uint64 with at least N entries")
    else:
        fp_out = np.zeros(n, np.uint64)
        pos_out = np.zeros(n, np.uint64)
    mp = ctypes.c_void_p()
    ml = ctypes.c_uint64()
    err = ctypes.create_string_buffer(1024)
    if num_gpus == 1 and devices is None and not flags:
        rc = LIB.s3imph_build_host(device, _np_ptr(blob), _np_ptr(offsets), _np_ptr(pos), n, _np_ptr(fp_out),
                                   _np_ptr(pos_out), ctypes.byref(mp), ctypes.byref(ml), err, 1024)
    else:
        if devices is not None:
            num_gpus = len(devices)
        devs = None if devices is None else (ctypes.c_int * num_gpus)(*devices)
        rc = LIB.s3imph_build_host_multi(num_gpus, devs, flags, _np_ptr(blob), _np_ptr(offsets), _np_ptr(pos), n,
                                         _np_ptr(fp_out), _np_ptr(pos_out), ctypes.byref(mp), ctypes.byref(ml), err,
                                         1024)
    _check(rc, err)
    mph = ctypes.string_at(mp.value, ml.value) if ml.value else b""
    if mp.value:
        LIB.s3imph_free(mp)
    return fp_out, pos_out, mph


def write_index_files(out_dir: str, mph_bin: bytes, fp: np.ndarray, pos: np.ndarray, blob: np.ndarray,
                      offsets: np.ndarray) -> None:
    """Emit mph.bin, mph_fp.u64, mph_pos.u64, prefix_blob.bin, prefix_offsets.u64 (reference framing)."""
    fp = np.ascontiguousarray(fp, np.uint64)
    pos = np.ascontiguousarray(pos, np.uint64)
    blob = np.ascontiguousarray(blob, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    err = ctypes.create_string_buffer(1024)
    rc = LIB.s3imph_write_index_files(out_dir.encode(), mph_bin, len(mph_bin), _np_ptr(fp), _np_ptr(pos),
                                      len(fp), _np_ptr(blob), _np_ptr(offsets), err, 1024)
    _check(rc, err)


def gen_keys(kind: int, seed: int, avg_len: int, lo: int, n: int) -> tuple[np.ndarray, np.ndarray]:
    """Deterministic synthetic prefixes [lo, lo+n) (see include/s3imph.h §6). Blob is padded to 8 bytes."""
    total = ctypes.c_uint64()
    _check(LIB.s3imph_gen_keys(kind, seed, avg_len, lo, n, None, None, ctypes.byref(total)))
    blob = np.zeros(((total.value + 7) // 8) * 8 + 8, np.uint8)
    offsets = np.zeros(n + 1, np.uint64)
    _check(LIB.s3imph_gen_keys(kind, seed, avg_len, lo, n, _np_ptr(blob), _np_ptr(offsets), ctypes.byref(total)))
    return blob, offsets


# ----------------------------------------------------------------- device builders --
class DeviceBuilder:
    """A device context: device-resident builds, mph.bin marshalling, batched lookup."""

    def __init__(self, device: int = 0):
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        _check(LIB.s3imph_ctx_create(device, ctypes.byref(h), err, 512), err)
        self._h = h
        self.device = device
        self.last_info: dict | None = None

    def reserve(self, max_keys: int, max_global_keys: int = 0) -> None:
        _check(LIB.s3imph_ctx_reserve(self._h, max_keys, max_global_keys), None, "reserve")

    def set_profiling(self, on) -> None:
        """False/0 off, True/1 every stage, 2 the level-0 hash (or route) stage only."""
        LIB.s3imph_ctx_set_profiling(self._h, int(on))

    def stage_times(self) -> dict:
        ms = (ctypes.c_float * 64)()
        cnt = ctypes.c_int()
        names = ctypes.create_string_buffer(2048)
        LIB.s3imph_ctx_stage_times(self._h, ms, 64, ctypes.byref(cnt), names, 2048)
        keys = names.value.decode().split(",") if cnt.value else []
        return {k: ms[i] for i, k in enumerate(keys)}

    def last_error(self) -> str:
        return LIB.s3imph_ctx_last_error(self._h).decode(errors="replace")

    def build(self, d_blob, d_offsets, n: int, d_fp_out, d_pos_out, d_pos=None, stream=None) -> dict:
        info = BuildInfo()
        rc = LIB.s3imph_build_device(self._h, _dev_ptr(d_blob), _dev_ptr(d_offsets), _dev_ptr(d_pos), n,
                                     _dev_ptr(d_fp_out), _dev_ptr(d_pos_out), _stream_ptr(stream),
                                     ctypes.byref(info))
        if rc != OK:
            raise MPHFError(rc, f"build MPHF: {self.last_error() or status_string(rc)}")
        self.last_info = info.as_dict()
        return self.last_info

    def mph_bin(self) -> bytes:
        ln = ctypes.c_uint64()
        LIB.s3imph_ctx_mph_bin(self._h, None, 0, ctypes.byref(ln))
        buf = ctypes.create_string_buffer(max(ln.value, 1))
        _check(LIB.s3imph_ctx_mph_bin(self._h, buf, ln.value, ctypes.byref(ln)), None, "marshal MPHF")
        return buf.raw[: ln.value]

    def load_mph_bin(self, mph: bytes) -> None:
        """OpenMPHF (mphf.go:186-247): this context's lookups now answer against `mph`."""
        rc = LIB.s3imph_ctx_load_mph_bin(self._h, mph if mph else None, len(mph))
        if rc != OK:
            raise MPHFError(rc, f"open MPHF: {self.last_error() or status_string(rc)}")

    def lookup(self, d_blob, d_offsets, n: int, d_fp, d_pos, count: int, d_result, stream=None) -> None:
        _check(LIB.s3imph_lookup_device(self._h, _dev_ptr(d_blob), _dev_ptr(d_offsets), n, _dev_ptr(d_fp),
                                        _dev_ptr(d_pos), count, _dev_ptr(d_result), _stream_ptr(stream)),
               None, "lookup")

    def finalize_index(self, d_blob, d_offsets, n: int, d_depths=None, stream=None) -> dict:
        """IndexBuilder.Finalize's arrays on the device (indexbuild.go:393-415,474-503,
        depthindex.go:32-96): torch tensors depth (int32), subtree_end (int64),
        max_depth_in_subtree (int32), depth_positions (int64), depth_offsets (int64), max_depth."""
        import torch
        dev = d_offsets.device
        depth = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        send = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        mds = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        dpos = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        md = ctypes.c_uint32()
        cap = 64
        for _ in range(2):
            doff = torch.empty(cap, dtype=torch.int64, device=dev)
            rc = LIB.s3imph_finalize_index_device(self._h, _dev_ptr(d_blob), _dev_ptr(d_offsets), _dev_ptr(d_depths),
                                                  n, _dev_ptr(depth), _dev_ptr(send), _dev_ptr(mds), _dev_ptr(dpos),
                                                  _dev_ptr(doff), cap, ctypes.byref(md), _stream_ptr(stream))
            if rc == OK:
                break
            if rc != ERR_INVALID or cap >= md.value + 2:
                raise MPHFError(rc, f"finalize index: {self.last_error() or status_string(rc)}")
            cap = md.value + 2
        return {"depth": depth[:n], "subtree_end": send[:n], "max_depth_in_subtree": mds[:n],
                "depth_positions": dpos[:n], "depth_offsets": doff[: md.value + 2], "max_depth": md.value}

    def close(self) -> None:
        if getattr(self, "_h", None):
            LIB.s3imph_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def finalize_index_host(blob: np.ndarray, offsets: np.ndarray, out_dir: str, depths: np.ndarray | None = None,
                        device: int = 0) -> None:
    """IndexBuilder.Finalize's depth / subtree / depth-index files (indexbuild.go:393-415,
    474-503; depthindex.go:32-96), computed on the GPU, written into out_dir."""
    blob = np.ascontiguousarray(blob, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    dp = None if depths is None else np.ascontiguousarray(depths, np.uint32)
    err = ctypes.create_string_buffer(1024)
    rc = LIB.s3imph_finalize_index_host(device, _np_ptr(blob), _np_ptr(offsets), _np_ptr(dp) if dp is not None else None,
                                        len(offsets) - 1, out_dir.encode(), err, 1024)
    _check(rc, err)


def write_manifest(out_dir: str, node_count: int, max_depth: int) -> None:
    """format.WriteManifest (pkg/format/manifest.go:33-95): manifest.json with the size and
    SHA-256 of every index file present in out_dir."""
    err = ctypes.create_string_buffer(1024)
    _check(LIB.s3imph_write_manifest(out_dir.encode(), node_count, max_depth, err, 1024), err)


def read_manifest(dir_: str) -> dict:
    """format.ReadManifest (manifest.go:97-111)."""
    import json
    with open(os.path.join(dir_, "manifest.json"), "rb") as f:
        return json.loads(f.read())


def verify_manifest(dir_: str) -> None:
    """format.VerifyManifest (manifest.go:113-138): every listed file's size and checksum;
    raises MPHFError (ERR_FORMAT on a mismatch, ERR_IO on a missing file)."""
    err = ctypes.create_string_buffer(1024)
    _check(LIB.s3imph_verify_manifest(dir_.encode(), err, 1024), err)


def sha256_file(path: str, portable: bool = False) -> str:
    """checksumFile (manifest.go:140-155): hex SHA-256 of a file."""
    err = ctypes.create_string_buffer(1024)
    out = ctypes.create_string_buffer(65)
    _check(LIB.s3imph_sha256_file(path.encode(), int(portable), out, err, 1024), err)
    return out.value.decode()


S3ID_MAGIC = 0x53334944  # pkg/format/format.go:6-45
S3ID_VERSION = 1
S3ID_HEADER = 20


def read_array(path: str, width: int = 8) -> np.ndarray:
    """OpenArray (pkg/format/reader.go:81-119): S3ID header checked (magic, version, the
    expected width, payload size), payload returned as little-endian u64 / u32
    (memory-mapped)."""
    raw = np.memmap(path, dtype=np.uint8, mode="r")
    if len(raw) < S3ID_HEADER:
        raise MPHFError(ERR_FORMAT, f"open array {path}: file too small")
    hdr = bytes(raw[:S3ID_HEADER])
    magic, version = int.from_bytes(hdr[0:4], "little"), int.from_bytes(hdr[4:8], "little")
    count, w = int.from_bytes(hdr[8:16], "little"), int.from_bytes(hdr[16:20], "little")
    if magic != S3ID_MAGIC or version != S3ID_VERSION or w != width or len(raw) != S3ID_HEADER + width * count:
        raise MPHFError(ERR_FORMAT, f"open array {path}: bad header")
    return raw[S3ID_HEADER:].view("<u8" if width == 8 else "<u4")


def read_u64_array(path: str) -> np.ndarray:
    """OpenArray for width-8 arrays (mph_fp.u64, mph_pos.u64, prefix_offsets.u64, ...)."""
    return read_array(path, 8)


class MPHF:
    """format.MPHF on the GPU (OpenMPHF / Lookup / VerifyMPHF, pkg/format/mphf.go:186-302,
    :372-393): mph.bin loaded into a device context, mph_fp / mph_pos in HBM, batched
    Lookup; prefix_blob.bin / prefix_offsets.u64 (when present) for VerifyMPHF."""

    def __init__(self, out_dir: str, device: int = 0):
        import torch
        mph = open(os.path.join(out_dir, "mph.bin"), "rb").read()
        self.ctx = DeviceBuilder(device)
        self.count = 0
        self.dev = f"cuda:{device}"
        self.blob = self.offsets = None
        if mph:
            fp = read_u64_array(os.path.join(out_dir, "mph_fp.u64"))
            pos = read_u64_array(os.path.join(out_dir, "mph_pos.u64"))
            if len(fp) != len(pos):
                raise MPHFError(ERR_FORMAT, "open MPHF: fingerprint and position arrays differ in length")
            self.count = len(fp)
            # read_u64_array may hand back a read-only view of the file: copy before torch takes it
            self.d_fp = torch.from_numpy(np.array(fp, dtype=np.uint64).view(np.int64)).to(self.dev)
            self.d_pos = torch.from_numpy(np.array(pos, dtype=np.uint64).view(np.int64)).to(self.dev)
        else:
            self.d_fp = self.d_pos = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.ctx.load_mph_bin(mph)
        bp, op = os.path.join(out_dir, "prefix_blob.bin"), os.path.join(out_dir, "prefix_offsets.u64")
        if os.path.exists(bp):
            self.offsets = np.ascontiguousarray(read_u64_array(op))
            self.blob = np.fromfile(bp, dtype=np.uint8)

    def lookup(self, keys) -> np.ndarray:
        """Lookup (mphf.go:275-302) of a batch: pos per key, or 2^64-1 when not found."""
        blob, offs = keys_to_blob(keys)
        return self.lookup_blob(blob, offs)

    def lookup_blob(self, blob: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        import torch
        n = len(offsets) - 1
        pad = np.zeros(((len(blob) + 7) // 8) * 8 + 8, np.uint8)
        pad[:len(blob)] = blob
        d_blob = torch.from_numpy(pad).to(self.dev)
        # offsets may be a read-only view of prefix_offsets.u64: copy before torch takes it
        d_offs = torch.from_numpy(np.array(offsets, dtype=np.uint64).view(np.int64)).to(self.dev)
        res = torch.empty(max(n, 1), dtype=torch.int64, device=self.dev)
        self.ctx.lookup(d_blob, d_offs, n, self.d_fp, self.d_pos, self.count, res)
        return res[:n].cpu().numpy().view(np.uint64)

    def verify(self) -> None:
        """VerifyMPHF (mphf.go:372-393): every prefix i of the blob looks up to i."""
        if self.offsets is None:
            raise MPHFError(ERR_STATE, "prefix blob not loaded")
        got = self.lookup_blob(self.blob, self.offsets)
        bad = np.nonzero(got != np.arange(len(got), dtype=np.uint64))[0]
        if len(bad):
            i = int(bad[0])
            raise MPHFError(ERR_INTERNAL, f"lookup returned wrong pos for prefix {i}: got {int(got[i])}, want {i}")

    def close(self) -> None:
        self.ctx.close()


def dist_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(LIB.s3imph_dist_unique_id(buf), None, "ncclGetUniqueId")
    return buf.raw


class DistBuilder(DeviceBuilder):
    """One rank of a multi-GPU build.  Collectives: RCCL (the library owns the
    communicator; `unique_id` from rank 0's dist_unique_id()), or, with `host_comm`,
    the given torch.distributed process group on host copies (test transport:
    several ranks may share one GPU)."""

    def __init__(self, device: int, unique_id: bytes | None, rank: int, nranks: int, host_comm=None):
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        if host_comm is None:
            idbuf = ctypes.create_string_buffer(unique_id, 128)
            _check(LIB.s3imph_ctx_create_dist(device, idbuf, rank, nranks, ctypes.byref(h), err, 512), err)
        else:
            self._comm = _TorchHostComm(None if host_comm is True else host_comm, nranks)
            _check(LIB.s3imph_ctx_create_dist_host(device, ctypes.byref(self._comm.cstruct), rank, nranks,
                                                   ctypes.byref(h), err, 512), err)
        self._h = h
        self.device = device
        self.rank, self.nranks = rank, nranks
        self.last_info = None

    def out_cap(self, n_global: int) -> int:
        return LIB.s3imph_dist_out_cap(self._h, n_global)

    def set_mode(self, mode: int) -> None:
        """DIST_ROUTE or DIST_BITMAP (every rank of a build must choose the same)."""
        _check(LIB.s3imph_ctx_set_dist_mode(self._h, mode), None, "set_dist_mode")

    def segments(self) -> list[tuple[int, int, int]]:
        """(global p, count, local offset) of this rank's outputs in the last build."""
        cnt = ctypes.c_uint64()
        LIB.s3imph_dist_segments(self._h, None, 0, ctypes.byref(cnt))
        buf = (ctypes.c_uint64 * max(3 * cnt.value, 1))()
        _check(LIB.s3imph_dist_segments(self._h, buf, cnt.value, ctypes.byref(cnt)), None, "segments")
        return [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(cnt.value)]

    def build_shard(self, d_blob, d_offsets, n_local: int, key_base: int, d_fp_out, d_pos_out, out_cap: int,
                    d_pos=None, stream=None) -> tuple[int, list, dict]:
        """Build this rank's share; returns (local outputs, segments, info)."""
        info = BuildInfo()
        cnt = ctypes.c_uint64()
        rc = LIB.s3imph_build_device_dist(self._h, _dev_ptr(d_blob), _dev_ptr(d_offsets), _dev_ptr(d_pos),
                                          n_local, key_base, _dev_ptr(d_fp_out), _dev_ptr(d_pos_out), out_cap,
                                          ctypes.byref(cnt), _stream_ptr(stream), ctypes.byref(info))
        if rc != OK:
            raise MPHFError(rc, f"build MPHF (dist): {self.last_error() or status_string(rc)}")
        self.last_info = info.as_dict()
        return cnt.value, self.segments(), self.last_info


class _TorchHostComm:
    """s3imph_host_comm over a torch.distributed process group (gloo), CPU tensors."""

    def __init__(self, group, nranks: int):
        import torch.distributed as tdist
        self.group, self.nranks, self.dist = group, nranks, tdist
        self.cstruct = HostComm(None, ALLGATHER_FN(self._allgather), ALLTOALLV_FN(self._alltoallv))

    def _allgather(self, _user, send, recv, nbytes):
        try:
            src = torch.frombuffer((ctypes.c_uint8 * max(nbytes, 1)).from_address(send), dtype=torch.uint8)[:nbytes]
            out = torch.empty(nbytes * self.nranks, dtype=torch.uint8)
            self.dist.all_gather_into_tensor(out, src.clone(), group=self.group)
            if nbytes:
                ctypes.memmove(recv, out.data_ptr(), nbytes * self.nranks)
            return 0
        except Exception:  # noqa: BLE001 - reported to the library as a failed collective
            import traceback
            traceback.print_exc()
            return 1

    def _alltoallv(self, _user, send, soff, sbytes, recv, roff, rbytes):
        try:
            P = self.nranks
            sb = [sbytes[q] for q in range(P)]
            rb = [rbytes[q] for q in range(P)]
            st, rt = sum(sb), sum(rb)
            src = torch.empty(st, dtype=torch.uint8)
            for q in range(P):
                if sb[q]:
                    ctypes.memmove(src.data_ptr() + sum(sb[:q]), send + soff[q], sb[q])
            out = torch.empty(rt, dtype=torch.uint8)
            self.dist.all_to_all_single(out, src, rb, sb, group=self.group)
            for q in range(P):
                if rb[q]:
                    ctypes.memmove(recv + roff[q], out.data_ptr() + sum(rb[:q]), rb[q])
            return 0
        except Exception:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            return 1


def assemble_dist(parts: list, n_global: int) -> tuple[np.ndarray, np.ndarray]:
    """Global (mph_fp, mph_pos) from every rank's (local fp, local pos, segments)."""
    fp = np.zeros(n_global, np.uint64)
    po = np.zeros(n_global, np.uint64)
    seen = np.zeros(n_global, bool)
    for lfp, lpo, segs in parts:
        for p0, cnt, off in segs:
            if seen[p0:p0 + cnt].any():
                raise ValueError("overlapping output segments")
            seen[p0:p0 + cnt] = True
            fp[p0:p0 + cnt] = lfp[off:off + cnt]
            po[p0:p0 + cnt] = lpo[off:off + cnt]
    if not seen.all():
        raise ValueError("output segments do not cover [0, N)")
    return fp, po


def _stream_ptr(stream):
    """hipStream_t for a call: an explicit stream, else torch's current stream when it is
    not the legacy default (the library's own stream is blocking, hence already ordered
    after work on the default stream)."""
    if stream is None:
        if torch is not None and torch.cuda.is_initialized():
            cur = torch.cuda.current_stream().cuda_stream
            return ctypes.c_void_p(cur) if cur else None
        return None
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


@dataclass
class ShardPlan:
    """Contiguous key-index shard of a global prefix set, balanced by key count."""
    rank: int
    nranks: int
    n_global: int

    @property
    def lo(self) -> int:
        return self.n_global * self.rank // self.nranks

    @property
    def hi(self) -> int:
        return self.n_global * (self.rank + 1) // self.nranks

    @property
    def n_local(self) -> int:
        return self.hi - self.lo
