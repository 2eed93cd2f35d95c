"""CPU oracle for the s3-inv-db MPHF-build path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.  The product path
(``s3-inv-db_amd``) never imports it and has no CPU fallback.

Two independent restatements live here:

* ``OracleLib``: ctypes binding of ``oracle/bbhash_oracle.c`` (fast; used for
  every parity check at size).
* ``py_*``: a pure-Python restatement of the same algorithm, written separately,
  used only on small key sets to cross-check the C restatement.

Reference anchors (``/root/reference``): FNV ``pkg/format/mphf.go:341-369``;
BBHash build ``pkg/format/mphf_streaming.go:141`` (relab/bbhash, restated per
SURVEY.md Appendix A — parity of ``mph.bin`` bytes is "vs restated spec");
positions/scatter ``mphf_streaming.go:176-204,237-261``; Lookup
``mphf.go:275-302``; S3ID framing ``format.go:6-45``, ``writer.go:113-140,212-237``.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

ORC_OK = 0
ORC_ERR_TOO_MANY_LEVELS = 3
ORC_ERR_KEY_ZERO = 4

MASK64 = (1 << 64) - 1
FNV_OFFSET64 = 0xCBF29CE484222325
FNV_PRIME64 = 0x100000001B3
HASH_M = 0x880355F21E6D1965
MIX_MUL = 0x2127599BF4325C37
MAX_LEVELS = 64

S3ID_MAGIC = 0x53334944
S3ID_VERSION = 1


def build_oracle() -> str:
    """Compile oracle/_build/liboracle.so with plain gcc (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class OracleMPHF:
    def __init__(self, lib: "OracleLib", handle):
        self._lib = lib
        self._h = handle

    def __del__(self):
        if self._h:
            self._lib.lib.orc_free(self._h)
            self._h = None

    @property
    def num_levels(self) -> int:
        return self._lib.lib.orc_num_levels(self._h)

    def find(self, key_hash: int) -> int:
        return self._lib.lib.orc_find(self._h, ctypes.c_uint64(key_hash))

    def marshal(self) -> bytes:
        n = self._lib.lib.orc_marshal_size(self._h)
        buf = (ctypes.c_uint8 * n)()
        self._lib.lib.orc_marshal(self._h, buf)
        return bytes(buf)

    def level_bits(self, lvl: int) -> np.ndarray:
        w = self._lib.lib.orc_level_word_count(self._h, lvl)
        ptr = self._lib.lib.orc_level_bits(self._h, lvl)
        return np.ctypeslib.as_array(ptr, shape=(w,)).copy()


class OracleLib:
    """ctypes binding of liboracle.so (the C restatement)."""

    def __init__(self, path: str = _LIB_PATH):
        if not os.path.exists(path):
            build_oracle()
        lib = ctypes.CDLL(path)
        u64, u8p, u64p = ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint64)
        vp = ctypes.c_void_p
        lib.orc_fnv1a64.restype = u64
        lib.orc_fnv1a64.argtypes = [ctypes.c_char_p, u64]
        lib.orc_fnv1_64.restype = u64
        lib.orc_fnv1_64.argtypes = [ctypes.c_char_p, u64]
        lib.orc_hash_keys.argtypes = [vp, vp, u64, vp, vp]
        lib.orc_bbhash_new.restype = ctypes.c_int
        lib.orc_bbhash_new.argtypes = [vp, u64, ctypes.POINTER(vp)]
        lib.orc_find.restype = u64
        lib.orc_find.argtypes = [vp, u64]
        lib.orc_marshal_size.restype = u64
        lib.orc_marshal_size.argtypes = [vp]
        lib.orc_marshal.argtypes = [vp, vp]
        lib.orc_unmarshal.restype = ctypes.c_int
        lib.orc_unmarshal.argtypes = [ctypes.c_char_p, u64, ctypes.POINTER(vp)]
        lib.orc_num_levels.restype = ctypes.c_uint32
        lib.orc_num_levels.argtypes = [vp]
        lib.orc_level_word_count.restype = u64
        lib.orc_level_word_count.argtypes = [vp, ctypes.c_uint32]
        lib.orc_level_bits.restype = u64p
        lib.orc_level_bits.argtypes = [vp, ctypes.c_uint32]
        lib.orc_free.argtypes = [vp]
        lib.orc_build.restype = ctypes.c_int
        lib.orc_build.argtypes = [vp, vp, vp, u64, vp, vp, ctypes.POINTER(vp)]
        lib.orc_build_mt.restype = ctypes.c_int
        lib.orc_build_mt.argtypes = [vp, vp, vp, u64, ctypes.c_int, vp, vp, ctypes.POINTER(vp)]
        lib.orc_build_revmap.restype = ctypes.c_int
        lib.orc_build_revmap.argtypes = [vp, vp, vp, u64, vp, vp]
        lib.orc_lookup.restype = ctypes.c_int
        lib.orc_lookup.argtypes = [vp, vp, vp, u64, ctypes.c_char_p, u64, u64p]
        lib.orc_level_hash.restype = u64
        lib.orc_level_hash.argtypes = [u64]
        lib.orc_key_hash.restype = u64
        lib.orc_key_hash.argtypes = [u64, u64]
        lib.orc_level_words.restype = u64
        lib.orc_level_words.argtypes = [u64]
        lib.orc_finalize.restype = ctypes.c_int
        lib.orc_finalize.argtypes = [vp, vp, vp, u64, vp, vp, vp, vp, u64, vp, ctypes.POINTER(ctypes.c_uint32)]
        self.lib = lib
        del u8p

    # -- hashes -----------------------------------------------------------
    def fnv1a64(self, b: bytes) -> int:
        return self.lib.orc_fnv1a64(b, len(b))

    def fnv1_64(self, b: bytes) -> int:
        return self.lib.orc_fnv1_64(b, len(b))

    def hash_keys(self, blob: np.ndarray, offsets: np.ndarray):
        n = len(offsets) - 1
        kh = np.empty(n, np.uint64)
        fp = np.empty(n, np.uint64)
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        self.lib.orc_hash_keys(_ptr(blob), _ptr(offsets), n, _ptr(kh), _ptr(fp))
        return kh, fp

    # -- bbhash -------------------------------------------------------------
    def bbhash_new(self, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        h = ctypes.c_void_p()
        st = self.lib.orc_bbhash_new(_ptr(keys), len(keys), ctypes.byref(h))
        return st, (OracleMPHF(self, h) if st == ORC_OK and h.value else None)

    def unmarshal(self, data: bytes):
        h = ctypes.c_void_p()
        st = self.lib.orc_unmarshal(data, len(data), ctypes.byref(h))
        return st, (OracleMPHF(self, h) if st == ORC_OK and h.value else None)

    def build(self, blob: np.ndarray, offsets: np.ndarray, pos: np.ndarray | None = None):
        """Returns (status, fp_out, pos_out, mph_bin_bytes)."""
        n = len(offsets) - 1
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        fp_out = np.zeros(n, np.uint64)
        pos_out = np.zeros(n, np.uint64)
        posp = None
        if pos is not None:
            pos = np.ascontiguousarray(pos, np.uint64)
            posp = _ptr(pos)
        h = ctypes.c_void_p()
        st = self.lib.orc_build(_ptr(blob), _ptr(offsets), posp, n, _ptr(fp_out), _ptr(pos_out), ctypes.byref(h))
        if st != ORC_OK:
            return st, None, None, None
        if n == 0:
            return st, fp_out, pos_out, b""
        m = OracleMPHF(self, h)
        return st, fp_out, pos_out, m.marshal()

    def build_mt(self, blob: np.ndarray, offsets: np.ndarray, pos: np.ndarray | None = None, threads: int = 8):
        """orc_build with the FNV pass and the placement on `threads` threads (same outputs)."""
        n = len(offsets) - 1
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        fp_out = np.zeros(n, np.uint64)
        pos_out = np.zeros(n, np.uint64)
        posp = None if pos is None else _ptr(np.ascontiguousarray(pos, np.uint64))
        h = ctypes.c_void_p()
        st = self.lib.orc_build_mt(_ptr(blob), _ptr(offsets), posp, n, threads, _ptr(fp_out), _ptr(pos_out),
                                   ctypes.byref(h))
        if st != ORC_OK:
            return st, None, None, None
        if n == 0:
            return st, fp_out, pos_out, b""
        return st, fp_out, pos_out, OracleMPHF(self, h).marshal()

    def build_revmap(self, blob: np.ndarray, offsets: np.ndarray, pos: np.ndarray | None = None):
        """The reference-shaped single-thread build (reverse map + hash map): (status, fp_out, pos_out)."""
        n = len(offsets) - 1
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        fp_out = np.zeros(n, np.uint64)
        pos_out = np.zeros(n, np.uint64)
        posp = None if pos is None else _ptr(np.ascontiguousarray(pos, np.uint64))
        st = self.lib.orc_build_revmap(_ptr(blob), _ptr(offsets), posp, n, _ptr(fp_out), _ptr(pos_out))
        return st, fp_out, pos_out

    def finalize(self, blob: np.ndarray, offsets: np.ndarray, depths: np.ndarray | None = None) -> dict:
        """IndexBuilder's finalize arrays (indexbuild.go:154-248,393-415,474-503; depthindex.go:32-96):
        depth, subtree_end, max_depth_in_subtree, depth_offsets, depth_positions, max_depth."""
        n = len(offsets) - 1
        blob = np.ascontiguousarray(blob, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        dp = None if depths is None else _ptr(np.ascontiguousarray(depths, np.uint32))
        depth = np.zeros(n, np.uint32)
        send = np.zeros(n, np.uint64)
        mds = np.zeros(n, np.uint32)
        dpos = np.zeros(n, np.uint64)
        maxd = ctypes.c_uint32()
        cap = 64
        while True:
            doff = np.zeros(cap, np.uint64)
            rc = self.lib.orc_finalize(_ptr(blob), _ptr(offsets), dp, n, _ptr(depth), _ptr(send), _ptr(mds),
                                       _ptr(doff), cap, _ptr(dpos), ctypes.byref(maxd))
            if rc != -1:
                break
            cap = maxd.value + 2
        assert rc == 0
        return {"depth": depth, "subtree_end": send, "max_depth_in_subtree": mds,
                "depth_offsets": doff[: maxd.value + 2].copy(), "depth_positions": dpos, "max_depth": maxd.value}

    def lookup(self, mph: OracleMPHF | None, fp_arr: np.ndarray, pos_arr: np.ndarray, key: bytes):
        out = ctypes.c_uint64()
        if mph is None:
            return None
        fp_arr = np.ascontiguousarray(fp_arr, np.uint64)
        pos_arr = np.ascontiguousarray(pos_arr, np.uint64)
        hit = self.lib.orc_lookup(mph._h, _ptr(fp_arr), _ptr(pos_arr), len(fp_arr), key, len(key), ctypes.byref(out))
        return out.value if hit else None


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


_LIB = None


def lib() -> OracleLib:
    global _LIB
    if _LIB is None:
        _LIB = OracleLib()
    return _LIB


# ---------------------------------------------------------------------------
# Pure-Python restatement (small inputs only), written independently of the C.
# ---------------------------------------------------------------------------

def py_fnv1a64(b: bytes) -> int:
    h = FNV_OFFSET64
    for c in b:
        h = ((h ^ c) * FNV_PRIME64) & MASK64
    return h


def py_fnv1_64(b: bytes) -> int:
    h = FNV_OFFSET64
    for c in b:
        h = ((h * FNV_PRIME64) & MASK64) ^ c
    return h


def _py_mix(h: int) -> int:
    h ^= h >> 23
    h = (h * MIX_MUL) & MASK64
    h ^= h >> 47
    return h


def py_pos(level: int, key: int, size: int) -> int:
    lh = (_py_mix(level) * HASH_M) & MASK64
    h = _py_mix(((lh ^ _py_mix(key)) * HASH_M) & MASK64)
    return h % size


def py_bbhash(keys: list[int]) -> list[list[int]]:
    """Levels as lists of u64 words (set semantics: positions hit exactly once)."""
    levels = []
    active = list(keys)
    lvl = 0
    while active:
        if lvl >= MAX_LEVELS:
            raise RuntimeError("too many levels")
        words = (2 * len(active) + 63) // 64
        size = 64 * words
        counts: dict[int, int] = {}
        idx = [py_pos(lvl, k, size) for k in active]
        for i in idx:
            counts[i] = counts.get(i, 0) + 1
        bits = [0] * words
        nxt = []
        for k, i in zip(active, idx):
            if counts[i] == 1:
                bits[i >> 6] |= 1 << (i & 63)
            else:
                nxt.append(k)
        levels.append(bits)
        active = nxt
        lvl += 1
    return levels


def py_find(levels: list[list[int]], key: int) -> int:
    base = 0
    for lvl, bits in enumerate(levels):
        i = py_pos(lvl, key, 64 * len(bits))
        w, b = i >> 6, i & 63
        if (bits[w] >> b) & 1:
            r = sum(bin(x).count("1") for x in bits[:w]) + bin(bits[w] & ((1 << b) - 1)).count("1")
            return base + r + 1
        base += sum(bin(x).count("1") for x in bits)
    return 0


def py_marshal(levels: list[list[int]]) -> bytes:
    out = struct.pack("<QQ", 1, len(levels))
    for bits in levels:
        out += struct.pack("<Q", len(bits)) + b"".join(struct.pack("<Q", w) for w in bits)
    return out


def py_build(keys: list[bytes], pos: list[int] | None = None):
    """StreamingMPHFBuilder.Build restated in Python: (fp_out, pos_out, mph_bin)."""
    n = len(keys)
    if n == 0:
        return [], [], b""
    kh = [py_fnv1a64(k) for k in keys]
    levels = py_bbhash(kh)
    fp_out = [0] * n
    pos_out = [0] * n
    for i, k in enumerate(keys):
        p = py_find(levels, kh[i]) - 1
        fp_out[p] = py_fnv1_64(k)
        pos_out[p] = pos[i] if pos is not None else i
    return fp_out, pos_out, py_marshal(levels)


# ---------------------------------------------------------------------------
# S3ID framing (format.go:6-45; writer.go:19-46,113-140,212-237)
# ---------------------------------------------------------------------------

def py_finalize(keys: list[bytes], depths: list[int] | None = None) -> dict:
    """Pure-Python restatement of the finalize arrays (small inputs): the subtree of prefix
    i is every later key it is a byte prefix of (keys are sorted, so a run), as the
    ancestor stack of indexbuild.go:201-248 produces; depth index per depthindex.go:32-96."""
    n = len(keys)
    depth = [k.count(b"/") for k in keys] if depths is None else list(depths)
    send, mds = [0] * n, [0] * n
    for i in range(n):
        j = i
        while j + 1 < n and keys[j + 1].startswith(keys[i]):
            j += 1
        # the stack closes node i at the first later key it is not a prefix of ... unless
        # an entry below it on the stack closes first; every entry below i is a prefix of
        # keys[i], hence of every key in its run, so the run is exact
        send[i] = j
        mds[i] = max(depth[i:j + 1])
    maxd = max(depth) if n else 0
    offs, dpos = [], []
    for d in range(maxd + 1):
        offs.append(len(dpos))
        dpos.extend(i for i in range(n) if depth[i] == d)
    offs.append(len(dpos))
    return {"depth": depth, "subtree_end": send, "max_depth_in_subtree": mds, "depth_offsets": offs,
            "depth_positions": dpos, "max_depth": maxd}


def s3id_u32_array(vals) -> bytes:
    """ArrayWriter of width 4 (format.go:25-32, writer.go:113-140)."""
    vals = list(vals)
    return s3id_header(len(vals), 4) + b"".join(struct.pack("<I", int(v)) for v in vals)


def s3id_header(count: int, width: int = 8) -> bytes:
    return struct.pack("<IIQI", S3ID_MAGIC, S3ID_VERSION, count, width)


def s3id_u64_array(vals) -> bytes:
    a = np.ascontiguousarray(vals, dtype="<u8")
    return s3id_header(len(a)) + a.tobytes()


def keys_to_blob(keys: list[bytes]):
    """Concatenate keys into (blob u8, offsets u64[N+1]) — prefix_blob.bin / prefix_offsets.u64 layout."""
    offs = np.zeros(len(keys) + 1, np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    blob = np.frombuffer(b"".join(keys), np.uint8) if keys else np.zeros(0, np.uint8)
    return blob.copy(), offs
