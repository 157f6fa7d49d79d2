"""ctypes wrapper of oracle/codec_oracle.c (TEST INFRASTRUCTURE ONLY — the parity checker for the
shard-routing and WAL-checksum kernels; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it).  Restates hashindex/shard.go:47-52,104-122 and
lsm/wal.go:31-62,98-133; see the C file's header for the pins."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcodec_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = C.CDLL(_LIB_PATH)
        vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
        L.codec_fnv32a.argtypes, L.codec_fnv32a.restype = [vp, u64], u32
        L.codec_fnv32a_batch.argtypes, L.codec_fnv32a_batch.restype = [vp, vp, u32, u64, vp], None
        L.codec_partition.argtypes, L.codec_partition.restype = [vp, u64, u32, vp, vp], C.c_int
        L.codec_crc32_ieee.argtypes, L.codec_crc32_ieee.restype = [vp, u64], u32
        L.codec_wal_crc.argtypes, L.codec_wal_crc.restype = [vp, vp, u64, vp, vp], None
        _lib = L
    return _lib


def _buf(b) -> np.ndarray:
    return np.frombuffer(b, np.uint8) if isinstance(b, (bytes, bytearray)) else np.ascontiguousarray(b, np.uint8)


def fnv32a(key: bytes) -> int:
    a = _buf(key)
    return lib().codec_fnv32a(a.ctypes.data if a.size else None, a.size)


def fnv32a_batch(data: np.ndarray, n: int, stride: int = 0, offsets: np.ndarray | None = None) -> np.ndarray:
    data = np.ascontiguousarray(data, np.uint8).ravel()
    out = np.empty(n, np.uint32)
    offp = None
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, np.uint64)
        offp = offsets.ctypes.data
    lib().codec_fnv32a_batch(data.ctypes.data if data.size else None, offp, stride, n, out.ctypes.data)
    return out


def partition(shard: np.ndarray, bits: int) -> tuple[np.ndarray, np.ndarray]:
    shard = np.ascontiguousarray(shard, np.uint16)
    nb = 1 << bits
    perm = np.empty(shard.size, np.uint32)
    begin = np.empty(nb + 1, np.uint64)
    if lib().codec_partition(shard.ctypes.data, shard.size, nb, perm.ctypes.data, begin.ctypes.data):
        raise MemoryError
    return perm, begin


def crc32_ieee(b) -> int:
    a = _buf(b)
    return lib().codec_crc32_ieee(a.ctypes.data if a.size else None, a.size)


def wal_crc(image: np.ndarray, offsets: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    image = _buf(image)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    crc = np.empty(n, np.uint32)
    ok = np.empty(n, np.uint8)
    lib().codec_wal_crc(image.ctypes.data, offsets.ctypes.data, n, crc.ctypes.data, ok.ctypes.data)
    return crc, ok
