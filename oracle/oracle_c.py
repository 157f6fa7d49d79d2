"""ctypes loader for oracle/_build/libbloom_oracle.so — TEST INFRASTRUCTURE ONLY (checker)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libbloom_oracle.so")
_lib = None

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)


def build_library() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build_library()
        L = C.CDLL(_LIB_PATH)
        L.oracle_params.argtypes = [C.c_int64, C.c_double, u64p, u32p]
        L.oracle_params.restype = C.c_int
        L.oracle_go_log.argtypes = [C.c_double]
        L.oracle_go_log.restype = C.c_double
        L.oracle_fnv1a64.argtypes = [u8p, C.c_uint64]
        L.oracle_fnv1a64.restype = C.c_uint64
        L.oracle_fnv1_64.argtypes = [u8p, C.c_uint64]
        L.oracle_fnv1_64.restype = C.c_uint64
        L.oracle_positions.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint32, u64p]
        L.oracle_build.argtypes = [u8p, C.c_uint64, C.c_uint32, u8p, u64p, C.c_uint32, C.c_uint64]
        L.oracle_probe.argtypes = [u8p, C.c_uint64, C.c_uint32, u8p, u64p, C.c_uint32, C.c_uint64, u8p]
        L.oracle_probe_multi.argtypes = [C.POINTER(u8p), u64p, u32p, C.c_uint32, u8p, u64p, C.c_uint32,
                                         C.c_uint64, u64p]
        L.oracle_build_mt.argtypes = [u8p, C.c_uint64, C.c_uint32, u8p, u64p, C.c_uint32, C.c_uint64, C.c_int]
        L.oracle_build_mt.restype = C.c_int
        L.oracle_probe_mt.argtypes = [u8p, C.c_uint64, C.c_uint32, u8p, u64p, C.c_uint32, C.c_uint64, u8p,
                                      C.c_int]
        L.oracle_probe_mt.restype = C.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray, t=u8p):
    return a.ctypes.data_as(t) if a is not None else None


def params(n: int, p: float) -> tuple[int, int]:
    m = C.c_uint64()
    k = C.c_uint32()
    if lib().oracle_params(n, p, C.byref(m), C.byref(k)) != 0:
        raise ValueError("outside the reference's defined range")
    return m.value, k.value


def go_log(x: float) -> float:
    return lib().oracle_go_log(x)


def fnv(key: bytes) -> tuple[int, int]:
    a = np.frombuffer(key, dtype=np.uint8) if key else np.zeros(1, np.uint8)
    return lib().oracle_fnv1a64(_p(a), len(key)), lib().oracle_fnv1_64(_p(a), len(key))


def positions(key: bytes, m: int, k: int) -> list[int]:
    a = np.frombuffer(key, dtype=np.uint8) if key else np.zeros(1, np.uint8)
    out = np.zeros(max(k, 1), dtype=np.uint64)
    lib().oracle_positions(_p(a), len(key), m, k, _p(out, u64p))
    return [int(x) for x in out[:k]]


def _keys_args(data: np.ndarray, offsets: np.ndarray | None, stride: int):
    data = np.ascontiguousarray(data).reshape(-1)
    if data.size == 0:
        data = np.zeros(1, np.uint8)
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    return data, off


def build(m: int, k: int, data: np.ndarray, n: int, stride: int = 0, offsets: np.ndarray | None = None,
          threads: int = 1, bits: np.ndarray | None = None) -> np.ndarray:
    d, off = _keys_args(data, offsets, stride)
    if bits is None:
        bits = np.zeros(max((m + 7) // 8, 1), dtype=np.uint8)
    if threads > 1:
        if lib().oracle_build_mt(_p(bits), m, k, _p(d), _p(off, u64p), stride, n, threads) != 0:
            raise RuntimeError(f"oracle_build_mt: {threads} threads could not all start or allocate")
    else:
        lib().oracle_build(_p(bits), m, k, _p(d), _p(off, u64p), stride, n)
    return bits[: (m + 7) // 8]


def probe(bits: np.ndarray, m: int, k: int, data: np.ndarray, n: int, stride: int = 0,
          offsets: np.ndarray | None = None, threads: int = 1) -> np.ndarray:
    d, off = _keys_args(data, offsets, stride)
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    if bits.size == 0:
        bits = np.zeros(1, np.uint8)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    if threads > 1:
        lib().oracle_probe_mt(_p(bits), m, k, _p(d), _p(off, u64p), stride, n, _p(out), threads)
    else:
        lib().oracle_probe(_p(bits), m, k, _p(d), _p(off, u64p), stride, n, _p(out))
    return out[:n]


def probe_multi(filters: list[tuple[np.ndarray, int, int]], data: np.ndarray, n: int, stride: int = 0,
                offsets: np.ndarray | None = None) -> np.ndarray:
    d, off = _keys_args(data, offsets, stride)
    nf = len(filters)
    keep = [np.ascontiguousarray(b, dtype=np.uint8) for b, _, _ in filters]
    arr = (u8p * nf)(*[_p(b) for b in keep])
    ms = np.array([m for _, m, _ in filters], dtype=np.uint64)
    ks = np.array([k for _, _, k in filters], dtype=np.uint32)
    out = np.zeros(max(n, 1), dtype=np.uint64)
    lib().oracle_probe_multi(arr, _p(ms, u64p), _p(ks, u32p), nf, _p(d), _p(off, u64p), stride, n,
                             _p(out, u64p))
    return out[:n]
