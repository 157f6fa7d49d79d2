"""Python host binding of libseb_bloom.so (the C ABI in include/seb_bloom.h), via ctypes.

`BloomFilter` mirrors the reference's Go API (lsm/bloom.go) one method per method, so the
parity tests read like the reference's own call sequences:

    NewBloomFilter(expectedKeys, fpr)  lsm/bloom.go:19   -> BloomFilter(n, p)
    (*BloomFilter).Add(key)            lsm/bloom.go:70   -> .add(key)            (deferred, batched)
    (*BloomFilter).MayContain(key)     lsm/bloom.go:82   -> .may_contain(key)
    (*BloomFilter).Encode()            lsm/bloom.go:96   -> .encode()
    DecodeBloomFilter(data)            lsm/bloom.go:105  -> BloomFilter.decode(data)  (None if < 12 B)

Every computation runs in the HIP library on the GPU: if the library is missing, or no gfx950
device is present, the device-resident and batch calls raise SebError.  The one exception is the
drop-in boundary's (SURVEY.md 8(b) error row): the Go API mirror (`BloomFilter`) keeps working on
its host copy when its device path fails, as the Go API has no error returns; `fallback_count()`
counts those uses and the GPU tests and smoke() assert it stays 0.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SEB_LIB_PATH") or os.path.join(_HERE, "lib", "libseb_bloom.so")  # override: A/B builds
HEADER = os.path.join(os.path.dirname(_HERE), "include", "seb_bloom.h")

SEB_OK = 0
SEB_BUILD_FRESH = 1
ERRORS = {-1: "SEB_ERR_INVALID", -2: "SEB_ERR_DEVICE", -3: "SEB_ERR_NOMEM", -4: "SEB_ERR_RANGE", -5: "SEB_ERR_SHORT",
          -6: "SEB_ERR_INTERNAL"}


class SebError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class seb_keys(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("n", C.c_uint64), ("stride", C.c_uint32),
                ("reserved", C.c_uint32)]


class seb_filter_ref(C.Structure):
    _fields_ = [("bits", C.c_void_p), ("num_bits", C.c_uint64), ("num_hashes", C.c_uint32),
                ("reserved", C.c_uint32)]


_lib = None
_vp = C.c_void_p
_u64 = C.c_uint64
_u32 = C.c_uint32
_i = C.c_int

_SIGS = {
    "seb_params": (_i, [C.c_int64, C.c_double, C.POINTER(_u64), C.POINTER(_u32)]),
    "seb_num_bytes": (_u64, [_u64]),
    "seb_words_bytes": (_u64, [_u64]),
    "seb_abi_version": (_i, []),
    "seb_last_error": (C.c_char_p, []),
    "seb_set_option": (_i, [C.c_char_p, C.c_int64]),
    "seb_get_option": (_i, [C.c_char_p, C.POINTER(C.c_int64)]),
    "seb_dev_build_workspace_size": (_u64, [_u64, _u64, _u32]),
    "seb_dev_build_ws": (_i, [C.POINTER(seb_keys), _vp, _u64, _u32, _vp, _u64, _vp]),
    "seb_device_check": (_i, [_i]),
    "seb_dev_clear": (_i, [_vp, _u64, _vp]),
    "seb_dev_build": (_i, [C.POINTER(seb_keys), _vp, _u64, _u32, _vp]),
    "seb_dev_build_fresh": (_i, [C.POINTER(seb_keys), _vp, _u64, _u32, _vp]),
    "seb_dev_probe": (_i, [C.POINTER(seb_keys), _vp, _u64, _u32, _vp, _vp]),
    "seb_dev_probe_multi": (_i, [C.POINTER(seb_keys), C.POINTER(seb_filter_ref), _u32, _vp, _u32, _vp]),
    "seb_dev_build_many": (_i, [C.POINTER(seb_keys), C.POINTER(_u64), C.POINTER(seb_filter_ref), _u32, _vp]),
    "seb_dev_alloc": (_i, [C.POINTER(_vp), _u64]),
    "seb_dev_free": (_i, [_vp]),
    "seb_host_alloc": (_i, [C.POINTER(_vp), _u64]),
    "seb_host_free": (_i, [_vp]),
    "seb_memcpy_h2d": (_i, [_vp, _vp, _u64, _vp]),
    "seb_memcpy_d2h": (_i, [_vp, _vp, _u64, _vp]),
    "seb_stream_sync": (_i, [_vp]),
    "seb_ctx_create": (_i, [_i, C.POINTER(_vp)]),
    "seb_ctx_destroy": (None, [_vp]),
    "seb_build": (_i, [_vp, C.POINTER(seb_keys), _vp, _u64, _u32, _u32]),
    "seb_probe": (_i, [_vp, C.POINTER(seb_keys), _vp, _u64, _u32, _vp]),
    "seb_probe_multi": (_i, [_vp, C.POINTER(seb_keys), C.POINTER(seb_filter_ref), _u32, _vp]),
    "seb_filter_new": (_vp, [C.c_int64, C.c_double]),
    "seb_filter_free": (None, [_vp]),
    "seb_filter_add": (_i, [_vp, _vp, _u64]),
    "seb_filter_add_batch": (_i, [_vp, C.POINTER(seb_keys)]),
    "seb_filter_may_contain": (_i, [_vp, _vp, _u64]),
    "seb_filter_may_contain_batch": (_i, [_vp, C.POINTER(seb_keys), _vp]),
    "seb_filter_encoded_size": (_u64, [_vp]),
    "seb_filter_encode": (_i, [_vp, _vp, _u64]),
    "seb_filter_decode": (_vp, [_vp, _u64]),
    "seb_filter_num_bits": (_u64, [_vp]),
    "seb_filter_num_hashes": (_u32, [_vp]),
    "seb_filter_pending": (_u64, [_vp]),
    "seb_filter_flush": (_i, [_vp]),
    "seb_fallback_count": (_u64, []),
    "seb_multiget_order_fallbacks": (_u64, []),
    "seb_registry_new": (_vp, [_i]),
    "seb_registry_free": (None, [_vp]),
    "seb_registry_put": (_i, [_vp, _u64, _i, _vp, _u64, _vp, _u64, _vp, _u64]),
    "seb_registry_remove": (_i, [_vp, _u64]),
    "seb_registry_slots": (_i, [_vp, C.POINTER(_u64), C.POINTER(C.c_int32), _u32]),
    "seb_registry_multiget": (_i, [_vp, C.POINTER(seb_keys), _vp]),
    "seb_registry_multiget_dev": (_i, [_vp, C.POINTER(seb_keys), _vp, _vp]),
    "seb_registry_max_candidates": (_i, [_vp]),
    "seb_registry_multiget_list": (_i, [_vp, C.POINTER(seb_keys), _vp, _u32]),
    "seb_registry_multiget_list_dev": (_i, [_vp, C.POINTER(seb_keys), _vp, _u32, _vp]),
    "seb_registry_multiget_files": (_i, [_vp, C.POINTER(seb_keys), _vp, _u32, C.POINTER(_u32)]),
    "seb_workspace_bytes": (_u64, []),
    "seb_dev_or_slices": (_i, [_vp, _u32, _u64, _vp, _vp]),
    "seb_workspace_release": (_i, []),
    "seb_dev_shard_route": (_i, [C.POINTER(seb_keys), _u32, _vp, _vp, _vp]),
    "seb_dev_shard_partition_workspace_size": (_u64, [_u64, _u32]),
    "seb_dev_shard_partition": (_i, [C.POINTER(seb_keys), _u32, _vp, _vp, _vp, _vp, _u64, _vp]),
    "seb_dev_wal_crc": (_i, [_vp, _vp, _u64, _i, _vp, _vp, _vp]),
    "seb_wal_scan": (_i, [_vp, _u64, _vp, _u64, C.POINTER(_u64)]),
    "seb_dev_pack_residues": (_i, [C.POINTER(seb_keys), _u64, _u32, _vp, _vp]),
    "seb_dev_probe_packed": (_i, [_vp, _u64, _vp, _u64, _u32, _vp, _vp]),
    "seb_dev_probe_emit_packed": (_i, [C.POINTER(seb_keys), _vp, _u64, _u32, _vp, _vp, _vp]),
    "seb_dev_probe_multi_packed": (_i, [_vp, _u64, C.POINTER(seb_filter_ref), _u32, _vp, _u32, _vp]),
    "seb_packed6_bytes": (_u64, [_u64]),
    "seb_dev_pack_residues6": (_i, [C.POINTER(seb_keys), _u64, _u32, _vp, _vp]),
    "seb_dev_probe_multi_packed6": (_i, [_vp, _u64, C.POINTER(seb_filter_ref), _u32, _vp, _u32, _vp]),
    "seb_timer_create": (_i, [C.POINTER(_vp)]),
    "seb_timer_record": (_i, [_vp, _vp]),
    "seb_timer_elapsed_ms": (_i, [_vp, _vp, C.POINTER(C.c_float)]),
    "seb_timer_destroy": (_i, [_vp]),
}

WAL_CRC, WAL_SEAL, WAL_VERIFY = 0, 1, 2


def build_library() -> str:
    """Compile libseb_bloom.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "csrc")], check=True)
    return LIB_PATH


def lib():
    """Load the HIP library; raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SebError(-2, f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        try:  # share torch's HIP runtime when torch is in the process (same SONAME)
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().seb_last_error() or b"").decode()


def check(rc: int) -> int:
    if rc < 0:
        raise SebError(rc, last_error())
    return rc


def params(n: int, p: float) -> tuple[int, int]:
    m, k = _u64(), _u32()
    check(lib().seb_params(n, p, C.byref(m), C.byref(k)))
    return m.value, k.value


def num_bytes(m: int) -> int:
    return lib().seb_num_bytes(m)


def words_bytes(m: int) -> int:
    return lib().seb_words_bytes(m)


def set_option(name: str, value: int) -> None:
    """Tuning knob (build_algo, probe_phases, bucket_min_keys, grid_cap, ...); results never change."""
    check(lib().seb_set_option(name.encode(), int(value)))


def get_option(name: str) -> int:
    v = C.c_int64()
    check(lib().seb_get_option(name.encode(), C.byref(v)))
    return v.value


class option:
    """Context manager: temporarily set a tuning knob."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, value

    def __enter__(self):
        self.old = get_option(self.name)
        set_option(self.name, self.value)

    def __exit__(self, *exc):
        set_option(self.name, self.old)


def fallback_count() -> int:
    """Go-API-mirror builds / probes that ran on the host copy because the device path failed."""
    return int(lib().seb_fallback_count())


def device_check(device: int = 0) -> None:
    check(lib().seb_device_check(device))


# ------------------------------------------------------------------ key batches (host) ----

class HostKeys:
    """A host key batch: fixed-stride (n, L) uint8 array, or (data, offsets) variable-length."""

    def __init__(self, data: np.ndarray, offsets: np.ndarray | None = None):
        if offsets is None:
            arr = np.ascontiguousarray(data, dtype=np.uint8)
            if arr.ndim != 2:
                raise ValueError("fixed-length keys must be a 2-D (n, L) uint8 array")
            self.n, self.stride = arr.shape
            self.data = arr
            self.offsets = None
        else:
            self.data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
            self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            self.n = self.offsets.shape[0] - 1
            self.stride = 0
        self._s = seb_keys(self.data.ctypes.data if self.data.size else None,
                           self.offsets.ctypes.data if self.offsets is not None else None,
                           self.n, self.stride, 0)

    @property
    def ref(self):
        return C.byref(self._s)


def as_keys(keys) -> HostKeys:
    if isinstance(keys, HostKeys):
        return keys
    if isinstance(keys, tuple):
        return HostKeys(keys[0], keys[1])
    if isinstance(keys, (list,)):
        lens = np.array([len(k) for k in keys], dtype=np.uint64)
        off = np.zeros(len(keys) + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        data = np.frombuffer(b"".join(keys), dtype=np.uint8) if len(keys) else np.zeros(0, np.uint8)
        return HostKeys(data, off)
    return HostKeys(keys)


# ------------------------------------------------------------------ host-buffer API ------

class Ctx:
    """seb_ctx: streams + scratch on one device; host-buffer build / probe (PCIe-inclusive)."""

    def __init__(self, device: int = 0):
        p = _vp()
        check(lib().seb_ctx_create(device, C.byref(p)))
        self._p = p

    def close(self):
        if self._p:
            lib().seb_ctx_destroy(self._p)
            self._p = None

    __del__ = close

    def build(self, keys, m: int, k: int, bits: np.ndarray | None = None) -> np.ndarray:
        kb = as_keys(keys)
        fresh = bits is None
        out = np.zeros(num_bytes(m), dtype=np.uint8) if fresh else bits
        check(lib().seb_build(self._p, kb.ref, out.ctypes.data, m, k, SEB_BUILD_FRESH if fresh else 0))
        return out

    def probe(self, keys, bits: np.ndarray, m: int, k: int) -> np.ndarray:
        kb = as_keys(keys)
        out = np.zeros(max(kb.n, 1), dtype=np.uint8)
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        check(lib().seb_probe(self._p, kb.ref, bits.ctypes.data, m, k, out.ctypes.data))
        return out[: kb.n]

    def probe_multi(self, keys, filters: list[tuple[np.ndarray, int, int]]) -> np.ndarray:
        kb = as_keys(keys)
        keep = [np.ascontiguousarray(b, dtype=np.uint8) for b, _, _ in filters]
        refs = (seb_filter_ref * len(filters))(*[seb_filter_ref(b.ctypes.data, m, k, 0)
                                                  for b, (_, m, k) in zip(keep, filters)])
        out = np.zeros(max(kb.n, 1), dtype=np.uint64)
        check(lib().seb_probe_multi(self._p, kb.ref, refs, len(filters), out.ctypes.data))
        return out[: kb.n]


# ------------------------------------------------------------- Go API mirror (handles) ----

class BloomFilter:
    """lsm/bloom.go's BloomFilter, backed by an HBM-resident bit array in libseb_bloom."""

    def __init__(self, expected_keys: int | None = None, fpr: float = 0.01, *, _handle=None):
        if _handle is None:
            _handle = lib().seb_filter_new(expected_keys, fpr)
            if not _handle:
                raise SebError(-4, last_error())
        self._h = _handle

    @classmethod
    def decode(cls, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        h = lib().seb_filter_decode(buf.ctypes.data, len(data))
        return cls(_handle=h) if h else None

    def close(self):
        if getattr(self, "_h", None):
            lib().seb_filter_free(self._h)
            self._h = None

    __del__ = close

    @property
    def num_bits(self) -> int:
        return lib().seb_filter_num_bits(self._h)

    @property
    def num_hashes(self) -> int:
        return lib().seb_filter_num_hashes(self._h)

    @property
    def pending(self) -> int:
        return lib().seb_filter_pending(self._h)

    def add(self, key: bytes) -> None:
        check(lib().seb_filter_add(self._h, key, len(key)))

    def add_batch(self, keys) -> None:
        kb = as_keys(keys)
        check(lib().seb_filter_add_batch(self._h, kb.ref))

    def may_contain(self, key: bytes) -> bool:
        return bool(check(lib().seb_filter_may_contain(self._h, key, len(key))))

    def may_contain_batch(self, keys) -> np.ndarray:
        kb = as_keys(keys)
        out = np.zeros(max(kb.n, 1), dtype=np.uint8)
        check(lib().seb_filter_may_contain_batch(self._h, kb.ref, out.ctypes.data))
        return out[: kb.n]

    def flush(self) -> None:
        check(lib().seb_filter_flush(self._h))

    def encode(self) -> bytes:
        size = lib().seb_filter_encoded_size(self._h)
        out = np.zeros(size, dtype=np.uint8)
        check(lib().seb_filter_encode(self._h, out.ctypes.data, size))
        return out.tobytes()


# ------------------------------------------- filter registry + batched LSM lookup (§8f) ----

class Registry:
    """Device-resident SSTable filter registry (seb_registry): put the bloom block of each open
    SSTable with its level and key range; multiget() returns, per key, a u64 mask of the slots
    LSM.Get would consult whose filter may contain the key (lsm/lsm.go:168-198)."""

    def __init__(self, device: int = 0):
        self._h = lib().seb_registry_new(device)
        if not self._h:
            raise SebError(-3, "seb_registry_new failed")

    def close(self):
        if getattr(self, "_h", None):
            lib().seb_registry_free(self._h)
            self._h = None

    __del__ = close

    def put(self, file_num: int, level: int, bloom_block: bytes, min_key: bytes, max_key: bytes) -> int:
        return check(lib().seb_registry_put(self._h, file_num, level, bloom_block, len(bloom_block), min_key,
                                            len(min_key), max_key, len(max_key)))

    def remove(self, file_num: int) -> None:
        check(lib().seb_registry_remove(self._h, file_num))

    MAX_FILES = 4096  # kRegMaxFiles (u16 slot ids)

    def slots(self) -> dict[int, tuple[int, int]]:
        cap = self.MAX_FILES
        fn = (_u64 * cap)()
        lv = (C.c_int32 * cap)()
        check(lib().seb_registry_slots(self._h, fn, lv, cap))
        return {s: (fn[s], lv[s]) for s in range(cap) if lv[s] >= 0}

    def max_candidates(self) -> int:
        """Longest Get walk: every L0 file plus one file per non-empty level 1..4."""
        return check(lib().seb_registry_max_candidates(self._h))

    def multiget_list(self, keys, cap: int | None = None) -> np.ndarray:
        """Per key, the slots of the files Get would consult whose filter may contain it, in
        visiting order, padded with 0xFFFF: an (n, cap) u16 array.  Any registry size."""
        kb = as_keys(keys)
        cap = max(self.max_candidates(), 1) if cap is None else cap
        out = np.zeros((max(kb.n, 1), cap), dtype=np.uint16)
        check(lib().seb_registry_multiget_list(self._h, kb.ref, out.ctypes.data, cap))
        return out[: kb.n]

    def multiget_list_dev(self, keys: "seb_keys", out, cap: int, stream=None) -> None:
        check(lib().seb_registry_multiget_list_dev(self._h, C.byref(keys), out.data_ptr(), cap, _stream(stream)))

    def multiget_files(self, keys, cap: int = 1) -> np.ndarray:
        """Per key, the file numbers Get would read whose filter may contain it, in visiting order,
        padded with 2^64-1: an (n, cap) u64 array from one atomic registry call (retried while the
        registry grows between sizing and lookup)."""
        kb = as_keys(keys)
        need = _u32()
        while True:
            out = np.zeros((max(kb.n, 1), cap), dtype=np.uint64)
            rc = lib().seb_registry_multiget_files(self._h, kb.ref, out.ctypes.data, cap, C.byref(need))
            if rc == -4 and need.value > cap:
                cap = need.value
                continue
            check(rc)
            return out[: kb.n]

    def multiget(self, keys) -> np.ndarray:
        kb = as_keys(keys)
        out = np.zeros(max(kb.n, 1), dtype=np.uint64)
        check(lib().seb_registry_multiget(self._h, kb.ref, out.ctypes.data))
        return out[: kb.n]

    def multiget_dev(self, keys: "seb_keys", out, stream=None) -> None:
        check(lib().seb_registry_multiget_dev(self._h, C.byref(keys), out.data_ptr(), _stream(stream)))


# ------------------------------------------------- device-resident API (torch tensors) ----

def workspace_bytes() -> int:
    """Bytes of library-owned scratch (per device and stream) currently held."""
    return int(lib().seb_workspace_bytes())


def workspace_release() -> None:
    """Synchronise the streams that own library scratch and free it."""
    check(lib().seb_workspace_release())


def _stream(stream=None) -> int:
    import torch
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


class Timer:
    """A HIP timing event without the system-scope completion fence (seb_timer_*): recording it
    between two kernels does not flush L2 the way torch.cuda.Event does."""

    def __init__(self):
        self._e = _vp()
        check(lib().seb_timer_create(C.byref(self._e)))

    def record(self, stream=None) -> None:
        check(lib().seb_timer_record(self._e, _stream(stream)))

    def elapsed_ms(self, end: "Timer") -> float:
        ms = C.c_float()
        check(lib().seb_timer_elapsed_ms(self._e, end._e, C.byref(ms)))
        return ms.value

    def __del__(self):
        if getattr(self, "_e", None) and _lib is not None:
            _lib.seb_timer_destroy(self._e)
            self._e = None


def dev_keys(data, offsets=None, n: int | None = None, stride: int = 16) -> seb_keys:
    """seb_keys over device tensors (uint8 data; optional uint64/int64 offsets of n+1).
    The returned struct keeps the tensors alive (the C struct holds raw device pointers)."""
    if offsets is not None:
        kd = seb_keys(data.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, 0, 0)
    else:
        nn = n if n is not None else data.numel() // stride
        kd = seb_keys(data.data_ptr(), None, nn, stride, 0)
    kd._keep = (data, offsets)
    return kd


def dev_or_slices(slices, num_slices: int, out, stream=None) -> None:
    """out = OR of the num_slices equal slices of `slices` (int32 tensors; the sharded build's
    reduction after the all-to-all)."""
    sw = out.numel()
    if slices.numel() < num_slices * sw:
        raise ValueError("slices holds fewer than num_slices * out.numel() words")
    check(lib().seb_dev_or_slices(slices.data_ptr(), num_slices, sw, out.data_ptr(), _stream(stream)))


def dev_clear(words, m: int, stream=None) -> None:
    check(lib().seb_dev_clear(words.data_ptr(), m, _stream(stream)))


def dev_build(keys: seb_keys, words, m: int, k: int, stream=None) -> None:
    check(lib().seb_dev_build(C.byref(keys), words.data_ptr(), m, k, _stream(stream)))


def dev_build_fresh(keys: seb_keys, words, m: int, k: int, stream=None) -> None:
    """A new filter from the keys: `words` need not be cleared (every word is written)."""
    check(lib().seb_dev_build_fresh(C.byref(keys), words.data_ptr(), m, k, _stream(stream)))


def dev_build_workspace_size(n: int, m: int, k: int) -> int:
    return lib().seb_dev_build_workspace_size(n, m, k)


def dev_build_ws(keys: seb_keys, words, m: int, k: int, ws, stream=None) -> None:
    check(lib().seb_dev_build_ws(C.byref(keys), words.data_ptr(), m, k, ws.data_ptr() if ws is not None else None,
                                 ws.numel() * ws.element_size() if ws is not None else 0, _stream(stream)))


def dev_probe(keys: seb_keys, words, m: int, k: int, out, stream=None) -> None:
    check(lib().seb_dev_probe(C.byref(keys), words.data_ptr(), m, k, out.data_ptr(), _stream(stream)))


def dev_pack_residues(keys: seb_keys, m: int, k: int, packed, stream=None) -> None:
    """8-byte packed residues per key (k == 7, m < 2^29) for a batch shared by same-size filters."""
    check(lib().seb_dev_pack_residues(C.byref(keys), m, k, packed.data_ptr(), _stream(stream)))


def dev_probe_packed(packed, n: int, words, m: int, k: int, out, stream=None) -> None:
    check(lib().seb_dev_probe_packed(packed.data_ptr(), n, words.data_ptr(), m, k, out.data_ptr(), _stream(stream)))


def dev_probe_emit_packed(keys: seb_keys, words, m: int, k: int, out, packed, stream=None) -> None:
    """dev_probe that also writes the batch's packed residues (the broadcast root's probe)."""
    check(lib().seb_dev_probe_emit_packed(C.byref(keys), words.data_ptr(), m, k, out.data_ptr(), packed.data_ptr(),
                                          _stream(stream)))


def dev_probe_multi_packed(packed, n: int, filters: list[tuple[object, int, int]], mask, stream=None) -> None:
    """dev_probe_multi over packed residues (filters of one (m, k); k == 7, m < 2^29)."""
    refs = (seb_filter_ref * len(filters))(*[seb_filter_ref(w.data_ptr(), m, k, 0) for w, m, k in filters])
    check(lib().seb_dev_probe_multi_packed(packed.data_ptr(), n, refs, len(filters), mask.data_ptr(),
                                           mask.element_size(), _stream(stream)))


PACK6_BITS = 21      # narrow packed residues: m < 2^21 (include/seb_bloom.h)
PACK6_BLOCK = 384    # bytes per 64-key block (64 u32 low words + 64 u16 high halves)


def packed6_bytes(n: int) -> int:
    """Bytes of an n-key batch of 6-byte packed residues (whole 64-key blocks)."""
    return -(-n // 64) * PACK6_BLOCK


def pack6_supported(m: int, k: int) -> bool:
    return k == 7 and 0 < m < (1 << PACK6_BITS)


def dev_pack_residues6(keys: seb_keys, m: int, k: int, packed6, stream=None) -> None:
    """6-byte packed residues per key in 64-key blocks (k == 7, m < 2^21): a quarter fewer bytes
    than dev_pack_residues for the batch a compaction-sized filter set shares."""
    check(lib().seb_dev_pack_residues6(C.byref(keys), m, k, packed6.data_ptr(), _stream(stream)))


def dev_probe_multi_packed6(packed6, n: int, filters: list[tuple[object, int, int]], mask, stream=None) -> None:
    """dev_probe_multi over 6-byte packed residues (filters of one (m, k); k == 7, m < 2^21)."""
    refs = (seb_filter_ref * len(filters))(*[seb_filter_ref(w.data_ptr(), m, k, 0) for w, m, k in filters])
    check(lib().seb_dev_probe_multi_packed6(packed6.data_ptr(), n, refs, len(filters), mask.data_ptr(),
                                            mask.element_size(), _stream(stream)))


def dev_probe_multi(keys: seb_keys, filters: list[tuple[object, int, int]], mask, stream=None) -> None:
    refs = (seb_filter_ref * len(filters))(*[seb_filter_ref(w.data_ptr(), m, k, 0) for w, m, k in filters])
    check(lib().seb_dev_probe_multi(C.byref(keys), refs, len(filters), mask.data_ptr(), mask.element_size(),
                                    _stream(stream)))


def dev_build_many(keys: seb_keys, key_begin: list[int], filters: list[tuple[object, int, int]],
                   stream=None) -> None:
    kbeg = (_u64 * len(key_begin))(*key_begin)
    refs = (seb_filter_ref * len(filters))(*[seb_filter_ref(w.data_ptr(), m, k, 0) for w, m, k in filters])
    check(lib().seb_dev_build_many(C.byref(keys), kbeg, refs, len(filters), _stream(stream)))


def new_words(m: int, device="cuda"):
    """Zeroed device word array for an m-bit filter (torch uint32 view, 16-B padded)."""
    import torch
    return torch.zeros(max(words_bytes(m) // 4, 4), dtype=torch.int32, device=device)


def words_to_bits(words, m: int) -> np.ndarray:
    """First ceil(m/8) bytes of a device word array = the reference's bits slice."""
    return words.cpu().numpy().view(np.uint8)[: (m + 7) // 8].copy()


# ------------------------------------------------ shard routing + WAL checksums (§8(f) row 4)

def _ptr(t):
    return t.data_ptr() if t is not None else None


def dev_shard_route(keys: seb_keys, shard_bits: int, shard=None, hash=None, stream=None) -> None:
    """shard[i] = FNV-1a32(key i) & (2^bits - 1) (hashindex/shard.go:47-52); hash[i] = the hash."""
    check(lib().seb_dev_shard_route(C.byref(keys), shard_bits, _ptr(shard), _ptr(hash), _stream(stream)))


def dev_shard_partition_workspace_size(n: int, shard_bits: int) -> int:
    return lib().seb_dev_shard_partition_workspace_size(n, shard_bits)


def dev_shard_partition(keys: seb_keys, shard_bits: int, perm, shard_begin=None, shard=None, ws=None,
                        stream=None) -> None:
    """Stable partition by shard (hashindex/shard.go:104-122): perm grouped by shard, input order
    inside a shard; shard_begin (2^bits + 1 u64) delimits the groups."""
    import torch
    if ws is None:
        ws = torch.empty(max(dev_shard_partition_workspace_size(keys.n, shard_bits), 1), dtype=torch.uint8,
                         device=perm.device)
    check(lib().seb_dev_shard_partition(C.byref(keys), shard_bits, _ptr(perm), _ptr(shard_begin), _ptr(shard),
                                        ws.data_ptr(), ws.numel(), _stream(stream)))


def dev_wal_crc(data, rec_off, mode: int = WAL_CRC, crc=None, ok=None, stream=None) -> None:
    """CRC32-IEEE of WAL records data[rec_off[i]+4, rec_off[i+1]) (lsm/wal.go:59); SEAL stores it,
    VERIFY sets ok[i] (framing + stored CRC, lsm/wal.go:123-133)."""
    check(lib().seb_dev_wal_crc(data.data_ptr(), rec_off.data_ptr(), rec_off.numel() - 1, mode, _ptr(crc), _ptr(ok),
                                _stream(stream)))


def wal_scan(image: bytes | np.ndarray) -> tuple[np.ndarray, int]:
    """ReadAll's framing walk (lsm/wal.go:98-121) on the host: (offsets[0..n], status)."""
    buf = np.frombuffer(image, np.uint8) if isinstance(image, (bytes, bytearray)) else image
    cap = buf.size // 21 + 2
    off = np.zeros(cap, np.uint64)
    n = _u64(0)
    rc = lib().seb_wal_scan(buf.ctypes.data, buf.size, off.ctypes.data, cap, C.byref(n))
    if rc not in (0, -5):
        check(rc)
    return off[: n.value + 1].copy(), rc
