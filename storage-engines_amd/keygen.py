"""Synthetic key batches for the bloom path (workload generator, numpy, host side).

key16(i) is the reference's benchmark key format at KeySize 16
(common/benchmark/keygen.go:89-109 formatKey): ASCII "user%010d" followed by the two
padding bytes byte(i) and byte(i+1) (padding < 8 bytes -> "sequential bytes" branch, :101-104).

Variable-length keys (BASELINE config C4): length 8+k, k in [0,248] drawn from the integer CDF in
keygen_zipf_cdf.json (the reference's Zipf(s=1.1, v=1), keygen.go:47, bounded); bytes 0-7 are
the key index little-endian (uniqueness), the rest a splitmix64 stream seeded with
12345 ^ (i * 0xD1B54A32D192ED03) (seed 12345: common/benchmark/compare.go:41).

Probe batches follow one rule everywhere: probe q is present (key(q)) when q is even and
absent (key(n + q)) when q is odd, for a filter built from key(0..n-1).
"""
from __future__ import annotations

import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_U64 = np.uint64
GOLDEN = _U64(0x9E3779B97F4A7C15)
PAYLOAD_MUL = _U64(0xD1B54A32D192ED03)
LEN_SEED = _U64(0x5EB10F1E5EED5EED)
KEY_SEED = _U64(12345)

with open(os.path.join(_HERE, "keygen_zipf_cdf.json")) as _f:
    _ZIPF = json.load(_f)
ZIPF_CDF = np.array(_ZIPF["cdf_u32"], dtype=np.uint64)
MIN_LEN = int(_ZIPF["min_len"])


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of (x + golden)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + GOLDEN
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
        return z ^ (z >> _U64(31))


def key16(idx: np.ndarray) -> np.ndarray:
    """(n, 16) uint8 array of reference-format keys for the given indices (0 <= i < 1e10)."""
    idx = np.asarray(idx, dtype=np.int64)
    n = idx.shape[0]
    out = np.empty((n, 16), dtype=np.uint8)
    out[:, 0:4] = np.frombuffer(b"user", dtype=np.uint8)
    v = idx.copy()
    for d in range(9, -1, -1):
        out[:, 4 + d] = (v % 10 + 48).astype(np.uint8)
        v //= 10
    out[:, 14] = (idx & 0xFF).astype(np.uint8)
    out[:, 15] = ((idx + 1) & 0xFF).astype(np.uint8)
    return out


def key16_bytes(i: int) -> bytes:
    return b"user%010d" % i + bytes([i & 0xFF, (i + 1) & 0xFF])


def probe_indices(n: int, q: np.ndarray | None = None, count: int | None = None) -> np.ndarray:
    """Key indices of the standard probe batch: even q -> q (present), odd q -> n + q (absent)."""
    if q is None:
        q = np.arange(n if count is None else count, dtype=np.int64)
    q = np.asarray(q, dtype=np.int64)
    return np.where(q % 2 == 0, q, n + q)


def varlen_lengths(idx: np.ndarray) -> np.ndarray:
    u = splitmix64(np.asarray(idx, dtype=np.uint64) ^ LEN_SEED) >> _U64(32)
    k = np.searchsorted(ZIPF_CDF, u, side="right")
    return (MIN_LEN + k).astype(np.int64)


def varlen_keys(idx: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Packed bytes and (n+1) uint64 prefix offsets of the C4 variable-length keys."""
    idx = np.asarray(idx, dtype=np.int64)
    lens = varlen_lengths(idx)
    offsets = np.zeros(idx.shape[0] + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    total = int(offsets[-1])
    data = np.empty(total, dtype=np.uint8)
    starts = offsets[:-1].astype(np.int64)
    # bytes 0..7: LE index
    ib = idx.astype("<u8").view(np.uint8).reshape(-1, 8)
    for b in range(8):
        data[starts + b] = ib[:, b]
    with np.errstate(over="ignore"):
        seed = KEY_SEED ^ (idx.astype(np.uint64) * PAYLOAD_MUL)
    rest = lens - 8
    maxw = int((rest.max() + 7) // 8) if idx.shape[0] else 0
    for w in range(maxw):
        sel = np.nonzero(rest > 8 * w)[0]
        if sel.size == 0:
            break
        with np.errstate(over="ignore"):
            word = splitmix64(seed[sel] + _U64(w) * GOLDEN)
        wb = word.astype("<u8").view(np.uint8).reshape(-1, 8)
        base = starts[sel] + 8 + 8 * w
        nb = np.minimum(rest[sel] - 8 * w, 8)
        for b in range(8):
            ok = nb > b
            data[base[ok] + b] = wb[ok, b]
    return data, offsets


# ---- synthetic LSM layout for the registry / MultiGet config (bench.py --config lsm)
LSM_LAYOUT = {"l0_files": 4, "l0_keys": 250_000, "l1_files": 8, "l1_keys": 1_000_000, "l2_files": 16,
              "l2_keys": 500_000, "probes": 10_000_000, "seed": 12345}

# The same key span cut into compaction-sized files (lsm/compaction.go:253, 100K entries per output
# file): 244 files, beyond the u64 mask form, answered in the candidate-list form.
LSM_WIDE_LAYOUT = {"l0_files": 4, "l0_keys": 250_000, "l1_files": 80, "l1_keys": 100_000, "l2_files": 160,
                   "l2_keys": 50_000, "probes": 10_000_000, "seed": 12345}


def lsm_files(lay=LSM_LAYOUT):
    """Synthetic LSM for the registry/MultiGet config: keys key16(2i).  L1 file j holds
    i in [j*1M, (j+1)*1M), L2 file j holds i in [j*500K, (j+1)*500K) (non-overlapping, ranges in
    key order), L0 file f holds 250K random i (overlapping).  Returns [(level, file_num, i_array)]
    in registration order (L2 files registered in reverse to exercise the MinKey sort)."""
    rng = np.random.default_rng(lay["seed"])
    span = lay["l1_files"] * lay["l1_keys"]
    files = []
    for j in reversed(range(lay["l2_files"])):
        files.append((2, 2000 + j, np.arange(j * lay["l2_keys"], (j + 1) * lay["l2_keys"])))
    for j in range(lay["l1_files"]):
        files.append((1, 1000 + j, np.arange(j * lay["l1_keys"], (j + 1) * lay["l1_keys"])))
    for f in range(lay["l0_files"]):
        files.append((0, 100 + f, np.sort(rng.choice(span, lay["l0_keys"], replace=False))))
    return files


def lsm_probe_indices(lay=LSM_LAYOUT):
    """q even -> key16(2r) (present in L1, L2 and maybe L0), q odd -> key16(2r+1) (absent, inside
    the level ranges), r uniform in the key span."""
    rng = np.random.default_rng(lay["seed"] + 1)
    n = lay["probes"]
    r = rng.integers(0, lay["l1_files"] * lay["l1_keys"], n)
    return np.where(np.arange(n) % 2 == 0, 2 * r, 2 * r + 1)


# ---- synthetic WAL image for the checksum config (bench.py --config wal)
WAL_LAYOUT = {"records": 2_000_000, "value_size": 100, "delete_every": 16, "seed": 12345}


def wal_image(n: int, value_size: int = 100, delete_every: int = 16, seal: bool = True):
    """A WAL image of n records laid out as lsm/wal.go:31-62 Append writes them:
    [crc32][seq u64][keySize u32][valueSize u32][deleted u8][key][value], little-endian.
    Record i: key16(i), seq i+1; every delete_every-th record (i % delete_every == delete_every-1)
    is a Delete (lsm/lsm.go:209: value nil, deleted 1), the rest carry value_size splitmix64
    bytes (the reference benchmark's 100-B random values, common/benchmark/compare.go:37).
    seal=True fills the CRC field with zlib.crc32(record[4:]) (= Go's crc32.ChecksumIEEE).
    Returns (uint8 image, uint64 offsets[n+1])."""
    import zlib
    idx = np.arange(n, dtype=np.int64)
    deleted = (idx % delete_every == delete_every - 1) if delete_every else np.zeros(n, bool)
    vlen = np.where(deleted, 0, value_size).astype(np.int64)
    rlen = 21 + 16 + vlen
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(rlen, out=off[1:])
    img = np.zeros(int(off[-1]), np.uint8)
    st = off[:-1].astype(np.int64)
    seq = (idx + 1).astype("<u8").view(np.uint8).reshape(-1, 8)
    for b in range(8):
        img[st + 4 + b] = seq[:, b]
    img[st + 12] = 16
    vl = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    for b in range(4):
        img[st + 16 + b] = vl[:, b]
    img[st + 20] = deleted.astype(np.uint8)
    keys = key16(idx)
    for b in range(16):
        img[st + 21 + b] = keys[:, b]
    if value_size:
        live = np.nonzero(~deleted)[0]
        words = (value_size + 7) // 8
        with np.errstate(over="ignore"):
            seed = KEY_SEED ^ (live.astype(np.uint64) * PAYLOAD_MUL)
        for w in range(words):
            with np.errstate(over="ignore"):
                wb = splitmix64(seed + _U64(w) * GOLDEN).astype("<u8").view(np.uint8).reshape(-1, 8)
            for b in range(min(8, value_size - 8 * w)):
                img[st[live] + 37 + 8 * w + b] = wb[:, b]
    if seal:
        mv = memoryview(img)
        crc = np.fromiter((zlib.crc32(mv[int(s) + 4:int(e)]) for s, e in zip(off[:-1], off[1:])), np.uint32, n)
        cb = crc.astype("<u4").view(np.uint8).reshape(-1, 4)
        for b in range(4):
            img[st + b] = cb[:, b]
    return img, off
