"""numpy restatement of the reference bloom filter — TEST INFRASTRUCTURE ONLY.

Independent of oracle/bloom_oracle.c (different language, vectorised over keys) so that the
two restatements can check each other.  Used in this container to generate the golden
fixtures under tests/golden/ and by the CPU test suite.  Never imported by the shipped
library (storage-engines_amd/).

Reference (intellect4all/storage-engines, Go; read as text):
  lsm/bloom.go:19-41  sizing            -> params()
  lsm/bloom.go:44-54  hash1/hash2       -> fnv1a64 / fnv1_64 (Go stdlib hash/fnv, go1.25.5)
  lsm/bloom.go:58-67  getHashes         -> positions()
  lsm/bloom.go:70-77  Add               -> build()
  lsm/bloom.go:82-92  MayContain        -> probe()
  lsm/bloom.go:96-120 Encode / Decode   -> encode() / decode()
Sizing uses Go's portable math.Log algorithm (src/math/log.go), restated in pure Python
floats (IEEE binary64, no FMA), and the const-folded Ln2*Ln2 = 0.48045301391820144.
"""
from __future__ import annotations

import math
import struct

import numpy as np

FNV_OFFSET = np.uint64(0xCBF29CE484222325)
FNV_PRIME = np.uint64(0x100000001B3)
LN2 = 0.6931471805599453
LN2SQ = 0.48045301391820144


def go_log(x: float) -> float:
    """Go math.Log (src/math/log.go, portable path)."""
    Ln2Hi = 6.93147180369123816490e-01
    Ln2Lo = 1.90821492927058770002e-10
    L1 = 6.666666666666735130e-01
    L2 = 3.999999999940941908e-01
    L3 = 2.857142874366239149e-01
    L4 = 2.222219843214978396e-01
    L5 = 1.818357216161805012e-01
    L6 = 1.531383769920937332e-01
    L7 = 1.479819860511658591e-01
    if math.isnan(x) or x == math.inf:
        return x
    if x < 0:
        return math.nan
    if x == 0:
        return -math.inf
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f)


def params(n: int, p: float) -> tuple[int, int]:
    """NewBloomFilter sizing (lsm/bloom.go:22-31) -> (numBits, numHashes)."""
    if n < 0 or not (0.0 < p < 1.0):
        raise ValueError("outside the reference's defined range")
    m = math.ceil(-float(n) * go_log(p) / LN2SQ)
    if n == 0:
        k = 0  # uint32(NaN)
    else:
        k = math.ceil(float(m) / float(n) * LN2)
    if k == 0:
        k = 1
    return int(m), int(k)


def num_bytes(m: int) -> int:
    return (m + 7) // 8


def fnv_fixed(keys: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """FNV-1a and FNV-1 64 over each row of a (n, L) uint8 array."""
    n, L = keys.shape
    h1 = np.full(n, FNV_OFFSET, dtype=np.uint64)
    h2 = np.full(n, FNV_OFFSET, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(L):
            b = keys[:, j].astype(np.uint64)
            h1 = (h1 ^ b) * FNV_PRIME
            h2 = (h2 * FNV_PRIME) ^ b
    return h1, h2


def fnv_varlen(data: np.ndarray, offsets: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """FNV-1a / FNV-1 over keys data[offsets[i]:offsets[i+1]] (vectorised by byte index)."""
    offsets = offsets.astype(np.int64)
    lens = offsets[1:] - offsets[:-1]
    n = lens.shape[0]
    h1 = np.full(n, FNV_OFFSET, dtype=np.uint64)
    h2 = np.full(n, FNV_OFFSET, dtype=np.uint64)
    maxlen = int(lens.max()) if n else 0
    with np.errstate(over="ignore"):
        for j in range(maxlen):
            idx = np.nonzero(lens > j)[0]
            b = data[offsets[idx] + j].astype(np.uint64)
            h1[idx] = (h1[idx] ^ b) * FNV_PRIME
            h2[idx] = (h2[idx] * FNV_PRIME) ^ b
    return h1, h2


def fnv_bytes(key: bytes) -> tuple[int, int]:
    a = np.frombuffer(key, dtype=np.uint8).reshape(1, -1) if key else np.zeros((1, 0), np.uint8)
    h1, h2 = fnv_fixed(a)
    return int(h1[0]), int(h2[0])


def positions(h1: np.ndarray, h2: np.ndarray, m: int, k: int) -> np.ndarray:
    """(n, k) bit positions: (h1 + i*h2) mod 2^64, then mod m (lsm/bloom.go:63-65)."""
    mm = np.uint64(m)
    out = np.empty((h1.shape[0], k), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(k):
            out[:, i] = (h1 + np.uint64(i) * h2) % mm
    return out


def build(h1: np.ndarray, h2: np.ndarray, m: int, k: int, bits: np.ndarray | None = None) -> np.ndarray:
    bits = np.zeros(num_bytes(m), dtype=np.uint8) if bits is None else bits
    pos = positions(h1, h2, m, k).ravel()
    np.bitwise_or.at(bits, (pos >> np.uint64(3)).astype(np.int64),
                     (np.uint8(1) << (pos & np.uint64(7)).astype(np.uint8)))
    return bits


def probe(bits: np.ndarray, h1: np.ndarray, h2: np.ndarray, m: int, k: int) -> np.ndarray:
    pos = positions(h1, h2, m, k)
    byte = bits[(pos >> np.uint64(3)).astype(np.int64)]
    hit = (byte >> (pos & np.uint64(7)).astype(np.uint8)) & 1
    return np.all(hit == 1, axis=1).astype(np.uint8) if k else np.ones(h1.shape[0], np.uint8)


def encode(bits: np.ndarray, m: int, k: int) -> bytes:
    return struct.pack("<QI", m, k) + bits.tobytes()


def decode(data: bytes):
    if len(data) < 12:
        return None
    m, k = struct.unpack_from("<QI", data, 0)
    return m, k, np.frombuffer(data[12:], dtype=np.uint8).copy()
