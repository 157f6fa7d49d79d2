"""SURVEY.md §8(f) row 4 on the CPU: the oracle for hash-index shard routing (FNV-1a 32,
hashindex/shard.go:47-52,104-122) and WAL record checksums (CRC32-IEEE, lsm/wal.go:31-62,98-133)
pinned to published known answers and to zlib; the WAL image generator; the C-ABI's host-side
framing walk (seb_wal_scan, no GPU)."""
from __future__ import annotations

import zlib

import numpy as np
import pytest

from oracle import codec_c as cc
import keygen as kg

FNV32A_KATS = [(b"", 0x811C9DC5), (b"a", 0xE40C292C), (b"ab", 0x4D2505CA), (b"abc", 0x1A47E90B),
               (b"foobar", 0xBF9CF968)]


@pytest.mark.parametrize("key,want", FNV32A_KATS)
def test_fnv32a_known_answers(key, want):
    assert cc.fnv32a(key) == want


def test_fnv32a_batch_layouts():
    rng = np.random.default_rng(3)
    keys = [bytes(rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8)) for _ in range(500)]
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    data = np.frombuffer(b"".join(keys), np.uint8)
    got = cc.fnv32a_batch(data, len(keys), offsets=off)
    assert [int(x) for x in got] == [cc.fnv32a(k) for k in keys]
    fixed = kg.key16(np.arange(300))
    assert np.array_equal(cc.fnv32a_batch(fixed, 300, stride=16),
                          [cc.fnv32a(fixed[i].tobytes()) for i in range(300)])


def test_crc32_known_answer_and_zlib():
    assert cc.crc32_ieee(b"123456789") == 0xCBF43926
    assert cc.crc32_ieee(b"") == 0
    rng = np.random.default_rng(4)
    for ln in [1, 2, 3, 4, 5, 7, 8, 63, 64, 65, 1000, 4099]:
        b = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        assert cc.crc32_ieee(b) == zlib.crc32(b)


@pytest.mark.parametrize("bits", [0, 1, 8, 12])
def test_partition_is_stable_grouping(bits):
    rng = np.random.default_rng(bits)
    shard = rng.integers(0, 1 << bits, 20000).astype(np.uint16)
    perm, begin = cc.partition(shard, bits)
    assert np.array_equal(perm, np.argsort(shard, kind="stable"))
    assert np.array_equal(begin, np.searchsorted(np.sort(shard), np.arange((1 << bits) + 1), side="left"))


def test_wal_image_layout_and_oracle():
    img, off = kg.wal_image(1000, value_size=100, delete_every=16)
    assert off[-1] == img.size and np.all(np.diff(off) == np.where(np.arange(1000) % 16 == 15, 37, 137))
    r = img[int(off[5]):int(off[6])].tobytes()  # record 5: seq 6, key16(5), live
    assert int.from_bytes(r[4:12], "little") == 6 and r[12:16] == (16).to_bytes(4, "little")
    assert r[16:20] == (100).to_bytes(4, "little") and r[20] == 0 and r[21:37] == kg.key16_bytes(5)
    assert int.from_bytes(r[:4], "little") == zlib.crc32(r[4:])
    d = img[int(off[15]):int(off[16])].tobytes()  # record 15: a Delete, empty value
    assert d[20] == 1 and d[16:20] == b"\0\0\0\0" and len(d) == 37
    crc, ok = cc.wal_crc(img, off)
    assert ok.all()
    assert np.array_equal(crc, img[off[:-1].astype(np.int64)[:, None] + np.arange(4)].copy().view("<u4").ravel())


def test_wal_oracle_flags_corruption():
    img, off = kg.wal_image(200, value_size=30)
    img = img.copy()
    st = off.astype(np.int64)
    img[st[3] + 40] ^= 1          # payload bit flip
    img[st[7]] ^= 0x80            # stored crc bit flip
    img[st[9] + 12] = 17          # keySize no longer matches the framing
    _, ok = cc.wal_crc(img, off)
    assert [i for i in range(200) if not ok[i]] == [3, 7, 9]
    short = off.copy()
    short[11] = short[10] + 20    # a 20-byte "record" cannot hold the header
    _, ok2 = cc.wal_crc(img, short[:12])
    assert ok2[10] == 0


def test_wal_scan_host_framing(seb):
    img, off = kg.wal_image(500, value_size=77, delete_every=5)
    got, rc = seb.wal_scan(img)
    assert rc == 0 and np.array_equal(got, off)
    got, rc = seb.wal_scan(img[: int(off[321]) + 10])  # truncated header
    assert rc == -5 and np.array_equal(got, off[:322])
    got, rc = seb.wal_scan(img[: int(off[100]) + 30])  # header complete, payload truncated
    assert rc == -5 and np.array_equal(got, off[:101])
    got, rc = seb.wal_scan(b"")
    assert rc == 0 and got.tolist() == [0]
