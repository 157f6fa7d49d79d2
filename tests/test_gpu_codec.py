"""GPU parity for SURVEY.md §8(f) row 4 through the C ABI: shard routing (FNV-1a 32,
hashindex/shard.go:47-52), the stable shard partition (UpdateBatch's distribution,
hashindex/shard.go:104-122) and WAL record CRC32-IEEE compute / seal / verify (lsm/wal.go:31-62,
98-133), each against oracle/codec_oracle.c element for element."""
import zlib

import numpy as np
import pytest

from oracle import codec_c as cc
import keygen as kg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch


def to_dev(torch, arr):
    return torch.from_numpy(np.array(arr, copy=True)).cuda()


def _varlen(rng, n, maxlen=90):
    keys = [bytes(rng.integers(0, 256, int(rng.integers(0, maxlen)), dtype=np.uint8)) for _ in range(n)]
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    return np.frombuffer(b"".join(keys) or b"\0", np.uint8), off


@pytest.mark.parametrize("layout", ["fixed16", "stride13", "varlen", "empty_keys"])
@pytest.mark.parametrize("bits", [0, 8, 16])
def test_shard_route_matches_oracle(seb, torch_cuda, layout, bits):
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 5003
    if layout == "fixed16":
        data = kg.key16(np.arange(n))
        kd = seb.dev_keys(to_dev(torch, data), n=n, stride=16)
        want = cc.fnv32a_batch(data, n, stride=16)
    elif layout == "stride13":
        data = rng.integers(0, 256, (n, 13), dtype=np.uint8)
        kd = seb.dev_keys(to_dev(torch, data.ravel()), n=n, stride=13)
        want = cc.fnv32a_batch(data, n, stride=13)
    elif layout == "varlen":
        data, off = _varlen(rng, n)
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off.view(np.int64)))
        want = cc.fnv32a_batch(data, n, offsets=off)
    else:
        data = np.zeros(1, np.uint8)
        off = np.zeros(n + 1, np.uint64)
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off.view(np.int64)))
        want = np.full(n, 0x811C9DC5, np.uint32)
    shard = torch.zeros(n, dtype=torch.int16, device="cuda")
    h = torch.zeros(n, dtype=torch.int32, device="cuda")
    seb.dev_shard_route(kd, bits, shard, h)
    torch.cuda.synchronize()
    assert np.array_equal(h.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(shard.cpu().numpy().view(np.uint16), (want & ((1 << bits) - 1)).astype(np.uint16))


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 100_003])
@pytest.mark.parametrize("bits", [0, 1, 8, 12])
def test_shard_partition_matches_oracle(seb, torch_cuda, n, bits):
    torch = torch_cuda
    data = kg.key16(np.arange(n)) if n else np.zeros((1, 16), np.uint8)
    kd = seb.dev_keys(to_dev(torch, data), n=n, stride=16)
    perm = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    begin = torch.zeros((1 << bits) + 1, dtype=torch.int64, device="cuda")
    shard = torch.zeros(max(n, 1), dtype=torch.int16, device="cuda")
    seb.dev_shard_partition(kd, bits, perm, begin, shard)
    torch.cuda.synchronize()
    want_shard = (cc.fnv32a_batch(data, n, stride=16) & ((1 << bits) - 1)).astype(np.uint16)
    want_perm, want_begin = cc.partition(want_shard, bits)
    assert np.array_equal(begin.cpu().numpy().view(np.uint64), want_begin)
    if n:
        assert np.array_equal(perm.cpu().numpy().view(np.uint32)[:n], want_perm)
        assert np.array_equal(shard.cpu().numpy().view(np.uint16)[:n], want_shard)


def test_shard_partition_skewed_and_varlen(seb, torch_cuda):
    """One shard holding almost every key (identical keys) and variable-length keys."""
    torch = torch_cuda
    rng = np.random.default_rng(12)
    keys = [b"same-key"] * 9000 + [bytes(rng.integers(0, 256, 20, dtype=np.uint8)) for _ in range(1000)]
    rng.shuffle(keys)
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    data = np.frombuffer(b"".join(keys), np.uint8)
    kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off.view(np.int64)))
    n = len(keys)
    perm = torch.zeros(n, dtype=torch.int32, device="cuda")
    begin = torch.zeros(257, dtype=torch.int64, device="cuda")
    seb.dev_shard_partition(kd, 8, perm, begin)
    torch.cuda.synchronize()
    want_perm, want_begin = cc.partition((cc.fnv32a_batch(data, n, offsets=off) & 255).astype(np.uint16), 8)
    assert np.array_equal(perm.cpu().numpy().view(np.uint32), want_perm)
    assert np.array_equal(begin.cpu().numpy().view(np.uint64), want_begin)


def _wal_varied(rng, n):
    """Records with value sizes 0..5000 (small, unaligned, large) in Append's layout."""
    recs = []
    for i in range(n):
        key = bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
        vs = int(rng.choice([0, 1, 3, 7, 100, 1000, 5000]))
        val = bytes(rng.integers(0, 256, vs, dtype=np.uint8))
        body = (i + 1).to_bytes(8, "little") + len(key).to_bytes(4, "little") + vs.to_bytes(4, "little") + \
            bytes([i % 3 == 0]) + key + val
        recs.append(zlib.crc32(body).to_bytes(4, "little") + body)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


@pytest.mark.parametrize("kind", ["bench_layout", "varied"])
def test_wal_crc_seal_verify(seb, torch_cuda, kind):
    torch = torch_cuda
    rng = np.random.default_rng(13)
    img, off = kg.wal_image(20000, value_size=100) if kind == "bench_layout" else _wal_varied(rng, 3000)
    n = off.size - 1
    want_crc, want_ok = cc.wal_crc(img, off)
    assert want_ok.all()
    d_img, d_off = to_dev(torch, img), to_dev(torch, off.view(np.int64))
    crc = torch.zeros(n, dtype=torch.int32, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    seb.dev_wal_crc(d_img, d_off, seb.WAL_VERIFY, crc, ok)
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), want_crc)
    assert ok.cpu().numpy().all()
    # seal: clear every CRC field, seal on the device, get the original image back
    blank = img.copy()
    st = off[:-1].astype(np.int64)
    for b in range(4):
        blank[st + b] = 0
    d_blank = to_dev(torch, blank)
    seb.dev_wal_crc(d_blank, d_off, seb.WAL_SEAL)
    torch.cuda.synchronize()
    assert np.array_equal(d_blank.cpu().numpy(), img)


def test_wal_verify_flags_exactly_the_corrupt_records(seb, torch_cuda):
    torch = torch_cuda
    img, off = kg.wal_image(5000, value_size=100)
    img = img.copy()
    st = off.astype(np.int64)
    bad = {17: 40, 999: 0, 2500: 12, 4999: 136}  # payload, crc field, keySize, last byte of the image
    for r, o in bad.items():
        img[st[r] + o] ^= 0x21
    short = off.copy()
    want_crc, want_ok = cc.wal_crc(img, short)
    assert sorted(np.nonzero(want_ok == 0)[0].tolist()) == sorted(bad)
    crc = torch.zeros(5000, dtype=torch.int32, device="cuda")
    ok = torch.zeros(5000, dtype=torch.uint8, device="cuda")
    seb.dev_wal_crc(to_dev(torch, img), to_dev(torch, short.view(np.int64)), seb.WAL_VERIFY, crc, ok)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), want_ok)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), want_crc)
    # framing violations: a record shorter than its header, and one of 0..3 bytes
    odd = np.array([0, 20, 20, 23, 160], np.uint64)
    ok2 = torch.zeros(4, dtype=torch.uint8, device="cuda")
    crc2 = torch.zeros(4, dtype=torch.int32, device="cuda")
    seb.dev_wal_crc(to_dev(torch, img[:200]), to_dev(torch, odd.view(np.int64)), seb.WAL_VERIFY, crc2, ok2)
    torch.cuda.synchronize()
    w_crc, w_ok = cc.wal_crc(img[:200], odd)
    assert np.array_equal(ok2.cpu().numpy(), w_ok) and not w_ok.any()
    assert np.array_equal(crc2.cpu().numpy().view(np.uint32), w_crc)
