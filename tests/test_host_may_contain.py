"""Single-key MayContain on the host copy ("a single-key MayContain stays on CPU";
VERDICT r02 item 3).  seb_filter_decode + seb_filter_may_contain touch no GPU, so these run in the
CPU suite: the product library's host path against the oracle (oracle/bloom_oracle.c), key by
key, on decoded filters (lsm/sstable.go:129 Decode, :206 MayContain; lsm/bloom.go:82-92)."""
import hashlib
import struct
import threading

import numpy as np
import pytest

import keygen as kg
from oracle import oracle_c as oc


def _block(m, k, bits):
    return struct.pack("<QI", m, k) + bits.tobytes()


def _probe_keys(n):
    return kg.key16(kg.probe_indices(n))


@pytest.mark.parametrize("n", [1, 7, 1000, 5000, 100_000])
def test_single_key_matches_oracle_on_golden(seb, golden, n):
    m, k = seb.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    block = _block(m, k, bits)
    row = {r["n"]: r for r in golden["fixed16"] if r["p"] == 0.01}[n]
    assert hashlib.sha256(block).hexdigest() == row["encode_sha256"]
    pk = _probe_keys(n)
    ref = oc.probe(bits, m, k, pk, n, stride=16)
    f = seb.BloomFilter.decode(block)
    try:
        got = np.array([f.may_contain(pk[i].tobytes()) for i in range(n)], dtype=np.uint8)
    finally:
        f.close()
    assert np.array_equal(got, ref)
    assert hashlib.sha256(got.tobytes()).hexdigest() == row["probe_sha256"]
    assert int(got.sum()) == row["probe_positives"]
    assert got[0::2].all()  # no false negatives


@pytest.mark.parametrize("m,k", [(1, 1), (2, 3), (10, 7), (64, 7), (9586, 1), (9586, 30), (958_506, 7),
                                 ((1 << 31) + 11, 7), ((1 << 32) + 5, 7)])
def test_single_key_modulus_and_k_edges(seb, m, k):
    rng = np.random.default_rng(m ^ k)
    n_build = 2000
    keys = rng.integers(0, 256, size=(2 * n_build, 24), dtype=np.uint8)
    bits = oc.build(m, k, keys[:n_build], n_build, stride=24)
    ref = oc.probe(bits, m, k, keys, 2 * n_build, stride=24)
    f = seb.BloomFilter.decode(_block(m, k, bits))
    try:
        got = np.array([f.may_contain(keys[i].tobytes()) for i in range(2 * n_build)], dtype=np.uint8)
        # each built key's own positions, as the oracle computes them
        for i in range(0, n_build, 97):
            assert all(bits[p >> 3] >> (p & 7) & 1 for p in oc.positions(keys[i].tobytes(), m, k))
    finally:
        f.close()
    assert np.array_equal(got, ref)
    assert got[:n_build].all()


def test_single_key_varlen_and_empty_keys(seb):
    n = 3000
    data, off = kg.varlen_keys(np.arange(2 * n))
    m, k = seb.params(n, 0.01)
    bits = oc.build(m, k, data, n, offsets=off[: n + 1])
    ref = oc.probe(bits, m, k, data, 2 * n, offsets=off)
    f = seb.BloomFilter.decode(_block(m, k, bits))
    try:
        got = np.array([f.may_contain(data[off[i]:off[i + 1]].tobytes()) for i in range(2 * n)], dtype=np.uint8)
        empty = f.may_contain(b"")
    finally:
        f.close()
    assert np.array_equal(got, ref)
    e_ref = all(bits[p >> 3] >> (p & 7) & 1 for p in oc.positions(b"", m, k))
    assert empty == e_ref


def test_k_zero_and_empty_filter(seb):
    # numHashes 0: the reference's loop has no positions and returns true
    f = seb.BloomFilter.decode(_block(64, 0, np.zeros(8, np.uint8)))
    assert f.may_contain(b"anything")
    f.close()
    # a fresh filter with no Add answers false, with no device involved
    g = seb.BloomFilter(1000, 0.01)
    assert not g.may_contain(b"user0000000001xy")
    g.close()


def test_short_decoded_bits_error(seb):
    f = seb.BloomFilter.decode(_block(1000, 7, np.zeros(10, np.uint8)))
    with pytest.raises(seb.SebError):
        f.may_contain(b"key")
    f.close()


def test_concurrent_readers_on_one_filter(seb):
    """Many threads call MayContain on one decoded filter at once (lsm/lsm.go:166: Get holds no
    lock across the SSTable loop); ctypes drops the GIL for each call."""
    n = 50_000
    m, k = seb.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    pk = _probe_keys(n)
    ref = oc.probe(bits, m, k, pk, n, stride=16)
    f = seb.BloomFilter.decode(_block(m, k, bits))
    keys = [pk[i].tobytes() for i in range(n)]
    results = [None] * 8

    def reader(t):
        out = np.zeros(n, np.uint8)
        for i in range(t, n + t):
            j = i % n
            out[j] = f.may_contain(keys[j])
        results[t] = out

    threads = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    f.close()
    for r in results:
        assert np.array_equal(r, ref)
