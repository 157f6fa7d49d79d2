"""CPU: the oracle restatements against the committed golden vectors and each other.

The oracle is the checker of the GPU path, so it is pinned first: public FNV known answers
(Go hash/fnv, go1.25.5), NewBloomFilter sizing, full Encode() bytes for small n and the sha256
digests of SURVEY.md §8(c).  Reference: lsm/bloom.go:19-120.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import bloom_np as bn
from oracle import oracle_c as oc
import keygen as kg


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def test_fnv_known_answers(golden):
    for kat in golden["fnv_kats"]:
        key = bytes.fromhex(kat["key_hex"])
        h1a, h1 = oc.fnv(key)
        assert f"{h1a:016x}" == kat["fnv1a_64"]
        assert f"{h1:016x}" == kat["fnv1_64"]
        assert bn.fnv_bytes(key) == (h1a, h1)


def test_sizing_table(golden):
    for row in golden["sizing"]:
        assert oc.params(row["n"], row["p"]) == (row["m"], row["k"]), row
        assert bn.params(row["n"], row["p"]) == (row["m"], row["k"]), row


def test_sizing_docs_example():
    # lsm/README.md:296-298 derives "m ~ 9585 bits, k ~ 7" for n=1000; the code's Ceil gives 9586.
    assert oc.params(1000, 0.01) == (9586, 7)


def test_sizing_invalid():
    for n, p in [(-1, 0.01), (10, 0.0), (10, 1.0), (10, -0.5), (10, float("nan"))]:
        with pytest.raises(ValueError):
            oc.params(n, p)


def test_go_log_one_ulp_insensitive():
    # Go's portable math.Log(0.01) and glibc's log(0.01) differ by one ulp; the ceil in the
    # sizing formula absorbs it for every n <= 20M at p = 0.01 (scanned).
    import math
    n = np.arange(1, 2_000_001, dtype=np.float64)
    a = np.ceil(-n * oc.go_log(0.01) / bn.LN2SQ)
    b = np.ceil(-n * math.log(0.01) / bn.LN2SQ)
    assert np.array_equal(a, b)
    assert abs(oc.go_log(0.01) - math.log(0.01)) <= 2 * np.spacing(4.6)


def test_positions(golden):
    for e in golden["positions"]:
        assert oc.positions(bytes.fromhex(e["key_hex"]), e["m"], e["k"]) == e["pos"]


def test_key16_format():
    assert kg.key16_bytes(0) == b"user0000000000\x00\x01"
    assert kg.key16_bytes(256) == b"user0000000256\x00\x01"
    assert kg.key16(np.array([0, 257, 9999999])).tobytes() == (
        kg.key16_bytes(0) + kg.key16_bytes(257) + kg.key16_bytes(9999999))


@pytest.mark.parametrize("n", [1, 7, 1000, 5000])
def test_small_encode_bytes(golden, n):
    row = next(r for r in golden["fixed16"] if r["n"] == n and r["p"] == 0.01)
    m, k = oc.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    assert bn.encode(bits, m, k).hex() == row["encode_hex"]


@pytest.mark.parametrize("n,p", [(100000, 0.01), (100000, 0.001), (100000, 0.1), (100000, 0.5)])
def test_fixed_digests(golden, n, p):
    row = next(r for r in golden["fixed16"] if r["n"] == n and r["p"] == p)
    m, k = oc.params(n, p)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    ans = oc.probe(bits, m, k, kg.key16(kg.probe_indices(n)), n, stride=16)
    assert sha(ans.tobytes()) == row["probe_sha256"]
    assert ans[0::2].all()  # no false negatives: the only property the reference's tests pin


def test_full_10m_digest(golden):
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n = row["n"]
    m, k = oc.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16, threads=8)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]


def test_multithreaded_matches_scalar():
    n = 50000
    m, k = oc.params(n, 0.01)
    keys = kg.key16(np.arange(n))
    a = oc.build(m, k, keys, n, stride=16)
    b = oc.build(m, k, keys, n, stride=16, threads=4)
    assert np.array_equal(a, b)
    pk = kg.key16(kg.probe_indices(n))
    assert np.array_equal(oc.probe(a, m, k, pk, n, stride=16), oc.probe(a, m, k, pk, n, stride=16, threads=4))


@pytest.mark.parametrize("n", [1000, 100000])
def test_varlen_digests(golden, n):
    row = next(r for r in golden["varlen"] if r["n"] == n)
    data, off = kg.varlen_keys(np.arange(n))
    assert sha(data.tobytes()) == row["keys_sha256"]
    m, k = oc.params(n, 0.01)
    bits = oc.build(m, k, data, n, offsets=off)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    h1, h2 = bn.fnv_varlen(data, off)
    assert np.array_equal(bn.build(h1, h2, m, k), bits)


def test_varlen_length_distribution():
    lens = kg.varlen_lengths(np.arange(200000))
    assert lens.min() == 8 and lens.max() <= 256
    assert abs(lens.mean() - 39.95) < 0.6
    assert abs((lens == 8).mean() - 0.207) < 0.01


def test_multi_digest(golden):
    row = golden["multi"][0]
    nf, per, npr = row["filters"], row["keys_per_filter"], row["probes"]
    m, k = oc.params(per, 0.01)
    filters = [(oc.build(m, k, kg.key16(f * per + np.arange(per)), per, stride=16), m, k) for f in range(nf)]
    for (b, _, _), h in zip(filters, row["filter_sha256"]):
        assert sha(bn.encode(b, m, k)) == h
    q = np.arange(npr, dtype=np.int64)
    half = q // 2
    pk = kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q))
    mask = oc.probe_multi(filters, pk, npr, stride=16)
    assert sha(mask.astype("<u8").tobytes()) == row["mask_sha256"]


def test_decode_roundtrip_and_nil():
    n = 1000
    m, k = oc.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    enc = bn.encode(bits, m, k)
    mm, kk, bb = bn.decode(enc)
    assert (mm, kk) == (m, k) and np.array_equal(bb, bits)
    assert bn.decode(enc[:11]) is None  # lsm/bloom.go:106-108


def test_bench_golden_digests_match_fixtures():
    """bench.py checks its runs against digests it carries inline (the GPU box has no generator);
    they must be the ones tests/golden/gen_golden.py wrote."""
    import json
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "bench.py")).read()
    gold = json.load(open(os.path.join(root, "tests", "golden", "golden.json")))
    consts = dict(re.findall(r'^(GOLDEN_[A-Z_0-9]+) = "([0-9a-f]{64})"', src, re.M))
    assert consts["GOLDEN_LSM"] == gold["lsm"]["mask_sha256"]
    assert consts["GOLDEN_LSM_WIDE"] == gold["lsm_wide"]["rows_sha256"]
    c4 = next(r for r in gold["varlen"] if r["n"] == 10_000_000)
    assert consts["GOLDEN_C4"] == c4["encode_sha256"] and consts["GOLDEN_C4_PROBE"] == c4["probe_sha256"]
    c2 = next(r for r in gold["fixed16"] if r["n"] == 10_000_000 and r["p"] == 0.01)
    assert consts["GOLDEN_C2"] == c2["encode_sha256"] and consts["GOLDEN_C3"] == c2["probe_sha256"]


def test_gather_count_tool(tmp_path):
    """tools/gather_count.py (the probe's gather count in the bench's gather_model): the phased
    walk answers as MayContain does and the positives equal the C1 golden count; the committed
    10M count is the one the bench reads."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "g.json"
    subprocess.run([sys.executable, os.path.join(root, "tools", "gather_count.py"), "--n", "100000", "--out", str(out)],
                   check=True, capture_output=True)
    r = json.loads(out.read_text())["c2c3"]["probe"]
    assert r["positives"] == 51233 and r["ranges"] == 1
    assert r["gathers_phased"] == r["gathers_reference_order"]  # one range: the same order
    with open(os.path.join(root, "profiles", "gathers_c2c3.json")) as f:
        full = json.load(f)["c2c3"]["probe"]
    assert full["n"] == 10_000_000 and full["positives"] == 5_233_107 and full["ranges"] == 3


def test_gather_count_c5_tool(tmp_path):
    """tools/gather_count_c5.py (the C5 line's gather_model): the keys whose 64-filter mask stays
    non-zero are exactly the keys the oracle's multi-filter probe answers 'maybe' for, and the
    committed 10M count is the one the bench reads."""
    import json
    import subprocess
    import sys

    import keygen as kg
    from oracle import oracle_c as oc

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "g.json"
    n = 20_000
    subprocess.run([sys.executable, os.path.join(root, "tools", "gather_count_c5.py"), "--n", str(n), "--out", str(out)],
                   check=True, capture_output=True)
    r = json.loads(out.read_text())["c5"]["probe"]
    nf, per = 64, 100_000
    m, k = oc.params(per, 0.01)
    filters = [(oc.build(m, k, kg.key16(f * per + np.arange(per)), per, stride=16), m, k) for f in range(nf)]
    q = np.arange(n)
    half = q // 2
    mask = oc.probe_multi(filters, kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q)), n,
                          stride=16)
    assert r["keys_with_a_maybe"] == int((mask != 0).sum())
    assert n * 7 >= r["gathers"] >= n  # at least one gather per key, at most k
    with open(os.path.join(root, "profiles", "gathers_c2c3.json")) as f:
        full = json.load(f)["c5"]["probe"]
    assert full["n"] == 10_000_000 and full["filters"] == 64 and full["slices"] == 4
