"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden vectors.

Bit-exact everywhere: the same bit array (byte h>>3, bit h&7) and the same MayContain answers
as the reference algorithm (lsm/bloom.go:19-120).  Sizes the oracle finishes in seconds are
compared element for element; the BASELINE full sizes (10M keys) are compared through the
committed sha256 digests plus size-independent properties (no false negatives, idempotence,
OR-linearity of builds over key partitions).
"""
import hashlib

import numpy as np
import pytest

from oracle import bloom_np as bn
from oracle import oracle_c as oc
import keygen as kg

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch


@pytest.fixture(scope="module")
def ctx(seb, torch_cuda):
    seb.device_check(0)
    c = seb.Ctx(0)
    yield c
    c.close()


def to_dev(torch, arr):
    return torch.from_numpy(np.array(arr, copy=True)).cuda()


def dev_build_bits(seb, torch, keys_dev, m, k):
    words = seb.new_words(m)
    seb.dev_build(keys_dev, words, m, k)
    torch.cuda.synchronize()
    return words, seb.words_to_bits(words, m)


# ---------------------------------------------------------------- Go-API mirror -------------

@pytest.mark.parametrize("n", [1, 7, 1000, 5000])
def test_go_api_sequence_small(seb, golden, torch_cuda, n):
    """Replays sstable_builder.go (New -> Add per sorted key -> Encode) and sstable.go
    (Decode -> MayContain per Get) on the golden small cases."""
    row = next(r for r in golden["fixed16"] if r["n"] == n and r["p"] == 0.01)
    f = seb.BloomFilter(n, 0.01)
    for i in range(n):
        f.add(kg.key16_bytes(i))
    enc = f.encode()
    assert enc.hex() == row["encode_hex"]
    g = seb.BloomFilter.decode(enc)
    probes = [kg.key16_bytes(int(i)) for i in kg.probe_indices(n)]
    ans = np.array([g.may_contain(p) for p in probes[:300]], dtype=np.uint8)
    m, k = row["m"], row["k"]
    ref = oc.probe(np.frombuffer(enc[12:], np.uint8), m, k, kg.key16(kg.probe_indices(n))[:300], min(n, 300),
                   stride=16)
    assert np.array_equal(ans[: len(ref)], ref)
    batch = g.may_contain_batch(kg.key16(kg.probe_indices(n)))
    assert sha(batch.tobytes()) == row["probe_sha256"]


def test_go_api_add_after_encode_accumulates(seb, torch_cuda):
    n = 3000
    f = seb.BloomFilter(n, 0.01)
    keys = kg.key16(np.arange(n))
    f.add_batch(keys[:1000])
    first = f.encode()
    for i in range(1000, 1500):
        f.add(keys[i].tobytes())
    f.add_batch(keys[1500:])
    m, k = oc.params(n, 0.01)
    ref_first = oc.build(m, k, keys[:1000], 1000, stride=16)
    assert first[12:] == ref_first.tobytes()
    ref = oc.build(m, k, keys, n, stride=16)
    assert f.encode()[12:] == ref.tobytes()
    assert f.pending == 0


def test_go_api_variable_keys_and_empty_key(seb, torch_cuda):
    rng = np.random.default_rng(3)
    keys = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 300, 2000)]
    keys[5] = b""
    f = seb.BloomFilter(len(keys), 0.01)
    for key in keys:
        f.add(key)
    m, k = f.num_bits, f.num_hashes
    lens = np.array([len(x) for x in keys], np.uint64)
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = np.frombuffer(b"".join(keys), np.uint8)
    ref = oc.build(m, k, data, len(keys), offsets=off)
    assert f.encode()[12:] == ref.tobytes()
    assert f.may_contain(b"") is True
    probes = keys[:100] + [bytes(rng.integers(0, 256, 20, dtype=np.uint8)) for _ in range(400)]
    got = np.array([f.may_contain(p) for p in probes[:40]], np.uint8)
    pb = seb.as_keys(probes)
    refp = oc.probe(ref, m, k, pb.data, pb.n, offsets=pb.offsets)
    assert np.array_equal(got, refp[:40])
    assert np.array_equal(f.may_contain_batch(probes), refp)


def test_go_api_uniform_then_mixed_lengths_and_republish(seb, torch_cuda):
    """The Add arena keeps no offsets while every key has one length (a fixed-stride build), and
    materialises them at the first key of another length; MayContain after more Adds sees them
    (the lock-free host copy is republished), from several threads at once."""
    import threading

    rng = np.random.default_rng(9)
    fixed = [kg.key16_bytes(i) for i in range(3000)]
    mixed = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 40, 1000)]
    f = seb.BloomFilter(4000, 0.01)
    m, k = f.num_bits, f.num_hashes
    for key in fixed[:2000]:
        f.add(key)
    assert f.may_contain(fixed[0]) and f.pending == 0  # flushed as one stride-16 batch
    for key in fixed[2000:] + mixed:
        f.add(key)
    keys = fixed + mixed
    lens = np.array([len(x) for x in keys], np.uint64)
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    ref = oc.build(m, k, np.frombuffer(b"".join(keys), np.uint8), len(keys), offsets=off)
    probes = keys[::3] + [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(3000)]
    pb = seb.as_keys(probes)
    want = oc.probe(ref, m, k, pb.data, pb.n, offsets=pb.offsets)
    results = [None] * 8

    def reader(t):
        results[t] = np.array([f.may_contain(p) for p in probes], np.uint8)

    threads = [threading.Thread(target=reader, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    for r in results:
        assert np.array_equal(r, want)
    assert f.encode()[12:] == ref.tobytes()


@pytest.mark.parametrize("n", [1, 500, 1024, 1025, 5000, 50_000, 100_003])
def test_image_build_fresh_and_accumulating(seb, torch_cuda, n):
    """The LDS-image build (build_algo 4): one workgroup writing the filter directly or G images
    OR-merged by the second kernel; a new filter's first build writes its words whole (no clear),
    later builds OR into them; the device API always ORs."""
    torch = torch_cuda
    keys = kg.key16(np.arange(2 * n))
    m, k = oc.params(n, 0.01)
    with seb.option("build_algo", 4):
        f = seb.BloomFilter(n, 0.01)
        f.add_batch(keys[:n])
        assert f.encode()[12:] == oc.build(m, k, keys[:n], n, stride=16).tobytes()
        f.add_batch(keys[n:])
        assert f.encode()[12:] == oc.build(m, k, keys, 2 * n, stride=16).tobytes()
        f.close()
        words = seb.new_words(m)
        seb.dev_build(seb.dev_keys(to_dev(torch, keys[n:]), n=n, stride=16), words, m, k)
        seb.dev_build(seb.dev_keys(to_dev(torch, keys[:n]), n=n, stride=16), words, m, k)
        torch.cuda.synchronize()
        assert np.array_equal(seb.words_to_bits(words, m), oc.build(m, k, keys, 2 * n, stride=16))
        tail = words.cpu().numpy().view(np.uint8)[(m + 7) // 8:]
        assert not tail.any() or (m % 8 and tail[0] >> (m % 8) == 0 and not tail[1:].any())


def test_go_api_errors_match_reference_panics(seb, torch_cuda):
    z = seb.BloomFilter.decode(bytes(12))  # numBits 0: Go panics with divide by zero
    with pytest.raises(seb.SebError):
        z.may_contain(b"a")
    k0 = seb.BloomFilter.decode(bytes.fromhex("400000000000000000000000") + bytes(8))  # k = 0
    assert k0.may_contain(b"anything") is True  # loop over zero hashes -> true
    k0.add(b"x")
    assert k0.encode() == bytes.fromhex("400000000000000000000000") + bytes(8)


# ------------------------------------------------------------- host-buffer API --------------

def test_c1_100k_host_api(seb, golden, ctx):
    """BASELINE C1 shape (100K x 16B @1%) through the PCIe-inclusive host API."""
    row = next(r for r in golden["fixed16"] if r["n"] == 100000 and r["p"] == 0.01)
    n, m, k = row["n"], row["m"], row["k"]
    bits = ctx.build(kg.key16(np.arange(n)), m, k)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    ans = ctx.probe(kg.key16(kg.probe_indices(n)), bits, m, k)
    assert sha(ans.tobytes()) == row["probe_sha256"]


@pytest.mark.parametrize("p", [0.001, 0.1, 0.5])
def test_other_fpr(seb, golden, ctx, p):
    row = next(r for r in golden["fixed16"] if r["n"] == 100000 and r["p"] == p)
    n, m, k = row["n"], row["m"], row["k"]
    bits = ctx.build(kg.key16(np.arange(n)), m, k)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    assert sha(ctx.probe(kg.key16(kg.probe_indices(n)), bits, m, k).tobytes()) == row["probe_sha256"]


def test_host_api_chunked_pipeline(seb, monkeypatch, torch_cuda):
    """Many small chunks through the double-buffered H2D/compute/D2H pipeline."""
    monkeypatch.setenv("SEB_CHUNK_BYTES", "4096")
    c = seb.Ctx(0)
    n = 50000
    m, k = oc.params(n, 0.01)
    keys = kg.key16(np.arange(n))
    bits = c.build(keys, m, k)
    assert np.array_equal(bits, oc.build(m, k, keys, n, stride=16))
    pk = kg.key16(kg.probe_indices(n))
    assert np.array_equal(c.probe(pk, bits, m, k), oc.probe(bits, m, k, pk, n, stride=16))
    data, off = kg.varlen_keys(np.arange(n))
    vb = c.build((data, off), m, k)
    assert np.array_equal(vb, oc.build(m, k, data, n, offsets=off))
    # a build that ORs into existing host bits
    acc = c.build(keys[: n // 2], m, k)
    acc = c.build(keys[n // 2:], m, k, bits=acc)
    assert np.array_equal(acc, bits)
    c.close()


# --------------------------------------------------------- device-resident API --------------

@pytest.fixture(params=[1, 2, 3, 4], ids=["atomic", "bucketed", "lds", "images"])
def build_algo(request, seb):
    """Build paths: device-scope atomics, radix-partitioned (bucketed), the LDS-resident filter
    with an atomic merge (algo 3) and LDS images merged by a second kernel (algo 4); a filter
    over 160 KiB takes atomics for 3 and 4."""
    with seb.option("build_algo", request.param):
        yield request.param


@pytest.fixture(params=[(0, 1 << 20), (1, 1 << 20), (2, 1 << 20), (7, 1 << 20), (0, 97), (1, 61)],
                ids=lambda v: f"phases{v[0]}-grid{v[1]}")
def probe_split(request, seb):
    """Probe paths: phased (auto or forced range counts), the sliced probe (one phase), and
    grid-stride loops (a capped grid)."""
    phases, grid = request.param
    with seb.option("probe_phases", phases), seb.option("grid_cap", grid):
        yield request.param


@pytest.fixture(params=[1, 0], ids=["compact", "dense"])
def probe_compact(request, seb):
    """Later phases of the phased probe: compacted rows of live keys, or every key's word and
    answer byte through every phase."""
    with seb.option("probe_compact", request.param):
        yield request.param


def test_c2_c3_10m_device_resident(seb, golden, torch_cuda, build_algo):
    """BASELINE C2 (build 10M x 16B @1%) and C3 (probe 10M, 50% present), digests + properties,
    for both build algorithms (device-scope atomics and the radix-partitioned LDS build)."""
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n, m, k = row["n"], row["m"], row["k"]
    keys = to_dev(torch, kg.key16(np.arange(n)))
    kd = seb.dev_keys(keys, n=n, stride=16)
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    assert int(np.unpackbits(bits).sum()) == row["popcount"]
    # padding words stay zero
    tail = words.cpu().numpy().view(np.uint8)[(m + 7) // 8:]
    assert not tail.any() or (m % 8 and tail[0] >> (m % 8) == 0 and not tail[1:].any())
    # idempotence: building the same keys again changes nothing
    seb.dev_build(kd, words, m, k)
    torch.cuda.synchronize()
    assert np.array_equal(seb.words_to_bits(words, m), bits)
    # OR-linearity: build over two key partitions into fresh words equals the whole
    w2 = seb.new_words(m)
    half = seb.dev_keys(keys[: n // 2], n=n // 2, stride=16)
    rest = seb.dev_keys(keys[n // 2:], n=n - n // 2, stride=16)
    seb.dev_build(rest, w2, m, k)
    seb.dev_build(half, w2, m, k)
    torch.cuda.synchronize()
    assert np.array_equal(seb.words_to_bits(w2, m), bits)
    # C3 probe
    probe_keys = to_dev(torch, kg.key16(kg.probe_indices(n)))
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    seb.dev_probe(seb.dev_keys(probe_keys, n=n, stride=16), words, m, k, out)
    torch.cuda.synchronize()
    ans = out.cpu().numpy()
    assert sha(ans.tobytes()) == row["probe_sha256"]
    assert int(ans.sum()) == row["probe_positives"]
    assert ans[0::2].all()  # no false negatives
    # spot-check answers element for element against the oracle on a slice
    sl = kg.probe_indices(n)[:200000]
    assert np.array_equal(ans[:200000], oc.probe(bits, m, k, kg.key16(sl), 200000, stride=16))


def test_probe_paths_and_phase_counts(seb, golden, torch_cuda):
    """The phased probe at any number of filter ranges (compacted later phases, or every key's
    word and answer through every phase), the sliced probe (one range, or an answer array that is
    not 4-byte aligned), give the C3 answers bit for bit, also for a ragged batch whose last
    workgroup (and group of 64 keys) is partly empty."""
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n, m, k = row["n"], row["m"], row["k"]
    kd = seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16)
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    pk = to_dev(torch, kg.key16(kg.probe_indices(n)))
    ragged = 999_983
    ref_ragged = oc.probe(bits, m, k, kg.key16(kg.probe_indices(n)[:ragged]), ragged, stride=16)
    for phases, shift, compact in ((0, 0, 1), (0, 0, 0), (2, 0, 1), (2, 0, 0), (4, 0, 1), (7, 0, 1), (7, 0, 0),
                                   (1, 0, 1), (0, 1, 1)):
        with seb.option("probe_phases", phases), seb.option("probe_compact", compact):
            buf = torch.full((n + 4,), 7, dtype=torch.uint8, device="cuda")
            seb.dev_probe(seb.dev_keys(pk, n=n, stride=16), words, m, k, buf[shift:shift + n])
            torch.cuda.synchronize()
            assert sha(buf[shift:shift + n].cpu().numpy().tobytes()) == row["probe_sha256"], (phases, shift, compact)
            outr = torch.full((ragged + 2,), 7, dtype=torch.uint8, device="cuda")
            seb.dev_probe(seb.dev_keys(pk[:ragged], n=ragged, stride=16), words, m, k, outr[shift:shift + ragged])
            torch.cuda.synchronize()
            got = outr.cpu().numpy()
            assert np.array_equal(got[shift:shift + ragged], ref_ragged), (phases, shift, compact)
            assert got[shift + ragged] == 7, (phases, shift)  # nothing written past the batch


@pytest.mark.parametrize("phases", [2, 3, 5])
def test_phased_probe_small_batches(seb, torch_cuda, phases, probe_compact):
    """Phased probes of batches that leave groups of 64 keys (and a wave's 4 groups) partly empty:
    1 to 4097 keys, fixed 16-B keys and packed residues, against the oracle; nothing is written
    past the batch."""
    torch = torch_cuda
    n_build = 100_000
    m, k = oc.params(n_build, 0.01)
    bkeys = kg.key16(np.arange(n_build))
    bits = oc.build(m, k, bkeys, n_build, stride=16)
    words, got_bits = dev_build_bits(seb, torch, seb.dev_keys(to_dev(torch, bkeys), n=n_build, stride=16), m, k)
    assert np.array_equal(got_bits, bits)
    with seb.option("probe_phases", phases):
        for n in (1, 2, 63, 64, 65, 129, 255, 256, 257, 4097):
            q = kg.key16(kg.probe_indices(n_build, count=n))
            want = oc.probe(bits, m, k, q, n, stride=16)
            qd = seb.dev_keys(to_dev(torch, q), n=n, stride=16)
            out = torch.full((n + 8,), 7, dtype=torch.uint8, device="cuda")
            seb.dev_probe(qd, words, m, k, out[:n])
            packed = torch.zeros(n, dtype=torch.int64, device="cuda")
            seb.dev_pack_residues(qd, m, k, packed)
            out2 = torch.full((n + 8,), 7, dtype=torch.uint8, device="cuda")
            seb.dev_probe_packed(packed, n, words, m, k, out2[:n])
            torch.cuda.synchronize()
            for o in (out, out2):
                got = o.cpu().numpy()
                assert np.array_equal(got[:n], want), (n, phases)
                assert (got[n:] == 7).all(), (n, phases)


def test_multi_packed_matches_multi(seb, golden, torch_cuda):
    """The C5 multi-filter probe over packed residues equals the probe over the keys (golden C5
    digest for 64 filters, u64 masks) and the oracle for 8 filters with a ragged batch; mixed
    filter sizes are rejected."""
    torch = torch_cuda
    nf, per, n = 64, 100_000, 10_000_000
    m, k = seb.params(per, 0.01)
    fkeys = torch.from_numpy(kg.key16(np.arange(nf * per))).cuda()
    filters = [(seb.new_words(m), m, k) for _ in range(nf)]
    seb.dev_build_many(seb.dev_keys(fkeys, n=nf * per, stride=16), [j * per for j in range(nf + 1)], filters)
    q = np.arange(n, dtype=np.int64)
    half = q // 2
    pk = seb.dev_keys(torch.from_numpy(kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf,
                                                          nf * per + q))).cuda(), n=n, stride=16)
    packed = torch.zeros(n, dtype=torch.int64, device="cuda")
    seb.dev_pack_residues(pk, m, k, packed)
    mask = torch.zeros(n, dtype=torch.int64, device="cuda")
    seb.dev_probe_multi_packed(packed, n, filters, mask)
    torch.cuda.synchronize()
    assert sha(mask.cpu().numpy().view(np.uint64).astype("<u8").tobytes()) == golden["c5"]["mask_sha256"]
    # 8 filters, u8 masks, ragged batch, against the oracle
    nn = 100_003
    sub = filters[:8]
    keys8 = kg.key16(np.where(q[:nn] % 2 == 0, (half[:nn] % 8) * per + half[:nn] // 8, nf * per + q[:nn]))
    pk8 = seb.dev_keys(torch.from_numpy(keys8).cuda(), n=nn, stride=16)
    p8 = torch.zeros(nn, dtype=torch.int64, device="cuda")
    seb.dev_pack_residues(pk8, m, k, p8)
    host = [(seb.words_to_bits(w, m), m, k) for w, m, k in sub]
    ref = oc.probe_multi(host, keys8, nn, stride=16)
    m8 = torch.full((nn + 1,), 7, dtype=torch.uint8, device="cuda")
    seb.dev_probe_multi_packed(p8, nn, sub, m8)
    torch.cuda.synchronize()
    got = m8.cpu().numpy()
    assert np.array_equal(got[:nn].astype(np.uint64), ref)
    assert got[nn] == 7
    m2, k2 = seb.params(per + 1, 0.01)
    with pytest.raises(seb.SebError):
        seb.dev_probe_multi_packed(p8, nn, sub + [(seb.new_words(m2), m2, k2)],
                                   torch.zeros(nn, dtype=torch.int16, device="cuda"))


def unpack6(buf: np.ndarray, n: int) -> np.ndarray:
    """Test-side reading of seb_dev_pack_residues6's 64-key blocks into one 48-bit word per key."""
    blocks = buf[: -(-n // 64) * 384].reshape(-1, 384)
    lo = blocks[:, :256].copy().view("<u4").astype(np.uint64)
    hi = blocks[:, 256:].copy().view("<u2").astype(np.uint64)
    return (lo | (hi << np.uint64(32))).ravel()[:n]


def test_multi_packed6(seb, golden, torch_cuda):
    """The narrow (6-byte, m < 2^21) packed residues: the same fields as the 8-byte form at 21-bit
    width, the C5 golden masks from them for 64 filters, an 8-filter ragged batch equal to the
    oracle (the bytes past the batch untouched), a pre-hashed variable-length batch equal to the
    probe of its keys, and the cases the narrow form cannot take rejected."""
    torch = torch_cuda
    nf, per, n = 64, 100_000, 10_000_000
    m, k = seb.params(per, 0.01)
    assert seb.pack6_supported(m, k) and seb.lib().seb_packed6_bytes(n) == seb.packed6_bytes(n) == 60_000_000
    fkeys = torch.from_numpy(kg.key16(np.arange(nf * per))).cuda()
    filters = [(seb.new_words(m), m, k) for _ in range(nf)]
    seb.dev_build_many(seb.dev_keys(fkeys, n=nf * per, stride=16), [j * per for j in range(nf + 1)], filters)
    q = np.arange(n, dtype=np.int64)
    half = q // 2
    pk = seb.dev_keys(torch.from_numpy(kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf,
                                                          nf * per + q))).cuda(), n=n, stride=16)
    p6 = torch.zeros(seb.packed6_bytes(n), dtype=torch.uint8, device="cuda")
    seb.dev_pack_residues6(pk, m, k, p6)
    mask = torch.zeros(n, dtype=torch.int64, device="cuda")
    seb.dev_probe_multi_packed6(p6, n, filters, mask)
    p8 = torch.zeros(n, dtype=torch.int64, device="cuda")
    seb.dev_pack_residues(pk, m, k, p8)
    torch.cuda.synchronize()
    assert sha(mask.cpu().numpy().view(np.uint64).astype("<u8").tobytes()) == golden["c5"]["mask_sha256"]
    # field by field against the 8-byte words (r0 | b << 29 | carries << 58)
    w6, w8 = unpack6(p6.cpu().numpy(), n), p8.cpu().numpy().view(np.uint64)
    f21, f29 = np.uint64((1 << 21) - 1), np.uint64((1 << 29) - 1)
    assert np.array_equal(w6 & f21, w8 & f29)
    assert np.array_equal((w6 >> np.uint64(21)) & f21, (w8 >> np.uint64(29)) & f29)
    assert np.array_equal(w6 >> np.uint64(42), w8 >> np.uint64(58))
    # 8 filters, u8 masks, a ragged batch (not a multiple of 64 keys) against the oracle
    nn = 100_003
    sub = filters[:8]
    keys8 = kg.key16(np.where(q[:nn] % 2 == 0, (half[:nn] % 8) * per + half[:nn] // 8, nf * per + q[:nn]))
    pk8 = seb.dev_keys(torch.from_numpy(keys8).cuda(), n=nn, stride=16)
    b6 = torch.full((seb.packed6_bytes(nn) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    seb.dev_pack_residues6(pk8, m, k, b6)
    host = [(seb.words_to_bits(w, m), m, k) for w, m, k in sub]
    ref = oc.probe_multi(host, keys8, nn, stride=16)
    m8 = torch.full((nn + 1,), 7, dtype=torch.uint8, device="cuda")
    seb.dev_probe_multi_packed6(b6, nn, sub, m8)
    torch.cuda.synchronize()
    got = m8.cpu().numpy()
    assert np.array_equal(got[:nn].astype(np.uint64), ref)
    assert got[nn] == 7
    assert (b6.cpu().numpy()[seb.packed6_bytes(nn):] == 0xA5).all()
    # a variable-length batch (pre-hashed on the device first) gives the masks of its keys
    nv = 70_001
    vd, vo = kg.varlen_keys(np.arange(nv))
    vkd = seb.dev_keys(torch.from_numpy(vd).cuda(), torch.from_numpy(vo.view(np.int64)).cuda())
    v6 = torch.zeros(seb.packed6_bytes(nv), dtype=torch.uint8, device="cuda")
    seb.dev_pack_residues6(vkd, m, k, v6)
    mv6 = torch.zeros(nv, dtype=torch.int64, device="cuda")
    seb.dev_probe_multi_packed6(v6, nv, filters, mv6)
    mvk = torch.zeros(nv, dtype=torch.int64, device="cuda")
    seb.dev_probe_multi(vkd, filters, mvk)
    torch.cuda.synchronize()
    assert torch.equal(mv6, mvk)
    # rejected: m >= 2^21, k != 7, mixed sizes, a misaligned buffer
    mb, kb = seb.params(300_000, 0.01)
    assert mb >= 1 << 21
    with pytest.raises(seb.SebError):
        seb.dev_pack_residues6(pk8, mb, kb, b6)
    with pytest.raises(seb.SebError):
        seb.dev_pack_residues6(pk8, m, 5, b6)
    m2, k2 = seb.params(per + 1, 0.01)
    with pytest.raises(seb.SebError):
        seb.dev_probe_multi_packed6(b6, nn, sub + [(seb.new_words(m2), m2, k2)], torch.zeros(nn, dtype=torch.int16,
                                                                                           device="cuda"))
    with pytest.raises(seb.SebError):
        seb.dev_probe_multi_packed6(b6[1:], nn, sub, m8)


def unpack_positions(packed: np.ndarray, m: int) -> np.ndarray:
    """Test-side decoding of seb_dev_pack_residues' words into the 7 positions (the recurrence
    of for_positions, in Python integers)."""
    mask = (1 << 29) - 1
    c = (1 << 64) % m
    out = np.zeros((packed.size, 7), np.uint64)
    for j, v in enumerate(int(x) for x in packed):
        r, b, f = v & mask, (v >> 29) & mask, v >> 58
        out[j, 0] = r
        for q in range(1, 7):
            r = (r + b - (c if (f >> (q - 1)) & 1 else 0)) % m
            out[j, q] = r
    return out


def test_packed_residues(seb, golden, torch_cuda, probe_compact):
    """Packed residues (the multi-GPU broadcast form): positions equal the oracle's
    (h1 + i*h2 mod 2^64) mod m, and probing them gives the C3 answers bit for bit, for fixed 16-B
    and variable-length batches; unsupported (k, m) are rejected."""
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n, m, k = row["n"], row["m"], row["k"]
    kd = seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16)
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    pidx = kg.probe_indices(n)
    pk = seb.dev_keys(to_dev(torch, kg.key16(pidx)), n=n, stride=16)
    packed = torch.zeros(n, dtype=torch.int64, device="cuda")
    seb.dev_pack_residues(pk, m, k, packed)
    out = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    seb.dev_probe_packed(packed, n, words, m, k, out)
    torch.cuda.synchronize()
    assert sha(out.cpu().numpy().tobytes()) == row["probe_sha256"]
    # the root's fused probe: the same answers and the same packed words in one pass
    packed2 = torch.zeros(n, dtype=torch.int64, device="cuda")
    out2 = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    seb.dev_probe_emit_packed(pk, words, m, k, out2, packed2)
    torch.cuda.synchronize()
    assert torch.equal(packed2, packed)
    assert torch.equal(out2, out)
    host = packed.cpu().numpy().view(np.uint64)
    sample = np.r_[0:2000, n - 2000:n]
    want = np.array([oc.positions(kg.key16_bytes(int(i)), m, k) for i in pidx[sample]], np.uint64)
    assert np.array_equal(unpack_positions(host[sample], m), want)
    # ragged tail and a variable-length batch against the oracle
    nv = 50001
    data, off = kg.varlen_keys(np.arange(nv))
    mv, kv = oc.params(nv, 0.01)
    vkd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
    vwords, vbits = dev_build_bits(seb, torch, vkd, mv, kv)
    pdata, poff = kg.varlen_keys(kg.probe_indices(nv))
    vpk = seb.dev_keys(to_dev(torch, pdata), to_dev(torch, poff))
    vpacked = torch.zeros(nv, dtype=torch.int64, device="cuda")
    seb.dev_pack_residues(vpk, mv, kv, vpacked)
    vout = torch.full((nv + 1,), 7, dtype=torch.uint8, device="cuda")
    seb.dev_probe_packed(vpacked, nv, vwords, mv, kv, vout)
    torch.cuda.synchronize()
    got = vout.cpu().numpy()
    assert np.array_equal(got[:nv], oc.probe(vbits, mv, kv, pdata, nv, offsets=poff))
    assert got[nv] == 7
    for bad_m, bad_k in ((1 << 29, 7), (m, 6)):
        with pytest.raises(seb.SebError):
            seb.dev_pack_residues(pk, bad_m, bad_k, packed)


@pytest.mark.parametrize("n", [1000, 100000, 1000000])
def test_c4_varlen_device(seb, golden, torch_cuda, n, build_algo):
    torch = torch_cuda
    row = next(r for r in golden["varlen"] if r["n"] == n)
    m, k = row["m"], row["k"]
    data, off = kg.varlen_keys(np.arange(n))
    kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    pdata, poff = kg.varlen_keys(kg.probe_indices(n))
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    seb.dev_probe(seb.dev_keys(to_dev(torch, pdata), to_dev(torch, poff)), words, m, k, out)
    torch.cuda.synchronize()
    assert sha(out.cpu().numpy().tobytes()) == row["probe_sha256"]


@pytest.mark.parametrize("tail", [0, 1, 2, 3])
@pytest.mark.parametrize("algo", [0, 2])
def test_c4_prehash_golden(seb, golden, torch_cuda, algo, tail):
    """C4's zipf lengths (the spans fit the LDS window, so the sorted and split-chain hashing
    paths run rather than the overflow fallback), pre-hashed to 16-B hashes (LDS-resident build,
    unphased probe) and to packed residues (bucketed build), reproduce the C4 golden digests;
    with the 64 v longest keys of a workgroup on 2 v tail waves, a lane per chain (varlen_tail v =
    1, 2, 3), and without (0)."""
    torch = torch_cuda
    n = 100000
    row = next(r for r in golden["varlen"] if r["n"] == n)
    m, k = row["m"], row["k"]
    data, off = kg.varlen_keys(np.arange(n))
    pdata, poff = kg.varlen_keys(kg.probe_indices(n))
    with seb.option("varlen_prehash_min_keys", 0), seb.option("build_algo", algo), seb.option("varlen_tail", tail):
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe(seb.dev_keys(to_dev(torch, pdata), to_dev(torch, poff)), words, m, k, out)
        torch.cuda.synchronize()
        assert sha(out.cpu().numpy().tobytes()) == row["probe_sha256"]


@pytest.mark.parametrize("tail", [0, 1, 2, 3])
def test_varlen_prehash_tiny_keys(seb, torch_cuda, tail):
    """Batches of only empty and 1-3-byte keys, so the tail waves' keys (a workgroup's longest) are
    empty or shorter than a word: FNV-1 of an empty key is the offset basis, and a 1-byte key's
    FNV-1 is the basis times the prime xor its byte (the tail lanes run FNV-1 as FNV-1a's recurrence
    over n - 1 bytes); a batch of all-empty keys too."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    for lens in (rng.choice([0, 1, 2, 3], size=5000, p=[0.4, 0.3, 0.2, 0.1]), np.zeros(3000, np.int64)):
        n = lens.size
        off = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        data = rng.integers(0, 256, max(int(off[-1]), 1), dtype=np.uint8)[: int(off[-1])]
        m, k = oc.params(n, 0.01)
        ref = oc.build(m, k, data, n, offsets=off)
        with seb.option("varlen_prehash_min_keys", 0), seb.option("varlen_tail", tail):
            kd = seb.dev_keys(to_dev(torch, np.concatenate([data, np.zeros(16, np.uint8)])), to_dev(torch, off))
            words, bits = dev_build_bits(seb, torch, kd, m, k)
            assert np.array_equal(bits, ref)
            out = torch.empty(n, dtype=torch.uint8, device="cuda")
            seb.dev_probe(kd, words, m, k, out)
            torch.cuda.synchronize()
            assert bool(out.all())


@pytest.mark.parametrize("prehash_min", [0, 1 << 40], ids=["prehash", "direct"])
def test_varlen_processing_order_invisible(seb, torch_cuda, prehash_min, build_algo):
    """The LDS-staged pre-hash and the direct byte walk give the same bit array and answers,
    including for empty keys and keys longer than 256 B (the last length bucket, and LDS spans
    that overflow the staging window)."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    n = 70000
    lens = rng.choice([0, 1, 3, 8, 15, 16, 17, 40, 64, 255, 256, 300, 1000], size=n)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    m, k = oc.params(n, 0.01)
    ref = oc.build(m, k, data, n, offsets=off)
    with seb.option("varlen_prehash_min_keys", prehash_min):
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        assert np.array_equal(bits, ref)
        pd = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
        pd[: int(off[n // 2])] = data[: int(off[n // 2])]  # first half present
        pkd = seb.dev_keys(to_dev(torch, pd), to_dev(torch, off))
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe(pkd, words, m, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), oc.probe(ref, m, k, pd, n, offsets=off))


@pytest.mark.parametrize("packed", [0, 1], ids=["small_filter", "packed_paths"])
@pytest.mark.parametrize("tail", [0, 1, 2, 3])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_varlen_prehash_edge_lengths(seb, torch_cuda, seed, tail, packed):
    """The pre-hash (448/384/320-key workgroups, 64-B window per key, with and without the tail
    waves) hashes like the oracle over lengths that mix empty, sub-word, bucket-edge, 48/49-B and
    window-overflowing keys, and a ragged last workgroup; the answers of a half-present batch
    equal the oracle's key by key; with a two-range filter and the bucketed build as well, so the
    packed paths (build from packed residues, phase 0 fused into the pre-hash) run."""
    torch = torch_cuda
    rng = np.random.default_rng(seed)
    n = 40000 + 77
    w = np.array([4, 4, 4, 4, 4, 4, 4, 8, 4, 8, 4, 8, 8, 4, 4, 4, 4, 4, 4, 3, 1, 4, 4], float)
    lens = rng.choice([0, 1, 2, 3, 4, 5, 7, 8, 9, 16, 31, 39, 40, 41, 63, 64, 65, 255, 256, 300, 2000, 48, 49],
                      size=n, p=w / w.sum())
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, int(off[-1]) + 1, dtype=np.uint8)[1:]  # odd base offset in the host copy
    m, k = (40_000_003, 7) if packed else oc.params(n, 0.01)
    ref = oc.build(m, k, data, n, offsets=off)
    pd = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    pd[: int(off[n // 2])] = data[: int(off[n // 2])]  # first half present
    want = oc.probe(ref, m, k, pd, n, offsets=off)
    with seb.option("varlen_prehash_min_keys", 0), seb.option("varlen_tail", tail), \
            seb.option("build_algo", 2 if packed else 0):
        pkd = seb.dev_keys(to_dev(torch, pd), to_dev(torch, off))
        dd = torch.zeros(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
        offd = to_dev(torch, off)
        for shift in (0, 3):  # key bytes at an unaligned device address too
            view = dd[shift: shift + int(off[-1])]
            view.copy_(torch.from_numpy(data).cuda())
            kd = seb.dev_keys(view, offd)
            words, bits = dev_build_bits(seb, torch, kd, m, k)
            assert np.array_equal(bits, ref), shift
            out = torch.empty(n, dtype=torch.uint8, device="cuda")
            seb.dev_probe(kd, words, m, k, out)
            torch.cuda.synchronize()
            assert bool(out.all()), shift
        seb.dev_probe(pkd, words, m, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("k", [7, 8])
@pytest.mark.parametrize("algo", [1, 2])
def test_varlen_prehash_packed_paths(seb, torch_cuda, k, algo, probe_compact):
    """Pre-hash to packed residues (k = 7: bucketed build from KeysPacked; the phased probe with
    phase 0 fused into the pre-hash (compacted) or from the dense packed words; pack_residues /
    emit_packed over variable-length keys) against the oracle, and the 16-B hash path (k = 8); a
    2-range filter so the k = 7 probe runs phased; keys up to 3000 B, so some workgroups take the
    pre-hash's straight-from-HBM path."""
    torch = torch_cuda
    packed = k == 7
    rng = np.random.default_rng(11 + packed)
    n = 600_001
    w = np.array([20, 10, 10, 10, 5, 3, 1, 1], float)
    lens = rng.choice([8, 9, 15, 16, 40, 100, 256, 3000], size=n, p=w / w.sum())
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    m = 40_000_003
    ref = oc.build(m, k, data, n, offsets=off, threads=16)
    pd = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    pd[: int(off[n // 2])] = data[: int(off[n // 2])]  # first half present
    want = oc.probe(ref, m, k, pd, n, offsets=off)
    with seb.option("build_algo", algo):
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        assert np.array_equal(bits, ref)
        pkd = seb.dev_keys(to_dev(torch, pd), to_dev(torch, off))
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe(pkd, words, m, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)
        if not packed:
            return
        pk = torch.zeros(n, dtype=torch.int64, device="cuda")
        seb.dev_pack_residues(pkd, m, k, pk)
        out2 = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe_packed(pk, n, words, m, k, out2)
        pk3 = torch.zeros(n, dtype=torch.int64, device="cuda")
        out3 = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe_emit_packed(pkd, words, m, k, out3, pk3)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)
        assert np.array_equal(out2.cpu().numpy(), want)
        assert np.array_equal(out3.cpu().numpy(), want)
        assert torch.equal(pk, pk3)


@pytest.mark.parametrize("k", [7, 8])
def test_varlen_bucketed_build_chunks(seb, torch_cuda, k):
    """A pre-hashed variable-length build larger than one bucketed launch (16.7M keys at k = 7)
    runs in chunks; every chunk must take its own slice of the hashes / packed residues."""
    torch = torch_cuda
    rng = np.random.default_rng(21)
    n = (1 << 24) + 123_457
    lens = rng.integers(8, 13, n)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    m = 160_000_001
    ref = oc.build(m, k, data, n, offsets=off, threads=16)
    with seb.option("build_algo", 2):
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        assert np.array_equal(bits, ref)


def test_c4_varlen_10m_properties(seb, golden, torch_cuda):
    """Full C4 size: the filter and the 10M answers match the golden digests (tests/golden varlen
    n = 10M, the oracle's), and every built key answers true."""
    torch = torch_cuda
    n = 10_000_000
    row = next(r for r in golden["varlen"] if r["n"] == n)
    m, k = oc.params(n, 0.01)
    assert (m, k) == (row["m"], row["k"])
    data, off = kg.varlen_keys(np.arange(n))
    pdata, poff = kg.varlen_keys(kg.probe_indices(n))
    kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off))
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    assert sha(bn.encode(bits, m, k)) == row["encode_sha256"]
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    seb.dev_probe(kd, words, m, k, out)  # every built key must answer true
    torch.cuda.synchronize()
    assert bool(out.all())
    seb.dev_probe(seb.dev_keys(to_dev(torch, pdata), to_dev(torch, poff)), words, m, k, out)
    torch.cuda.synchronize()
    assert sha(out.cpu().numpy().tobytes()) == row["probe_sha256"]


@pytest.mark.parametrize("stride", [0, 1, 3, 13, 16, 24, 33, 64])
def test_fixed_strides_and_alignment(seb, torch_cuda, stride, build_algo):
    torch = torch_cuda
    rng = np.random.default_rng(stride)
    n = 20000
    keys = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    m, k = oc.params(n, 0.01)
    ref = oc.build(m, k, keys, n, stride=stride)
    buf = torch.zeros(n * stride + 64, dtype=torch.uint8, device="cuda")
    for shift in (0, 1, 4):  # aligned and unaligned key buffers
        view = buf[shift: shift + n * stride]
        view.copy_(torch.from_numpy(keys.reshape(-1)).cuda())
        kd = seb.seb_keys(view.data_ptr(), None, n, stride, 0)
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        assert np.array_equal(bits, ref), shift
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        seb.dev_probe(kd, words, m, k, out)
        torch.cuda.synchronize()
        assert bool(out.all())


@pytest.mark.parametrize("algo", [1, 2])
@pytest.mark.parametrize("m,k", [(1, 1), (1, 7), (2, 3), (31, 7), (32, 7), (33, 7), (4096, 30), (1 << 30, 7),
                                 (3 * 2**29 + 1, 7), (2**31 - 2, 5), (2**31 - 1, 7), (2**31, 7), (2**31 + 1, 7),
                                 (2**32 - 5, 7), (2**32 + 977, 7), (3 * 2**32 + 12345, 9)])
def test_modulus_edge_cases(seb, torch_cuda, m, k, algo):
    """u32 residue path (m < 2^31, mod_m31) and u64 path, m at and around 2^31 and 2^32, runtime
    k != 7 (lsm/bloom.go:64 wraparound).
    algo 2 runs the radix-partitioned build where it applies (m <= 2^28), atomics elsewhere."""
    torch = torch_cuda
    seb.set_option("build_algo", algo)
    rng = np.random.default_rng(m % 1000)
    n = 4096
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    words = seb.new_words(m)
    kd = seb.dev_keys(to_dev(torch, keys), n=n, stride=16)
    seb.dev_build(kd, words, m, k)
    torch.cuda.synchronize()
    # compare positions touched: rebuild with the oracle sparsely (positions list)
    h1, h2 = bn.fnv_fixed(keys)
    pos = bn.positions(h1, h2, m, k).ravel()
    w = words.cpu().numpy().view(np.uint32)
    expect = np.zeros_like(w)
    np.bitwise_or.at(expect, (pos >> np.uint64(5)).astype(np.int64),
                     (np.uint32(1) << (pos & np.uint64(31)).astype(np.uint32)))
    assert np.array_equal(w, expect)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    seb.dev_probe(kd, words, m, k, out)
    torch.cuda.synchronize()
    assert bool(out.all())
    seb.set_option("build_algo", 0)


@pytest.mark.parametrize("m", [(1 << 29) - 3, 1 << 29, 33_554_433, 33_554_432 * 2 + 7])
def test_phased_probe_ranges(seb, torch_cuda, m):
    """The phased probe (default) at the edges of its domain: m just under 2^29 (the packed
    residue width, 16 ranges), m = 2^29 (falls back to the sliced probe), filters one bit over
    one and two 4 MiB ranges (2 and 3 ranges), and an answer array that is not 4-byte aligned
    (falls back).  Answers equal the oracle's for present and absent keys."""
    torch = torch_cuda
    k = 7
    rng = np.random.default_rng(m % 997)
    n = 60_000
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    words = seb.new_words(m)
    seb.dev_build(seb.dev_keys(to_dev(torch, keys), n=n, stride=16), words, m, k)
    probe = np.concatenate([keys[: n // 2], rng.integers(0, 256, (n - n // 2, 16), dtype=np.uint8)])
    # the oracle's answers: every position of the key set in the built words
    h1, h2 = bn.fnv_fixed(probe)
    pos = bn.positions(h1, h2, m, k)
    w = words.cpu().numpy().view(np.uint32)
    want = np.all((w[(pos >> np.uint64(5)).astype(np.int64)] >> (pos & np.uint64(31)).astype(np.uint32)) & 1,
                  axis=1).astype(np.uint8)
    assert want[: n // 2].all()
    pk = seb.dev_keys(to_dev(torch, probe), n=n, stride=16)
    buf = torch.full((n + 8,), 7, dtype=torch.uint8, device="cuda")
    for off in (0, 1):  # aligned (phased where it applies) and unaligned (fallback)
        out = buf[off: off + n]
        seb.dev_probe(pk, words, m, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want), off
    if m < (1 << 29):  # packed forms
        packed = torch.zeros(n, dtype=torch.int64, device="cuda")
        out = buf[:n]
        seb.dev_probe_emit_packed(pk, words, m, k, out, packed)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)
        out.fill_(7)
        seb.dev_probe_packed(packed, n, words, m, k, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)


def test_probe_split_variants(seb, golden, torch_cuda, probe_split):
    """The split-round probe (first-round gathers, the rest only where all bits so far are set)
    returns exactly the single-round answers."""
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 100000 and r["p"] == 0.01)
    n, m, k = row["n"], row["m"], row["k"]
    kd = seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16)
    words, bits = dev_build_bits(seb, torch, kd, m, k)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    seb.dev_probe(seb.dev_keys(to_dev(torch, kg.key16(kg.probe_indices(n))), n=n, stride=16), words, m, k, out)
    torch.cuda.synchronize()
    assert sha(out.cpu().numpy().tobytes()) == row["probe_sha256"]
    for nn in (1, 255, 513, 1001):  # ragged tails of the multi-key threads
        pk = kg.key16(kg.probe_indices(nn))
        o = torch.full((nn + 8,), 7, dtype=torch.uint8, device="cuda")
        seb.dev_probe(seb.dev_keys(to_dev(torch, pk), n=nn, stride=16), words, m, k, o)
        torch.cuda.synchronize()
        got = o.cpu().numpy()
        assert np.array_equal(got[:nn], oc.probe(bits, m, k, pk, nn, stride=16))
        assert (got[nn:] == 7).all()  # nothing written past n


def test_dev_build_with_caller_workspace(seb, golden, torch_cuda):
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 100000 and r["p"] == 0.01)
    n, m, k = row["n"], row["m"], row["k"]
    kd = seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16)
    with seb.option("build_algo", 2):
        need = seb.dev_build_workspace_size(n, m, k)
        assert need > 0
        ws = torch.empty(need, dtype=torch.uint8, device="cuda")
        words = seb.new_words(m)
        seb.dev_build_ws(kd, words, m, k, ws)
        torch.cuda.synchronize()
        assert sha(bn.encode(seb.words_to_bits(words, m), m, k)) == row["encode_sha256"]
        with pytest.raises(seb.SebError):
            seb.dev_build_ws(kd, words, m, k, ws[: need // 2])


def test_empty_batches(seb, ctx, torch_cuda, build_algo):
    torch = torch_cuda
    m, k = oc.params(100, 0.01)
    words = seb.new_words(m)
    kd = seb.seb_keys(None, None, 0, 16, 0)
    seb.dev_build(kd, words, m, k)
    out = torch.empty(1, dtype=torch.uint8, device="cuda")
    seb.dev_probe(kd, words, m, k, out)
    torch.cuda.synchronize()
    assert not words.any()
    assert ctx.build(np.zeros((0, 16), np.uint8), m, k).sum() == 0
    assert ctx.probe(np.zeros((0, 16), np.uint8), np.zeros(seb.num_bytes(m), np.uint8), m, k).size == 0


def test_fuzz_against_oracle(seb, ctx, build_algo):
    rng = np.random.default_rng(11)
    for trial in range(12):
        n = int(rng.integers(1, 3000))
        p = float(rng.choice([0.5, 0.1, 0.01, 1e-4, 1e-7]))
        m, k = seb.params(n, p)
        lens = rng.integers(0, 80, n)
        keys = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in lens]
        kb = seb.as_keys(keys)
        bits = ctx.build(kb, m, k)
        ref = oc.build(m, k, kb.data, n, offsets=kb.offsets)
        assert np.array_equal(bits, ref), (trial, n, p)
        probes = seb.as_keys(keys[::2] + [bytes(rng.integers(0, 256, 9, dtype=np.uint8)) for _ in range(n)])
        assert np.array_equal(ctx.probe(probes, bits, m, k),
                              oc.probe(ref, m, k, probes.data, probes.n, offsets=probes.offsets))


def shared_prefix_keys(rng, n):
    """(n, 16) u8 keys in blocks of 64 whose keys share their first L words (L = 0..4 per block;
    4: the block is one key repeated), with blocks where one lane breaks the prefix: the shapes a
    sorted flush batch gives a wave (the scalar-prefix hashing measured on them)."""
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    for b0 in range(0, n, 64):
        blk = keys[b0:b0 + 64]
        L = int(rng.integers(0, 5))
        blk[:, :4 * L] = blk[0, :4 * L]
        if L and rng.random() < 0.25:  # one lane differs in the shared words
            j = int(rng.integers(0, blk.shape[0]))
            blk[j, int(rng.integers(0, 4 * L))] ^= 0x5A
    return keys


@pytest.mark.parametrize("n", [1, 63, 64 * 37 + 13, 300_001])
def test_keys16_shared_prefix_waves(seb, torch_cuda, build_algo, probe_compact, n):
    """Fixed 16-B keys whose waves share 0-4 leading words (a sorted batch), ragged tails and
    duplicate keys: build bits and probe answers equal the oracle's for every build path and
    both probe layouts."""
    torch = torch_cuda
    rng = np.random.default_rng(n)
    keys = shared_prefix_keys(rng, n)
    m, k = seb.params(max(n, 2), 0.01)
    words = seb.new_words(m)
    seb.dev_build(seb.dev_keys(to_dev(torch, keys), n=n, stride=16), words, m, k)
    torch.cuda.synchronize()
    ref = oc.build(m, k, keys, n, stride=16)
    assert np.array_equal(seb.words_to_bits(words, m), ref)
    probes = np.concatenate([keys[::2], shared_prefix_keys(rng, n)])
    out = torch.empty(probes.shape[0], dtype=torch.uint8, device="cuda")
    seb.dev_probe(seb.dev_keys(to_dev(torch, probes), n=probes.shape[0], stride=16), words, m, k, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oc.probe(ref, m, k, probes, probes.shape[0], stride=16))


# ------------------------------------------------------------- multi-filter (C5) ------------

@pytest.mark.parametrize("which", [0, 1])
def test_multi_filter_probe(seb, golden, torch_cuda, which):
    torch = torch_cuda
    row = golden["multi"][which]
    nf, per, npr, m, k = row["filters"], row["keys_per_filter"], row["probes"], row["m"], row["k"]
    filters = []
    for f in range(nf):
        keys = to_dev(torch, kg.key16(f * per + np.arange(per)))
        words, bits = dev_build_bits(seb, torch, seb.dev_keys(keys, n=per, stride=16), m, k)
        assert sha(bn.encode(bits, m, k)) == row["filter_sha256"][f]
        filters.append((words, m, k))
    q = np.arange(npr, dtype=np.int64)
    half = q // 2
    pk = to_dev(torch, kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q)))
    kd = seb.dev_keys(pk, n=npr, stride=16)
    mask = torch.zeros(npr, dtype=torch.int64, device="cuda")
    seb.dev_probe_multi(kd, filters, mask)
    torch.cuda.synchronize()
    got = mask.cpu().numpy().view(np.uint64)
    assert sha(got.astype("<u8").tobytes()) == row["mask_sha256"]
    if nf <= 8:  # 1-byte mask plane (one GPU's share in the 8-GPU C5 layout)
        m8 = torch.zeros(npr, dtype=torch.uint8, device="cuda")
        seb.dev_probe_multi(kd, filters, m8)
        torch.cuda.synchronize()
        assert np.array_equal(m8.cpu().numpy(), (got & np.uint64(0xFF)).astype(np.uint8))
    # mixed (m, k) filters take the per-filter path
    m2, k2 = oc.params(per // 2, 0.001)
    w2 = seb.new_words(m2)
    seb.dev_build(seb.dev_keys(to_dev(torch, kg.key16(np.arange(per // 2))), n=per // 2, stride=16), w2, m2, k2)
    mixed = [filters[0], (w2, m2, k2)]
    mm = torch.zeros(npr, dtype=torch.uint8, device="cuda")
    seb.dev_probe_multi(kd, mixed, mm)
    torch.cuda.synchronize()
    b0 = seb.words_to_bits(filters[0][0], m)
    b1 = seb.words_to_bits(w2, m2)
    ref = oc.probe_multi([(b0, m, k), (b1, m2, k2)], kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf,
                                                                      nf * per + q)), npr, stride=16)
    assert np.array_equal(mm.cpu().numpy(), ref.astype(np.uint8))


@pytest.mark.parametrize("interleave,aligned", [(0, True), (1, True), (1, False)])
def test_multi_filter_interleaved_vs_direct(seb, golden, torch_cuda, interleave, aligned):
    """The interleaved (bit-transposed) table path and the per-filter path give identical masks; the
    table is built by wave ballots from 16-B aligned filters and entry by entry otherwise (word
    arrays starting 4 bytes into their buffers)."""
    torch = torch_cuda
    row = golden["multi"][1]  # 64 filters x 2000 keys
    nf, per, npr, m, k = row["filters"], row["keys_per_filter"], row["probes"], row["m"], row["k"]
    keys = to_dev(torch, kg.key16(np.arange(nf * per)))
    nw = seb.words_bytes(m) // 4
    filters = [((seb.new_words(m) if aligned else torch.zeros(nw + 4, dtype=torch.int32, device="cuda")[1:nw + 1]),
                m, k) for _ in range(nf)]
    seb.dev_build_many(seb.dev_keys(keys, n=nf * per, stride=16), [f * per for f in range(nf + 1)], filters)
    q = np.arange(npr, dtype=np.int64)
    half = q // 2
    kd = seb.dev_keys(to_dev(torch, kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q))),
                      n=npr, stride=16)
    with seb.option("multi_interleave", interleave):
        for dt, nsub in ((torch.int64, 64), (torch.int32, 32), (torch.int16, 16), (torch.uint8, 8), (torch.int64, 37),
                         (torch.uint8, 5)):
            mask = torch.zeros(npr, dtype=dt, device="cuda")
            seb.dev_probe_multi(kd, filters[:nsub], mask)
            torch.cuda.synchronize()
            got = mask.cpu().numpy().astype(np.int64).view(np.uint64) & np.uint64((1 << nsub) - 1 if nsub < 64 else
                                                                                   0xFFFFFFFFFFFFFFFF)
            if nsub == 64:
                assert sha(got.astype("<u8").tobytes()) == row["mask_sha256"]
            else:
                bits = [seb.words_to_bits(w, m) for w, _, _ in filters[:nsub]]
                ref = oc.probe_multi([(b, m, k) for b in bits], kg.key16(np.where(q % 2 == 0, (half % nf) * per +
                                                                                   half // nf, nf * per + q)), npr,
                                     stride=16)
                assert np.array_equal(got, ref), nsub


def test_multi_filter_host_api(seb, golden, ctx):
    row = golden["multi"][0]
    nf, per, npr, m, k = row["filters"], row["keys_per_filter"], row["probes"], row["m"], row["k"]
    filters = [(oc.build(m, k, kg.key16(f * per + np.arange(per)), per, stride=16), m, k) for f in range(nf)]
    q = np.arange(npr, dtype=np.int64)
    half = q // 2
    pk = kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q))
    got = ctx.probe_multi(pk, filters)
    assert sha(got.astype("<u8").tobytes()) == row["mask_sha256"]


@pytest.mark.parametrize("splits", [0, 1, 3, 8])
def test_build_many_splits(seb, torch_cuda, splits):
    """Compaction filters whose keys are split over several workgroups (atomic OR merge) equal the
    oracle; ragged key counts, an empty filter, and filters that already hold bits (OR-accumulate)."""
    torch = torch_cuda
    counts = [100_000, 33_333, 0, 65_537, 100_000, 1]
    begin = np.concatenate([[0], np.cumsum(counts)]).tolist()
    n = begin[-1]
    keys = kg.key16(np.arange(n) * 3 + 7)
    m, k = oc.params(100_000, 0.01)
    pre = kg.key16(np.arange(5000) * 5 + 1)  # bits already set in every filter
    filters = []
    for _ in counts:
        w = seb.new_words(m)
        seb.dev_build(seb.dev_keys(to_dev(torch, pre), n=5000, stride=16), w, m, k)
        filters.append((w, m, k))
    with seb.option("many_splits", splits):
        seb.dev_build_many(seb.dev_keys(to_dev(torch, keys), n=n, stride=16), begin, filters)
    torch.cuda.synchronize()
    for f, c in enumerate(counts):
        ref = oc.build(m, k, np.concatenate([pre, keys[begin[f]:begin[f + 1]]]), 5000 + c, stride=16)
        assert np.array_equal(seb.words_to_bits(filters[f][0], m), ref), f


def test_build_many_compaction_batch(seb, golden, torch_cuda):
    """Batched compaction-output build (lsm/compaction.go:286, 100K-key filters) in one launch:
    small filters built in LDS, one filter larger than LDS through the global path."""
    torch = torch_cuda
    row = golden["multi"][0]
    nf, per, m, k = row["filters"], row["keys_per_filter"], row["m"], row["k"]
    keys = to_dev(torch, kg.key16(np.arange((nf + 1) * per)))
    kd = seb.dev_keys(keys, n=(nf + 1) * per, stride=16)
    filters = [(seb.new_words(m), m, k) for _ in range(nf)]
    big_m, big_k = oc.params(2 * per * 10, 0.01)  # > 160 KiB of words -> global atomics path
    filters.append((seb.new_words(big_m), big_m, big_k))
    begin = [f * per for f in range(nf + 2)]  # filter f <- keys [begin[f], begin[f+1])
    seb.dev_build_many(kd, begin, filters)
    torch.cuda.synchronize()
    for f in range(nf):
        assert sha(bn.encode(seb.words_to_bits(filters[f][0], m), m, k)) == row["filter_sha256"][f], f
    last = kg.key16(np.arange(nf * per, (nf + 1) * per))
    assert np.array_equal(seb.words_to_bits(filters[-1][0], big_m), oc.build(big_m, big_k, last, per, stride=16))
    # C1-size compaction filters (100K keys, 119,814 B each) fit the LDS path
    m1, k1 = oc.params(100000, 0.01)
    assert seb.words_bytes(m1) <= 160 * 1024
    keys1 = to_dev(torch, kg.key16(np.arange(300000)))
    f1 = [(seb.new_words(m1), m1, k1) for _ in range(3)]
    seb.dev_build_many(seb.dev_keys(keys1, n=300000, stride=16), [0, 100000, 200000, 300000], f1)
    torch.cuda.synchronize()
    c1 = next(r for r in golden["fixed16"] if r["n"] == 100000 and r["p"] == 0.01)
    assert sha(bn.encode(seb.words_to_bits(f1[0][0], m1), m1, k1)) == c1["encode_sha256"]


@pytest.mark.parametrize("n,expected", [(1000, 1000), (100000, 100000), (70000, 100000), (1, 1)])
def test_c_harness_replays_sstable_sequence(seb, golden, n, expected):
    """storage-engines_amd/harness/sstable_replay.c: the exact call sequence the cgo shim makes for
    SSTableBuilder (New -> Add per entry -> Encode) and SSTable (Decode -> MayContain per Get);
    (70000, 100000) is a compaction output file sized for 100K keys (lsm/compaction.go:286)."""
    import json
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(seb.LIB_PATH), "sstable_replay")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(os.path.dirname(seb.LIB_PATH), "..", "harness")], check=True)
    out = subprocess.run([exe, str(n), str(expected)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout)
    assert res["batch_matches_single"]
    m, k = oc.params(expected, 0.01)
    assert (res["num_bits"], res["num_hashes"]) == (m, k)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    assert res["encode_sha256"] == sha(bn.encode(bits, m, k))
    ans = oc.probe(bits, m, k, kg.key16(kg.probe_indices(n)), n, stride=16)
    assert res["probe_sha256"] == sha(ans.tobytes())
    row = next((r for r in golden["fixed16"] if r["n"] == n and r["p"] == 0.01), None)
    if row is not None and expected == n:
        assert res["encode_sha256"] == row["encode_sha256"]
        assert res["probe_sha256"] == row["probe_sha256"]


def test_flush_bench_harness_parity(seb, golden):
    """harness/flush_bench.c (bench.py --config flush): New -> Add per key -> Encode at flush and
    compaction sizes, then Decode -> single-key MayContain on 1 and 8 threads at once and the
    batched GPU MayContain; every digest against the oracle (and the C1 golden row at 100K)."""
    import json
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(seb.LIB_PATH), "flush_bench")
    out = subprocess.run([exe, "--reps", "2", "--threads", "8", "1", "1000", "50000", "100000"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    res = json.loads(out.stdout)
    for r in res["sizes"]:
        n = r["n"]
        m, k = oc.params(n, 0.01)
        bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
        assert r["encode_sha256"] == sha(bn.encode(bits, m, k)), n
        ans = oc.probe(bits, m, k, kg.key16(kg.probe_indices(n)), n, stride=16)
        assert r["probe_sha256"] == sha(ans.tobytes()), n
        assert r["batch_matches_single"]
        row = next((g for g in golden["fixed16"] if g["n"] == n and g["p"] == 0.01), None)
        if row is not None:
            assert r["encode_sha256"] == row["encode_sha256"] and r["probe_sha256"] == row["probe_sha256"]


@pytest.mark.parametrize("n,expected", [(1000, 1000), (70000, 100000)])
def test_c_harness_under_host_asan(seb, golden, n, expected):
    """The SSTable replay harness against libseb_bloom.so built with host-side AddressSanitizer +
    UndefinedBehaviorSanitizer (tools/sanitize/Makefile; device code unchanged): the C ABI's host
    code (arena, chunked H2D pipeline, context pool, Encode/Decode) runs clean on the GPU and gives
    the same digests as the oracle."""
    import json
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(seb.LIB_PATH), "asan", "sstable_replay_asan")
    if not os.path.exists(exe):
        pytest.skip("host-ASan build missing: make -C tools/sanitize (part of __graft_entry__.build())")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe, str(n), str(expected)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-3000:]
    res = json.loads(out.stdout)
    m, k = oc.params(expected, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    assert res["batch_matches_single"]
    assert res["encode_sha256"] == sha(bn.encode(bits, m, k))
    assert res["probe_sha256"] == sha(oc.probe(bits, m, k, kg.key16(kg.probe_indices(n)), n, stride=16).tobytes())


# ------------------------------------------- registry + batched LSM lookup ----

def _lsm_get_model(files, key: bytes):
    """lsm/lsm.go:168-198 candidate walk over (slot, level, min, max, bits, m, k, seq) records:
    every L0 file in insertion order, then per level 1..4 the first file (by MinKey) whose range
    covers the key.  Returns the slots visited whose filter may contain the key, as a mask."""
    mask = 0
    for s in _lsm_get_walk(files, key):
        mask |= 1 << s
    return mask


def _lsm_get_walk(files, key: bytes):
    """The same walk as _lsm_get_model; the slots in visiting order (the list form)."""
    visited = []
    l0 = sorted((f for f in files if f["level"] == 0), key=lambda f: f["seq"])
    visited += l0
    for lvl in range(1, 5):
        for f in sorted((f for f in files if f["level"] == lvl), key=lambda f: (f["min"], f["seq"])):
            if f["min"] <= key <= f["max"]:
                visited.append(f)
                break
    out = []
    for f in visited:
        kb = np.frombuffer(key, np.uint8).reshape(1, -1) if key else np.zeros((1, 0), np.uint8)
        if oc.probe(f["bits"], f["m"], f["k"], kb, 1, stride=len(key))[0]:
            out.append(f["slot"])
    return out


def test_registry_multiget_matches_lsm_get_walk(seb, torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(17)
    reg = seb.Registry(0)
    files = []
    seq = 0

    def add(file_num, level, keys):
        nonlocal seq
        m, k = oc.params(max(len(keys), 1), 0.01)
        arr = np.frombuffer(b"".join(keys), np.uint8)
        lens = np.array([len(x) for x in keys], np.uint64)
        off = np.zeros(len(keys) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        bits = oc.build(m, k, arr, len(keys), offsets=off)
        mn, mx = min(keys), max(keys)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), mn, mx)
        files.append(dict(file=file_num, level=level, min=mn, max=mx, bits=bits, m=m, k=k, seq=seq, slot=slot))
        seq += 1

    universe = sorted({kg.key16_bytes(int(i)) for i in rng.integers(0, 200000, 30000)})
    # L0: 3 overlapping flushes of random subsets
    for f in range(3):
        add(100 + f, 0, sorted(rng.choice(universe, 2000, replace=False).tolist()))
    # L1..L3: non-overlapping contiguous ranges, added out of MinKey order
    for lvl, parts in ((1, 4), (2, 6), (3, 3)):
        chunks = np.array_split(np.array(universe, dtype=object), parts)
        for j in rng.permutation(parts):
            add(1000 * lvl + int(j), lvl, list(chunks[j]))
    # probes: present keys, absent keys inside ranges, keys outside every range, varied lengths
    probes = list(rng.choice(universe, 3000).tolist()) + [kg.key16_bytes(int(i)) for i in rng.integers(200000, 400000, 2000)]
    probes += [b"", b"a", b"user", b"zzzz" * 10, universe[0], universe[-1], universe[0][:-1]]
    got = reg.multiget(probes)
    want = np.array([_lsm_get_model(files, p) for p in probes], dtype=np.uint64)
    assert np.array_equal(got, want)
    # device-resident form on fixed 16-B keys
    fixed = [p for p in probes if len(p) == 16]
    dk = seb.dev_keys(to_dev(torch, np.frombuffer(b"".join(fixed), np.uint8)), n=len(fixed), stride=16)
    out = torch.zeros(len(fixed), dtype=torch.int64, device="cuda")
    reg.multiget_dev(dk, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), np.array([_lsm_get_model(files, p) for p in fixed],
                                                                      dtype=np.uint64))
    # compaction removes L0 files; slots are reused
    for f in [f for f in files if f["level"] == 0]:
        reg.remove(f["file"])
    files = [f for f in files if f["level"] != 0]
    add(4000, 4, sorted(rng.choice(universe, 5000, replace=False).tolist()))
    got = reg.multiget(probes)
    assert np.array_equal(got, np.array([_lsm_get_model(files, p) for p in probes], dtype=np.uint64))
    slots = reg.slots()
    assert len(slots) == len(files) and {v[0] for v in slots.values()} == {f["file"] for f in files}
    with pytest.raises(seb.SebError):
        reg.remove(123456)
    reg.close()


def test_registry_multiget_overlap_long_keys_generic_k(seb, torch_cuda):
    """The branches the LSM bench layout does not reach: an overlapping level (the reference's
    first-cover linear scan, lsm/lsm.go:184-196), range keys longer than the 16-byte LDS prefix
    that tie on it (HBM tail compare), prefix-of relations, and filters with k != 7."""
    rng = np.random.default_rng(29)
    reg = seb.Registry(0)
    files = []

    def add(file_num, level, keys, fpr, seq):
        m, k = oc.params(max(len(keys), 1), fpr)
        arr = np.frombuffer(b"".join(keys), np.uint8)
        lens = np.array([len(x) for x in keys], np.uint64)
        off = np.zeros(len(keys) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        bits = oc.build(m, k, arr, len(keys), offsets=off)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k, seq=seq,
                          slot=slot))

    pre = b"tenant/0000000/" + b"x"  # 16-byte shared prefix
    universe = sorted({pre + b"%06d" % int(i) + b"z" * int(rng.integers(0, 12)) for i in rng.integers(0, 50000, 6000)})
    universe += [pre[:-1], pre, pre + b"\x00", pre[:10]]
    universe = sorted(set(universe))
    seq = 0
    for lvl, parts, fpr in ((1, 5, 0.001), (2, 3, 0.05)):
        chunks = np.array_split(np.array(universe, dtype=object), parts)
        for j in range(parts):
            lo = max(0, len(chunks[0]) * j - 200)  # overlap the previous chunk by ~200 keys
            keys = universe[lo:lo + len(chunks[j]) + 200]
            add(1000 * lvl + j, lvl, keys, fpr, seq)
            seq += 1
    add(3000, 3, universe[::7], 0.2, seq)
    probes = list(rng.choice(universe, 2000).tolist())
    probes += [pre + b"%06d" % int(i) for i in rng.integers(0, 50000, 1500)]
    probes += [pre, pre[:-1], pre[:15] + b"y", pre + b"\x00", pre + b"\x00\x00", b"", b"tenant/", universe[-1] + b"!"]
    got = reg.multiget(probes)
    want = np.array([_lsm_get_model(files, p) for p in probes], dtype=np.uint64)
    assert np.array_equal(got, want)
    reg.close()


def _walk_rows(files, probes, cap):
    want = np.full((len(probes), cap), 0xFFFF, dtype=np.uint16)
    for i, p in enumerate(probes):
        w = _lsm_get_walk(files, p)
        want[i, : len(w)] = w
    return want


def test_registry_multiget_list_beyond_64_files(seb, torch_cuda):
    """A registry past 64 files (an LSM with populated L1/L2: 400 MB / ~4 MB files,
    lsm/levels.go:10-14, lsm/compaction.go:253): the slot table is read from HBM instead of LDS
    and the answer is the list form, the slots Get would consult whose filter may contain the key
    in visiting order.  The u64 mask form refuses slots >= 64; cap below the longest walk is
    refused; the list form at <= 64 files (LDS table) agrees with the mask form."""
    torch = torch_cuda
    rng = np.random.default_rng(41)
    reg = seb.Registry(0)
    files = []
    seq = 0

    def add(file_num, level, keys):
        nonlocal seq
        m, k = oc.params(max(len(keys), 1), 0.01)
        arr = np.frombuffer(b"".join(keys), np.uint8)
        bits = oc.build(m, k, arr, len(keys), stride=16)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k, seq=seq,
                          slot=slot))
        seq += 1

    universe = sorted({kg.key16_bytes(int(i)) for i in rng.integers(0, 400000, 40000)})
    for f in range(3):
        add(100 + f, 0, sorted(rng.choice(universe, 1500, replace=False).tolist()))
    for lvl, parts in ((1, 20), (2, 90), (3, 7)):
        chunks = np.array_split(np.array(universe, dtype=object), parts)
        for j in rng.permutation(parts):
            add(1000 * lvl + int(j), lvl, list(chunks[j]))
    assert len(files) == 120 and max(f["slot"] for f in files) == 119
    assert reg.max_candidates() == 3 + 3
    probes = list(rng.choice(universe, 3000).tolist()) + [kg.key16_bytes(int(i)) for i in rng.integers(400000, 800000, 2000)]
    probes += [universe[0], universe[-1], b"\x00" * 16, b"\xff" * 16]
    got = reg.multiget_list(probes)
    assert got.shape == (len(probes), 6)
    assert np.array_equal(got, _walk_rows(files, probes, 6))
    # a wider row pads with 0xFFFF
    got8 = reg.multiget_list(probes[:500], cap=8)
    assert np.array_equal(got8, _walk_rows(files, probes[:500], 8))
    with pytest.raises(seb.SebError):
        reg.multiget(probes[:10])
    with pytest.raises(seb.SebError):
        reg.multiget_list(probes[:10], cap=5)
    # device-resident form on fixed 16-B keys (rng.choice's bytes array drops trailing NULs)
    fixed = [p for p in probes if len(p) == 16]
    dk = seb.dev_keys(to_dev(torch, np.frombuffer(b"".join(fixed), np.uint8)), n=len(fixed), stride=16)
    out = torch.zeros((len(fixed), 6), dtype=torch.int16, device="cuda")
    reg.multiget_list_dev(dk, out, 6)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), _walk_rows(files, fixed, 6))
    # rows of <= 16 slots are stored as u64 / u32 / u16 words by cap and alignment, wider rows
    # slot by slot: every cap and a 2-B-aligned output give the same rows
    want_rows = {cap: _walk_rows(files, fixed, cap) for cap in (6, 7, 8, 12, 16, 17, 20)}
    for cap, want_c in want_rows.items():
        for shift in (0, 1):
            flat = torch.full((len(fixed) * cap + 1,), 7, dtype=torch.int16, device="cuda")
            view = flat[shift:shift + len(fixed) * cap].view(len(fixed), cap)
            reg.multiget_list_dev(dk, view, cap)
            torch.cuda.synchronize()
            assert np.array_equal(view.cpu().numpy().view(np.uint16), want_c), (cap, shift)
            assert int(flat[len(fixed) * cap if shift == 0 else 0].item()) == 7  # nothing written past the rows
    # L2 compacted away: 30 files (LDS slot table), but L3 keeps slots 113..119, beyond a u64 mask
    for f in [f for f in files if f["level"] == 2]:
        reg.remove(f["file"])
    files = [f for f in files if f["level"] != 2]
    assert reg.max_candidates() == 5
    assert np.array_equal(reg.multiget_list(probes), _walk_rows(files, probes, 5))
    with pytest.raises(seb.SebError):
        reg.multiget(probes[:10])
    # L3 gone too: every slot < 64, and the mask form agrees with the list form
    for f in [f for f in files if f["level"] == 3]:
        reg.remove(f["file"])
    files = [f for f in files if f["level"] < 2]
    assert reg.max_candidates() == 4
    assert np.array_equal(reg.multiget_list(probes), _walk_rows(files, probes, 4))
    mask = reg.multiget(probes)  # every remaining slot is < 64: the mask form works again
    want = np.zeros(len(probes), np.uint64)
    for i, row in enumerate(_walk_rows(files, probes, 4)):
        for s in row[row != 0xFFFF]:
            want[i] |= np.uint64(1) << np.uint64(s)
    assert np.array_equal(mask, want)
    reg.close()


def test_registry_multiget_key_range_order(seb, torch_cuda):
    """multiget_order: a batch of >= 64K keys is walked in key-range order over the registry's
    disjoint level with the most files (bucket = files whose MinKey <= key).  Every answer must
    equal the batch-order walk's, for masks and lists, host (variable-length) and device keys,
    keys below the first file, between files and above the last; a model check on a sample."""
    torch = torch_cuda
    rng = np.random.default_rng(53)
    reg = seb.Registry(0)
    files = []
    seq = 0

    def add(file_num, level, keys):
        nonlocal seq
        m, k = oc.params(max(len(keys), 1), 0.01)
        arr = np.frombuffer(b"".join(keys), np.uint8)
        lens = np.array([len(x) for x in keys], np.uint64)
        off = np.zeros(len(keys) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        bits = oc.build(m, k, arr, len(keys), offsets=off)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k, seq=seq,
                          slot=slot))
        seq += 1

    universe = [kg.key16_bytes(int(i)) for i in range(1000, 61000, 2)]  # sorted: key16 sorts as i
    for f in range(2):
        add(100 + f, 0, sorted(rng.choice(universe, 3000, replace=False).tolist()))
    chunks = np.array_split(np.array(universe, dtype=object), 40)
    for j in rng.permutation(40):  # the partition level: 40 disjoint files, registered out of order
        add(1000 + int(j), 1, [c for c in chunks[j]][::3])
    for j in range(3):  # an overlapping level (linear first-cover scan)
        add(2000 + j, 2, universe[j * 8000: j * 8000 + 14000:5])
    n = 120_000
    idx = rng.integers(0, 64000, n)
    probes = [kg.key16_bytes(int(i)) for i in idx]
    probes[:4] = [b"", b"a", b"user0000000000", b"zzzz"]
    with seb.option("multiget_order", 0):
        want_mask = reg.multiget(probes)
        want_list = reg.multiget_list(probes)
        want_odd = reg.multiget_list(probes, cap=5)  # odd rows: the unpermute moves u16 granules
        want_wide = reg.multiget_list(probes, cap=20)  # 40-B rows: u32 granules staged in 3 passes
    # multiget_xcd: the XCD-contiguous block remap walks the same rows; order 1 reads fixed keys
    # through segment tables, order 2 (round 5's form) moves them by a scatter pass
    for order, xcd in ((1, 0), (1, 1), (2, 1)):
        with seb.option("multiget_order", order), seb.option("multiget_xcd", xcd):
            got_mask = reg.multiget(probes)
            got_list = reg.multiget_list(probes)
            got_odd = reg.multiget_list(probes, cap=5)
            got_wide = reg.multiget_list(probes, cap=20)
        assert np.array_equal(got_wide, want_wide) and np.array_equal(got_wide[:, :4], want_list), xcd
        assert np.array_equal(got_mask, want_mask), xcd
        assert np.array_equal(got_list, want_list), xcd
        assert np.array_equal(got_odd, want_odd) and np.array_equal(got_odd[:, :4], want_list), xcd
    sample = list(range(0, n, 97)) + [0, 1, 2, 3]
    assert np.array_equal(got_list[sample], _walk_rows(files, [probes[i] for i in sample], got_list.shape[1]))
    fixed = np.frombuffer(b"".join(p for p in probes if len(p) == 16), np.uint8)
    nf = fixed.size // 16
    dk = seb.dev_keys(to_dev(torch, fixed), n=nf, stride=16)
    outs, lists = [], []
    for order in (0, 1, 2):
        with seb.option("multiget_order", order):
            out = torch.zeros(nf, dtype=torch.int64, device="cuda")
            reg.multiget_dev(dk, out)
            lst = torch.zeros((nf, want_list.shape[1]), dtype=torch.int16, device="cuda")
            reg.multiget_list_dev(dk, lst, want_list.shape[1])  # list form with the keys moved
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
            lists.append(lst.cpu().numpy().view(np.uint16))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert np.array_equal(lists[0], lists[1]) and np.array_equal(lists[0], lists[2])
    # a batch walked in ordered pieces (multiget_piece_mib 1: 64K-key pieces, the last ragged)
    with seb.option("multiget_order", 1), seb.option("multiget_piece_mib", 1):
        out = torch.zeros(nf, dtype=torch.int64, device="cuda")
        reg.multiget_dev(dk, out)
        lst = torch.zeros((nf, want_list.shape[1]), dtype=torch.int16, device="cuda")
        reg.multiget_list_dev(dk, lst, want_list.shape[1])
        torch.cuda.synchronize()
        assert nf > 65536 and np.array_equal(out.cpu().numpy(), outs[0])
        assert np.array_equal(lst.cpu().numpy().view(np.uint16), lists[0])
        assert np.array_equal(reg.multiget(probes), want_mask)
    # The order's scratch cannot be had (a 1 MiB workspace cap; its first request is ~2.6 MB):
    # MultiGet falls back to batch order and answers the same.  A failed HIP call made just before
    # (the caller's hipMalloc of 2^60 B, its error left unread) must not leak into the MultiGet's
    # launch check.
    import ctypes

    seb.workspace_release()
    hip = ctypes.CDLL("libamdhip64.so")
    fell = int(seb.lib().seb_multiget_order_fallbacks())
    with seb.option("multiget_order", 1), seb.option("workspace_limit_mib", 1):
        out = torch.zeros(nf, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(1 << 60)) != 0  # left unread in HIP's state
        reg.multiget_dev(dk, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), outs[0])
        assert np.array_equal(reg.multiget(probes), want_mask)
        assert np.array_equal(reg.multiget_list(probes), want_list)
        assert int(seb.lib().seb_multiget_order_fallbacks()) >= fell + 3  # each counted as batch order
        with pytest.raises(seb.SebError):  # a build whose scratch is over the cap fails loudly
            big = seb.dev_keys(to_dev(torch, kg.key16(np.arange(1_000_000))), n=1_000_000, stride=16)
            with seb.option("build_algo", 2):
                seb.dev_build(big, seb.new_words(9_585_059), 9_585_059, 7)
    seb.workspace_release()
    fixed_rows = np.array([i for i, p in enumerate(probes) if len(p) == 16])
    assert np.array_equal(lists[1], want_list[fixed_rows])
    # host fixed 16-B chunks: staged into aligned device buffers, so the keys move as well
    host16 = fixed.reshape(nf, 16)
    with seb.option("multiget_order", 1):
        assert np.array_equal(reg.multiget(host16), want_mask[fixed_rows])
        assert np.array_equal(reg.multiget_list(host16), want_list[fixed_rows])
        # file numbers from one atomic call equal the list form mapped through the slot table
        files_got = reg.multiget_files(probes[:70000])
    by_slot = {s: fn for s, (fn, _) in reg.slots().items()}
    want_files = np.full((70000, files_got.shape[1]), np.iinfo(np.uint64).max, np.uint64)
    for i, row in enumerate(want_list[:70000]):
        for j, s in enumerate(row[row != 0xFFFF]):
            want_files[i, j] = by_slot[int(s)]
    assert files_got.shape[1] == reg.max_candidates()
    assert np.array_equal(files_got, want_files)
    # a batch past 8192 tiles x 2048 keys: tiles of two LDS-sorted chunks, the last one ragged
    nbig = 17_000_003
    big = to_dev(torch, kg.key16(rng.integers(0, 64000, nbig)))
    dbig = seb.dev_keys(big, n=nbig, stride=16)
    res = []
    for order in (0, 1, 2):
        with seb.option("multiget_order", order):
            out = torch.zeros(nbig, dtype=torch.int64, device="cuda")
            reg.multiget_dev(dbig, out)
            torch.cuda.synchronize()
            res.append(out.cpu().numpy())
    assert np.array_equal(res[0], res[1]) and np.array_equal(res[0], res[2])
    reg.close()


@pytest.mark.parametrize("nfiles", [31, 32, 254, 255])
def test_registry_multiget_narrow_sorted_rows(seb, torch_cuda, nfiles):
    """The key-range order's sorted rows travel narrow when the slots allow: masks as u32 when
    every slot is < 32 (one L0 file + 31 partition files: slots 0-31), list rows of <= 16 slots as
    u8 when every slot is < 255 (0xFF = none; 1 + 254 files: slots 0-254).  One slot more keeps
    the wide rows.  Every form equals the batch-order walk, for device and host keys, two batch
    sizes, both ordering forms and ordered pieces; list caps 2 / 4 / 6 (narrow when even) and
    5 / 20 (wide)."""
    torch = torch_cuda
    rng = np.random.default_rng(nfiles)
    reg = seb.Registry(0)
    universe = [kg.key16_bytes(int(i)) for i in range(1000, 61000, 2)]

    def add(file_num, level, keys):
        m, k = oc.params(len(keys), 0.01)
        bits = oc.build(m, k, np.frombuffer(b"".join(keys), np.uint8), len(keys), stride=16)
        return reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))

    slots = [add(100, 0, sorted(rng.choice(universe, 3000, replace=False).tolist()))]
    for j, c in enumerate(np.array_split(np.array(universe, dtype=object), nfiles)):
        slots.append(add(1000 + j, 1, list(c)[::3]))
    assert max(slots) == nfiles  # the largest slot id in use
    masks = nfiles < 64
    for n in (65_536, 200_003):
        keys = kg.key16(rng.integers(0, 64000, n))
        dk = seb.dev_keys(to_dev(torch, keys), n=n, stride=16)
        got, lists = [], {}
        # order 1 also in ordered pieces of 64K keys (multiget_piece_mib 1), the last one ragged
        for order, piece in ((0, 1024), (1, 1024), (2, 1024), (1, 1)):
            with seb.option("multiget_order", order), seb.option("multiget_piece_mib", piece):
                if masks:
                    out = torch.full((n,), -1, dtype=torch.int64, device="cuda")
                    reg.multiget_dev(dk, out)
                    torch.cuda.synchronize()
                    got.append(out.cpu().numpy())
                    if order:
                        assert np.array_equal(reg.multiget(keys), got[0])  # host keys, staged and moved
                for cap in (2, 4, 5, 6, 20):
                    lst = torch.full((n, cap), -7, dtype=torch.int16, device="cuda")
                    reg.multiget_list_dev(dk, lst, cap)
                    torch.cuda.synchronize()
                    lists.setdefault(cap, []).append(lst.cpu().numpy().view(np.uint16))
        if masks:
            assert all(np.array_equal(got[0], g) for g in got[1:])
            if nfiles == 32:
                assert (got[0] >> 32 != 0).any()  # slot 32 answers: the u64 rows carry bits past 31
        for cap, ls in lists.items():
            assert all(np.array_equal(ls[0], x) for x in ls[1:]), cap
            assert np.array_equal(ls[0][:, :2], lists[2][0]), cap  # a longer row extends the short one
        if nfiles == 255:
            assert (lists[4][0] == 255).any()  # slot 255 answers: the u16 rows carry it
    reg.close()


def test_registry_l0_group_table(seb, torch_cuda):
    """The L0 files sharing (m, k) are tested through one bit-interleaved table (multiget_l0_group):
    every answer, mask and list form, equals the per-file walk (option off) and the Python model of
    LSM.Get's walk, with a differently sized L0 file between the members (visiting order kept), as
    members are removed (group of 3 -> 2 -> none), for 5 members (8-bit entries) and for k != 7."""
    rng = np.random.default_rng(67)

    def run(layout_l0, p=0.01, probes_n=20_000):
        reg = seb.Registry(0)
        files = []
        universe = [kg.key16_bytes(int(i)) for i in range(0, 60_000, 2)]

        def add(file_num, level, keys, fpr):
            m, k = oc.params(max(len(keys), 1), fpr)
            arr = np.frombuffer(b"".join(keys), np.uint8)
            bits = oc.build(m, k, arr, len(keys), stride=16)
            slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
            files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k,
                              seq=len(files), slot=slot))

        for f, nkeys in enumerate(layout_l0):
            add(10 + f, 0, sorted(rng.choice(universe, nkeys, replace=False).tolist()), p)
        chunks = np.array_split(np.array(universe, dtype=object), 10)
        for j in rng.permutation(10):
            add(1000 + int(j), 1, list(chunks[j])[::3], 0.01)
        idx = rng.integers(0, 64_000, probes_n)
        probes = kg.key16(idx)
        return reg, files, probes

    def check(reg, files, probes):
        cap = reg.max_candidates()
        res = {}
        for grp in (1, 0):
            with seb.option("multiget_l0_group", grp):
                res[grp] = (reg.multiget_list(probes, cap=cap),
                            reg.multiget(probes) if max(f["slot"] for f in files) < 64 else None)
        assert np.array_equal(res[1][0], res[0][0])
        if res[1][1] is not None:
            assert np.array_equal(res[1][1], res[0][1])
        sample = list(range(0, len(probes), 97))
        assert np.array_equal(res[1][0][sample], _walk_rows(files, [probes[i].tobytes() for i in sample], cap))
        return res[1][0]

    # A, B, D (other size), C: group {A, B, C} with 4-bit entries, D tested alone between B and C
    reg, files, probes = run([2000, 2000, 1500, 2000])
    rows = check(reg, files, probes)
    assert all((rows == f["slot"]).any() for f in files if f["level"] == 0)  # each L0 file answers "maybe"
    for fn in (11, 10):  # group of 2 (2-bit entries), then none (C alone shares no shape)
        reg.remove(fn)
        files[:] = [f for f in files if f["file"] != fn]
        check(reg, files, probes)
    reg.close()
    # five members: 8-bit entries; and a k = 4 group (p = 0.1: the generic-k position walk)
    for layout, p in (([1000] * 5, 0.01), ([3000, 3000, 3000], 0.1)):
        reg, files, probes = run(layout, p)
        check(reg, files, probes)
        reg.close()


@pytest.mark.parametrize("parts", [1020, 255, 256])
def test_registry_key_range_order_wide_partition_level(seb, torch_cuda, parts):
    """Key-range order over a partition level of 1020 files (1021 buckets, near kMgMaxBuckets =
    1025: the block scans run 4 buckets per thread), with an L1 of 60 files over it and two L0
    files, on a 300K-key batch with keys below, between and above the files: the list rows equal
    the batch-order walk's and, on a sample, the Python model of LSM.Get's walk.  255 and 256
    files straddle the bucket ids' switch from u8 (at most 256 buckets, ids up to 255) to u16."""
    torch = torch_cuda
    rng = np.random.default_rng(61)
    reg = seb.Registry(0)
    files = []

    def add(file_num, level, keys):
        m, k = oc.params(max(len(keys), 1), 0.01)
        arr = np.frombuffer(b"".join(keys), np.uint8)
        bits = oc.build(m, k, arr, len(keys), stride=16)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k,
                          seq=len(files), slot=slot))

    universe = [kg.key16_bytes(int(i)) for i in range(10_000, 10_000 + 2 * 40_800, 2)]  # sorted
    for f in range(2):
        add(10 + f, 0, sorted(rng.choice(universe, 500, replace=False).tolist()))
    for lvl, nparts in ((1, 60), (2, parts)):
        chunks = np.array_split(np.array(universe, dtype=object), nparts)
        for j in rng.permutation(nparts):
            add(10_000 * lvl + int(j), lvl, list(chunks[j])[::2])
    assert reg.max_candidates() == 4
    n = 300_000
    pk = kg.key16(rng.integers(0, 100_000, n))
    probes = pk.reshape(n, 16)
    with seb.option("multiget_order", 0):
        want = reg.multiget_list(probes)
    with seb.option("multiget_order", 1):
        got = reg.multiget_list(probes)
        dk = seb.dev_keys(to_dev(torch, pk), n=n, stride=16)
        out = torch.zeros((n, 4), dtype=torch.int16, device="cuda")
        reg.multiget_list_dev(dk, out, 4)
        torch.cuda.synchronize()
    with seb.option("multiget_order", 2):  # round 5's scatter form
        got2 = reg.multiget_list(probes)
    assert np.array_equal(got, want) and np.array_equal(got2, want)
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    sample = list(range(0, n, 499))
    assert np.array_equal(want[sample], _walk_rows(files, [probes[i].tobytes() for i in sample], 4))
    reg.close()


def test_registry_key_range_order_long_min_keys(seb, torch_cuda):
    """Key-range order over a partition level whose MinKeys are longer than 16 bytes and share
    their first 16 bytes: the bucket pass must break the tie with the HBM tail compare.  Probes
    share that 16-byte prefix and differ only after byte 16 (host variable-length keys, which
    go through the index, and a device stride-22 batch, which is not moved)."""
    torch = torch_cuda
    rng = np.random.default_rng(59)
    reg = seb.Registry(0)
    files = []
    pre = b"tenant/0000042/x"  # 16 bytes shared by every key and every MinKey
    assert len(pre) == 16
    universe = [pre + b"%06d" % i for i in range(0, 90000, 3)]  # sorted

    def add(file_num, level, keys, seq):
        m, k = oc.params(len(keys), 0.01)
        lens = np.array([len(x) for x in keys], np.uint64)
        off = np.zeros(len(keys) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        bits = oc.build(m, k, np.frombuffer(b"".join(keys), np.uint8), len(keys), offsets=off)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k, seq=seq,
                          slot=slot))

    chunks = np.array_split(np.array(universe, dtype=object), 24)
    for seq, j in enumerate(rng.permutation(24)):
        add(500 + int(j), 1, list(chunks[j])[::2], seq)
    add(900, 0, universe[::50], 99)
    n = 70_000
    idx = rng.integers(0, 92000, n)
    probes = [pre + b"%06d" % int(i) for i in idx]
    probes[:6] = [pre, pre[:15], pre + b"\x00", pre + b"000000", pre + b"999999", pre[:15] + b"y"]
    with seb.option("multiget_order", 0):
        want = reg.multiget_list(probes)
    with seb.option("multiget_order", 1):
        got = reg.multiget_list(probes)
    assert np.array_equal(got, want)
    sample = list(range(0, n, 131)) + list(range(6))
    assert np.array_equal(got[sample], _walk_rows(files, [probes[i] for i in sample], got.shape[1]))
    dev = np.frombuffer(b"".join(p for p in probes if len(p) == 22), np.uint8)
    rows = np.array([i for i, p in enumerate(probes) if len(p) == 22])
    dk = seb.dev_keys(to_dev(torch, dev), n=rows.size, stride=22)
    for order in (0, 1):
        with seb.option("multiget_order", order):
            out = torch.zeros((rows.size, want.shape[1]), dtype=torch.int16, device="cuda")
            reg.multiget_list_dev(dk, out, want.shape[1])
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint16), want[rows])
    reg.close()


def test_shared_stream_threads_and_workspace_release(seb, golden, torch_cuda):
    """Library scratch is per (device, stream); two host threads calling on ONE stream must not
    interleave launches on it or free it under each other (growing batch sizes force the grow
    path).  seb_workspace_release frees it all; the next call re-allocates."""
    import threading
    torch = torch_cuda
    m, k = seb.params(10_000_000, 0.01)  # a 12 MB filter: the phased probe keeps packed scratch
    keys = kg.key16(np.arange(1_000_000)).reshape(-1)
    words = seb.new_words(m)
    dk_all = seb.dev_keys(to_dev(torch, keys), n=1_000_000, stride=16)
    seb.dev_build(dk_all, words, m, k)
    qn = [200_000, 1_000_000]
    qkeys = [kg.key16(kg.probe_indices(1_000_000, count=q)).reshape(-1) for q in qn]
    qdev = [to_dev(torch, q) for q in qkeys]
    want = [oc.probe(oc.build(m, k, keys, 1_000_000, stride=16), m, k, q, q.size // 16, stride=16) for q in qkeys]
    stream = torch.cuda.current_stream()
    errors = []

    def worker(t):
        try:
            dk = seb.dev_keys(qdev[t], n=qn[t], stride=16)
            for it in range(12):
                out = torch.zeros(qn[t], dtype=torch.uint8, device="cuda")
                seb.dev_probe(dk, words, m, k, out, stream=stream)
                stream.synchronize()
                if not np.array_equal(out.cpu().numpy(), want[t]):
                    errors.append((t, it))
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    seb.workspace_release()
    assert seb.workspace_bytes() == 0
    th = [threading.Thread(target=worker, args=(t,)) for t in (0, 1, 0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert seb.workspace_bytes() > 0
    seb.workspace_release()
    assert seb.workspace_bytes() == 0
    out = torch.zeros(qn[1], dtype=torch.uint8, device="cuda")
    seb.dev_probe(seb.dev_keys(qdev[1], n=qn[1], stride=16), words, m, k, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want[1])


def test_workspace_release_after_context_streams_destroyed(seb, torch_cuda):
    """A context's (and a registry's) streams hold library scratch while they live: destroying the
    context gives it back, so a later seb_workspace_release never synchronises a dead stream."""
    m, k = seb.params(10_000_000, 0.01)  # phased probe: packed scratch on the context's stream
    keys = kg.key16(np.arange(200_000)).reshape(-1)
    q = kg.key16(kg.probe_indices(200_000, count=300_000)).reshape(-1)
    bits = oc.build(m, k, keys, 200_000, stride=16)
    want = oc.probe(bits, m, k, q, 300_000, stride=16)
    seb.workspace_release()
    for _ in range(3):
        ctx = seb.Ctx(0)
        assert np.array_equal(ctx.probe(seb.HostKeys(q.reshape(-1, 16)), bits, m, k), want)
        assert seb.workspace_bytes() > 0
        ctx.close()
        assert seb.workspace_bytes() == 0
        seb.workspace_release()
    reg = seb.Registry(0)
    for f in range(3):
        fk = [kg.key16_bytes(int(i)) for i in range(f * 1000, f * 1000 + 1000)]
        fm, fkk = oc.params(len(fk), 0.01)
        fb = oc.build(fm, fkk, np.frombuffer(b"".join(fk), np.uint8), len(fk), stride=16)
        reg.put(10 + f, 0, bn.encode(fb, fm, fkk), min(fk), max(fk))
    probes = [kg.key16_bytes(int(i)) for i in range(0, 6000, 3)]
    got = reg.multiget(probes)
    reg.close()
    seb.workspace_release()
    assert seb.workspace_bytes() == 0
    assert got.shape == (len(probes),)


def test_registry_full_capacity(seb, torch_cuda):
    """4096 files (the u16 slot-id capacity): one L0 file and 4095 one-key L1 files.  The
    4097th put is refused; the list form still answers every key as Get's walk does, and a key
    between two files' ranges visits only L0."""
    reg = seb.Registry(0)
    files = []

    def add(file_num, level, keys, seq):
        m, k = oc.params(len(keys), 0.01)
        bits = oc.build(m, k, np.frombuffer(b"".join(keys), np.uint8), len(keys), stride=16)
        slot = reg.put(file_num, level, bn.encode(bits, m, k), min(keys), max(keys))
        files.append(dict(file=file_num, level=level, min=min(keys), max=max(keys), bits=bits, m=m, k=k, seq=seq,
                          slot=slot))

    add(1, 0, [kg.key16_bytes(2 * j) for j in range(0, 8190, 7)], 0)
    for j in range(4095):
        add(10 + j, 1, [kg.key16_bytes(2 * j)], 1 + j)
    assert max(f["slot"] for f in files) == 4095
    m, k = oc.params(1, 0.01)
    with pytest.raises(seb.SebError):
        reg.put(99999, 1, bn.encode(np.zeros((m + 7) // 8, np.uint8), m, k), b"zz", b"zz")
    rng = np.random.default_rng(3)
    probes = [kg.key16_bytes(int(i)) for i in rng.integers(0, 8190, 300)]
    probes = [p for p in probes if len(p) == 16]
    assert reg.max_candidates() == 2
    got = reg.multiget_list(probes)
    assert np.array_equal(got, _walk_rows(files, probes, 2))
    reg.close()


@pytest.mark.parametrize("case", ["duplicates", "skewed", "large_m"])
def test_bucketed_build_overflow_and_lds_limits(seb, torch_cuda, case):
    """Radix-partitioned build paths a hash-distributed batch never takes: runs that overflow
    their fixed-capacity region (identical keys put a tile's positions into 7 buckets; skewed: a
    few distinct keys repeated) fall back to device-scope atomic OR, and a filter with more
    buckets than the 5-keys-per-thread LDS layout holds (m = 200M bits) uses 4 keys per thread.
    The bit array must equal the oracle's either way."""
    torch = torch_cuda
    seb.set_option("build_algo", 2)
    try:
        rng = np.random.default_rng(5)
        if case == "duplicates":
            n, m, k = 400_000, 3_834_024, 7
            keys = np.tile(kg.key16(np.array([42])), (n, 1))
        elif case == "skewed":
            n, m, k = 400_000, 3_834_024, 7
            keys = kg.key16(rng.integers(0, 50, n))
        else:
            n, m, k = 300_000, 200_000_000, 7
            keys = kg.key16(np.arange(n))
        kd = seb.dev_keys(to_dev(torch, keys), n=n, stride=16)
        words, bits = dev_build_bits(seb, torch, kd, m, k)
        uniq = np.unique(keys, axis=0)
        ref = oc.build(m, k, np.ascontiguousarray(uniq).ravel(), len(uniq), stride=16)
        assert np.array_equal(bits, ref)
    finally:
        seb.set_option("build_algo", 0)


@pytest.mark.parametrize("bins", [1, 0], ids=["bins", "counting"])
@pytest.mark.parametrize("case", ["nb513", "c2m", "nb2274", "duplicates", "skewed"])
def test_bucketed_scatter_bins(seb, torch_cuda, case, bins):
    """The radix-partitioned build's two scatters (scatter_bins 1: fixed LDS bins, runs padded to
    16-B chunks; 0: the counting sort) against the oracle, both as a fresh build into garbage words
    and OR-ed into a filter: ordinary keys at the smallest and largest bucket counts the bins take
    (513 and 2274 buckets: shorter rounds below 94M bits) and at C2's m, plus runs that pass their
    bin and then their region (every key identical: 7 buckets get every position of a tile) or
    skewed (50 distinct keys)."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    m = {"nb513": 33_580_000, "nb2274": 149_000_000}.get(case, 95_850_584)
    k = 7
    if case == "duplicates":
        n = 400_000
        keys = np.tile(kg.key16(np.array([42])), (n, 1))
    elif case == "skewed":
        n = 400_000
        keys = kg.key16(rng.integers(0, 50, n))
    else:
        n = 1_000_003
        keys = kg.key16(rng.permutation(3 * n)[:n])
    uniq = np.unique(keys, axis=0)
    ref = oc.build(m, k, np.ascontiguousarray(uniq).ravel(), len(uniq), stride=16)
    kd = seb.dev_keys(to_dev(torch, keys), n=n, stride=16)
    with seb.option("build_algo", 2), seb.option("scatter_bins", bins):
        words = seb.new_words(m)
        for rep in range(2):
            words.view(torch.uint8).fill_(0xC3 if rep == 0 else 0xFF)
            seb.dev_build_fresh(kd, words, m, k)
            torch.cuda.synchronize()
            raw = words.cpu().numpy().view(np.uint8)
            assert np.array_equal(raw[: (m + 7) // 8], ref), (case, bins, rep)
            assert not raw[(m + 7) // 8:].any()
        # OR-accumulating build: half the keys into a fresh filter, then all of them
        w2 = seb.new_words(m)
        seb.dev_build(seb.dev_keys(to_dev(torch, keys[: n // 2]), n=n // 2, stride=16), w2, m, k)
        seb.dev_build(kd, w2, m, k)
        torch.cuda.synchronize()
        assert np.array_equal(seb.words_to_bits(w2, m), ref), (case, bins)


@pytest.mark.parametrize("bins", [1, 0], ids=["bins", "counting"])
@pytest.mark.parametrize("src", ["stride20", "stride13", "varlen_direct", "varlen_prehash"])
def test_bucketed_scatter_key_sources(seb, torch_cuda, src, bins):
    """Both scatters over every key source the radix-partitioned build reads at a filter size the
    bins take (95.85M bits, 1463 buckets): 4-B-aligned strided keys, byte-strided keys, and
    variable-length keys walked per lane or pre-hashed into packed residues; against the oracle."""
    torch = torch_cuda
    n, m, k = 300_001, 95_850_584, 7
    idx = np.random.default_rng(5).permutation(4 * n)[:n]
    if src.startswith("stride"):
        stride = int(src[6:])
        base = kg.key16(idx)
        host = np.zeros((n, stride), np.uint8)
        host[:, : min(16, stride)] = base[:, : min(16, stride)]
        host[:, min(16, stride):] = (idx[:, None] * 7 + np.arange(stride - min(16, stride))) % 251
        ref = oc.build(m, k, np.ascontiguousarray(host).ravel(), n, stride=stride)
        kd = seb.dev_keys(to_dev(torch, host.ravel()), n=n, stride=stride)
    else:
        data, off = kg.varlen_keys(idx)
        ref = oc.build(m, k, data, n, offsets=off)
        kd = seb.dev_keys(to_dev(torch, data), to_dev(torch, off.astype(np.int64)))
    prehash = 0 if src == "varlen_prehash" else 1 << 40
    with seb.option("build_algo", 2), seb.option("scatter_bins", bins), \
            seb.option("varlen_prehash_min_keys", prehash):
        words = seb.new_words(m)
        words.view(torch.uint8).fill_(0x3C)
        seb.dev_build_fresh(kd, words, m, k)
        torch.cuda.synchronize()
        raw = words.cpu().numpy().view(np.uint8)
        assert np.array_equal(raw[: (m + 7) // 8], ref), (src, bins)
        assert not raw[(m + 7) // 8:].any()


@pytest.mark.parametrize("algo", [0, 1, 2, 3, 4])
def test_fresh_build_overwrites_garbage(seb, golden, torch_cuda, algo):
    """seb_dev_build_fresh: words full of garbage (never cleared) become the filter of the keys, bit
    for bit, padding zero: the C2 golden at 10M (radix-partitioned: written whole) and 100K keys
    (the small-filter paths clear first); twice in a row on one buffer."""
    torch = torch_cuda
    with seb.option("build_algo", algo):
        for n in (10_000_000, 100_000):
            row = next(r for r in golden["fixed16"] if r["n"] == n)
            m, k = row["m"], row["k"]
            if algo in (3, 4) and seb.words_bytes(m) > 160 * 1024:
                continue
            kd = seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16)
            words = seb.new_words(m)
            for rep in range(2):
                words.view(torch.uint8).fill_(0xA5 if rep == 0 else 0x5A)
                seb.dev_build_fresh(kd, words, m, k)
                torch.cuda.synchronize()
                raw = words.cpu().numpy().view(np.uint8)
                bits = raw[: (m + 7) // 8]
                assert sha(bn.encode(bits, m, k)) == row["encode_sha256"], (algo, n, rep)
                assert not raw[(m + 7) // 8:].any(), (algo, n, rep)


@pytest.mark.parametrize("case", ["duplicates", "skewed"])
def test_fresh_build_overflow(seb, torch_cuda, case):
    """A fresh radix-partitioned build whose runs overflow their regions: the overflowed positions
    go to the overflow bitmap, which apply folds into the (never cleared) words and leaves zero:
    the next fresh build on the same stream, of ordinary keys, equals the oracle too."""
    torch = torch_cuda
    rng = np.random.default_rng(9)
    n, m, k = 400_000, 3_834_024, 7
    keys = np.tile(kg.key16(np.array([42])), (n, 1)) if case == "duplicates" else kg.key16(rng.integers(0, 50, n))
    uniq = np.unique(keys, axis=0)
    ref = oc.build(m, k, np.ascontiguousarray(uniq).ravel(), len(uniq), stride=16)
    plain = kg.key16(np.arange(n))
    ref2 = oc.build(m, k, plain, n, stride=16)
    with seb.option("build_algo", 2):
        words = seb.new_words(m)
        for ks, want in ((keys, ref), (plain, ref2), (keys, ref), (plain, ref2)):
            words.view(torch.uint8).fill_(0xFF)
            seb.dev_build_fresh(seb.dev_keys(to_dev(torch, ks), n=n, stride=16), words, m, k)
            torch.cuda.synchronize()
            raw = words.cpu().numpy().view(np.uint8)
            assert np.array_equal(raw[: (m + 7) // 8], want)
            assert not raw[(m + 7) // 8:].any()


# ------------------------------------------------ sharded build of one filter (§8(e)) ----

def test_or_slices_kernel(seb, torch_cuda):
    """seb_dev_or_slices: out = OR of the slices, vector (multiple of 4 words, aligned) and scalar
    (odd slice length) paths, 1..8 slices."""
    torch = torch_cuda
    rng = np.random.default_rng(3)
    for ns, sw in ((1, 4096), (2, 1000), (3, 7), (8, 65536), (5, 12345)):
        host = rng.integers(-2**31, 2**31, ns * sw, dtype=np.int64).astype(np.int32)
        host[rng.random(host.size) < 0.5] = 0
        slices = torch.from_numpy(host).cuda()
        out = torch.full((sw + 1,), 77, dtype=torch.int32, device="cuda")
        seb.dev_or_slices(slices, ns, out[:sw])
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got[:sw], np.bitwise_or.reduce(host.reshape(ns, sw), axis=0)), (ns, sw)
        assert got[sw] == 77


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_build_emulated_on_one_gpu(seb, torch_cuda, world):
    """dist_build's data path with the collectives done by hand on one GPU: partial filters of
    `world` key shards (the bucketed HIP build), the all-to-all as slice copies, the OR kernel per
    slice, the all-gather as a concatenation.  Equals the single build of all keys (the oracle)."""
    import dist_build as db
    torch = torch_cuda
    n = 1_000_003
    m, k = seb.params(n, 0.01)
    per = db.slice_words(m, world)
    parts = []
    for r in range(world):
        lo, hi = db.shard_bounds(n, world, r)
        w = torch.zeros(per * world, dtype=torch.int32, device="cuda")
        seb.dev_build(seb.dev_keys(to_dev(torch, kg.key16(np.arange(lo, hi))), n=hi - lo, stride=16), w, m, k)
        parts.append(w)
    full = torch.empty(per * world, dtype=torch.int32, device="cuda")
    for g in range(world):
        recv = torch.cat([p[g * per:(g + 1) * per] for p in parts])
        seb.dev_or_slices(recv, world, full[g * per:(g + 1) * per])
    torch.cuda.synchronize()
    want = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    assert np.array_equal(seb.words_to_bits(full, m), want)


def test_sharded_build_nccl_one_rank(seb, golden, torch_cuda):
    """The nccl (RCCL) backend carries the collectives of the multi-GPU paths (dist_build's int32
    all-to-all single, all-gather into a tensor and gather; dist_probe's answer planes as byte
    views; the broadcast batch dtypes), on a one-rank group in this process; ShardedBuild at
    world 1 gives the C2 filter (golden digest)."""
    import socket
    import torch.distributed as dist
    import dist_build as db
    torch = torch_cuda
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        x = torch.arange(16, dtype=torch.int32, device="cuda")
        y = torch.empty_like(x)
        dist.all_to_all_single(y, x)
        z = torch.empty_like(x)
        dist.all_gather_into_tensor(z, x)
        g = [torch.empty_like(x)]
        dist.gather(x, gather_list=g, dst=0)
        torch.cuda.synchronize()
        assert torch.equal(y, x) and torch.equal(z, x) and torch.equal(g[0], x)
        # dist_probe / bench c5: answer planes of every width travel as byte views (an int16 plane,
        # 9-16 filters per rank, has no RCCL type), packed batches as int64, keys as uint8
        import dist_probe as dp
        for dt in (torch.uint8, torch.int16, torch.int32, torch.int64):
            plane = torch.arange(1000, device="cuda").to(dt)
            got = dp.gather_planes(plane, 1)
            gl = [torch.empty_like(plane)]
            dist.gather(dp.comm_view(plane), gather_list=[dp.comm_view(t) for t in gl], dst=0)
            torch.cuda.synchronize()
            assert got[0].dtype == dt and torch.equal(got[0], plane) and torch.equal(gl[0], plane), dt
        for dt in (torch.int64, torch.uint8):
            b = torch.arange(64, device="cuda").to(dt)
            dist.broadcast(b, src=0, async_op=True).wait()
            torch.cuda.synchronize()
            assert torch.equal(b, torch.arange(64, device="cuda").to(dt))
        # bench c2c3's default N > 1 batch path: the in-place all-gather of each rank's packed part
        # (dist_probe.AllGatherPipeline on RCCL), a different batch every step
        nb_, steps, lead = 10_000, 5, 2
        mp_, kp_ = seb.params(nb_, 0.01)
        kbs = [seb.dev_keys(to_dev(torch, kg.key16(b * nb_ + np.arange(nb_))), n=nb_, stride=16)
               for b in range(steps + lead)]
        want = []
        for kb in kbs:
            w_ = torch.zeros(nb_, dtype=torch.int64, device="cuda")
            seb.dev_pack_residues(kb, mp_, kp_, w_)
            want.append(w_)
        bufs = [torch.zeros(nb_, dtype=torch.int64, device="cuda") for _ in range(lead + 1)]
        pipe = dp.AllGatherPipeline(bufs, lead, 0, 1, produce=lambda b, part: seb.dev_pack_residues(kbs[b], mp_, kp_, part))
        assert pipe.in_place
        pipe.prologue()
        for j in range(steps):
            buf = pipe.acquire(j)
            seb.dev_pack_residues(kbs[j + lead], mp_, kp_, pipe.target(j))
            assert torch.equal(buf, want[j]), j
            pipe.end_step(j)
        pipe.drain()
    finally:
        dist.destroy_process_group()
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n, m, k = row["n"], row["m"], row["k"]
    sb = db.ShardedBuild(m, k, 1, 0, "cuda")
    build_fn, or_fn = db.gpu_fns(seb)
    words = sb.build(seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16), build_fn, or_fn)
    torch.cuda.synchronize()
    bits = seb.words_to_bits(words, m)
    assert sha(m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()) == row["encode_sha256"]


def test_partitioned_probe_one_rank(seb, golden, torch_cuda):
    """dist_build.PartitionedProbe on one rank through the HIP probe: the C3 answers (golden)."""
    import dist_build as db
    torch = torch_cuda
    row = next(r for r in golden["fixed16"] if r["n"] == 10_000_000)
    n, m, k = row["n"], row["m"], row["k"]
    words = torch.zeros(db.slice_words(m, 1), dtype=torch.int32, device="cuda")
    seb.dev_build(seb.dev_keys(to_dev(torch, kg.key16(np.arange(n))), n=n, stride=16), words, m, k)
    pp = db.PartitionedProbe(n, 1, 0, "cuda")
    kd = seb.dev_keys(to_dev(torch, kg.key16(kg.probe_indices(n))), n=n, stride=16)
    ans = pp.probe(kd, words, m, k, db.gpu_probe_fn(seb))
    torch.cuda.synchronize()
    assert sha(ans.cpu().numpy().tobytes()) == row["probe_sha256"]


def test_dev_clear(seb, torch_cuda):
    """seb_dev_clear zeroes exactly seb_words_bytes(m) (the 16-B store kernel), and leaves the
    words past it alone; a pointer that is not 16-B aligned takes hipMemsetAsync."""
    torch = torch_cuda
    for m in (1, 127, 128, 129, 958_506, 95_850_584):
        nw = seb.words_bytes(m) // 4
        buf = torch.full((nw + 8,), -1, dtype=torch.int32, device="cuda")
        seb.dev_clear(buf, m)
        torch.cuda.synchronize()
        assert int(buf[:nw].abs().sum()) == 0 and bool((buf[nw:] == -1).all()), m
        view = buf[1:]  # 4-B aligned only
        buf.fill_(-1)
        seb.dev_clear(view, m)
        torch.cuda.synchronize()
        assert int(buf[0]) == -1 and int(buf[1:nw + 1].abs().sum()) == 0 and bool((buf[nw + 1:] == -1).all()), m
