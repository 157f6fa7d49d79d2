"""CPU: the drop-in boundary's CPU fallback (SURVEY.md 8(b) error row).

The Go API has no error returns (lsm/bloom.go:19-41,70-77,96-102 never fail on valid input), so
the Go API mirror (seb_filter_*, the cgo shim's calls) must keep working when its device path
fails: a build or batched probe that gets SEB_ERR_DEVICE / SEB_ERR_NOMEM is done on the filter's
host copy (product code in csrc/seb_host.cpp, not the oracle) and counted by seb_fallback_count().

The device error is forced with the test-only option fault_inject (and, in this container, also
happens for real: there is no GPU).  Each case runs in a child process, so the fallbacks it
causes never show in the counter that the GPU suite (tests/conftest.py) and smoke() require to
be 0.  The results are checked against the golden Encode() / answer digests (tests/golden) and
the oracle.
"""
import hashlib
import multiprocessing as mp

import numpy as np
import pytest

import keygen as kg
from oracle import oracle_c as oc


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def _go_sequence(seb, n, p=0.01, singles=500):
    """sstable_builder.go (New -> Add per key -> Encode) then sstable.go (Decode -> MayContain)."""
    f = seb.BloomFilter(n, p)
    for i in range(min(singles, n)):
        f.add(kg.key16_bytes(i))
    if n > singles:
        f.add_batch(kg.key16(np.arange(singles, n)))
    enc = f.encode()
    g = seb.BloomFilter.decode(enc)
    probe = kg.key16(kg.probe_indices(n))
    ans = g.may_contain_batch(probe)
    singles_ok = all(g.may_contain(bytes(probe[q])) == bool(ans[q]) for q in range(0, n, max(1, n // 300)))
    return {"encode_sha256": sha(enc), "probe_sha256": sha(ans.tobytes()), "positives": int(ans.sum()),
            "singles_ok": singles_ok}


def _child(case, args, q):
    try:
        import seb_bloom as seb

        out = {}
        if case == "inject":
            seb.set_option("fault_inject", 1)
            out["rows"] = {(n, p): _go_sequence(seb, n, p) for n, p in args}
        elif case == "no_fallback":
            seb.set_option("fault_inject", 1)
            seb.set_option("cpu_fallback", 0)
            f = seb.BloomFilter(1000, 0.01)
            f.add(b"key")
            try:
                f.encode()
                out["raised"] = None
            except seb.SebError as e:
                out["raised"] = e.code
            seb.set_option("cpu_fallback", 1)  # the kept keys build on the next call
            out["after"] = sha(f.encode())
            m, k = seb.params(1000, 0.01)
            bits = oc.build(m, k, np.frombuffer(b"key", np.uint8), 1, offsets=np.array([0, 3], np.uint64))
            out["want"] = sha(m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes())
        elif case == "internal":  # an internal error (a library bug) is reported, never absorbed
            seb.set_option("fault_inject", 2)
            f = seb.BloomFilter(1000, 0.01)
            f.add(b"key")
            try:
                f.encode()
                out["raised"] = None
            except seb.SebError as e:
                out["raised"] = e.code
            try:
                f.may_contain_batch([b"key"])
                out["raised_probe"] = None
            except seb.SebError as e:
                out["raised_probe"] = e.code
        elif case == "varlen":
            seb.set_option("fault_inject", 1)
            rng = np.random.default_rng(7)
            keys = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 300, 3000)]
            keys[5] = b""
            m, k = seb.params(len(keys), 0.01)
            f = seb.BloomFilter(len(keys), 0.01)
            for key in keys[:100]:
                f.add(key)
            f.add_batch(keys[100:])
            enc = f.encode()
            off = np.zeros(len(keys) + 1, np.uint64)
            np.cumsum([len(x) for x in keys], out=off[1:])
            data = np.frombuffer(b"".join(keys), np.uint8)
            want = oc.build(m, k, data, len(keys), offsets=off)
            out["equal"] = enc[12:] == want.tobytes()
            probes = keys[::2] + [b"absent-%d" % i for i in range(1000)]
            ans = seb.BloomFilter.decode(enc).may_contain_batch(probes)
            poff = np.zeros(len(probes) + 1, np.uint64)
            np.cumsum([len(x) for x in probes], out=poff[1:])
            want_ans = oc.probe(want, m, k, np.frombuffer(b"".join(probes), np.uint8), len(probes), offsets=poff)
            out["answers_equal"] = bool(np.array_equal(ans, want_ans))
        elif case == "recover":  # GPU: device build, a fallback, then the device again (host bits re-uploaded)
            n = 5000
            f = seb.BloomFilter(n, 0.01)
            f.add_batch(kg.key16(np.arange(2000)))
            seb.set_option("fault_inject", 1)
            f.add_batch(kg.key16(np.arange(2000, 4000)))
            seb.set_option("fault_inject", 0)
            f.add_batch(kg.key16(np.arange(4000, n)))
            out["encode_sha256"] = sha(f.encode())
            ans = f.may_contain_batch(kg.key16(kg.probe_indices(n)))  # the device probe, from the re-uploaded bits
            out["probe_sha256"] = sha(ans.tobytes())
        elif case == "fresh_nomem":
            # A new filter's first build takes a pooled device buffer without clearing it and fails
            # after that (scratch over workspace_limit_mib) with the fallback off: the Adds stay
            # pending and the retry must start from zeros, not from the recycled buffer's bits.
            n = 300_000
            old = seb.BloomFilter(n, 0.01)  # the same size class; a small batch (atomic build, no scratch)
            old.add_batch(kg.key16(10_000_000 + np.arange(2000)))
            old.encode()
            old.close()  # its (non-zero) words go to the pool
            seb.set_option("cpu_fallback", 0)
            seb.set_option("workspace_limit_mib", 1)
            f = seb.BloomFilter(n, 0.01)
            for i in range(n):
                f.add(kg.key16_bytes(i))
            try:
                f.encode()
                out["raised"] = None
            except seb.SebError as e:
                out["raised"] = e.code
            seb.set_option("workspace_limit_mib", 0)
            seb.set_option("cpu_fallback", 1)
            m, k = seb.params(n, 0.01)
            enc = f.encode()
            out["equal"] = enc[12:] == oc.build(m, k, kg.key16(np.arange(n)), n, stride=16).tobytes()
        elif case == "no_device":
            out["rows"] = {(n, p): _go_sequence(seb, n, p) for n, p in args}
        out["fallbacks"] = seb.fallback_count()
        q.put(out)
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put({"error": f"{type(e).__name__}: {e}"})


def _run(case, args=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(case, list(args), q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=60)
    assert "error" not in out, out["error"]
    return out


def test_injected_device_fault_gives_golden_filters(golden):
    rows = [(r["n"], r["p"]) for r in golden["fixed16"] if r["n"] <= 100_000]
    out = _run("inject", rows)
    for r in golden["fixed16"]:
        if r["n"] > 100_000:
            continue
        got = out["rows"][(r["n"], r["p"])]
        assert got["encode_sha256"] == r["encode_sha256"], r["n"]
        assert got["positives"] == r["probe_positives"] and got["probe_sha256"] == r["probe_sha256"], r["n"]
        assert got["singles_ok"]
    assert out["fallbacks"] > 0


def test_fallback_off_reports_the_error_and_keeps_the_keys():
    out = _run("no_fallback")
    assert out["raised"] == -2  # SEB_ERR_DEVICE
    assert out["after"] == out["want"]  # the failed build kept the Add; the next Encode built it


def test_internal_error_is_not_absorbed():
    """Only unavailability (SEB_ERR_DEVICE) and allocation failures (SEB_ERR_NOMEM) fall back; a
    rejected launch or kernel fault (SEB_ERR_INTERNAL) reaches the caller with the fallback on."""
    out = _run("internal")
    assert out["raised"] == -6 and out["raised_probe"] == -6  # SEB_ERR_INTERNAL
    assert out["fallbacks"] == 0


def test_fallback_variable_length_keys():
    out = _run("varlen")
    assert out["equal"] and out["answers_equal"]


def test_no_device_at_all():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the device path works, see test_injected_device_fault_gives_golden_filters")
    out = _run("no_device", [(1000, 0.01), (100_000, 0.01)])
    assert out["rows"][(100_000, 0.01)]["encode_sha256"] == "5c339ef1b8a07e85ae0afd0e623f6a329efc05be098f110c28ff5757bc8b5064"
    assert out["fallbacks"] > 0


@pytest.mark.gpu
def test_fallback_and_back_to_the_device(golden):
    """On the GPU: a filter built on the device, then one batch through the fallback (host copy,
    device copy dropped), then the device again (the host bits uploaded first) = the golden n=5000
    filter and answers."""
    out = _run("recover")
    row = next(r for r in golden["fixed16"] if r["n"] == 5000 and r["p"] == 0.01)
    assert out["encode_sha256"] == row["encode_sha256"] and out["probe_sha256"] == row["probe_sha256"]
    assert out["fallbacks"] == 1


@pytest.mark.gpu
def test_failed_fresh_build_retries_from_zeros():
    """a failed first build of a New must not leave the recycled device words behind."""
    out = _run("fresh_nomem")
    assert out["raised"] == -3  # SEB_ERR_NOMEM
    assert out["equal"]
    assert out["fallbacks"] == 0


@pytest.mark.gpu
def test_injected_device_fault_on_gpu(golden):
    rows = [(1000, 0.01), (100_000, 0.01)]
    out = _run("inject", rows)
    for r in golden["fixed16"]:
        if (r["n"], r["p"]) in rows:
            got = out["rows"][(r["n"], r["p"])]
            assert got["encode_sha256"] == r["encode_sha256"] and got["probe_sha256"] == r["probe_sha256"]
