"""CPU: the C-ABI library loads, exports every symbol include/seb_bloom.h declares, and its
host-only logic (sizing, Encode of an untouched filter, Decode's nil rule) matches the oracle.
No compute call is made here (there is no GPU in the build container)."""
import ctypes
import re
import subprocess

import numpy as np
import pytest

from oracle import bloom_np as bn
from oracle import oracle_c as oc


def declared_functions(header):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(seb_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(seb):
    names = declared_functions(seb.HEADER)
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", seb.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (seb_[a-z0-9_]+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    L = seb.lib()
    for n in names:
        assert getattr(L, n) is not None
    assert set(names) == set(seb._SIGS), "binding signature table out of sync with the header"


def test_library_is_gfx950_code_object(seb):
    blob = open(seb.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob  # embedded offload bundle target


def test_abi_version(seb):
    assert seb.lib().seb_abi_version() == 1


def test_params_match_oracle(seb, golden):
    for row in golden["sizing"]:
        assert seb.params(row["n"], row["p"]) == (row["m"], row["k"]), row
    rng = np.random.default_rng(7)
    for _ in range(2000):
        n = int(rng.integers(0, 10**9))
        p = float(rng.uniform(1e-12, 0.999))
        assert seb.params(n, p) == oc.params(n, p), (n, p)


def test_params_invalid(seb):
    for n, p in [(-1, 0.01), (10, 0.0), (10, 1.0), (10, 2.0), (10, float("nan"))]:
        with pytest.raises(seb.SebError) as e:
            seb.params(n, p)
        assert e.value.code == -4


def test_sizes(seb):
    for m in [0, 1, 7, 8, 9, 127, 128, 129, 95850584]:
        assert seb.num_bytes(m) == (m + 7) // 8
        assert seb.words_bytes(m) == -(-m // 128) * 16
        assert seb.words_bytes(m) >= seb.num_bytes(m)


def test_encode_untouched_filter_host_only(seb):
    # NewBloomFilter + Encode with no Add never reaches the device.
    f = seb.BloomFilter(1000, 0.01)
    assert (f.num_bits, f.num_hashes) == (9586, 7)
    enc = f.encode()
    assert enc == bn.encode(np.zeros(1199, np.uint8), 9586, 7)


def test_new_zero_keys(seb):
    f = seb.BloomFilter(0, 0.01)  # m = 0, k = 1 as in Go (uint32(NaN) -> 0 -> 1)
    assert (f.num_bits, f.num_hashes) == (0, 1)
    assert f.encode() == bytes.fromhex("000000000000000001000000")
    with pytest.raises(seb.SebError):  # Go: integer divide by zero panic in Add
        f.add(b"x")


def test_decode_rules(seb):
    assert seb.BloomFilter.decode(b"\x00" * 11) is None  # lsm/bloom.go:106-108
    data = bytes.fromhex("0a0000000000000007000000ee01")
    f = seb.BloomFilter.decode(data)
    assert (f.num_bits, f.num_hashes) == (10, 7)
    assert f.encode() == data  # copied verbatim, re-encoded identically
    long = data + b"\xff\xff"  # trailing bytes are kept as part of bits (len(data)-12)
    assert seb.BloomFilter.decode(long).encode() == long
    short = bytes.fromhex("ff00000000000000070000000102")  # m=255 needs 32 bytes
    g = seb.BloomFilter.decode(short)
    with pytest.raises(seb.SebError) as e:
        g.may_contain(b"k")
    assert e.value.code == -5


def test_filter_new_invalid(seb):
    with pytest.raises(seb.SebError):
        seb.BloomFilter(10, 1.5)


def test_no_silent_fallback_without_library(seb, monkeypatch, tmp_path):
    import importlib
    mod = importlib.import_module("seb_bloom")
    monkeypatch.setattr(mod, "_lib", None)
    monkeypatch.setattr(mod, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(mod.SebError):
        mod.params(10, 0.01)


OPTION_NAMES = ["build_algo", "multi_interleave", "multiget_order", "multiget_l0_group", "varlen_prehash_min_keys",
                "bucket_min_keys", "lds_min_keys", "many_splits", "probe_phases", "probe_compact", "grid_cap",
                "workspace_limit_mib", "multiget_piece_mib"]


def test_options_round_trip_and_reject_bad_values(seb):
    """Every knob reads back what was set, bad values are refused and leave the knob unchanged; the
    rejected variants of earlier rounds are gone from the library."""
    for name in OPTION_NAMES:
        old = seb.get_option(name)
        seb.set_option(name, old)
        assert seb.get_option(name) == old
    with seb.option("probe_phases", 5):
        assert seb.get_option("probe_phases") == 5
    for name, bad in (("build_algo", 5), ("probe_phases", 65), ("many_splits", -1), ("grid_cap", 0),
                      ("multiget_order", 3), ("multiget_piece_mib", 0), ("multiget_l0_group", 2), ("probe_compact", 2), ("nonexistent", 1), ("probe_mode", 8), ("scatter_xcd", 0),
                      ("clear_kernel", 1)):
        before = seb.get_option(name) if name in OPTION_NAMES else None
        with pytest.raises(seb.SebError):
            seb.set_option(name, bad)
        if before is not None:
            assert seb.get_option(name) == before


def test_options_from_environment(seb):
    """SEB_<NAME> sets a knob's initial value in a fresh process; an out-of-range value is ignored."""
    code = ("import sys; sys.path.insert(0, 'storage-engines_amd'); import seb_bloom as s; "
            "print(s.get_option('many_splits'), s.get_option('build_algo'), s.get_option('probe_phases'))")
    import os
    env = dict(os.environ, SEB_MANY_SPLITS="12", SEB_BUILD_ALGO="13", SEB_PROBE_PHASES="5")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run(["python", "-c", code], env=env, cwd=root, capture_output=True, text=True, check=True)
    splits, algo, phases = map(int, out.stdout.split())
    assert splits == 12 and phases == 5
    assert algo == 0  # 13 is not a valid build_algo: the default stays
