"""CPU: the checker itself under the host sanitizers (race detection / sanitizers).

tools/sanitize/oracle_check.c drives oracle/bloom_oracle.c + codec_oracle.c over the golden
cases.  Built with -fsanitize=address,undefined (no recovery: any report fails the run) and with
-fsanitize=thread for the multi-threaded build/probe, its Encode() bytes and answers must still
match tests/golden (the same digests the GPU path is held to)."""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tools", "sanitize", "oracle_check.c"), os.path.join(ROOT, "oracle", "bloom_oracle.c"),
       os.path.join(ROOT, "oracle", "codec_oracle.c")]
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def _build(tmp, flags, name):
    exe = os.path.join(tmp, name)
    cmd = ["gcc", "-std=c11", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer", *flags, "-o", exe, *SRC,
           "-lm", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-400:]}")
    return exe


def _run(exe, tmp, threads, ns, env_extra):
    out = os.path.join(tmp, "out")
    os.makedirs(out, exist_ok=True)
    kats = "".join(r["key_hex"] + "\n" for r in GOLDEN["fnv_kats"])
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, out, str(threads), *map(str, ns)], input=kats, capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "ERROR: " not in r.stderr, r.stderr[-3000:]
    return out, r.stdout


def _check_against_golden(out, stdout, ns):
    lines = stdout.split("\n")
    fnv = {p[1][1:]: (p[2], p[3]) for p in (ln.split() for ln in lines if ln.startswith("fnv"))}
    for row in GOLDEN["fnv_kats"]:
        assert fnv[row["key_hex"]] == (row["fnv1a_64"], row["fnv1_64"]), row
    assert "crc cbf43926" in stdout and stdout.rstrip().endswith("ok")
    rows = {r["n"]: r for r in GOLDEN["fixed16"] if r["p"] == 0.01}
    for n in ns:
        enc = open(os.path.join(out, f"enc_{n}.bin"), "rb").read()
        ans = open(os.path.join(out, f"ans_{n}.bin"), "rb").read()
        assert hashlib.sha256(enc).hexdigest() == rows[n]["encode_sha256"], n
        assert hashlib.sha256(ans).hexdigest() == rows[n]["probe_sha256"], n


def test_oracle_under_asan_ubsan(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    tmp = str(tmp_path)
    exe = _build(tmp, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], "oracle_asan")
    ns = [1, 7, 1000, 5000, 100_000]
    out, stdout = _run(exe, tmp, 4, ns, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                                         "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    _check_against_golden(out, stdout, ns)


def test_oracle_threads_under_tsan(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    tmp = str(tmp_path)
    exe = _build(tmp, ["-fsanitize=thread"], "oracle_tsan")
    ns = [1000, 100_000]
    out, stdout = _run(exe, tmp, 8, ns, {"TSAN_OPTIONS": "halt_on_error=1"})
    _check_against_golden(out, stdout, ns)
