"""bench.py's rank launcher (`--gpus N` without torchrun): the driver runs `bench.py --gpus N`, so
the script itself must start N rank processes and report n_gpus = N.
CPU only: --launch-check forms the process group on gloo without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(extra)
    return e


def _run(args, env=None, timeout=120):
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env or _env())


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-check"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["rank_sum"] == n * (n + 1) // 2
    assert d["master"].startswith("127.0.0.1:")
    # the per-rank records the N-GPU line carries, here on gloo without a GPU
    recs = d["per_rank"]
    assert [r["rank"] for r in recs] == list(range(n))
    for r in recs:
        assert r["world_size"] == n and r["allreduce_ones"] == n and r["backend"] == "gloo"
        assert r["device"] is None and r["local_rank"] == r["rank"] and r["host"]
        assert set(r) >= {"kernel_ms", "wait_ms", "wait_host_ms", "elapsed_s"}
    assert d["devices"] == 0 and d["problems"] == []
    # the default N > 1 line: the headline's batch broadcast from rank 0 (the
    # north star's form), then in the same processes its all-gather and resident forms and C5 in
    # its three forms (north star configs[4])
    assert [(v["key"], v["config"]) for v in d["variants"]] == [
        ("all_gather_spread", "c2c3"), ("resident_batch", "c2c3"), ("c5", "c5"), ("c5_spread", "c5"),
        ("c5_2d", "c5_2d")]
    assert d["variants"][2]["overrides"]["batch_origin"] == "root"
    assert d["variants"][3]["overrides"]["batch_origin"] == "spread"
    # each form's batch, 6-byte packed residues of the 10M keys: every rank probes every key
    # against its 64/N filters (root, spread) or its 1/N of the keys against all 64 (grid)
    keys, blk = 10_000_000, 384
    plans = {f: [r["c5_plan"][i] for r in recs] for i, f in enumerate(("root", "spread", "grid"))}
    for f, rows in plans.items():
        assert [p["rank"] for p in rows] == list(range(n)) and all(p["form"] == f for p in rows)
    total = -(-keys // 64) * blk  # 60 MB: 6 B per key in 64-key blocks
    assert sum(p["filters"] for p in plans["root"]) == 64
    assert plans["root"][0]["pack_keys"] == keys and all(p["pack_keys"] == 0 for p in plans["root"][1:])
    assert plans["root"][0]["send_bytes"] == total and all(p["recv_bytes"] == total for p in plans["root"][1:])
    assert all(p["probe_keys"] == keys for p in plans["root"] + plans["spread"])
    assert sum(p["pack_keys"] for p in plans["spread"]) == keys
    assert all(p["send_bytes"] % blk == 0 and p["recv_bytes"] == p["send_bytes"] * (n - 1) for p in plans["spread"])
    assert sum(p["probe_keys"] for p in plans["grid"]) == keys and all(p["filters"] == 64 for p in plans["grid"])
    assert plans["grid"][0]["send_bytes"] == sum(p["recv_bytes"] for p in plans["grid"][1:])
    assert all(p["recv_bytes"] % blk == 0 for p in plans["grid"])


def test_variant_failing_on_every_rank_is_reported_and_the_line_prints():
    """A variant that raises on every rank (e.g. an operation the backend rejects) becomes an
    error entry; the variants after it still run and rank 0 still prints its one line."""
    r = _run(["--gpus", "2", "--launch-check"], env=_env(SEB_BENCH_FAIL_VARIANT="c5"))
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])["variant_results"]
    assert "injected failure" in res["c5"]["error"] and res["c5"]["config"] == "c5"
    for key in ("all_gather_spread", "resident_batch", "c5_spread", "c5_2d"):
        assert res[key]["ranks"] == 2, key  # the stand-in's all-reduce over both ranks
    assert "variant c5 failed" in r.stderr


def test_variant_failing_on_one_rank_ends_the_run():
    """A variant that fails on one rank only leaves its peers in a collective it never joins: the
    failing rank's bounded barrier on the gloo side group times out and the run exits non-zero
    (as an uncaught error would) instead of hanging."""
    r = _run(["--gpus", "2", "--launch-check"],
             env=_env(SEB_BENCH_FAIL_VARIANT="c5@1", SEB_BENCH_VARIANT_VOTE_S="5"), timeout=180)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_c5_plan_alignment():
    """The 6-byte form's slices start at multiples of 64 keys at every world size the driver runs;
    the 8-byte form keeps key-granular slices."""
    sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))
    import dist_probe as dp

    for world in (2, 3, 4, 8):
        for n in (10_000_000, 1_000_003, 130):
            spread = [dp.spread_bounds(n, world, r, align=64) for r in range(world)]
            assert spread[0][0] == 0 and spread[-1][1] == n
            assert all((lo % 64 == 0 or lo == n) and hi >= lo for lo, hi, _ in spread)
            assert all(a[1] == b[0] for a, b in zip(spread, spread[1:]))
            g = [dp.KeyFilterGrid(64, r, world, world, align=64) for r in range(world)]
            bounds = [g[0].key_bounds(n, x) for x in range(world)]
            assert bounds[0][0] == 0 and bounds[-1][1] == n and all(lo % 64 == 0 or lo == n for lo, _ in bounds)
            assert g[0].width(n) == max(hi - lo for lo, hi in bounds)
            for r in range(world):
                p = dp.c5_rank_plan(n, world, r, "spread", 8)
                lo, hi, w = dp.spread_bounds(n, world, r)
                assert p["pack_keys"] == hi - lo and p["send_bytes"] == 8 * w
    lay = dp.Packed6Layout()
    assert lay.span(128, 200) == (768, 1536) and lay.rows(65) == 768
    with pytest.raises(ValueError):
        lay.span(1, 64)


def test_rank_report_summary():
    """rank_report.summarize: distinct GPUs by (host, PCI address); an RCCL run whose ranks share a
    GPU, disagree on the world size or miss an all-reduce contribution is flagged."""
    sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))
    import rank_report as rr

    def rec(rank, pci, ones=2, world=2, backend="nccl", elapsed=1.0):
        dev = {"index": rank, "current_device": rank, "pci": pci, "name": "x", "arch": "gfx950", "uuid": ""}
        r = rr.rank_record(rank, rank, world, backend, dev, ones, {"build": 0.2, "probe": 0.3}, 0.05, 0.01, elapsed)
        r["host"] = "h"
        return r

    ok = rr.summarize([rec(0, "0000:05:00.0"), rec(1, "0000:15:00.0", elapsed=1.5)], 2, "nccl")
    assert ok["devices"] == 2 and ok["problems"] == [] and ok["slowest_rank"] == 1
    assert ok["elapsed_s_spread"] == 0.5 and ok["wait_ms_max"] == 0.05
    same = rr.summarize([rec(0, "0000:05:00.0"), rec(1, "0000:05:00.0")], 2, "nccl")
    assert same["devices"] == 1 and any("distinct GPU" in p for p in same["problems"])
    assert rr.summarize([rec(0, "a", backend="gloo"), rec(1, "a", backend="gloo")], 2, "gloo")["problems"] == []
    bad = rr.summarize([rec(0, "a", ones=1), rec(1, "b", world=3)], 2, "nccl")
    assert len(bad["problems"]) == 2


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--launch-check"], env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_rccl_needs_n_gpus(monkeypatch):
    import importlib.util

    import torch

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    args = type("A", (), {"gpus": 4, "launch_check": False, "dist_backend": "nccl"})()
    assert bench.launch_ranks(args, []) == 3  # refuses before starting any rank


def test_rank_envs():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    envs = bench.rank_envs(4, 12345, base={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "12345"
               and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["X"] == "1" for e in envs)
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
