"""GPU: bench.py's multi-rank paths on the one GPU of the box (two ranks on cuda:0, gloo moving
the device tensors), at the BASELINE sizes, so the N > 1 code the driver's 8-GPU run takes stays
bit-exact between scaling runs.  The times of such a rehearsal mean nothing (gloo stages every
transfer through host memory); only `parity` is asserted.

  * c5 (the north star's split): 64 filters over the ranks, a new batch broadcast every step,
    planes gathered to rank 0; its resident_batch secondary broadcasts the batch once;
  * c5_2d (dist_probe.KeyFilterGrid): key groups x filter slots, shards sent and planes returned
    in one exchange per step (the collective transport under gloo);
  * c2c3 (the headline): a filter per rank, a new packed batch in every step, broadcast from
    rank 0 (default) or spread over the ranks and all-gathered (its all_gather_spread secondary
    and --batch-origin spread); the resident_batch secondary broadcasts one batch once; then C5
    in its three forms (c5, c5_spread, c5_2d) as the default line's same-process variants.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench(*args, timeout=170):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--steps", "3", "--warmup",
                        "2", "--time-every", "1", *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    # the per-rank records: both ranks on the box's one GPU under gloo
    recs = d["per_rank"]
    assert len(recs) == 2 and [r["rank"] for r in recs] == [0, 1]
    assert d["devices"] == 1 and d["rank_check"]["problems"] == []
    for r in recs:
        assert r["backend"] == "gloo" and r["world_size"] == 2 and r["allreduce_ones"] == 2
        assert r["device"]["arch"].startswith("gfx950") and r["device"]["pci"] == recs[0]["device"]["pci"]
        assert r["kernel_ms"] and r["elapsed_s"] > 0 and r["wait_ms"] is not None
    return d


def _variant_ok(v, n_ranks=2):
    assert v["parity"].startswith("bit-exact"), v
    assert v["value"] > 0 and v["ms_per_step"] > 0
    assert v["roofline"]["achieved"] > 0 and v["roofline"]["algorithmic_bytes_per_launch"] > 0
    assert [r["rank"] for r in v["per_rank"]] == list(range(n_ranks))
    assert all(r["wait_ms"] is not None and r["kernel_ms"] for r in v["per_rank"]), v["per_rank"]


def test_c5_filter_split_two_ranks():
    d = _bench("--config", "c5")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "6-B packed residues" in d["config"]["workload"]
    _variant_ok(d["c5_spread"])
    assert d["resident_batch"]["parity"].startswith("bit-exact"), d["resident_batch"]


def test_c5_8_byte_batch_two_ranks():
    d = _bench("--config", "c5", "--pack6", "0", "--no-secondary")
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "8-B packed residues" in d["config"]["workload"]


@pytest.mark.parametrize("groups", [2, 1])
def test_c5_2d_grid_two_ranks(groups):
    d = _bench("--config", "c5_2d", "--c5-groups", str(groups), "--no-secondary")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert f"key groups {groups}" in d["config"]["parallelism"]
    assert "6-B packed residues" in d["config"]["workload"]


def test_c2c3_spread_batch_per_step_two_ranks():
    """The default N > 1 line: the headline's batch broadcast from rank 0 every step (the north
    star's form), then in the same processes its all-gather and resident forms and the north
    star's C5 in its three forms, every one bit-exact with per-rank waits."""
    d = _bench("--config", "c2c3", timeout=420)
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "RCCL-broadcast from rank 0 in every step" in d["config"]["workload"]
    for key in ("all_gather_spread", "c5", "c5_spread", "c5_2d"):
        _variant_ok(d[key])
    assert "all-gather" in d["all_gather_spread"]["workload"]
    assert d["c5"]["scaling"] == "strong" and "6-B packed" in d["c5"]["workload"]
    assert d["resident_batch"]["parity"].startswith("bit-exact"), d["resident_batch"]


def test_c2c3_broadcast_per_step_two_ranks():
    d = _bench("--config", "c2c3", "--batch-origin", "spread", "--no-secondary")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "all-gather" in d["config"]["workload"] and "all-gathered" in d["config"]["parallelism"]
