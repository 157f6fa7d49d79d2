"""GPU: bench.py's multi-rank paths on the one GPU of the box (two ranks on cuda:0, gloo moving
the device tensors), at the BASELINE sizes, so the N > 1 code the driver's 8-GPU run takes stays
bit-exact between scaling runs.  The times of such a rehearsal mean nothing (gloo stages every
transfer through host memory); only `parity` is asserted.

  * c5 (the north star's split): 64 filters over the ranks, a new batch broadcast every step,
    planes gathered to rank 0; its resident_batch secondary broadcasts the batch once;
  * c5_2d (dist_probe.KeyFilterGrid): key groups x filter slots, shards sent and planes returned
    in one exchange per step (the collective transport under gloo);
  * c2c3 (the headline): a filter per rank, a new packed batch in every step, spread over the
    ranks and all-gathered (default), or broadcast from rank 0 (its root_broadcast secondary and
    --batch-origin root); the resident_batch secondary broadcasts one batch once.
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


def test_c5_filter_split_two_ranks():
    d = _bench("--config", "c5")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert d["resident_batch"]["parity"].startswith("bit-exact"), d["resident_batch"]


@pytest.mark.parametrize("groups", [2, 1])
def test_c5_2d_grid_two_ranks(groups):
    d = _bench("--config", "c5_2d", "--c5-groups", str(groups), "--no-secondary")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert f"key groups {groups}" in d["config"]["parallelism"]


def test_c2c3_spread_batch_per_step_two_ranks():
    d = _bench("--config", "c2c3")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "all-gather" in d["config"]["workload"] and "all-gathered" in d["config"]["parallelism"]
    assert d["root_broadcast"]["parity"].startswith("bit-exact"), d["root_broadcast"]
    assert d["resident_batch"]["parity"].startswith("bit-exact"), d["resident_batch"]


def test_c2c3_broadcast_per_step_two_ranks():
    d = _bench("--config", "c2c3", "--batch-origin", "root", "--no-secondary")
    assert d["n_gpus"] == 2
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert "RCCL-broadcast from rank 0 in every step" in d["config"]["workload"]
