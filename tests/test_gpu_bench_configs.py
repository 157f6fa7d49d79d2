"""GPU: every bench.py config at N = 1 runs through the same timed loop the driver's bench uses
(warm-up, timed steps, the kernel_timing steps after them) and reports its golden parity, so a
config that no secondary line covers (route, wal, many, c2_sharded, c3_partitioned, c5_2d, the
overlapped c2c3 / c4 steps) cannot rot between rounds.  Times are not asserted."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


@pytest.mark.parametrize("args", [
    ["--config", "route"],
    ["--config", "wal"],
    ["--config", "many"],
    ["--config", "c2_sharded"],
    ["--config", "c3_partitioned"],
    ["--config", "c5_2d"],
    ["--config", "c2c3", "--overlap", "1"],
    ["--config", "c4", "--overlap", "1"],
    ["--config", "c2c3", "--fresh-build", "0"],
], ids=lambda a: "_".join(x.lstrip("-") for x in a[1:]))
def test_bench_config_one_gpu(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, *args, "--steps", "4", "--warmup", "1", "--kernel-reps", "2",
                        "--no-cpu-baseline", "--no-secondary", "--no-host-inclusive"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["parity"].startswith("bit-exact"), d["parity"]
    assert d["cpu_fallbacks"] == 0
    assert d["kernel_timing"]["reps"] == 2
