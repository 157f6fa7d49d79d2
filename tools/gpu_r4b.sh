#!/bin/bash
# Round 4: the pre-hash fill (varlen_tail 2) — parity, A/B against varlen_tail 1, kernel trace + SQ counters.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "varlen or c4" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for t in 1 2 0; do
    timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --varlen-tail $t \
        > $O/ab_t${t}_$i.json 2> $O/ab_t${t}_$i.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for t in 1 2 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/trace_t$t" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config c4 --steps 5 --warmup 2 --no-cpu-baseline --varlen-tail $t > "$ROOT/$O/trace_t$t.log" 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
      -d "$ROOT/$O/pmc_t$t" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config c4 --steps 2 --warmup 1 --no-cpu-baseline --varlen-tail $t > "$ROOT/$O/pmc_t$t.log" 2>&1 || exit 1
done
bash "$ROOT/tools/gpu_r4c.sh" || exit 1
