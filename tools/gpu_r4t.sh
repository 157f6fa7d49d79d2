#!/bin/bash
# Round 4 (session 2): the probe batch packed on a second stream while the filter builds.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/cob
timeout -k 10 300 python tools/ab_cobuild.py > gpurun_out/cob/ab.jsonl 2> gpurun_out/cob/ab.err || { tail -5 gpurun_out/cob/ab.err; exit 1; }
cat gpurun_out/cob/ab.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/cob/trace" -o run --output-format csv -- \
    python3 "$ROOT/tools/ab_cobuild.py" > "$ROOT/gpurun_out/cob/trace.log" 2>&1
