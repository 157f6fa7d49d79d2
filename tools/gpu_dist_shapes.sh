#!/bin/bash
# Profile the N > 1 paths' per-rank kernels on the one GPU (tools/dist_shapes.py run): kernel trace,
# then one PMC pass each for FETCH_SIZE and WRITE_SIZE.  Usage: tools/gpu_dist_shapes.sh TAG
# Writes gpurun_out/prof_TAG/; summarise here with: python tools/dist_shapes.py summarize TAG
set -e
TAG=${1:-r06_dist}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o shapes --output-format csv -- \
    python3 "$ROOT/tools/dist_shapes.py" run > "$OUT/trace.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o shapes --output-format csv -- \
        python3 "$ROOT/tools/dist_shapes.py" run > "$OUT/pmc$i.log" 2>&1
done
