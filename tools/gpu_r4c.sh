#!/bin/bash
# Round 4: WRITE_SIZE calibration for the scatter's u16 run stores (tools/ubench/runs.hip).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r4c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in "0" "1" "1 --stream" "2"; do
  tag=$(echo $m | tr -d ' -')
  timeout -k 10 60 "$ROOT/tools/ubench/runs" $m > $O/run_$tag.json 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$tag -o run --output-format csv -- "$ROOT/tools/ubench/runs" $m > $O/pmc_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$tag -o run --output-format csv -- "$ROOT/tools/ubench/runs" $m > $O/pmcf_$tag.log 2>&1 || exit 1
done
