#!/bin/bash
# Round 4 end-to-end check on one MI355X: the GPU suite, smoke(), the default bench line (with its
# secondary lines), and the 4-rank gloo rehearsal of every N > 1 path.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r4e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 900 bash tools/gpu_rehearse.sh 4 > $O/rehearse4.txt 2>&1 || exit 1
