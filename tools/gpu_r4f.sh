#!/bin/bash
# Round 4: SDWA byte selects in the FNV steps — parity of the hashing paths, then A/B against the
# library of the previous commit (tools/ab_lib/base, tools/rev_lib.sh) on c2c3 and c4.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_fallback.py \
    -m gpu -k "c2_c3 or c4 or varlen or fallback or fresh or go_api or fuzz or multi" > $O/tests.log 2>&1 || exit 1
bash tools/gpu_ab_lib.sh sdwa_c2c3 tools/ab_lib/base/libseb_bloom.so > $O/ab_c2c3.txt 2>&1 || exit 1
bash tools/gpu_ab_lib.sh sdwa_c4 tools/ab_lib/base/libseb_bloom.so --config c4 > $O/ab_c4.txt 2>&1 || exit 1
