set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multirank.py > gpurun_out/r4a_multirank.log 2>&1 &&
timeout -k 10 200 python bench.py --config c5_2d --steps 10 --warmup 3 > gpurun_out/r4a_c5_2d_n1.json 2> gpurun_out/r4a_c5_2d_n1.err &&
timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/r4a_c5_n1.json 2> gpurun_out/r4a_c5_n1.err
