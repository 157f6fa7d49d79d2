#!/bin/bash
# C4 pre-hash tail-wave count A/B (varlen_tail 1/2/3): varlen/c4 parity tests, then alternating bench runs.
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "varlen or c4 or prehash" > gpurun_out/r5x/tests.log 2>&1 || { tail -30 gpurun_out/r5x/tests.log; exit 1; }
tail -1 gpurun_out/r5x/tests.log
for r in 1 2 3; do for v in 1 2 3; do
  timeout -k 10 200 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline --varlen-tail $v > gpurun_out/r5x/t$v.$r.json 2> gpurun_out/r5x/err || { tail gpurun_out/r5x/err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], d['ms_per_step'], d.get('build_ms'), d.get('probe_ms'), d['parity'][:12])" gpurun_out/r5x/t$v.$r.json
done; done
