#!/bin/bash
# Checkpoint at HEAD: the whole GPU suite, smoke(), then the default bench line (with its
# CPU baseline legs and secondary lines).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-checkpoint}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 \
    || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['parity'][:30], d['roofline']['frac'])
cb=d['cpu_baseline']; print('cpu', cb['value'], cb['build_mkeys_s'], cb['probe_mkeys_s'], {k:(cb[k]['build_mkeys_s'],cb[k]['probe_mkeys_s'],cb[k]['cores']) for k in ('multi_thread','all_cpus') if k in cb}, cb['host'])
for s in d.get('secondary',[]): print(s['config'], s.get('value'), s.get('ms_per_step'), (s.get('parity') or '')[:20], s.get('cpu_baseline',{}).get('value'))
"
