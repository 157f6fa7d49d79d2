set -e
for r in 1 2; do
 for v in base s768_6 s768_5; do
  if [ $v = base ]; then L=""; else L="SEB_LIB_PATH=$PWD/tools/ab_lib/$v/libseb_bloom.so"; fi
  env $L timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-secondary > gpurun_out/abs_${v}_$r.json
  python3 -c "import json;d=json.loads(open('gpurun_out/abs_${v}_$r.json').read().splitlines()[-1]);print('$v',d['value'],d['build_ms'],d['probe_ms'],d['parity'][:9])"
 done
done
