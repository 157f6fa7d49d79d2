set -e
for cb in 67108864 33554432 16777216 8388608; do
  SEB_CHUNK_BYTES=$cb timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/chunk_$cb.json
  python3 -c "import json;d=json.loads(open('gpurun_out/chunk_$cb.json').read().splitlines()[-1]);print($cb, d['host_inclusive'])"
done
