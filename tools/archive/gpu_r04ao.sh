#!/bin/bash
# r04ao: cached ctypes argument list in Batch.render -- GPU suite, then C1 / C2 / C5 one-tile latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; stop $rc tests
for c in c1 c5 c2; do
  timeout -k 10 300 python3 bench.py --only $c --no-cpu --steps 3 --warmup 1 --png-tiles 0 > gpurun_out/$c.json 2> gpurun_out/$c.err
  stop $? $c
  python3 -c "
import json; d=json.load(open('gpurun_out/$c.json')); c=d.get('configs',{}).get('$c'.upper(),d)
print('$c p50', c.get('p50_tile_ms'), 'p99', c.get('p99_tile_ms'))" | tee -a gpurun_out/lat.txt
done
