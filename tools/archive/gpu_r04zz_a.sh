#!/bin/bash
# r04zz (a): closing run on the final library build -- the GPU suite and the
# bench line (N=1, all configs, CPU baselines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('C2', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('p50_tile_ms'))
for k, c in d.get('configs', {}).items(): print(k, json.dumps(c)[:300])"
