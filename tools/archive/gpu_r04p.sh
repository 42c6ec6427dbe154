#!/bin/bash
# r04p: decile selection over the key range (linear buckets) -- decile
# parity tests, C4 deciles timing and per-launch trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dec_tests.log; stop $rc dec_tests
timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err
stop $? c4
python3 -c "
import json; d=json.load(open('gpurun_out/c4.json')); c=d.get('configs',{}).get('C4',d)
print(json.dumps(c.get('deciles'))); print('descriptors_ms', c.get('descriptors_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 2 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
