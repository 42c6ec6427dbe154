#!/bin/bash
# r04w: drill descriptors with pinned window / offset upload -- drill GPU
# tests, breakdown, C4 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_drill_geom.py tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "drill or descriptor or c4 or geom" -x -q --timeout 300 --timeout-method thread > gpurun_out/drill_tests.log 2>&1
rc=$?; tail -3 gpurun_out/drill_tests.log; stop $rc drill_tests
timeout -k 10 200 python3 tools/c4_desc.py --label pinned --reps 20 >> gpurun_out/c4_desc.jsonl
stop $? c4_desc
cat gpurun_out/c4_desc.jsonl
timeout -k 10 300 python3 bench.py --only c4 --no-cpu --no-deciles --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err
stop $? c4
python3 -c "
import json; d=json.load(open('gpurun_out/c4.json')); c=d.get('configs',{}).get('C4',d); print('descriptors_ms', c.get('descriptors_ms'))"
