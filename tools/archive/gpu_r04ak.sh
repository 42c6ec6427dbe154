#!/bin/bash
# r04ak: oracle-free warp checks (longlat / sinusoidal -> 3857), parity suite for planning, C1 latency
# with the lane-parallel transformer set-up.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_warp_exact.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/warp_exact.log 2>&1
rc=$?; grep -E "warp vs exact|PASS|FAIL|Error" gpurun_out/warp_exact.log | head -20; stop $rc warp_exact
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -2 gpurun_out/parity.log; stop $rc parity
timeout -k 10 300 python3 bench.py --only c1 --no-cpu --steps 3 --warmup 1 > gpurun_out/c1.json 2> gpurun_out/c1.err
stop $? c1
python3 -c "
import json; d=json.load(open('gpurun_out/c1.json')); c=d.get('configs',{}).get('C1',d); print('C1 p50', c['p50_tile_ms'], 'p99', c['p99_tile_ms'])"
