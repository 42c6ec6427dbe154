#!/bin/bash
# r03i: GPU suite (deciles: no-atomic key cache, 4 workgroups per CU, grouped
# radix fallback, 16-pixel transpose tile, parallel TimeSeries rows; bilinear
# fast path: all taps inside -> no per-tap rules, no division); rocprofv3
# stats of C3 and C4; the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --only c3 --no-cpu > gpurun_out/prof_c3.log 2>&1
stop $? prof_c3
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
