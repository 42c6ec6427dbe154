#!/bin/bash
# r03c: GPU suite on the new defaults (NN rows per wave by batch size, fp32
# bilinear weights, counters zeroed in the prologue); rocprofv3 kernel stats of
# C4 (deciles breakdown) and C3; FETCH_SIZE / WRITE_SIZE calibration of the
# 2-B / 4-B gathers and 4-B stores (tools/calib/fetch_calib); the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --only c3 --no-cpu > gpurun_out/prof_c3.log 2>&1
stop $? prof_c3
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/calib_f -o run --output-format csv -- \
  ./tools/calib/fetch_calib 3 > gpurun_out/calib_f.log 2>&1
stop $? calib_fetch
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/calib_w -o run --output-format csv -- \
  ./tools/calib/fetch_calib 3 > gpurun_out/calib_w.log 2>&1
stop $? calib_write
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
