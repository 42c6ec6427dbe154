#!/bin/bash
# r05w: Lambert Conformal Conic on the GPU -- the new parity / exact tests,
# then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_warp_exact.py -m gpu -k "lambert or extent" -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r05w_lcc.txt 2>&1
rc=$?; grep -E "PASS|FAIL|lambert warp" gpurun_out/r05w_lcc.txt | tail -12; stop $rc lcc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05w_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r05w_tests.txt; stop $rc tests
