#!/bin/bash
# r04aj: oracle-free warp checks for longlat -> 3857 and sinusoidal -> 3857.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_warp_exact.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/warp_exact.log 2>&1
rc=$?; grep -E "warp vs exact|PASS|FAIL|Error|assert" gpurun_out/warp_exact.log | head -20; tail -2 gpurun_out/warp_exact.log; exit $rc
