#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "extent" -v --timeout 200 --timeout-method thread > gpurun_out/r05u_extent.txt 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/r05u_extent.txt | head -20; exit $rc
