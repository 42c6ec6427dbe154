#!/bin/bash
# r06: the whole GPU suite (one pytest process) + smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06s}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/${T}_gpu_tests.txt; echo "[suite] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_smoke.txt; echo "[smoke] rc=$rc"; exit $rc
