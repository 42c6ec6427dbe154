#!/bin/bash
# r05v: service soak -- 64 client processes, 6 x 20 s, daemon RSS per segment
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/soak_service.py --segments 6 --seconds 20 --workers 64 > gpurun_out/r05v_soak.txt 2> gpurun_out/r05v_soak.err
rc=$?; cat gpurun_out/r05v_soak.txt; echo "[soak] rc=$rc"; exit $rc
