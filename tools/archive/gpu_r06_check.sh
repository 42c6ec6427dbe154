#!/bin/bash
# r06: full-size identity (C2, C5) + parity suite, then render timings of the
# product against gsky_amd/libgskyhip_ab.so (the previous build) on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06c}
CFGS=${2:-"c2 c5"}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full_identical" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
bash tools/gpu_r06_time.sh $T "$CFGS"
