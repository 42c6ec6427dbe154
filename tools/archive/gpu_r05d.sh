#!/bin/bash
# r05d: pair footprint hook test + C5 bench line with its roofline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x -k "pair_info or warp_windows" \
  --timeout 200 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05d_tests.log; stop $rc tests
timeout -k 10 300 python3 bench.py --only c5 --no-cpu --steps 10 --warmup 3 > gpurun_out/r05d_c5.json 2> gpurun_out/r05d_c5.err
stop $? c5
python3 -c "
import json; c=json.load(open('gpurun_out/r05d_c5.json'))['configs']['C5']; print(json.dumps(c)[:1500])"
