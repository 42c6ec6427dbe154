#!/bin/bash
# r04ap: reference-order drill mean -- pixel loads in flight per lane 8 / 16 / 32 (A/B build), C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DRILL_U=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k drill -x -q --timeout 200 --timeout-method thread > gpurun_out/drill_tests.log 2>&1
rc=$?; tail -1 gpurun_out/drill_tests.log; stop $rc drill_tests
for u in 16 32 8 16 32; do
  GSKYHIP_LIB=ab GSKYHIP_DRILL_U=$u timeout -k 10 300 python3 bench.py --only c4 --no-cpu --no-deciles --steps 10 --warmup 2 > gpurun_out/c4_$u.json 2> gpurun_out/c4_$u.err
  stop $? c4_$u
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$u.json')); c=d.get('configs',{}).get('C4',d)
print('u=$u reference_order', c['reference_order']['ms_per_step'], c['reference_order']['roofline']['frac'])" | tee -a gpurun_out/sweep.txt
done
