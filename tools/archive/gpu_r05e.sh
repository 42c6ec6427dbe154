#!/bin/bash
# r05e: netCDF-4 GPU test; fused deciles select with 16-byte loads + merged
# bucket runs (A/B build) -- parity tests, then the C4 deciles step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_netcdf4.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/r05e_nc4.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_nc4.log; stop $rc nc4
GSKYHIP_LIB=ab GSKYHIP_DEC_VEC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k decile -x -q --timeout 200 --timeout-method thread > gpurun_out/r05e_dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05e_dec_tests.log; stop $rc dec_tests
for cfg in "0 8" "1 8" "1 16" "0 8b" "1 8b"; do
  set -- $cfg
  u=${2%b}
  GSKYHIP_LIB=ab GSKYHIP_DEC_VEC=$1 GSKYHIP_DEC_U=$u timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05e_c4_$1_$2.json 2> gpurun_out/r05e_c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; c=json.load(open('gpurun_out/r05e_c4_$1_$2.json'))['configs']['C4']
print('vec=$1 u=$2 deciles', c['deciles']['ms_per_step'])" | tee -a gpurun_out/r05e_dec_sweep.txt
done
