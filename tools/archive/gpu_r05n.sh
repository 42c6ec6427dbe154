#!/bin/bash
# r05n: fused deciles select with 128-thread workgroups (twice the segments
# in flight per CU) and 8 / 16 KB of LDS, A/B build; CF transverse_mercator
# netCDF GPU test on the product build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n_ingest.txt 2>&1
rc=$?; tail -2 gpurun_out/r05n_ingest.txt; stop $rc ingest
GSKYHIP_LIB=ab GSKYHIP_DEC_FNT=128 GSKYHIP_DEC_LDS_KB=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k decile -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n_dec_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r05n_dec_tests.txt; stop $rc dec_tests
for cfg in "256 16" "128 8" "128 16" "256 16" "128 8"; do
  set -- $cfg
  GSKYHIP_LIB=ab GSKYHIP_DEC_FNT=$1 GSKYHIP_DEC_LDS_KB=$2 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05n_c4_$1_$2.json 2> gpurun_out/r05n_c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; c=json.load(open('gpurun_out/r05n_c4_$1_$2.json'))['configs']['C4']
print('nt=$1 lds=$2 deciles', c['deciles']['ms_per_step'])" | tee -a gpurun_out/r05n_dec_sweep.txt
done
