#!/bin/bash
# r04aa: decile select with register-resident keys (A/B build, GSKYHIP_DEC_REG) and kU=8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for r in 32 16; do
GSKYHIP_LIB=ab GSKYHIP_DEC_REG=$r GSKYHIP_DEC_LDS_KB=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests_$r.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests_$r.log; stop $rc dec_tests_$r
done
for cfg in "0 20 16" "0 20 8" "32 8 16" "32 20 16" "24 8 16" "16 8 16" "16 20 16"; do
  set -- $cfg
  GSKYHIP_LIB=ab GSKYHIP_DEC_REG=$1 GSKYHIP_DEC_LDS_KB=$2 GSKYHIP_DEC_U=$3 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$1_$2_$3.json 2> gpurun_out/c4_$1_$2_$3.err
  stop $? c4_$1_$2_$3
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$1_$2_$3.json')); c=d.get('configs',{}).get('C4',d)
print('reg=$1 lds=$2 u=$3', c['deciles']['ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
