#!/bin/bash
# r04y: decile select workgroup shape sweep (A/B build: threads x LDS KB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DEC_NT=128 GSKYHIP_DEC_LDS_KB=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests.log; stop $rc dec_tests
for cfg in "256 20" "256 16" "256 24" "256 28" "128 12" "128 16" "128 20"; do
  set -- $cfg
  GSKYHIP_LIB=ab GSKYHIP_DEC_NT=$1 GSKYHIP_DEC_LDS_KB=$2 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$1_$2.json 2> gpurun_out/c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$1_$2.json')); c=d.get('configs',{}).get('C4',d)
print('nt=$1 lds=$2', c['deciles']['ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
