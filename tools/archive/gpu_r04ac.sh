#!/bin/bash
# r04ac: product select (kU 8, 8 waves/SIMD, 16 KB) parity; deciles vs band chunk size (A/B GSKYHIP_DEC_WS_LOG2) + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile or drill" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests.log; stop $rc dec_tests
GSKYHIP_LIB=ab GSKYHIP_DEC_WS_LOG2=33 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests33.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests33.log; stop $rc dec_tests33
for w in 30 31 32 33; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_WS_LOG2=$w timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$w.json 2> gpurun_out/c4_$w.err
  stop $? c4_$w
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$w.json')); c=d.get('configs',{}).get('C4',d)
print('ws_log2=$w', c['deciles']['ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
for w in 30 33; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_WS_LOG2=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run -- python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_$w.log 2>&1
  stop $? prof_$w
done
