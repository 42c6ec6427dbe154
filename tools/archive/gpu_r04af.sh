#!/bin/bash
# r04af: readData with deciles -- the mean pass writes the band-major rows + key ranges (fused) vs the transpose path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile or drill" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests.log; stop $rc dec_tests
GSKYHIP_LIB=ab GSKYHIP_DEC_FUSED_LOG2=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests_nf.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests_nf.log; stop $rc dec_tests_nofused
for cfg in "prod -" "ab 33" "ab 0" "prod -"; do
  set -- $cfg
  if [ "$1" = prod ]; then L=""; else L=ab; fi
  GSKYHIP_LIB=$L GSKYHIP_DEC_FUSED_LOG2=$2 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$1_$2.json 2> gpurun_out/c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$1_$2.json')); c=d.get('configs',{}).get('C4',d)
print('lib=$1 fused_log2=$2 deciles', c['deciles']['ms_per_step'], 'ref_order', c['reference_order']['ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1
stop $? prof
