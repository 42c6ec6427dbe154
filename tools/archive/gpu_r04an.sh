#!/bin/bash
# r04an: fused deciles -- select LDS (histogram + key cache) sweep, A/B build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DEC_LDS_KB=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k decile -x -q --timeout 200 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -1 gpurun_out/dec_tests.log; stop $rc dec_tests
for kb in 16 12 20 24 32 40 16; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_LDS_KB=$kb timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$kb.json 2> gpurun_out/c4_$kb.err
  stop $? c4_$kb
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$kb.json')); c=d.get('configs',{}).get('C4',d)
print('lds_kb=$kb deciles', c['deciles']['ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
