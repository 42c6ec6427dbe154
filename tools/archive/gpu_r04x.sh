#!/bin/bash
# r04x: decile select with 256-thread workgroups (GSKYHIP_DEC_NT=256, A/B
# build) at 20 / 36 KB of LDS vs 512 threads; parity of the 256 variant;
# the packed drill descriptors (drill tests, breakdown, C4 line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DEC_NT=256 GSKYHIP_DEC_LDS_KB=20 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dec_tests.log; stop $rc dec_tests
for cfg in "512 36" "256 20" "256 36" "256 12"; do
  set -- $cfg
  GSKYHIP_LIB=ab GSKYHIP_DEC_NT=$1 GSKYHIP_DEC_LDS_KB=$2 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$1_$2.json 2> gpurun_out/c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$1_$2.json')); c=d.get('configs',{}).get('C4',d)
print('nt=$1 lds=$2', c['deciles']['ms_per_step'], 'descriptors', c['descriptors_ms'])"
done
timeout -k 10 600 python -u -m pytest tests/test_drill_geom.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/drill_tests.log 2>&1
rc=$?; tail -2 gpurun_out/drill_tests.log; stop $rc drill_tests
timeout -k 10 200 python3 tools/c4_desc.py --label packed --reps 20 >> gpurun_out/c4_desc.jsonl
stop $? c4_desc
cat gpurun_out/c4_desc.jsonl
