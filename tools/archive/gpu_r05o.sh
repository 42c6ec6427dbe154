#!/bin/bash
# r05o: masked stack entries with every data + mask gather of a row in flight
# together (GSKYHIP_NN_MASKB=1, A/B build) -- mask / C5 parity tests, then the
# C5 band kernel A/B with the oracle check and the C5 bench step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_NN_MASKB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "c5 or mask or merge" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05o_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r05o_tests.txt; stop $rc tests
for m in 0 1 0 1; do
  GSKYHIP_NN_MASKB=$m timeout -k 10 300 python3 tools/ab_render.py --config c5 --label "c5 maskb=$m" >> gpurun_out/r05o_c5.jsonl 2>> gpurun_out/r05o_c5.err
  stop $? c5_$m
done
GSKYHIP_NN_MASKB=1 timeout -k 10 300 python3 tools/ab_render.py --config c5 --oracle --label "c5 maskb=1 oracle" >> gpurun_out/r05o_c5.jsonl 2>> gpurun_out/r05o_c5.err
stop $? c5_oracle
for m in 0 1; do
  GSKYHIP_NN_MASKB=$m timeout -k 10 300 python3 bench.py --only c5 --no-cpu --steps 20 --warmup 3 > gpurun_out/r05o_bench_c5_$m.json 2>> gpurun_out/r05o_c5.err
  stop $? bench_c5_$m
  python3 -c "
import json; c=json.load(open('gpurun_out/r05o_bench_c5_$m.json'))['configs']['C5']
print('maskb=$m C5 ms', c['ms_per_step'], 'p50', c['p50_tile_ms'], 'kernel', c['roofline']['kernel_ms'])" | tee -a gpurun_out/r05o_c5.txt
done
cat gpurun_out/r05o_c5.jsonl
