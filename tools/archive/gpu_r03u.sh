#!/bin/bash
# r03u: A/B (A/B build) of the deciles transpose with all 32 loads per lane in
# one round (GSKYHIP_DEC_TR1) on C4, its deciles parity tests against the
# oracle with the variant on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DEC_TR1=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -k deciles \
  -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/tr1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tr1_tests.log; stop $rc tr1_tests
for v in 0 1 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_TR1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tr$v -o run \
    --output-format csv -- python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_tr$v.json 2>> gpurun_out/ab.err
  stop $? "c4_tr$v"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['configs']['C4']['deciles']['ms_per_step'])" gpurun_out/c4_tr$v.json
  grep -h "decile_transpose" gpurun_out/prof_tr$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,150-
done
