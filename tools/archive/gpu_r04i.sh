#!/bin/bash
# r04i: NN band kernel prologue in one load round + tile-plan e0 + all rows'
# RowFix in one vector load (VFETCH) -- C2/C5 against the round-3 library,
# VFETCH off and 16 rows per wave (A/B build), oracle identity; GPU tests of
# the render paths; service leg trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 5 --oracle --label new >> gpurun_out/ab.jsonl
stop $? oracle_c2
timeout -k 10 200 python3 tools/ab_render.py --config c5 --reps 5 --oracle --label new >> gpurun_out/ab.jsonl
stop $? oracle_c5
for i in 1 2; do
  for c in c2 c5; do
    timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label new >> gpurun_out/ab.jsonl
    stop $? "ab_new_$c"
    GSKYHIP_LIB=r03 timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label r03 >> gpurun_out/ab.jsonl
    stop $? "ab_r03_$c"
  done
  GSKYHIP_LIB=ab GSKYHIP_NN_VFETCH=0 timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label vfetch0 >> gpurun_out/ab.jsonl
  stop $? ab_vfetch0
  GSKYHIP_LIB=ab GSKYHIP_NN_RPW=16 timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label rpw16 >> gpurun_out/ab.jsonl
  stop $? ab_rpw16
  GSKYHIP_LIB=ab GSKYHIP_AB_MODE=1 timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label storeonly >> gpurun_out/ab.jsonl
  stop $? ab_storeonly
done
GSKYHIP_LIB=ab GSKYHIP_NN_RPW=16 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 3 --oracle --label rpw16 >> gpurun_out/ab.jsonl
stop $? oracle_rpw16
cat gpurun_out/ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_graph.py tests/test_service.py tests/test_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc gpu_tests
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_svc -o run --output-format csv -- \
  python3 bench.py --only svc --no-cpu --svc-jobs 256 > gpurun_out/prof_svc.log 2>&1
stop $? prof_svc
timeout -k 10 400 python3 bench.py --only svc --no-cpu --steps 3 --warmup 1 > gpurun_out/svc.json 2> gpurun_out/svc.err
stop $? svc
python3 -c "
import json; d=json.load(open('gpurun_out/svc.json'))['configs']['service']
for k in ('workers_16','workers_64'): print(k, json.dumps(d[k]))"
