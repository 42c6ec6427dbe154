#!/bin/bash
# r03j: GPU suite (bilinear fast path branch-free; the LDS-staged NN kernel in
# the A/B variants); C2 A/B of the staged kernel vs the product path, checked
# against the oracle; C3 bilinear timing; rocprofv3 of C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; stop $rc tests
for v in 0 1 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_NN_STAGED=$v timeout -k 10 300 python -u tools/ab_render.py --config c2 \
    --reps 30 --oracle --label "staged$v" >> gpurun_out/ab_c2.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c2_staged$v"
done
cat gpurun_out/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_c3.py --reps 20 --oracle --label "bil_fast" > gpurun_out/ab_c3.jsonl 2>> gpurun_out/ab.err
stop $? ab_c3
cat gpurun_out/ab_c3.jsonl
GSKYHIP_LIB=ab GSKYHIP_NN_STAGED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s -o run \
  --output-format csv -- python3 tools/ab_render.py --config c2 --reps 5 > gpurun_out/prof_c2s.log 2>&1
stop $? prof_c2s
for v in "36 16" "48 16" "36 8" "48 8" "24 16"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_DEC_LDS_KB=$1 GSKYHIP_DEC_U=$2 timeout -k 10 300 python -u bench.py --only c4 --no-cpu \
    --steps 3 --warmup 1 > gpurun_out/c4_lds$1_u$2.json 2>> gpurun_out/ab.err
  stop $? "c4_lds$1_u$2"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['configs']['C4']['deciles']['ms_per_step'])" gpurun_out/c4_lds$1_u$2.json
done
GSKYHIP_LIB=ab GSKYHIP_PLAN_STAMPS=1 timeout -k 10 300 python -u bench.py --only c1 --no-cpu --c1-reps 30 \
  > gpurun_out/c1_stamps.json 2> gpurun_out/c1_stamps.err
stop $? c1_stamps
grep plan_small_stamps gpurun_out/c1_stamps.err | tail -5
