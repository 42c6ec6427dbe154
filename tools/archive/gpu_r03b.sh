#!/bin/bash
# r03b: GPU suite (new bilinear kernel, new rasterizer, partition ranks),
# A/B of the NN band kernel (rows per wave x deferred stores, C2 + C5) and of
# the bilinear kernel (C3), each checked against the oracle; then the full
# default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
for v in "0 0 4" "1 0 4" "0 0 2" "0 8 4" "1 8 4"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_BIL_F32=$1 GSKYHIP_BIL_RPW=${2/0/4} GSKYHIP_BIL_HP=$3 timeout -k 10 300 python -u tools/ab_c3.py \
    --oracle --label "f32=$1 rpw=${2/0/4} hp=$3" >> gpurun_out/ab_c3.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c3_$1_$2_$3"
done
for c in c2 c5; do
  for rpw in 4 8 16; do
    for pipe in 0 1; do
      GSKYHIP_LIB=ab GSKYHIP_NN_RPW=$rpw GSKYHIP_NN_PIPE=$pipe timeout -k 10 300 python -u tools/ab_render.py \
        --config $c --reps 30 --oracle --label "rpw$rpw pipe$pipe" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
      stop $? "ab_${c}_rpw${rpw}_pipe${pipe}"
    done
  done
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- \
  python3 bench.py --only c1 --no-cpu --c1-reps 200 > gpurun_out/prof_c1.log 2>&1
stop $? prof_c1
