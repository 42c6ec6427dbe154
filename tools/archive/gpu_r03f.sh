#!/bin/bash
# r03f: the scale+palette LUT (render_nn.h: RAW-domain canvases, one 4-B
# table load per pixel instead of ~10 VALU + an LDS read) A/B on C2 with and
# without the single-entry prefetch path, and on C5 with one / four rows per
# wave for masked stacks -- each checked against the oracle; the deciles
# select kernel with pipelined passes (rocprofv3 of C4); C1 with the fused
# one-launch planner; GPU suite and the bench line on the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
tail -3 gpurun_out/gpu_tests.log
for v in "0 0" "1 0" "1 1" "0 1" "0 0" "1 0" "1 1"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_NN_LUT=$1 GSKYHIP_NN_ONE=$2 timeout -k 10 300 python -u tools/ab_render.py --config c2 \
    --reps 30 --oracle --label "lut$1 one$2" >> gpurun_out/ab_c2.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c2_lut$1_one$2"
done
cat gpurun_out/ab_c2.jsonl
for v in "0 4" "0 1" "1 1" "1 4" "0 4" "1 1"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_NN_LUT=$1 GSKYHIP_NN_MASK_RPW=$2 timeout -k 10 300 python -u tools/ab_render.py \
    --config c5 --reps 30 --oracle --label "lut$1 mask_rpw$2" >> gpurun_out/ab_c5.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c5_lut$1_rpw$2"
done
cat gpurun_out/ab_c5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- \
  python3 bench.py --only c1 --no-cpu --c1-reps 200 > gpurun_out/prof_c1.log 2>&1
stop $? prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
