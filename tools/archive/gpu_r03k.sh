#!/bin/bash
# r03k: (+ deciles transpose in 32-band tiles; + C1: SuggestedWarpOutput2 transforms inlined in the workgroup planner) GPU suite (NN: window-edge rows of `inside` entries take a fast body
# with the window test instead of the general per-pixel rules); C2 / C5
# render timing checked against the oracle; rocprofv3 stats of C2; bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
for c in c2 c5 c2 c5; do
  timeout -k 10 300 python -u tools/ab_render.py --config $c --reps 30 --oracle --label "partial_$c" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_$c"
done
cat gpurun_out/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python3 bench.py --only c2 --no-cpu > gpurun_out/prof_c2.log 2>&1
stop $? prof_c2
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
GSKYHIP_LIB=ab GSKYHIP_PLAN_STAMPS=1 timeout -k 10 300 python -u bench.py --only c1 --no-cpu --c1-reps 30 \
  > gpurun_out/c1_stamps.json 2> gpurun_out/c1_stamps.err
stop $? c1_stamps
grep plan_small_stamps gpurun_out/c1_stamps.err | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- \
  python3 bench.py --only c1 --no-cpu --c1-reps 200 > gpurun_out/prof_c1.log 2>&1
stop $? prof_c1
