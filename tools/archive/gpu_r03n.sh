#!/bin/bash
# r03n: GPU suite (entry-window group skipping in the bilinear / NN edge
# bodies); C3, C2, C5 render timing checked against the oracle; PMC of
# render_nn_kernel (C2) on this library build -> the bench line's traffic;
# rocprofv3 stats of the C2 bench command; the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
timeout -k 10 300 python -u tools/ab_c3.py --reps 20 --oracle --label "bil_skip" > gpurun_out/ab_c3.jsonl 2>> gpurun_out/ab.err
stop $? ab_c3
cat gpurun_out/ab_c3.jsonl
for c in c2 c5; do
  timeout -k 10 300 python -u tools/ab_render.py --config $c --reps 30 --oracle --label "skip_$c" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_$c"
done
cat gpurun_out/ab.jsonl
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python3 bench.py --only c2 --no-cpu > gpurun_out/prof_c2.log 2>&1
stop $? prof_c2
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
