#!/bin/bash
# r03a: first GPU pass of the round-3 NN band kernel: the GPU suite, C2/C5
# render-phase timing, C2 bench line, rocprofv3 kernel stats, PMC passes of
# render_nn_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
for c in c2 c5; do
  timeout -k 10 300 python -u tools/ab_render.py --config $c --reps 30 --oracle >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  stop $? ab_$c
done
timeout -k 10 300 python -u bench.py --only c2 --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_c2.json 2> gpurun_out/bench.err
stop $? bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python3 tools/ab_render.py --config c2 --reps 10 > gpurun_out/prof_c2.log 2>&1
stop $? prof_c2
PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2 timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1
stop $? pmc
