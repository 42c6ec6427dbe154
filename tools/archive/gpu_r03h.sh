#!/bin/bash
# r03h: GPU suite on the product library (deciles: 11-bit bucket pass +
# candidate compaction); rocprofv3 stats of C4 (deciles) and C3; PMC passes of
# render_bil_kernel (C3) and render_nn_kernel (C2, current build); the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
  python3 bench.py --only c3 --no-cpu > gpurun_out/prof_c3.log 2>&1
stop $? prof_c3
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" bash tools/pmc.sh
stop $? pmc_c3
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
