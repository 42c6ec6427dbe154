#!/bin/bash
# r03v: closing measurement (+ speculative SuggestedWarpOutput2 grid points, one-round deciles transpose; C1 phase stamps) on the final library build: GPU suite; PMC passes
# of render_nn_kernel (C2) and render_bil_kernel (C3) -> profiles/pmc_*.json
# (the bench line's traffic, matched by library hash); rocprofv3 kernel stats
# of the C2, C3, C4 and C1 bench commands; the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
GSKYHIP_LIB=ab GSKYHIP_PLAN_STAMPS=1 timeout -k 10 300 python -u bench.py --only c1 --no-cpu --c1-reps 30 \
  > gpurun_out/c1_stamps.json 2> gpurun_out/c1_stamps.err
stop $? c1_stamps
grep plan_small_stamps gpurun_out/c1_stamps.err | tail -2
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c3
for c in c2 c3 c4 c1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 bench.py --only $c --no-cpu --steps 5 --warmup 2 --c1-reps 200 > gpurun_out/prof_$c.log 2>&1
  stop $? prof_$c
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
