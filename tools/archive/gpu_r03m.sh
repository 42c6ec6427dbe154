#!/bin/bash
# r03m: GPU suite (deciles: bucket ranks by wave-ballot selection; drill
# stack pixel rows 128-byte aligned); C4 bench + rocprofv3 stats; PMC passes
# of render_bil_kernel (C3); the bench line.
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
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" \
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;FETCH_SIZE;WRITE_SIZE;TA_BUSY_avr TA_TA_BUSY_sum;GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_ANY;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c3
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
