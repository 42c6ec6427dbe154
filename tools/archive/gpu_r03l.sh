#!/bin/bash
# r03l: C1 plan_small phase stamps (inside SuggestedWarpOutput2); C4 deciles
# timing with the 32-band transpose; PMC passes of the deciles kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_PLAN_STAMPS=1 timeout -k 10 300 python -u bench.py --only c1 --no-cpu --c1-reps 30 \
  > gpurun_out/c1_stamps.json 2> gpurun_out/c1_stamps.err
stop $? c1_stamps
grep plan_small_stamps gpurun_out/c1_stamps.err | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
PMC_OUT=gpurun_out/pmc_c4 PMC_CMD="python3 bench.py --only c4 --no-cpu --steps 1 --warmup 0" \
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS;SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c4
