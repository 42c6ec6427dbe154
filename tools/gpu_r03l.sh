#!/bin/bash
# r03l: PMC passes of the deciles kernels (select, transpose) on C4, one
# counter group per rocprofv3 run: instruction mix, waits, LDS conflicts,
# occupancy, HBM bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_OUT=gpurun_out/pmc_c4 PMC_CMD="python3 bench.py --only c4 --no-cpu --steps 1 --warmup 0" \
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS;SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;MeanOccupancyPerCU" \
  bash tools/pmc.sh
echo "pmc rc=$?"
