#!/bin/bash
# r04am: PMC of the fused deciles path on C4 (drill_sum_kernel<*, true> and decile_select_kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_OUT=gpurun_out/pmc_c4 PMC_CMD="python3 bench.py --only c4 --no-cpu --steps 1 --warmup 1" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR;MeanOccupancyPerCU" \
  bash tools/pmc.sh
