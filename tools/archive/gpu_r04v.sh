#!/bin/bash
# r04v: PMC of decile_select_kernel (C4 deciles): waits, LDS conflicts,
# instruction mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
PMC_OUT=gpurun_out/pmc_dec PMC_CMD="python3 bench.py --only c4 --no-cpu --steps 1 --warmup 1" \
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY;FETCH_SIZE;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_dec
