#!/bin/bash
# r06: PMC passes of C2's planner kernels (plan_rows_kernel, plan_pairs_kernel)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_OUT=gpurun_out/pmc_plan PMC_CMD="python3 tools/ab_render.py --config c2 --reps 1" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64;SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;MeanOccupancyPerCU" \
  bash tools/pmc.sh || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_plan "plan_rows_kernel" gpurun_out/pmc_plan_rows_c2.json > /dev/null
python3 tools/pmc_summary.py gpurun_out/pmc_plan "plan_pairs_kernel" gpurun_out/pmc_plan_pairs_c2.json > /dev/null
cat gpurun_out/pmc_plan_rows_c2.json; echo; cat gpurun_out/pmc_plan_pairs_c2.json
