#!/bin/bash
# r05s: the LDS-staged NN kernel (GSKYHIP_NN_STAGED=1, A/B build) against
# the product body now that the texture data unit is known to be the
# product's bound; oracle check; its counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 1 0 1; do
  GSKYHIP_NN_STAGED=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "staged=$m" >> gpurun_out/r05s_staged.jsonl 2>> gpurun_out/r05s.err
  stop $? staged_$m
done
GSKYHIP_NN_STAGED=1 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "staged=1 oracle" >> gpurun_out/r05s_staged.jsonl 2>> gpurun_out/r05s.err
stop $? staged_oracle
cat gpurun_out/r05s_staged.jsonl
GSKYHIP_NN_STAGED=1 PMC_GROUPS="TD_TD_BUSY_sum TD_TC_STALL_sum;GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE MeanOccupancyPerCU" PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2_staged bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_staged render_nn_stage gpurun_out/pmc_c2_staged.json && cat gpurun_out/pmc_c2_staged.json
