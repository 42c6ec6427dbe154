#!/bin/bash
# r05t: RGBA rows through LDS as 16-byte stores (GSKYHIP_NN_STAGE=1, A/B
# build) vs 4-byte stores -- time, oracle check, texture-data-unit counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 1 0 1; do
  GSKYHIP_NN_STAGE=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "stage16=$m" >> gpurun_out/r05t.jsonl 2>> gpurun_out/r05t.err
  stop $? st_$m
done
GSKYHIP_NN_STAGE=1 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "stage16=1 oracle" >> gpurun_out/r05t.jsonl 2>> gpurun_out/r05t.err
stop $? st_oracle
cat gpurun_out/r05t.jsonl
GSKYHIP_NN_STAGE=1 PMC_GROUPS="TD_TD_BUSY_sum TD_TC_STALL_sum;GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_WRITE_sum" PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2_stage16 bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_stage16 render_nn_kernel gpurun_out/pmc_c2_stage16.json && cat gpurun_out/pmc_c2_stage16.json
