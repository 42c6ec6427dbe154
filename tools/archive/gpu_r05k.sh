#!/bin/bash
# r05k: C2 NN kernel in column-group-major order (GSKYHIP_NN_COLG=1, A/B
# build) vs row-major; oracle check; L1 counters of the COLG variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 1 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_NN_COLG=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "colg=$m" >> gpurun_out/r05k_c2_colg.jsonl 2> gpurun_out/r05k_c2_colg.err
  stop $? c2_colg_$m
done
GSKYHIP_LIB=ab GSKYHIP_NN_COLG=1 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "colg=1, oracle check" >> gpurun_out/r05k_c2_colg.jsonl 2>> gpurun_out/r05k_c2_colg.err
stop $? c2_colg_oracle
GSKYHIP_LIB=ab GSKYHIP_NN_COLG=1 timeout -k 10 300 python3 tools/ab_render.py --config c5 --oracle --label "c5 colg=1, oracle check" >> gpurun_out/r05k_c2_colg.jsonl 2>> gpurun_out/r05k_c2_colg.err
stop $? c5_colg_oracle
cat gpurun_out/r05k_c2_colg.jsonl
export GSKYHIP_LIB=ab GSKYHIP_NN_COLG=1
export PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3"
export PMC_OUT=gpurun_out/pmc_c2_colg
export PMC_GROUPS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum;TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum;TD_TD_BUSY_sum TD_TC_STALL_sum;GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU;FETCH_SIZE"
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_colg render_nn_kernel gpurun_out/pmc_c2_colg.json && cat gpurun_out/pmc_c2_colg.json
