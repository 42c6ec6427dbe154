#!/bin/bash
# r05j: C2 render_nn_kernel memory-pipeline counters (L1 / texture units):
# where a gather instruction's ~40 CU cycles go
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3"
export PMC_OUT=gpurun_out/pmc_c2_l1
export PMC_GROUPS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum;TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum;TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum;TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum;TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum TCP_TCC_WRITE_REQ_sum;GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;TA_BUFFER_WRITE_WAVEFRONTS_sum TA_BUFFER_COALESCED_READ_CYCLES_sum;TD_TD_BUSY_sum TD_TC_STALL_sum"
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_l1 render_nn_kernel gpurun_out/pmc_c2_l1.json && cat gpurun_out/pmc_c2_l1.json
