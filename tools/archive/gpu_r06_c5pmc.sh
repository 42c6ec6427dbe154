#!/bin/bash
# r06: PMC passes of the C5 band kernel (render_nn_kernel<int16, mask>) on
# the current library, summarised; plus the C5 render timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06v}
timeout -k 10 200 python -u tools/ab_render.py --config c5 --reps 20 --label $T > gpurun_out/${T}_c5.jsonl 2>/dev/null
rc=$?; cat gpurun_out/${T}_c5.jsonl; [ $rc -ne 0 ] && exit $rc
PMC_OUT=gpurun_out/${T}_pmc_c5 PMC_CMD="python3 tools/ab_render.py --config c5 --reps 3" PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64;MeanOccupancyPerCU;TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum;TD_TD_BUSY_sum TD_TC_STALL_sum;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" bash tools/pmc.sh
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 tools/pmc_summary.py gpurun_out/${T}_pmc_c5 "render_nn_kernel<" gpurun_out/${T}_pmc_render_c5.json > /dev/null
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_pmc_render_c5.json'))
c=d['counters_per_launch']; print(json.dumps({k: round(v) for k,v in c.items()}))
print({k: d[k] for k in d if k not in ('counters_per_launch',)})"
