#!/bin/bash
# PMC passes for one kernel, one counter group per rocprofv3 run (kernel-trace
# only, never combined with sys/runtime traces), each under its own time limit.
#   PMC_CMD   the program to profile (default: the C2 A/B tool, direct variant)
#   PMC_OUT   output dir (default gpurun_out/pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 tools/ab_render.py --variant nn_4x4 --reps 3"}
i=${PMC_FIRST:-0}
# PMC_GROUPS: ';'-separated counter groups replacing the default list
if [ -n "${PMC_GROUPS:-}" ]; then
  IFS=';' read -r -a GROUPS_ARR <<< "$PMC_GROUPS"
else
  GROUPS_ARR=()
fi
if [ ${#GROUPS_ARR[@]} -eq 0 ]; then GROUPS_ARR=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "MeanOccupancyPerCU"); fi
for grp in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    $CMD > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
