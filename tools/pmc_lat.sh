#!/bin/bash
# Latency PMC passes (Little's law: SQ_INST_LEVEL_x / SQ_INSTS_x = cycles in flight per instruction)
# and scalar/instruction cache hit rates for one A/B variant.  One counter group per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmc_lat}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 tools/ab_render.py --variant nn_4x2 --reps 3"}
i=0
for grp in "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INST_LEVEL_LDS" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES" \
           "SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_IFETCH SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    $CMD > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
