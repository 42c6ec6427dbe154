#!/bin/bash
# r04zz (b): PMC passes of render_nn_kernel (C2) and render_bil_kernel (C3)
# on the final build (-> profiles/pmc_render_c2.json / pmc_bil_c3.json, the
# bench line's traffic by library hash) and rocprofv3 kernel stats of the
# C1, C2, C3, C4, C5 bench commands.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c3
for c in c2 c3 c4 c1 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 bench.py --only $c --no-cpu --steps 5 --warmup 2 --c1-reps 200 --png-tiles 0 > gpurun_out/prof_$c.log 2>&1
  stop $? prof_$c
done
