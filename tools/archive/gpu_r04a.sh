#!/bin/bash
# r04a: fixed-point NN rows (RowFix) -- GPU suite, C2/C5 render A/B against the
# round-3 product library (libgskyhip_r03.so), oracle identity, PMC of C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; [ -n "${SKIP_TESTS:-}" ] || { tail -3 gpurun_out/gpu_tests.log; stop $rc tests; }
for i in 1 2; do
  for lib in default r03; do
    for c in c2 c5; do
      GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label "$lib" >> gpurun_out/ab.jsonl
      stop $? "ab_${lib}_$c"
    done
  done
done
timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 5 --oracle --label fix >> gpurun_out/ab.jsonl
stop $? oracle_c2
timeout -k 10 200 python3 tools/ab_render.py --config c5 --reps 5 --oracle --label fix >> gpurun_out/ab.jsonl
stop $? oracle_c5
cat gpurun_out/ab.jsonl
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c2
