#!/bin/bash
# r04b: fixed-point NN rows (RowFix, restrict kernel parameter, fallback rows
# in a second loop) -- C2/C5 render A/B against the round-3 product library,
# oracle identity, PMC of C2's render_nn_kernel; FETCH_SIZE/WRITE_SIZE
# calibration (tools/calib/fetch_calib.hip); C5 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for i in 1 2; do
  for lib in default r03; do
    for c in c2 c5; do
      GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label "$lib" >> gpurun_out/ab.jsonl
      stop $? "ab_${lib}_$c"
    done
  done
done
for i in 1 2; do
  for lib in default r03; do
    GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_c3.py --reps 10 --label "c3_$lib" >> gpurun_out/ab.jsonl
    stop $? "ab_c3_$lib"
  done
done
timeout -k 10 300 python3 tools/ab_c3.py --reps 3 --oracle --label c3_fix >> gpurun_out/ab.jsonl
stop $? oracle_c3
timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 5 --oracle --label fix >> gpurun_out/ab.jsonl
stop $? oracle_c2
timeout -k 10 200 python3 tools/ab_render.py --config c5 --reps 5 --oracle --label fix >> gpurun_out/ab.jsonl
stop $? oracle_c5
cat gpurun_out/ab.jsonl
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c2
PMC_OUT=gpurun_out/calib PMC_CMD="./tools/calib/fetch_calib 3" PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc.sh
stop $? calib
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- \
  python3 bench.py --only c5 --no-cpu --steps 5 --warmup 2 > gpurun_out/prof_c5.log 2>&1
stop $? prof_c5
timeout -k 10 300 python -u -m pytest tests/test_drill_geom.py tests/test_ingest.py tests/test_geoloc.py -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_geom.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_geom.log; stop $rc tests_geom
timeout -k 10 300 python3 bench.py --only c4 --no-cpu --no-deciles --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err
stop $? c4
