#!/bin/bash
# r03e: GPU suite (chunk-parallel deciles transpose + LDS-cached selection,
# one-workgroup small-batch planner), A/B of the producer / store-wave
# bilinear kernel on C3, FETCH_SIZE calibration with live 16-bit kernels,
# rocprofv3 stats of C1 and C4, the bench line; NN row-pair A/B on C2 and
# PMC passes of the default NN kernel (tools/pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
tail -3 gpurun_out/gpu_tests.log
for ws in 0 3 7 0; do
  GSKYHIP_LIB=ab GSKYHIP_BIL_WS=$ws timeout -k 10 300 python -u tools/ab_c3.py --oracle --label "bil ws$ws" \
    >> gpurun_out/ab_c3.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c3_ws$ws"
done
cat gpurun_out/ab_c3.jsonl
for v in "PAIR 0" "PAIR 8" "PAIR 4" "ONE 8" "ONE 4" "PAIR 0" "PAIR 8" "ONE 8"; do
  set -- $v
  env GSKYHIP_LIB=ab GSKYHIP_NN_$1=$2 timeout -k 10 300 python -u tools/ab_render.py --config c2 --reps 30 \
    --oracle --label "$1 $2" >> gpurun_out/ab_pair.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_$1_$2"
done
cat gpurun_out/ab_pair.jsonl
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/calib_f -o run --output-format csv -- \
  ./tools/calib/fetch_calib 3 > gpurun_out/calib_f.log 2>&1
stop $? calib_fetch
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- \
  python3 bench.py --only c1 --no-cpu --c1-reps 200 > gpurun_out/prof_c1.log 2>&1
stop $? prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2 bash tools/pmc.sh
