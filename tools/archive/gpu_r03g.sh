#!/bin/bash
# r03g: GPU suite (A/B-build variants in child processes); C2 A/B of the
# single-entry path and of LDS-staged 16-B stores, each checked against the
# oracle; rocprofv3 stats of C2 and C4 (deciles: wave-parallel bucket search,
# cached workspace); the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
stop $? tests
tail -3 gpurun_out/gpu_tests.log
for v in "1 0" "0 0" "1 1" "0 1" "1 0" "1 1"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_NN_ONE=$1 GSKYHIP_NN_STAGE=$2 timeout -k 10 300 python -u tools/ab_render.py --config c2 \
    --reps 30 --oracle --label "one$1 stage$2" >> gpurun_out/ab_c2.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c2_one$1_stage$2"
done
cat gpurun_out/ab_c2.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python3 bench.py --only c2 --no-cpu > gpurun_out/prof_c2.log 2>&1
stop $? prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_c4.log 2>&1
stop $? prof_c4
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
