#!/bin/bash
# r05b: C3 separable-row kernel A/B (variants of the A/B build, each against
# the oracle), then the full C3 test on the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
run_ab() {  # label, env...
  local label=$1; shift
  env GSKYHIP_LIB=ab "$@" timeout -k 10 300 python3 tools/ab_c3.py --reps 10 --oracle --label $label >> gpurun_out/r05b_ab_c3.jsonl 2> gpurun_out/r05b_ab_c3_$label.err
  stop $? ab_c3_$label
}
run_ab sep0 GSKYHIP_BIL_SEP=0
run_ab sep1 GSKYHIP_BIL_SEP=1
run_ab sep1_hp8 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_HP=8
run_ab sep1_rpw8 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_RPW=8
run_ab sep1_rpw16 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_RPW=16
run_ab sep0b GSKYHIP_BIL_SEP=0
cat gpurun_out/r05b_ab_c3.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -m gpu -v -x -k "c3" \
  --timeout 300 --timeout-method thread > gpurun_out/r05b_tests_c3.log 2>&1
rc=$?; tail -3 gpurun_out/r05b_tests_c3.log; stop $rc tests_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b_prof_c3 -o run --output-format csv -- \
  python3 bench.py --only c3 --no-cpu --steps 5 --warmup 2 > gpurun_out/r05b_prof_c3.log 2>&1
stop $? prof_c3
