#!/bin/bash
# r05c: C3 separable-row kernel A/B (variants of the A/B build, each against
# the oracle), then the full C3 test on the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
run_ab() {  # label, env...
  local label=$1; shift
  env GSKYHIP_LIB=ab "$@" timeout -k 10 300 python3 tools/ab_c3.py --reps 10 --oracle --label $label >> gpurun_out/r05c_ab_c3.jsonl 2> gpurun_out/r05c_ab_c3_$label.err
  stop $? ab_c3_$label
}
run_ab sep0 GSKYHIP_BIL_SEP=0
run_ab sep1 GSKYHIP_BIL_SEP=1
run_ab sep1_hp8w6 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_HP=8
run_ab sep1_pipe_w8 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_HP=0
run_ab sep1_pipe_w6 GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_HP=10
run_ab sep0b GSKYHIP_BIL_SEP=0
GSKYHIP_LIB=ab GSKYHIP_BIL_SEP=1 GSKYHIP_BIL_SEPSTAT=1 timeout -k 10 300 python3 tools/ab_c3.py --reps 1 --label stat > gpurun_out/r05c_sepstat.json 2> gpurun_out/r05c_sepstat.err
stop $? sepstat
grep bil_sep_stat gpurun_out/r05c_sepstat.err | tail -2
cat gpurun_out/r05c_ab_c3.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -m gpu -v -x -k "c3" \
  --timeout 300 --timeout-method thread > gpurun_out/r05c_tests_c3.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_tests_c3.log; stop $rc tests_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof_c3 -o run --output-format csv -- \
  python3 bench.py --only c3 --no-cpu --steps 5 --warmup 2 > gpurun_out/r05c_prof_c3.log 2>&1
stop $? prof_c3
# fused deciles select: workgroup size x LDS (A/B build)
GSKYHIP_LIB=ab GSKYHIP_DEC_FNT=1024 GSKYHIP_DEC_LDS_KB=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k decile -x -q --timeout 200 --timeout-method thread > gpurun_out/r05c_dec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05c_dec_tests.log; stop $rc dec_tests
for cfg in "256 16" "1024 64" "512 32" "1024 48" "512 64" "256 16"; do
  set -- $cfg
  GSKYHIP_LIB=ab GSKYHIP_DEC_FNT=$1 GSKYHIP_DEC_LDS_KB=$2 timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05c_c4_$1_$2.json 2> gpurun_out/r05c_c4_$1_$2.err
  stop $? c4_$1_$2
  python3 -c "
import json; c=json.load(open('gpurun_out/r05c_c4_$1_$2.json'))['configs']['C4']
print('fnt=$1 lds_kb=$2 deciles', c['deciles']['ms_per_step'])" | tee -a gpurun_out/r05c_dec_sweep.txt
done
