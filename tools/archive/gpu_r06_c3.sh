#!/bin/bash
# r06: C3 full-canvas bilinear test + C3 render timings, product vs libgskyhip_ab.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06c3}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c3" -m gpu > gpurun_out/${T}_full.txt 2>&1
rc=$?; tail -2 gpurun_out/${T}_full.txt; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${T}_c3.jsonl
for rep in 1 2; do
  for lib in default ab; do
    if [ $lib = ab ]; then export GSKYHIP_LIB=ab; else unset GSKYHIP_LIB; fi
    timeout -k 10 200 python -u tools/ab_c3.py --reps 10 --label $T-$lib >> gpurun_out/${T}_c3.jsonl 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "c3 $lib rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/${T}_c3.jsonl
