#!/bin/bash
# r06: render timings of the product library against libgskyhip_prev.so (the
# last committed build, GSKYHIP_LIB=prev), alternating, with the oracle check
# on the first pass, after the GPU tests selected by $3.
#   bash tools/gpu_r06_ab2.sh <tag> "<configs>" "<pytest -k expr>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06ab}
CFGS=${2:-"c5"}
K=${3:-""}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${T}_tests.txt 2>&1
  rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -ne 0 ] && exit $rc
fi
: > gpurun_out/${T}_render.jsonl
for rep in 1 2 3; do
  for lib in product prev; do
    if [ $lib = prev ]; then export GSKYHIP_LIB=prev; else unset GSKYHIP_LIB; fi
    for c in $CFGS; do
      O=""; [ $rep = 1 ] && O="--oracle"
      timeout -k 10 300 python -u tools/ab_render.py --config $c --reps 20 --label $T-$lib $O >> gpurun_out/${T}_render.jsonl 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "render $lib $c rc=$rc"; exit $rc; }
    done
  done
done
cat gpurun_out/${T}_render.jsonl
