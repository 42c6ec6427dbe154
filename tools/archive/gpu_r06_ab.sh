#!/bin/bash
# r06: correctness (full C2 / C5, parity suite) + render timings of the
# product and the A/B library on C2 and C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06x}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full_identical" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
: > gpurun_out/${T}_render.jsonl
for rep in 1 2; do
for lib in default ab; do
  for c in c5 c2; do
    if [ $lib = ab ]; then export GSKYHIP_LIB=ab; else unset GSKYHIP_LIB; fi
    timeout -k 10 200 python -u tools/ab_render.py --config $c --reps 20 --label $T-$lib >> gpurun_out/${T}_render.jsonl 2>/dev/null
    stop $? render_${lib}_$c
  done
done
done
unset GSKYHIP_LIB
tail -2 gpurun_out/${T}_full.txt gpurun_out/${T}_parity.txt; cat gpurun_out/${T}_render.jsonl
