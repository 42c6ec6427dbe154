#!/bin/bash
# r06: two-entry rows folded with one per-lane-address gather per pixel
# (nn_pair_row) -- full C2 / C5 identity, the parity suite, render A/B
# against the previous build (libgskyhip_prev.so), alternating, tile classes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06pair}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
for rep in 1 2 3; do
  for lib in prev default; do
    GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 200 python -u tools/ab_render.py --config c2 --reps 30 --label ${T}_$lib >> gpurun_out/${T}_render.jsonl 2>/dev/null
    stop $? render_${lib}
  done
done
timeout -k 10 400 python -u tools/c2_classes.py > gpurun_out/${T}_classes.jsonl 2>/dev/null
stop $? classes
tail -1 gpurun_out/${T}_full.txt gpurun_out/${T}_parity.txt; cat gpurun_out/${T}_render.jsonl gpurun_out/${T}_classes.jsonl
