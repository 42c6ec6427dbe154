#!/bin/bash
# r06: render timings (phase 2) of the product library against
# gsky_amd/libgskyhip_ab.so (GSKYHIP_LIB=ab), alternating, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${1:-r06t}
CFGS=${2:-"c5 c2"}
: > gpurun_out/${T}_render.jsonl
for rep in 1 2; do
for lib in default ab; do
  for c in $CFGS; do
    if [ $lib = ab ]; then export GSKYHIP_LIB=ab; else unset GSKYHIP_LIB; fi
    timeout -k 10 200 python -u tools/ab_render.py --config $c --reps 20 --label $T-$lib >> gpurun_out/${T}_render.jsonl 2>/dev/null
    rc=$?; if [ $rc -ne 0 ]; then echo "render $lib $c rc=$rc"; exit $rc; fi
  done
done
done
cat gpurun_out/${T}_render.jsonl
