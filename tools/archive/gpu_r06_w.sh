#!/bin/bash
# r06: C5 masked one-row kernel compiled for 5 (product) / 6 / 8 waves per
# SIMD (A/B build, GSKYHIP_NN_MASK_WPE), checked against the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06w}
: > gpurun_out/${T}_c5.jsonl
for rep in 1 2; do
  for v in product 0 6 8; do
    if [ $v = product ]; then unset GSKYHIP_LIB GSKYHIP_NN_MASK_WPE; else export GSKYHIP_LIB=ab GSKYHIP_NN_MASK_WPE=$v; fi
    O=""; [ $rep = 1 ] && O="--oracle"
    timeout -k 10 300 python -u tools/ab_render.py --config c5 --reps 20 --label $T-$v $O >> gpurun_out/${T}_c5.jsonl 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "c5 $v rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/${T}_c5.jsonl
