#!/bin/bash
# r06: C5 masked fold with the mask rows' sameness tested in the prefetch
# lanes (75 VGPRs: 6 waves / SIMD) -- masked parity tests incl. full C5, then
# render timings (product; A/B build at 8 waves / SIMD) against the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06x}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c5_full or render_c5" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${T}_c5.jsonl
for rep in 1 2; do
  for v in product 7 8; do
    if [ $v = product ]; then unset GSKYHIP_LIB GSKYHIP_NN_MASK_WPE; else export GSKYHIP_LIB=ab GSKYHIP_NN_MASK_WPE=$v; fi
    O=""; [ $rep = 1 ] && O="--oracle"
    timeout -k 10 300 python -u tools/ab_render.py --config c5 --reps 20 --label $T-$v $O >> gpurun_out/${T}_c5.jsonl 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "c5 $v rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/${T}_c5.jsonl
