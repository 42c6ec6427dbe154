#!/bin/bash
# r06: C3 separable-row tap reuse -- full-canvas test on the product, render
# timings and canvas hashes of the A/B build's variants (GSKYHIP_BIL_REUSE
# 0 = round 5, 6 / 8 = reuse at 6 / 8 waves per SIMD) beside the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06t}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_parity.py -k "c3 or bil or lds" -m gpu > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/${T}_tests.txt; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${T}_c3.jsonl
for rep in 1 2; do
  for v in product 0 6 8; do
    if [ $v = product ]; then unset GSKYHIP_LIB GSKYHIP_BIL_REUSE; else export GSKYHIP_LIB=ab GSKYHIP_BIL_REUSE=$v; fi
    timeout -k 10 200 python -u tools/ab_c3.py --reps 10 --label $T-$v >> gpurun_out/${T}_c3.jsonl 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "c3 $v rc=$rc"; exit $rc; }
  done
done
unset GSKYHIP_LIB GSKYHIP_BIL_REUSE
cat gpurun_out/${T}_c3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
  python3 tools/ab_c3.py --reps 10 > gpurun_out/${T}_prof.txt 2>&1
rc=$?; echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats_c3.csv
cut -d, -f1-4 gpurun_out/${T}_kernel_stats_c3.csv | cut -c1-140 | head -6
