#!/bin/bash
# r03qr: (r03q + r03r in one call) the bench line on the final build (C2 and C3 rooflines now carry the
# PMC traffic of this build; C3's roofline times the band kernel alone); A/B of
# the two-entry straight-line fold (GSKYHIP_NN_U2) on C2; the A/B variant tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
for v in 0 1 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_NN_U2=$v timeout -k 10 300 python -u tools/ab_render.py --config c2 --reps 30 --oracle \
    --label "u2_$v" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_c2_u2_$v"
done
cat gpurun_out/ab.jsonl
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/variants.log 2>&1
rc=$?; tail -3 gpurun_out/variants.log; stop $rc variants
