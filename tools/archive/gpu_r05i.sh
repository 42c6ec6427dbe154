#!/bin/bash
# r05i: Transverse Mercator (UTM / MGA) on the GPU -- the new parity and
# exact-transform tests, then the whole GPU suite; C2 bound probes (A/B build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_warp_exact.py -m gpu -k "utm" -v -s -x --timeout 200 --timeout-method thread > gpurun_out/r05i_utm.log 2>&1
rc=$?; grep -E "PASS|FAIL|utm warp" gpurun_out/r05i_utm.log | tail -8; stop $rc utm
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_tests.log; stop $rc tests
for m in 0 8 1 2 0 8 1 2; do
  GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "ab_mode=$m" >> gpurun_out/r05h_c2_bound.jsonl 2> gpurun_out/r05h_c2_bound.err
  stop $? c2_$m
done
cat gpurun_out/r05h_c2_bound.jsonl
