#!/bin/bash
# r05h: C2 render_nn_kernel bound probes (A/B build): product body (0), the
# lower-bound body with near-free index math (8), no gathers (1), no stores (2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 8 1 2 0 8 1 2; do
  GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "ab_mode=$m" >> gpurun_out/r05h_c2_bound.jsonl 2> gpurun_out/r05h_c2_bound.err
  stop $? c2_$m
done
cat gpurun_out/r05h_c2_bound.jsonl
