#!/bin/bash
# r04k: where render_nn_kernel's time goes on C2 (A/B build): full, no
# gathers (1), no stores (2), Scale without the palette lookup (3), neither
# Scale nor palette (4); bilinear fp64 fold inline again (C3 vs round 3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for i in 1 2; do
  for m in 0 1 2 3 4; do
    GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "mode$m" >> gpurun_out/ab.jsonl
    stop $? "ab_mode$m"
  done
  for lib in default r03; do
    GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_c3.py --reps 10 --label "c3_$lib" >> gpurun_out/ab.jsonl
    stop $? "ab_c3_$lib"
  done
done
timeout -k 10 300 python3 tools/ab_c3.py --reps 3 --oracle --label c3_new >> gpurun_out/ab.jsonl
stop $? oracle_c3
cat gpurun_out/ab.jsonl
