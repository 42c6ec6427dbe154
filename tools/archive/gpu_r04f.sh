#!/bin/bash
# r04f: what bounds render_nn_kernel on C2 -- the same kernel with its
# gathers skipped (GSKYHIP_AB_MODE=1: store-only) and with its stores skipped
# (2: gather-only), A/B build; kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for i in 1 2; do
  for m in 0 1 2; do
    GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "mode$m" >> gpurun_out/ab.jsonl
    stop $? "ab_mode$m"
  done
done
cat gpurun_out/ab.jsonl
for m in 0 1 2; do
  GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m$m -o run --output-format csv -- \
    python3 tools/ab_render.py --config c2 --reps 5 > gpurun_out/prof_m$m.log 2>&1
  stop $? prof_m$m
done
timeout -k 10 400 python3 bench.py --only svc --no-cpu --steps 3 --warmup 1 > gpurun_out/svc.json 2> gpurun_out/svc.err
stop $? svc
cut -c1-2000 gpurun_out/svc.json
for th in 16 8 4 1; do
  GSKYHIP_DRILL_THREADS=$th timeout -k 10 200 python3 tools/c4_desc.py --label "th$th" >> gpurun_out/c4_desc.jsonl
  stop $? c4_desc_$th
done
cat gpurun_out/c4_desc.jsonl
