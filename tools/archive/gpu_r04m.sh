#!/bin/bash
# r04l: dword-wide gathers (GSKYHIP_NN_WIDE, A/B build) vs 16-bit gathers on C2,
# oracle identity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_NN_WIDE=1 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 3 --oracle --label wide1 >> gpurun_out/ab.jsonl
stop $? oracle_wide
for i in 1 2; do
  for pr in 0 1; do
    GSKYHIP_LIB=ab GSKYHIP_NN_WIDE=$pr timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "wide$pr" >> gpurun_out/ab.jsonl
    stop $? "ab_wide$pr"
  done
  GSKYHIP_LIB=ab GSKYHIP_NN_WIDE=1 GSKYHIP_AB_MODE=2 timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "wide1_nostore" >> gpurun_out/ab.jsonl
  stop $? "ab_wide_nostore"
done
cat gpurun_out/ab.jsonl
