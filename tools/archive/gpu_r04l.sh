#!/bin/bash
# r04l: two rows' gathers in flight per wave (GSKYHIP_NN_PAIR, A/B build, 6
# waves per SIMD) vs one row on C2, oracle identity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_NN_PAIR=1 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 3 --oracle --label pair1 >> gpurun_out/ab.jsonl
stop $? oracle_pair
for i in 1 2; do
  for pr in 0 1; do
    GSKYHIP_LIB=ab GSKYHIP_NN_PAIR=$pr timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "pair$pr" >> gpurun_out/ab.jsonl
    stop $? "ab_pair$pr"
  done
  GSKYHIP_LIB=ab GSKYHIP_NN_PAIR=1 GSKYHIP_AB_MODE=2 timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "pair1_nostore" >> gpurun_out/ab.jsonl
  stop $? "ab_pair_nostore"
done
cat gpurun_out/ab.jsonl
