#!/bin/bash
# r04u: NN band kernel item order -- every block of a tile on one XCD, tiles
# dealt round-robin over the XCDs (GSKYHIP_NN_XCD=1, A/B build) vs linear, C2
# and C5, oracle identity; FETCH_SIZE of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_NN_XCD=1 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 3 --oracle --label xcd1 >> gpurun_out/ab.jsonl
stop $? oracle_xcd
for i in 1 2; do
  for x in 0 1; do
    for c in c2 c5; do
      GSKYHIP_LIB=ab GSKYHIP_NN_XCD=$x timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label "xcd$x" >> gpurun_out/ab.jsonl
      stop $? "ab_xcd${x}_$c"
    done
  done
done
cat gpurun_out/ab.jsonl
for x in 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_NN_XCD=$x PMC_OUT=gpurun_out/pmc_xcd$x PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" \
    PMC_GROUPS="FETCH_SIZE" bash tools/pmc.sh
  stop $? pmc_xcd$x
done
