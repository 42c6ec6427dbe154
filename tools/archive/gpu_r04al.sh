#!/bin/bash
# r04al: C5 / C2 / C1 one-tile request latency with the one-workgroup small-batch planner on / off (A/B build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for sm in 1 0 1 0; do
  for c in c5 c1; do
    GSKYHIP_LIB=ab GSKYHIP_PLAN_SMALL=$sm timeout -k 10 300 python3 bench.py --only $c --no-cpu --steps 3 --warmup 1 --png-tiles 0 > gpurun_out/${c}_$sm.json 2> gpurun_out/${c}_$sm.err
    stop $? ${c}_$sm
    python3 -c "
import json; d=json.load(open('gpurun_out/${c}_$sm.json')); c=d.get('configs',{}).get('${c}'.upper(),d)
print('$c small=$sm p50', c.get('p50_tile_ms'), 'p99', c.get('p99_tile_ms'), 'ms_per_step', c.get('ms_per_step'))" | tee -a gpurun_out/ab.txt
  done
done
