#!/bin/bash
# r04d: gather issue rate microbenchmark; cooperative-load NN body (A/B build,
# GSKYHIP_NN_COOP=1) vs per-lane gathers on C2 with the oracle check; C4
# descriptors with the fast GeoJSON parser.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 120 ./tools/calib/gather_rate 5 > gpurun_out/gather_rate.json
stop $? gather_rate
cat gpurun_out/gather_rate.json
for i in 1 2; do
  for co in 0 1; do
    GSKYHIP_LIB=ab GSKYHIP_NN_COOP=$co timeout -k 10 120 python3 tools/ab_render.py --config c2 --reps 20 --label "coop$co" >> gpurun_out/ab.jsonl
    stop $? "ab_coop$co"
  done
done
GSKYHIP_LIB=ab GSKYHIP_NN_COOP=1 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 5 --oracle --label coop1 >> gpurun_out/ab.jsonl
stop $? oracle_coop
cat gpurun_out/ab.jsonl
timeout -k 10 300 python3 bench.py --only c4 --no-cpu --no-deciles --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err
stop $? c4
python3 -c "import json; d=json.load(open('gpurun_out/c4.json')); c=d.get('configs',{}).get('C4',d); print('descriptors_ms', c.get('descriptors_ms'))"
