#!/bin/bash
# r04j: fixed-point rows only on the single-entry NN path / off for bilinear
# -- C2, C3, C5 against the round-3 library with the oracle check; service
# leg with the barrier-started load generator; C2 with the PNG encode leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for c in c2 c5; do
  timeout -k 10 200 python3 tools/ab_render.py --config $c --reps 5 --oracle --label new >> gpurun_out/ab.jsonl
  stop $? oracle_$c
done
timeout -k 10 300 python3 tools/ab_c3.py --reps 3 --oracle --label c3_new >> gpurun_out/ab.jsonl
stop $? oracle_c3
for i in 1 2; do
  for lib in default r03; do
    for c in c2 c5; do
      GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label $lib >> gpurun_out/ab.jsonl
      stop $? "ab_${lib}_$c"
    done
    GSKYHIP_LIB=$lib timeout -k 10 120 python3 tools/ab_c3.py --reps 10 --label "c3_$lib" >> gpurun_out/ab.jsonl
    stop $? "ab_c3_$lib"
  done
done
cat gpurun_out/ab.jsonl
timeout -k 10 400 python3 bench.py --only svc,c2 --no-cpu --steps 10 --warmup 3 > gpurun_out/b.json 2> gpurun_out/b.err
stop $? bench
python3 -c "
import json; d=json.load(open('gpurun_out/b.json'))['configs']
s=d['service']
for k in ('workers_16','workers_64'): print(k, json.dumps(s[k]))
print('png', json.dumps(d['C2'].get('png')))
print('c2', d['C2']['ms_per_step'], d['C2']['roofline']['kernel_ms'], d['C2']['p50_tile_ms'])"
