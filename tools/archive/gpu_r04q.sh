#!/bin/bash
# r04q: decile select occupancy (A/B: LDS per workgroup 12 / 20 / 36 KB ->
# key cache 1k / 3k / 7k keys) on C4 deciles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for kb in 36 20 12; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_LDS_KB=$kb timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_$kb.json 2> gpurun_out/c4_$kb.err
  stop $? c4_$kb
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_$kb.json')); c=d.get('configs',{}).get('C4',d)
print('lds_kb=$kb', c['deciles']['ms_per_step'], c['deciles']['roofline']['kernel_ms'])"
done
for th in 16 1; do
  GSKYHIP_DRILL_THREADS=$th timeout -k 10 200 python3 tools/c4_desc.py --label "th$th" >> gpurun_out/c4_desc.jsonl
  stop $? c4_desc_$th
done
cat gpurun_out/c4_desc.jsonl
