#!/bin/bash
# r06: deciles select with segment keys in VGPRs (kR) -- parity tests, C4
# deciles at kR 0 (round 5) / 16 / 32 / 48 in the A/B build and the product;
# C1 after the one-tile planner schedule (tile plan beside the row records,
# serial extent scan, parallel transformer copy) with its phase stamps;
# kernel stats of C4 and C1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06s}
stop() { echo "[$2] rc=$1"; [ "$1" -ne 0 ] && exit "$1"; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "decile or c4_full or render_c1 or small_batch or graph or warp_windows_c1 or dropin or c5" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; stop $rc tests
: > gpurun_out/${T}_dec.txt
for rep in 1 2; do
  for kr in product 0 16 32 48; do
    if [ $kr = product ]; then unset GSKYHIP_LIB GSKYHIP_DEC_KR; else export GSKYHIP_LIB=ab GSKYHIP_DEC_KR=$kr; fi
    timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 10 > gpurun_out/${T}_c4_$kr.json 2>gpurun_out/${T}_err.txt
    stop $? bench_c4_$kr
    python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c4_$kr.json').read().strip().splitlines()[-1]); dd=d['configs']['C4'].get('deciles',{})
print('kr $kr dec_ms', dd.get('ms_per_step'), 'kernel_ms', dd.get('roofline',{}).get('kernel_ms'))" >> gpurun_out/${T}_dec.txt
  done
done
unset GSKYHIP_LIB GSKYHIP_DEC_KR
cat gpurun_out/${T}_dec.txt
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --only c1 --no-cpu --c1-reps 1000 > gpurun_out/${T}_c1_$rep.json 2>>gpurun_out/${T}_err.txt
  stop $? bench_c1
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c1_$rep.json').read().strip().splitlines()[-1]); c=d['configs']['C1']
print('c1 p50', c['p50_tile_ms'], 'p99', c['p99_tile_ms'], 'graph', c['p50_tile_ms_graph'])"
done
export GSKYHIP_LIB=ab GSKYHIP_PLAN_STAMPS=1
timeout -k 10 200 python -u bench.py --only c1 --no-cpu --c1-reps 200 > /dev/null 2> gpurun_out/${T}_stamps.txt
stop $? stamps
unset GSKYHIP_LIB GSKYHIP_PLAN_STAMPS
grep plan_small_stamps gpurun_out/${T}_stamps.txt | tail -200 | python3 -c "
import sys,re,statistics as S
rows=[list(map(float,re.findall(r'=([0-9.]+)',l))) for l in sys.stdin]
print('stamps median', [round(S.median(c),2) for c in zip(*rows)])"
for c in c4 c1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$c -o run --output-format csv -- \
    python3 bench.py --only $c --no-cpu --steps 5 --warmup 2 --c1-reps 200 > gpurun_out/${T}_prof_$c.txt 2>&1
  stop $? prof_$c
  f=$(find gpurun_out/${T}_prof_$c -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats_$c.csv
done
python3 - <<PY
import csv
for c in ["c4","c1"]:
    for r in csv.DictReader(open("gpurun_out/${T}_kernel_stats_%s.csv" % c)):
        if "gsky" in r["Name"] and float(r["AverageNs"]) > 3000:
            print(c, "%-70s %6s %9.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"])/1e3))
PY
