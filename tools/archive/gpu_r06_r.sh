#!/bin/bash
# r06: GPU suite on the wave-per-segment deciles select + small-batch complex
# tiles in the band kernel; C4 deciles and C1 timings against the A/B build's
# round-5 paths (GSKYHIP_DEC_WAVE=0 / GSKYHIP_NN_GEN=0); plan_small phase
# stamps; kernel stats of C4 and C1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06r}
stop() { echo "[$2] rc=$1"; [ "$1" -ne 0 ] && exit "$1"; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/${T}_gpu_tests.txt; stop $rc suite
: > gpurun_out/${T}_ab.txt
for rep in 1 2; do
  for v in product ab; do
    if [ $v = ab ]; then export GSKYHIP_LIB=ab GSKYHIP_DEC_WAVE=0 GSKYHIP_NN_GEN=0; else unset GSKYHIP_LIB GSKYHIP_DEC_WAVE GSKYHIP_NN_GEN; fi
    timeout -k 10 300 python -u bench.py --only c4,c1 --no-cpu --steps 10 --c1-reps 500 > gpurun_out/${T}_b_${v}_$rep.json 2>gpurun_out/${T}_b_err.txt
    stop $? bench_$v
    python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_b_${v}_$rep.json').read().strip().splitlines()[-1]); c=d['configs']
dd=c['C4'].get('deciles',{}); c1=c['C1']
print('$v', 'dec_ms', dd.get('ms_per_step'), 'dec_kernel', json.dumps(dd.get('roofline'))[:200], 'c1_p50', c1['p50_tile_ms'], 'c1_p99', c1['p99_tile_ms'])" >> gpurun_out/${T}_ab.txt
  done
done
unset GSKYHIP_DEC_WAVE GSKYHIP_NN_GEN
cat gpurun_out/${T}_ab.txt
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
  cut -d, -f1-4 gpurun_out/${T}_kernel_stats_$c.csv | cut -c1-150 | head -8
done
