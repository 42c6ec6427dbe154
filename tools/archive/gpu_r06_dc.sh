#!/bin/bash
# r06: deciles with the mean pass's loads one chunk ahead of its band-row
# stores -- decile parity tests, then C4 deciles product vs the A/B build's
# round-5 walk (GSKYHIP_DRILL_EMIT_PIPE=0), kernel stats of the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06dc}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decile or c4_full" > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${T}_dec.txt
for rep in 1 2; do
  for v in product 0; do
    if [ $v = product ]; then unset GSKYHIP_LIB GSKYHIP_DRILL_EMIT_PIPE; else export GSKYHIP_LIB=ab GSKYHIP_DRILL_EMIT_PIPE=$v; fi
    timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 10 > gpurun_out/${T}_c4_$v.json 2>gpurun_out/${T}_err.txt
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -3 gpurun_out/${T}_err.txt; exit $rc; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_c4_$v.json').read().strip().splitlines()[-1]); dd=d['configs']['C4'].get('deciles',{})
print('$v dec_ms', dd.get('ms_per_step'), 'kernel_ms', dd.get('roofline',{}).get('kernel_ms'))" >> gpurun_out/${T}_dec.txt
  done
done
unset GSKYHIP_LIB GSKYHIP_DRILL_EMIT_PIPE
cat gpurun_out/${T}_dec.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 5 --warmup 2 > gpurun_out/${T}_prof.txt 2>&1
rc=$?; echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats_c4.csv
python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/${T}_kernel_stats_c4.csv")):
    if "gsky" in r["Name"] and float(r["AverageNs"]) > 50000:
        print("%-70s %6s %9.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"])/1e3))
PY
