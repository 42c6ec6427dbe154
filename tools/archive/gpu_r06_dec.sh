#!/bin/bash
# r06: wave-per-segment deciles select -- parity tests, then C4 deciles timing
# (product vs the A/B build's round-5 workgroup select), then kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06q}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "decile" > gpurun_out/${T}_dec_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_dec_tests.txt; echo "[tests] rc=$rc"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  unset GSKYHIP_LIB GSKYHIP_DEC_WAVE
  timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 10 > gpurun_out/${T}_c4_wave_$rep.json 2>gpurun_out/${T}_c4_err.txt
  rc=$?; [ $rc -ne 0 ] && { echo "bench wave rc=$rc"; tail gpurun_out/${T}_c4_err.txt; exit $rc; }
  export GSKYHIP_LIB=ab GSKYHIP_DEC_WAVE=0
  timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 10 > gpurun_out/${T}_c4_wg_$rep.json 2>>gpurun_out/${T}_c4_err.txt
  rc=$?; [ $rc -ne 0 ] && { echo "bench wg rc=$rc"; exit $rc; }
done
unset GSKYHIP_LIB GSKYHIP_DEC_WAVE
for f in gpurun_out/${T}_c4_w*.json; do echo "$f"; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['configs']['C4']; print(json.dumps(c.get('deciles'))[:600])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --only c4 --no-cpu --steps 5 --warmup 2 > gpurun_out/${T}_prof.txt 2>&1
rc=$?; echo "[prof] rc=$rc"; f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/${T}_kernel_stats_c4.csv && cut -c1-160 gpurun_out/${T}_kernel_stats_c4.csv | head -8
exit $rc
