#!/bin/bash
# r06: deciles select with a prefix key cache (a segment larger than the LDS
# cache keeps its first keys there; only the rest is streamed twice), at the
# product's 16 KB and at 24 / 32 / 40 KB of LDS per workgroup
# (libgskyhip_s<KB>.so); previous product = libgskyhip_t.so.  Deciles parity
# tests on every build, then C4 deciles timing alternating, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06dp}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for lib in default s24 s32 s40; do
  GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "decile" > gpurun_out/${T}_dec_tests_$lib.txt 2>&1
  stop $? tests_$lib
  tail -1 gpurun_out/${T}_dec_tests_$lib.txt
done
for rep in 1 2; do
  for lib in t default s24 s32 s40; do
    GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 10 > gpurun_out/${T}_c4_${lib}_$rep.json 2>gpurun_out/${T}_c4_err.txt
    stop $? bench_${lib}_$rep
    python3 -c "import json; d=json.loads(open('gpurun_out/${T}_c4_${lib}_$rep.json').read().strip().splitlines()[-1]); c=d['configs']['C4']['deciles']; print('$lib', c['ms_per_step'], c['step_ms'], c['roofline']['kernel_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --only c4 --no-cpu --steps 5 --warmup 2 > gpurun_out/${T}_prof.txt 2>&1
stop $? prof
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats_c4.csv; cut -c1-160 gpurun_out/${T}_kernel_stats_c4.csv | head -6
