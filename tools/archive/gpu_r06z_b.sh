#!/bin/bash
# r06z (b): closing run, part 2: the bench line (python bench.py, N=1, with
# the committed PMC summaries of this build) and rocprofv3 kernel stats of the
# bench commands per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
# part 1's PMC summaries of this build, when run in the same call (bench.py
# reads profiles/ and takes them only when their lib_sha16 is this library's)
for f in pmc_render_c2.json pmc_bil_c3.json pmc_render_c5.json; do
  if [ -f gpurun_out/$f ]; then cp gpurun_out/$f profiles/$f; fi
done
timeout -k 10 900 python -u bench.py > gpurun_out/r06z_bench.json 2> gpurun_out/r06z_bench.err
stop $? bench
python3 -c "
import json; d=json.load(open('gpurun_out/r06z_bench.json'))
print('C2', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('p50_tile_ms'))
for k, c in d.get('configs', {}).items(): print(k, json.dumps(c)[:300])"
for c in c2 c3 c4 c1 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 bench.py --only $c --no-cpu --steps 5 --warmup 2 --c1-reps 200 --png-tiles 0 > gpurun_out/r06z_prof_$c.txt 2>&1
  stop $? prof_$c
done
