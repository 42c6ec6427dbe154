#!/bin/bash
# r06: C5 masked fold (shared mask index, fill-mode slot skips) + touched bytes:
# full C5 / C2 identity, the parity suite, render timings, bench C5 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06h}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full_identical" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
for c in c5 c2; do
  timeout -k 10 200 python -u tools/ab_render.py --config $c --reps 20 --label $T > gpurun_out/${T}_render_$c.json 2>&1
  stop $? render_$c
done
timeout -k 10 300 python -u bench.py --only c5 --no-cpu --steps 20 --warmup 3 > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err
stop $? bench_c5
tail -2 gpurun_out/${T}_full.txt gpurun_out/${T}_parity.txt; cat gpurun_out/${T}_render_c5.json gpurun_out/${T}_render_c2.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench_c5.json')); c=d['configs']['C5'] if 'configs' in d else d
print(json.dumps(c)[:1500])" 2>&1 | tail -3
