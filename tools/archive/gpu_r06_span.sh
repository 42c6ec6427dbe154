#!/bin/bash
# r06 span: rows leaving the band folded over their in-band span (multi-entry
# C2 tiles, C5 entries whose span misses the block): full C2 / C5 identity,
# the parity suite, then render-phase A/B against the previous build
# (gsky_amd/libgskyhip_base.so, GSKYHIP_LIB=base), alternating, + bench C2/C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06span}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full or c3" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
for rep in 1 2; do
  for lib in base default; do
    for c in c2 c5; do
      GSKYHIP_LIB=$([ $lib = base ] && echo base || echo "") timeout -k 10 200 python -u tools/ab_render.py --config $c --reps 30 --label $T >> gpurun_out/${T}_render.jsonl 2>/dev/null
      stop $? render_${lib}_$c
    done
  done
done
for lib in base default; do
  GSKYHIP_LIB=$([ $lib = base ] && echo base || echo "") timeout -k 10 300 python -u bench.py --only c2 --no-cpu --steps 20 --warmup 3 --png-tiles 0 > gpurun_out/${T}_bench_c2_$lib.json 2>/dev/null
  stop $? bench_c2_$lib
done
tail -2 gpurun_out/${T}_full.txt gpurun_out/${T}_parity.txt; cat gpurun_out/${T}_render.jsonl
for lib in base default; do python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench_c2_$lib.json')); print('$lib', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['plan_ms'], d['roofline']['frac'])"; done
