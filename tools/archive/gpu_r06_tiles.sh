#!/bin/bash
# r06 tiles: the merge planner's per-tile passes in registers (plan_tiles_kernel
# 70 us on C5's 128-pair tiles) -- the whole GPU suite, then bench C5 / C1 on
# the pre-span build (GSKYHIP_LIB=base), spans + register tile passes
# (GSKYHIP_LIB=t) and this one (+ spans in the masked rows); render A/B, and kernel stats of C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06tiles}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread --ignore=tests/test_warp_exact.py > gpurun_out/${T}_gpu_tests.txt 2>&1
stop $? gpu_tests
for rep in 1 2; do
  for lib in base t default; do
    for c in c5 c2; do
      GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 200 python -u tools/ab_render.py --config $c --reps 30 --label ${T}_$lib >> gpurun_out/${T}_render.jsonl 2>/dev/null
      stop $? render_${lib}_$c
    done
  done
done
for lib in base t default; do
  for c in c5 c1; do
    GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 300 python -u bench.py --only $c --no-cpu --steps 20 --warmup 3 --png-tiles 0 > gpurun_out/${T}_bench_${c}_$lib.json 2>/dev/null
    stop $? bench_${c}_$lib
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c5 -o run --output-format csv -- \
  python3 bench.py --only c5 --no-cpu --steps 5 --warmup 2 --png-tiles 0 > gpurun_out/${T}_prof_c5.txt 2>&1
stop $? prof_c5
tail -2 gpurun_out/${T}_gpu_tests.txt; cat gpurun_out/${T}_render.jsonl
for lib in base t default; do python3 -c "
import json
for c in ['c5','c1']:
    d=json.load(open('gpurun_out/${T}_bench_'+c+'_$lib.json')); x=d['configs'][c.upper()] if 'configs' in d else d
    print('$lib', c, json.dumps({k: x.get(k) for k in ('ms_per_step','step_ms','p50_tile_ms','p99_tile_ms')}), json.dumps({k: x.get('roofline',{}).get(k) for k in ('kernel_ms','plan_ms','frac')}))"; done
