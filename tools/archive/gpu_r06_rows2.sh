#!/bin/bash
# r06: planner -- plan_rows split into a separable-only kernel (84 VGPRs) and a full-transform one
# full C2/C3/C5 identity, the parity
# suite, then bench C5 / C2 on the previous build (libgskyhip_prev.so) and
# this one, alternating, + C5 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r06rows2}
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full.py -k "c5 or c2_full or c3" -m gpu > gpurun_out/${T}_full.txt 2>&1
stop $? full
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_warp_exact.py -m gpu > gpurun_out/${T}_parity.txt 2>&1
stop $? parity
for rep in 1 2; do
  for lib in prev default; do
    for c in c5 c2; do
      GSKYHIP_LIB=$([ $lib = default ] && echo "" || echo $lib) timeout -k 10 300 python -u bench.py --only $c --no-cpu --steps 20 --warmup 3 --png-tiles 0 > gpurun_out/${T}_bench_${c}_${lib}_$rep.json 2>/dev/null
      stop $? bench_${c}_${lib}
      python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench_${c}_${lib}_$rep.json')); x=d['configs']['${c}'.upper()] if '${c}' != 'c2' else d
print('$lib', '$c', x['ms_per_step'], x['step_ms'], x['roofline']['kernel_ms'], x['roofline']['plan_ms'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run --output-format csv -- \
  python3 bench.py --only c2 --no-cpu --steps 5 --warmup 2 --png-tiles 0 > gpurun_out/${T}_prof_c2.txt 2>&1
stop $? prof_c2
tail -1 gpurun_out/${T}_full.txt gpurun_out/${T}_parity.txt
