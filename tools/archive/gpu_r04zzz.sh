#!/bin/bash
# r04zzz (also r04zzzz): validation + closing run on the final library build in one call:
# oracle-free warp checks, the GPU suite, PMC passes of render_nn_kernel (C2) /
# render_bil_kernel (C3) summarised into the box's profiles/ (so the bench line
# carries `traffic`), the bench line, rocprofv3 kernel stats of C1-C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_warp_exact.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/warp_exact.log 2>&1
rc=$?; grep -E "warp vs exact|PASSED|FAILED" gpurun_out/warp_exact.log | head; echo "[warp_exact] rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then stop $rc warp_exact; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread --ignore=tests/test_warp_exact.py > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; stop $rc tests
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c3
python3 tools/pmc_summary.py gpurun_out/pmc_c2 "render_nn_kernel<" profiles/pmc_render_c2.json > gpurun_out/pmc_c2_summary.txt 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_c3 "render_bil" profiles/pmc_bil_c3.json > gpurun_out/pmc_c3_summary.txt 2>&1
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
stop $? bench
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('C2', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('p50_tile_ms'))
for k, c in d.get('configs', {}).items(): print(k, json.dumps(c)[:240])"
for c in c2 c3 c4 c1 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 bench.py --only $c --no-cpu --steps 5 --warmup 2 --c1-reps 200 --png-tiles 0 > gpurun_out/prof_$c.log 2>&1
  stop $? prof_$c
done
