#!/bin/bash
# r06z (a): closing run, part 1, on the final library build: oracle-free warp
# checks, the GPU suite, smoke(), PMC passes of the band kernels of C2
# (render_nn_kernel), C3 (render_bil_kernel) and C5 (render_nn_kernel, masked
# stacks), summarised into gpurun_out/ (committed to profiles/ so the bench
# line carries `traffic`).  Part 2 (gpu_r06z_b.sh): bench + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_warp_exact.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r06z_warp_exact.txt 2>&1
rc=$?; grep -E "vs exact|PASSED|FAILED" gpurun_out/r06z_warp_exact.txt | head; stop $rc warp_exact
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread --ignore=tests/test_warp_exact.py > gpurun_out/r06z_gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r06z_gpu_tests.txt; stop $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06z_smoke.txt 2>&1
rc=$?; tail -1 gpurun_out/r06z_smoke.txt; stop $rc smoke
PMC_OUT=gpurun_out/pmc_c2 PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" bash tools/pmc.sh
stop $? pmc_c2
python3 tools/pmc_summary.py gpurun_out/pmc_c2 "render_nn_kernel<" gpurun_out/pmc_render_c2.json > /dev/null
PMC_OUT=gpurun_out/pmc_c3 PMC_CMD="python3 tools/ab_c3.py --reps 3" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;MeanOccupancyPerCU" \
  bash tools/pmc.sh
stop $? pmc_c3
python3 tools/pmc_summary.py gpurun_out/pmc_c3 "render_bil" gpurun_out/pmc_bil_c3.json > /dev/null
PMC_OUT=gpurun_out/pmc_c5 PMC_CMD="python3 tools/ab_render.py --config c5 --reps 3" bash tools/pmc.sh
stop $? pmc_c5
python3 tools/pmc_summary.py gpurun_out/pmc_c5 "render_nn_kernel<" gpurun_out/pmc_render_c5.json > /dev/null
grep -h "lib_sha16\|hbm_bytes_per_launch" gpurun_out/pmc_render_c2.json gpurun_out/pmc_bil_c3.json gpurun_out/pmc_render_c5.json
