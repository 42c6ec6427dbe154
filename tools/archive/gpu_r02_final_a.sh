#!/bin/bash
# r02 final measurement, part A (final library build): GPU suite, PMC passes
# of the C2 render kernel and their summary (copied to profiles/ before part B).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
PMC_CMD="python3 tools/ab_render.py --stride --variant nn_4x1_s_w8_mask4x1 --reps 3" PMC_OUT=gpurun_out/pmc bash tools/pmc.sh
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/pmc_summary.py gpurun_out/pmc "render_nn_kernel<" profiles/pmc_render_c2.json > gpurun_out/pmc_render_c2.json
rc=$?; echo "pmc summary rc=$rc"; [ $rc -ne 0 ] && exit $rc
exit 0
