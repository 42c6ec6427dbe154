#!/bin/bash
# r02h: full GPU suite (separable planning, linear item order), A/B, plan stats, PMC of the NN kernel.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_render.py --config c5 > gpurun_out/ab_c5.jsonl 2>> gpurun_out/ab.err
rc=$?; echo "ab5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/plan_stats.py > gpurun_out/plan_stats.jsonl 2> gpurun_out/plan_stats.err
rc=$?; echo "plan_stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_OUT=gpurun_out/pmc_nn bash tools/pmc.sh
rc=$?; echo "pmc rc=$rc"; exit $rc
