#!/bin/bash
# r02g: typed-kernel parity subset first (new NN kernel), then A/B, plan stats, C3 diagnostic.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_render.py --config c5 > gpurun_out/ab_c5.jsonl 2>> gpurun_out/ab.err
rc=$?; echo "ab5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/plan_stats.py c2 c5 > gpurun_out/plan_stats.jsonl 2> gpurun_out/plan_stats.err
rc=$?; echo "plan_stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/diag_c3.py > gpurun_out/diag_c3.log 2>&1
rc=$?; echo "diag rc=$rc"; exit $rc
