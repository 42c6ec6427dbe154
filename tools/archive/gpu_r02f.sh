#!/bin/bash
# r02f: plan statistics + typed/generic timings, C3 diagnostic, typed-kernel parity subset.
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/plan_stats.py c2 c5 > gpurun_out/plan_stats.jsonl 2> gpurun_out/plan_stats.err
rc=$?; echo "plan_stats rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 240 python -u tools/diag_c3.py > gpurun_out/diag_c3.log 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -rf -k "lds or c2 or c5 or mixed" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc
