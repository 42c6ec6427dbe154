#!/bin/bash
# r02k: third-generation NN band kernel: GPU suite, A/B against the second generation on C2 and C5.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_render.py --config c5 > gpurun_out/ab_c5.jsonl 2>> gpurun_out/ab.err
rc=$?; echo "ab5 rc=$rc"; exit $rc
