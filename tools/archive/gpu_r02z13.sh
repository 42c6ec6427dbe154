#!/bin/bash
# r02z13: parity of every band-kernel A/B variant (tests/test_gpu_variants.py).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -m gpu -v -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_variants.log 2>&1
rc=$?; echo "variants rc=$rc"; tail -22 gpurun_out/gpu_tests_variants.log; exit $rc
