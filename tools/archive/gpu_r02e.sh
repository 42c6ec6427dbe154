#!/bin/bash
# r02e: C3 typed-vs-generic diagnostic, then the GPU parity suite.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_c3.py > gpurun_out/diag_c3.log 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc
