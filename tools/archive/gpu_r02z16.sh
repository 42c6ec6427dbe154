#!/bin/bash
# r02z16: closing check of the round: the whole GPU suite and the default bench (as the driver runs them).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_close.json 2> gpurun_out/bench_close.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_close.json; exit $rc
