#!/bin/bash
# r02u: GPU suite (band-math), C4 bench with deciles.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --only c4 --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; echo "bench c4 rc=$rc"; exit $rc
