#!/bin/bash
# r02z3: planning prologue + clamped-value Scale LUT in render_nn_kernel; LUT A/B (GSKYHIP_NN_LUT).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --only c2,c5 --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_lut1.json 2> gpurun_out/bench.err
rc=$?; echo "bench lut1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
GSKYHIP_NN_LUT=0 timeout -k 10 300 python -u bench.py --only c2,c5 --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_lut0.json 2>> gpurun_out/bench.err
rc=$?; echo "bench lut0 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --only c2,c5 --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_lut1b.json 2>> gpurun_out/bench.err
rc=$?; echo "bench lut1b rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --only c2 --no-cpu --steps 20 --warmup 5 > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"; exit $rc
