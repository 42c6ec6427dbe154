#!/bin/bash
# r02q: GPU suite (speculative border test in plan_pairs, bilinear band kernel), C2/C3 bench, C3 A/B.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --only c2,c3 --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_c2c3.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
GSKYHIP_BIL_KERNEL=0 timeout -k 10 300 python -u bench.py --only c3 --no-cpu > gpurun_out/bench_c3_old.json 2>> gpurun_out/bench.err
rc=$?; echo "bench old rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --only c3 --no-cpu > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc"; exit $rc
