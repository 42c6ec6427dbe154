#!/bin/bash
# r02 final measurement, part B: the default bench (N=1, CPU baseline, traffic
# from profiles/pmc_render_c2.json of this build), rocprofv3 stats of C2 and C3.
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_final.json | cut -c1-600; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --only c2 --no-cpu --steps 20 --warmup 5 > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --only c3 --no-cpu --steps 20 --warmup 5 > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc"; exit $rc
