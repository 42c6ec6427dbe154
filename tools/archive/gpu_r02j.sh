#!/bin/bash
# r02j: baseline of the restored tree: full bench line, rocprof kernel stats of C2 and C3.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --only c2 --no-cpu --steps 20 --warmup 5 > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --only c3 --no-cpu --c3-steps 3 > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "prof c3 rc=$rc"; exit $rc
