#!/bin/bash
# r02z19: rocprofv3 kernel stats of C4 and C5 on the final build, and PMC passes of the C4 drill kernels.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --only c4 --no-cpu --steps 10 --warmup 3 > gpurun_out/prof_c4.log 2>&1
rc=$?; echo "prof c4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --only c5 --no-cpu --steps 10 --warmup 3 > gpurun_out/prof_c5.log 2>&1
rc=$?; echo "prof c5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_CMD="python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1" PMC_OUT=gpurun_out/pmc_c4 bash tools/pmc.sh
rc=$?; echo "pmc c4 rc=$rc"; exit $rc
