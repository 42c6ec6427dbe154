#!/bin/bash
# r02r: GPU suite (extent op), bilinear kernel lane-shape A/B on C3.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2 3 4 0; do
  GSKYHIP_BIL_KERNEL=$k timeout -k 10 200 python -u bench.py --only c3 --no-cpu > gpurun_out/bench_c3_bil$k.json 2>> gpurun_out/bench.err
  rc=$?; echo "bench bil=$k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
