#!/bin/bash
# r02z12: render_bil_kernel shapes at 8 waves per SIMD (GSKYHIP_BIL_KERNEL=7: 2x1, 8: 4x1 spilling) vs 5; C3 parity + bench.
# (Both variants lost and were removed after this run; the knob values now fall back to the default.)
mkdir -p gpurun_out
for k in 7 8; do
  GSKYHIP_BIL_KERNEL=$k timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf -k "c3 or bil or coverage or wcs" > gpurun_out/gpu_tests_bil$k.log 2>&1
  rc=$?; echo "tests bil=$k rc=$rc"; tail -1 gpurun_out/gpu_tests_bil$k.log; [ $rc -ne 0 ] && exit $rc
done
for k in 5 7 8 5 7 8; do
  GSKYHIP_BIL_KERNEL=$k timeout -k 10 300 python -u bench.py --only c3 --no-cpu --steps 20 --warmup 5 >> gpurun_out/bench_c3_bil$k.jsonl 2>> gpurun_out/bench.err
  rc=$?; echo "bench c3 bil=$k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
