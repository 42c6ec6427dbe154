#!/bin/bash
# r02z6: strided lane pixels in render_bil_kernel (GSKYHIP_BIL_KERNEL=5: 4x1, 6: 4x2): C3 parity + bench A/B.
mkdir -p gpurun_out
for k in 5 6; do
  GSKYHIP_BIL_KERNEL=$k timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf -k "c3 or bil or coverage or wcs" > gpurun_out/gpu_tests_bil$k.log 2>&1
  rc=$?; echo "tests bil=$k rc=$rc"; tail -2 gpurun_out/gpu_tests_bil$k.log; [ $rc -ne 0 ] && exit $rc
done
for k in 1 5 6 1 5 6; do
  GSKYHIP_BIL_KERNEL=$k timeout -k 10 300 python -u bench.py --only c3 --no-cpu --steps 20 --warmup 5 >> gpurun_out/bench_c3_bil$k.jsonl 2>> gpurun_out/bench.err
  rc=$?; echo "bench c3 bil=$k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
