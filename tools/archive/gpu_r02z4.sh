#!/bin/bash
# r02z4: strided lane pixels in render_nn_kernel (GSKYHIP_NN_STRIDE=1): GPU suite with it on, C2/C5 A/B.
mkdir -p gpurun_out
GSKYHIP_NN_STRIDE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  GSKYHIP_NN_STRIDE=$v timeout -k 10 300 python -u bench.py --only c2,c5 --no-cpu --steps 20 --warmup 5 >> gpurun_out/bench_stride$v.jsonl 2>> gpurun_out/bench.err
  rc=$?; echo "bench stride=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
GSKYHIP_NN_STRIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --only c2 --no-cpu --steps 20 --warmup 5 > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "prof c2 rc=$rc"; exit $rc
