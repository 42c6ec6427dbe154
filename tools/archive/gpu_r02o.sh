#!/bin/bash
# r02o: GPU suite (express path, pipelined batch), C2 bench over chunk counts, A/B of the NN kernels.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for c in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --only c2 --no-cpu --steps 20 --warmup 5 --c2-chunks $c > gpurun_out/bench_c2_k$c.json 2> gpurun_out/bench_k$c.err
  rc=$?; echo "bench chunks=$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; exit $rc
