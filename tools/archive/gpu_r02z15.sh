#!/bin/bash
# r02z15: HIP-graph replay of a render (RenderGraph, set_tiles): parity tests + C1 latency eager vs graph.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py -m gpu -v -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_graph.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -5 gpurun_out/gpu_tests_graph.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --only c1 > gpurun_out/bench_c1_graph.json 2> gpurun_out/bench.err
rc=$?; echo "bench c1 rc=$rc"; cat gpurun_out/bench_c1_graph.json | cut -c1-200; exit $rc
