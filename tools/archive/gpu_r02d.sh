#!/bin/bash
# r02d: parity suite, C2 kernel A/B, C3 + C5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --only c3,c5 --no-cpu --steps 10 --warmup 2 > gpurun_out/bench_c3c5.json 2> gpurun_out/bench.err
echo "bench rc=$?"
