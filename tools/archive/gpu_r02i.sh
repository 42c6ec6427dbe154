#!/bin/bash
# r02i: full GPU suite (wave-parallel merge planner), plan stats.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/plan_stats.py > gpurun_out/plan_stats.jsonl 2> gpurun_out/plan_stats.err
rc=$?; echo "plan_stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_render.py --probes > gpurun_out/ab_probes.jsonl 2> gpurun_out/ab.err
rc=$?; echo "probes rc=$rc"; exit $rc
