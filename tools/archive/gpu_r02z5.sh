#!/bin/bash
# r02z5/z7/z10: lane-pixel layout A/B (strided, LDS-collected output rows, ...) on C2 and C5 against the oracle.
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_render.py --stride --config c2 --oracle --reps 20 > gpurun_out/ab_c2_stride.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab c2 rc=$rc"; cat gpurun_out/ab_c2_stride.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_render.py --stride --config c5 --oracle --reps 20 > gpurun_out/ab_c5_stride.jsonl 2>> gpurun_out/ab.err
rc=$?; echo "ab c5 rc=$rc"; cat gpurun_out/ab_c5_stride.jsonl; exit $rc
