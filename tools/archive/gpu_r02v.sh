#!/bin/bash
# r02v: NN gen-3 with 16-B source-row loads: A/B on C2 (with oracle diff) and C5.
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_render.py --oracle > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_render.py --config c5 --oracle > gpurun_out/ab_c5.jsonl 2>> gpurun_out/ab.err
rc=$?; echo "ab5 rc=$rc"; exit $rc
