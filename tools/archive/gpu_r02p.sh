#!/bin/bash
# r02p: bisect the C5 mismatch over the NN kernel variants (oracle comparison).
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_render.py --config c5 --oracle --reps 3 > gpurun_out/ab_c5.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab5 rc=$rc"; exit $rc
