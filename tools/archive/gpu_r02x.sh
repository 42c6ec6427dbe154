#!/bin/bash
# r02x: rows-per-wave A/B of the NN kernel on C2 (oracle diff).
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_render.py --oracle > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; exit $rc
