#!/bin/bash
# r02m: NN gen-3 after the bitwise fold (no sunk gathers): A/B on C2.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; exit $rc
