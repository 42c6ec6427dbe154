#!/bin/bash
# r02l: NN gen-3 occupancy variants A/B on C2 + PMC passes of gen 2 (4x2) and gen 3 (4x1).
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_render.py > gpurun_out/ab_c2.jsonl 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_OUT=gpurun_out/pmc_nn2 PMC_CMD="python3 tools/ab_render.py --variant nn_4x2 --reps 3" bash tools/pmc.sh
rc=$?; echo "pmc nn2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_OUT=gpurun_out/pmc_nn3 PMC_CMD="python3 tools/ab_render.py --variant nn3_4x1 --reps 3" bash tools/pmc.sh
rc=$?; echo "pmc nn3 rc=$rc"; exit $rc
