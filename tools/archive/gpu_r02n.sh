#!/bin/bash
# r02n: latency PMC of the gen-2 (4x2) and gen-3 (4x1) NN kernels.
mkdir -p gpurun_out
PMC_OUT=gpurun_out/lat_nn2 PMC_CMD="python3 tools/ab_render.py --variant nn_4x2 --reps 3" bash tools/pmc_lat.sh
rc=$?; echo "lat nn2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
PMC_OUT=gpurun_out/lat_nn3 PMC_CMD="python3 tools/ab_render.py --variant nn3_4x1 --reps 3" bash tools/pmc_lat.sh
rc=$?; echo "lat nn3 rc=$rc"; exit $rc
