#!/bin/bash
# r02z8: timing probes of the strided NN kernel (1: gathers without traffic, 2: stores only, 3: no stores, 4: no Scale/palette).
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_render.py --probes --config c2 --reps 20 > gpurun_out/ab_c2_probes.jsonl 2> gpurun_out/ab.err
rc=$?; echo "probes rc=$rc"; cat gpurun_out/ab_c2_probes.jsonl; exit $rc
