#!/bin/bash
# r02z17: block entry list in render_nn_kernel (wave 0 lists the entries overlapping the block in LDS): variant parity + C2/C5 A/B.
# (C2 +0.7-2.6 %, C5 -0.5-2.7 %: not kept; the code was removed after the run, the A/B is in profiles/r02z17_*.)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/gpu_tests_variants.log 2>&1
rc=$?; echo "variants rc=$rc"; tail -2 gpurun_out/gpu_tests_variants.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r02z5.sh
