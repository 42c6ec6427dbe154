#!/bin/bash
# r03d: A/B of the producer / store-wave NN kernel (render_nn_ws_kernel, 3 or 7
# producer waves per store wave) against render_nn_kernel on C2, each checked
# against the oracle; then the r03c steps (GPU suite, rocprofv3 stats of C4 /
# C3, FETCH/WRITE calibration, bench line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
for v in "0 0" "3 0" "7 0" "3 1" "7 1" "0 0" "3 0"; do
  set -- $v
  GSKYHIP_LIB=ab GSKYHIP_NN_WS=$1 GSKYHIP_NN_XCD=$2 timeout -k 10 300 python -u tools/ab_render.py --config c2 \
    --reps 30 --oracle --label "ws$1 xcd$2" >> gpurun_out/ab_ws.jsonl 2>> gpurun_out/ab.err
  stop $? "ab_ws$1_xcd$2"
done
cat gpurun_out/ab_ws.jsonl
bash tools/gpu_r03c.sh
