#!/bin/bash
# r04c: issue rate of the NN kernel's candidate load shapes (tools/calib/gather_rate.hip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib/gather_rate 5 > gpurun_out/gather_rate.json
echo "[gather_rate] rc=$?"
cat gpurun_out/gather_rate.json
