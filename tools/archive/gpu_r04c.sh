#!/bin/bash
# r04c: issue rate of the NN kernel's candidate load shapes (tools/calib/gather_rate.hip)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/calib/gather_rate 5 > gpurun_out/gather_rate.json
echo "[gather_rate] rc=$?"
cat gpurun_out/gather_rate.json
timeout -k 10 300 python3 bench.py --only c4 --no-cpu --no-deciles --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err
echo "[c4] rc=$?"
python3 -c "import json; d=json.load(open('gpurun_out/c4.json')); c=d.get('configs',{}).get('C4',d); print('descriptors_ms', c.get('descriptors_ms'))"
