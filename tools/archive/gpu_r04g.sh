#!/bin/bash
# r04g: write bandwidth of the NN output pattern (tools/calib/store_rate.hip);
# the host CPUs this process may run on; the service leg with the daemon's
# warp-batch phase timers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
echo "nproc=$(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
timeout -k 10 120 ./tools/calib/store_rate 5 > gpurun_out/store_rate.json
stop $? store_rate
cat gpurun_out/store_rate.json
timeout -k 10 400 python3 bench.py --only svc --no-cpu --steps 3 --warmup 1 > gpurun_out/svc.json 2> gpurun_out/svc.err
stop $? svc
python3 -c "
import json; d=json.load(open('gpurun_out/svc.json'))['configs']['service']
for k in ('workers_16','workers_64'): print(k, json.dumps(d[k]))"
