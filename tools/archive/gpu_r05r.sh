#!/bin/bash
# r05r: service leg planning on the A/B daemon -- the one-workgroup small
# planner (batches of <= 4 windows) vs the multi-launch planner for every batch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_DAEMON=$PWD/gsky_amd/gskyhipd_ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 1 0 1 0; do
  GSKYHIP_PLAN_SMALL=$m timeout -k 10 300 python3 bench.py --only svc --no-cpu > gpurun_out/r05r_svc_$m.json 2>> gpurun_out/r05r_svc.err
  stop $? svc_$m
  python3 -c "
import json; s=json.load(open('gpurun_out/r05r_svc_$m.json'))['configs']['service']
print('plan_small=$m', {k: (v['requests_per_s'], v['p50_ms'], v['daemon_batch_phases_ms_mean']['gpu_wait']) for k, v in s.items() if k.startswith('workers')})" | tee -a gpurun_out/r05r_svc.txt
done
