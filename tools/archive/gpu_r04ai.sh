#!/bin/bash
# r04ai: service transport -- persistent worker connections, replies sent from the batch result and
# received straight into the caller's buffer: service tests + the bench's service leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_service.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/svc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/svc_tests.log; stop $rc svc_tests
timeout -k 10 400 python3 bench.py --only svc --no-cpu --steps 3 --warmup 1 > gpurun_out/svc.json 2> gpurun_out/svc.err
stop $? svc
python3 -c "
import json; d=json.load(open('gpurun_out/svc.json')); s=d.get('configs',{}).get('service',d)
for k in ('workers_16','workers_64'): print(k, {x: s[k][x] for x in ('requests_per_s','p50_ms','p99_ms','mean_batch','daemon_batch_ms_mean','daemon_resident_ms_mean','errors')})"
