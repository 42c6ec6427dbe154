#!/bin/bash
# r05f: warp_job_kernel with 4 pixels per thread (GSKYHIP_SVC_PX=4) vs 1 --
# the whole GPU suite under PX=4, then the service leg under both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_SVC_PX=4 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05f_tests_px4.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests_px4.log; stop $rc tests_px4
for px in 1 4 1 4; do
  GSKYHIP_SVC_PX=$px timeout -k 10 300 python3 bench.py --only svc --no-cpu > gpurun_out/r05f_svc_px$px.json 2> gpurun_out/r05f_svc_px$px.err
  stop $? svc_px$px
  python3 -c "
import json; c=json.load(open('gpurun_out/r05f_svc_px$px.json'))
s=c.get('service') or c.get('configs',{}).get('service') or c
print('px=$px', json.dumps(s)[:1500])" | tee -a gpurun_out/r05f_svc.txt
done
