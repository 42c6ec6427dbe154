#!/bin/bash
# r05g: warp_job_kernel packed stores (default PX=4) -- the dtype/ragged
# drop-in tests under PX=1/4/8, the whole GPU suite at the default, then the
# service leg at PX=4 vs 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for px in 1 8; do
  GSKYHIP_SVC_PX=$px timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "warp_operation_fast" -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g_dt_px$px.log 2>&1
  rc=$?; tail -2 gpurun_out/r05g_dt_px$px.log; stop $rc dt_px$px
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05g_tests.log; stop $rc tests
for px in 4 8 4 8; do
  GSKYHIP_SVC_PX=$px timeout -k 10 300 python3 bench.py --only svc --no-cpu > gpurun_out/r05g_svc_px$px.json 2> gpurun_out/r05g_svc_px$px.err
  stop $? svc_px$px
  python3 -c "
import json; c=json.load(open('gpurun_out/r05g_svc_px$px.json'))
s=c.get('service') or c.get('configs',{}).get('service') or c
print('px=$px', {k: (v['requests_per_s'], v['p50_ms'], v['daemon_batch_phases_ms_mean']['gpu_wait']) for k, v in s.items() if k.startswith('workers')})" | tee -a gpurun_out/r05g_svc.txt
done
# C2 single-entry row loop: split on cover && full (default) vs one merged loop
# (GSKYHIP_AB_MODE=7, round 4), A/B build, alternating
for m in 0 7 0 7; do
  GSKYHIP_LIB=ab GSKYHIP_AB_MODE=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "ab_mode=$m" >> gpurun_out/r05g_ab_c2_cf.jsonl 2> gpurun_out/r05g_ab_c2_cf.err
  stop $? ab_c2_$m
done
GSKYHIP_LIB=ab timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "split, oracle check" >> gpurun_out/r05g_ab_c2_cf.jsonl 2>> gpurun_out/r05g_ab_c2_cf.err
stop $? ab_c2_oracle
cat gpurun_out/r05g_ab_c2_cf.jsonl
