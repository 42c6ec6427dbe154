#!/bin/bash
# r05a: the pipelined service (two batches in flight, GPU-written reply
# arenas): service + drop-in parity tests, then the steady-state service leg
# at a few batching windows and with staged windows, then a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_service.py tests/test_gpu_parity.py tests/test_geoloc.py -m gpu -v -x \
  --timeout 300 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05a_tests.log; stop $rc tests
for sep in 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_BIL_SEP=$sep timeout -k 10 300 python3 tools/ab_c3.py --reps 10 --oracle --label sep$sep >> gpurun_out/r05a_ab_c3.jsonl 2> gpurun_out/r05a_ab_c3_$sep.err
  stop $? ab_c3_sep$sep
done
cat gpurun_out/r05a_ab_c3.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -m gpu -v -x -k "c3 or coverage" \
  --timeout 300 --timeout-method thread > gpurun_out/r05a_tests_c3.log 2>&1
rc=$?; tail -3 gpurun_out/r05a_tests_c3.log; stop $rc tests_c3
for w in 0 200; do
  timeout -k 10 300 python -u bench.py --only svc --svc-window-us $w > gpurun_out/r05a_svc_w$w.json 2> gpurun_out/r05a_svc_w$w.err
  stop $? svc_w$w
  python3 -c "
import json; d=json.load(open('gpurun_out/r05a_svc_w$w.json'))['configs']['service']
for k in ('workers_16','workers_64'): print('w$w', k, json.dumps(d.get(k)))
print('cpu', d.get('cpu_baseline'))"
done
GSKYHIP_SVC_DIRECT=0 timeout -k 10 300 python -u bench.py --only svc --no-cpu > gpurun_out/r05a_svc_staged.json 2> gpurun_out/r05a_svc_staged.err
stop $? svc_staged
python3 -c "
import json; d=json.load(open('gpurun_out/r05a_svc_staged.json'))['configs']['service']
for k in ('workers_16','workers_64'): print('staged', k, json.dumps(d.get(k)))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05a_prof_svc -o run --output-format csv -- \
  python3 bench.py --only svc --no-cpu --svc-seconds 1 > gpurun_out/r05a_prof_svc.log 2>&1
stop $? prof_svc
