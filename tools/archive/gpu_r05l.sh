#!/bin/bash
# r05l: tmerc out of line -- GPU suite, then C1 / C2 bench lines (planning)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05l_tests.log; stop $rc tests
timeout -k 10 400 python3 bench.py --only c2,c1,c5 --no-cpu > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err
stop $? bench
python3 -c "
import json; b=json.load(open('gpurun_out/r05l_bench.json'))
print('C2', b['ms_per_step'], b['roofline']['frac'], b.get('plan_ms'), b.get('render_ms'))
c=b['configs']
print('C1', json.dumps(c.get('C1'))[:400])
print('C5', json.dumps(c.get('C5'))[:400])"
