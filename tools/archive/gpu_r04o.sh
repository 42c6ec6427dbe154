#!/bin/bash
# r04o: deciles selected straight from the stack (GSKYHIP_DEC_DIRECT=1, A/B
# build: no transposed copy, XCD-grouped workgroups) -- the decile parity
# tests and the C4 deciles timing against the transpose path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
GSKYHIP_LIB=ab GSKYHIP_DEC_DIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -k "decile" -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dec_tests.log; stop $rc dec_tests
for d in 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_DEC_DIRECT=$d timeout -k 10 300 python3 bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_d$d.json 2> gpurun_out/c4_d$d.err
  stop $? c4_d$d
  python3 -c "
import json; d=json.load(open('gpurun_out/c4_d$d.json')); c=d.get('configs',{}).get('C4',d)
print('direct=$d', json.dumps(c.get('deciles')))"
done
