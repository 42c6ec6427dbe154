#!/bin/bash
# r04s: GPU deflate of the PNG encoder -- PNG tests (inflate + row identity),
# the C2 PNG leg against host zlib.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/png_tests.log 2>&1
rc=$?; tail -15 gpurun_out/png_tests.log; stop $rc png_tests
timeout -k 10 400 python3 bench.py --only c2 --no-cpu --steps 5 --warmup 2 > gpurun_out/c2.json 2> gpurun_out/c2.err
stop $? c2
python3 -c "
import json; d=json.load(open('gpurun_out/c2.json')); print(json.dumps(d.get('png')))"
