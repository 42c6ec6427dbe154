#!/bin/bash
# r04t: PNG encode phase times (GPU deflate) on the C2 sample.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/png_tests.log 2>&1 && tail -2 gpurun_out/png_tests.log && GSKYHIP_PNG_TRACE=1 timeout -k 10 400 python3 bench.py --only c2 --no-cpu --steps 3 --warmup 1 --png-tiles 1024 > gpurun_out/c2.json 2> gpurun_out/c2.err
stop $? c2
grep "png tiles" gpurun_out/c2.err
python3 -c "
import json; d=json.load(open('gpurun_out/c2.json')); print(json.dumps(d.get('png')))"
