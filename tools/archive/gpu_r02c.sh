#!/bin/bash
# r02c: counter listing, PMC passes of the C2 band kernel, then the full bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1
echo "list rc=$?"
bash tools/pmc.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
