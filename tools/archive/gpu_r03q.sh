#!/bin/bash
# r03q: the bench line on the final build (C2 and C3 rooflines now carry the
# PMC traffic of this build; C3's roofline times the band kernel alone).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "[bench] rc=$?"
