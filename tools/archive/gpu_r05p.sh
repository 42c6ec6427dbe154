#!/bin/bash
# r05p: C1 legs -- eager, graph with the descriptor upload, graph replay
# alone, the upload alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --only c1 --no-cpu > gpurun_out/r05p_c1.json 2> gpurun_out/r05p_c1.err
rc=$?; echo "[c1] rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; print(json.dumps(json.load(open('gpurun_out/r05p_c1.json'))['configs']['C1']))"
