#!/bin/bash
# r05q: kernel stats of the service leg (the daemon's warp batches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_svc -o run --output-format csv -- \
  python3 bench.py --only svc --no-cpu > gpurun_out/r05q_svc.json 2> gpurun_out/r05q_svc.err
rc=$?; echo "[svc] rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_svc -name "*kernel_stats.csv" | head
for f in $(find gpurun_out/prof_svc -name "*kernel_stats.csv"); do head -6 $f | cut -c1-200; done
