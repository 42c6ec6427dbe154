#!/bin/bash
# r04h: kernel + copy trace of the service leg (daemon subprocess included).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_svc -o run --output-format csv -- \
  python3 bench.py --only svc --no-cpu --svc-jobs 256 > gpurun_out/prof_svc.log 2>&1
stop $? prof_svc
find gpurun_out/prof_svc -name "*stats*" | head
