#!/bin/bash
# r04n: per-launch kernel trace of the C4 deciles (decileCount 9).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_c4 -o run --output-format csv -- \
  python3 bench.py --only c4 --no-cpu --steps 2 --warmup 1 > gpurun_out/tr_c4.log 2>&1
stop $? tr_c4
f=$(find gpurun_out/tr_c4 -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if "decile" in n or "compact" in n:
        print(n.split("(")[0][-40:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
PY
