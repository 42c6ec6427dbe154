#!/bin/bash
# r04r: C4 descriptor breakdown with the describe_all trace (spawn / main
# thread / join) at 16 and 1 host threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for th in 16 4 1; do
  GSKYHIP_DRILL_TRACE=1 GSKYHIP_DRILL_THREADS=$th timeout -k 10 200 python3 tools/c4_desc.py --label "th$th" --reps 10 >> gpurun_out/c4_desc.jsonl 2> gpurun_out/c4_desc_$th.err
  stop $? c4_desc_$th
  tail -4 gpurun_out/c4_desc_$th.err
done
cat gpurun_out/c4_desc.jsonl
