#!/bin/bash
# r03o: A/B in one run: the product library (NN edge bodies without the
# window-group skip) vs the A/B build (with it; also the parallel rank / slot
# set-up of the deciles select) on C2 and C5, each checked against the
# oracle; GPU suite of the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2"; exit "$1"; fi; }
for v in prod ab prod ab; do
  for c in c2 c5; do
    if [ $v = ab ]; then L=ab; else L=default; fi
    GSKYHIP_LIB=$L timeout -k 10 300 python -u tools/ab_render.py --config $c --reps 30 --oracle --label "$v" >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
    stop $? "ab_${v}_$c"
  done
done
cat gpurun_out/ab.jsonl
GSKYHIP_LIB=ab timeout -k 10 300 python -u bench.py --only c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/c4_ab.json 2>> gpurun_out/ab.err
stop $? c4_ab
python3 -c "import json; d=json.load(open('gpurun_out/c4_ab.json')); print('deciles ab', d['configs']['C4']['deciles']['ms_per_step'])"
