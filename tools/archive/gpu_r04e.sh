#!/bin/bash
# r04e: RGBA store cache policy of render_nn_kernel (A/B build,
# GSKYHIP_NN_STPOL 0 nt / 1 sc1 / 2 sc0 sc1 / 3 plain) on C2 and C5 with the
# oracle check and FETCH_SIZE per policy; gather_rate with live u16 loads;
# the service leg on the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
timeout -k 10 120 ./tools/calib/gather_rate 5 > gpurun_out/gather_rate.json
stop $? gather_rate
cat gpurun_out/gather_rate.json
for i in 1 2; do
  for sp in 0 1 2 3; do
    for c in c2 c5; do
      GSKYHIP_LIB=ab GSKYHIP_NN_STPOL=$sp timeout -k 10 120 python3 tools/ab_render.py --config $c --reps 20 --label "stpol$sp" >> gpurun_out/ab.jsonl
      stop $? "ab_stpol${sp}_$c"
    done
  done
done
GSKYHIP_LIB=ab GSKYHIP_NN_STPOL=1 timeout -k 10 200 python3 tools/ab_render.py --config c2 --reps 5 --oracle --label stpol1 >> gpurun_out/ab.jsonl
stop $? oracle_stpol1
cat gpurun_out/ab.jsonl
for sp in 0 1; do
  GSKYHIP_LIB=ab GSKYHIP_NN_STPOL=$sp PMC_OUT=gpurun_out/pmc_stpol$sp PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" \
    PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc.sh
  stop $? pmc_stpol$sp
done
timeout -k 10 400 python3 bench.py --only svc --no-cpu --steps 3 --warmup 1 > gpurun_out/svc.json 2> gpurun_out/svc.err
stop $? svc
cut -c1-1500 gpurun_out/svc.json
