#!/bin/bash
# r05m: XCD-contiguous item order (GSKYHIP_NN_XCD=2: XCD x runs the x-th
# eighth of the items) for C3's bilinear and C2's NN kernel, A/B build;
# FETCH_SIZE of each order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 2 0 2; do
  GSKYHIP_NN_XCD=$m timeout -k 10 300 python3 tools/ab_c3.py --label "c3 xcd=$m" >> gpurun_out/r05m_xcd.jsonl 2>> gpurun_out/r05m_xcd.err
  stop $? c3_$m
  GSKYHIP_NN_XCD=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "c2 xcd=$m" >> gpurun_out/r05m_xcd.jsonl 2>> gpurun_out/r05m_xcd.err
  stop $? c2_$m
done
GSKYHIP_NN_XCD=2 timeout -k 10 300 python3 tools/ab_c3.py --oracle --label "c3 xcd=2 oracle" >> gpurun_out/r05m_xcd.jsonl 2>> gpurun_out/r05m_xcd.err
stop $? c3_oracle
GSKYHIP_NN_XCD=2 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "c2 xcd=2 oracle" >> gpurun_out/r05m_xcd.jsonl 2>> gpurun_out/r05m_xcd.err
stop $? c2_oracle
cat gpurun_out/r05m_xcd.jsonl
for m in 0 2; do
  export GSKYHIP_NN_XCD=$m PMC_GROUPS="FETCH_SIZE;WRITE_SIZE"
  PMC_CMD="python3 tools/ab_c3.py --reps 3" PMC_OUT=gpurun_out/pmc_c3_xcd$m bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c3_xcd$m render_bil_kernel gpurun_out/pmc_c3_xcd$m.json
  stop $? pmc_c3_$m
  PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2_xcd$m bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_xcd$m render_nn_kernel gpurun_out/pmc_c2_xcd$m.json
  stop $? pmc_c2_$m
done
grep -h "FETCH_SIZE\|traffic" gpurun_out/pmc_c*_xcd*.json
