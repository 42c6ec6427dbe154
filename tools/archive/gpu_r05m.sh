#!/bin/bash
# r05m: C2 NN rows by column pairs (GSKYHIP_NN_PAIR=1: one aligned dword
# gather per pixel pair where it serves both, 8-byte stores) vs the product
# body, oracle check, L1 counters; XCD-contiguous item order
# (GSKYHIP_NN_XCD=2: XCD x runs the x-th eighth of the items) for C3's
# bilinear and C2's NN kernel; FETCH_SIZE of each order.  A/B build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 1 0 1; do
  GSKYHIP_NN_PAIR=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "c2 pair=$m" >> gpurun_out/r05m_pair.jsonl 2>> gpurun_out/r05m_pair.err
  stop $? c2_pair_$m
done
GSKYHIP_NN_PAIR=1 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "c2 pair=1 oracle" >> gpurun_out/r05m_pair.jsonl 2>> gpurun_out/r05m_pair.err
stop $? c2_pair_oracle
GSKYHIP_NN_PAIR=1 timeout -k 10 300 python3 tools/ab_render.py --config c5 --oracle --label "c5 pair=1 oracle" >> gpurun_out/r05m_pair.jsonl 2>> gpurun_out/r05m_pair.err
stop $? c5_pair_oracle
cat gpurun_out/r05m_pair.jsonl
GSKYHIP_NN_PAIR=1 PMC_GROUPS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;TD_TD_BUSY_sum TD_TC_STALL_sum;GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2_pair bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_pair render_nn_kernel gpurun_out/pmc_c2_pair.json
stop $? pmc_pair
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
