#!/bin/bash
# r05x: C2 NN rows reusing the row above's gathered pixels
# (GSKYHIP_NN_REUSE=1: a gather only for the lanes whose source offset
# changed) vs the product body; oracle check on C2 and C5; texture-path
# counters.  A/B build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GSKYHIP_LIB=ab
stop() { echo "[$2] rc=$1"; if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi; }
for m in 0 1 0 1; do
  GSKYHIP_NN_REUSE=$m timeout -k 10 300 python3 tools/ab_render.py --config c2 --label "c2 reuse=$m" >> gpurun_out/r05x_reuse.jsonl 2>> gpurun_out/r05x_reuse.err
  stop $? c2_reuse_$m
done
GSKYHIP_NN_REUSE=1 timeout -k 10 300 python3 tools/ab_render.py --config c2 --oracle --label "c2 reuse=1 oracle" >> gpurun_out/r05x_reuse.jsonl 2>> gpurun_out/r05x_reuse.err
stop $? c2_reuse_oracle
GSKYHIP_NN_REUSE=1 timeout -k 10 300 python3 tools/ab_render.py --config c5 --oracle --label "c5 reuse=1 oracle" >> gpurun_out/r05x_reuse.jsonl 2>> gpurun_out/r05x_reuse.err
stop $? c5_reuse_oracle
cat gpurun_out/r05x_reuse.jsonl
GSKYHIP_NN_REUSE=1 PMC_GROUPS="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;TD_TD_BUSY_sum TD_TC_STALL_sum;GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" PMC_CMD="python3 tools/ab_render.py --config c2 --reps 3" PMC_OUT=gpurun_out/pmc_c2_reuse bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out/pmc_c2_reuse render_nn_kernel gpurun_out/pmc_c2_reuse.json
stop $? pmc_reuse
