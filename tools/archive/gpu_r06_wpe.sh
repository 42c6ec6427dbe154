set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for rep in 1 2 3; do for w in 7 8 6; do
  GSKYHIP_LIB=ab GSKYHIP_NN_MASK_WPE=$w timeout -k 10 200 python -u tools/ab_render.py --config c5 --reps 30 --label wpe$w >> gpurun_out/r06wpe_c5.jsonl 2>/dev/null || exit 1
done; done
cat gpurun_out/r06wpe_c5.jsonl
