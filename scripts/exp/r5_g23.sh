# decode-attention key split for the config-5 rank (1 kv head per rank: few
# attention workgroups) and the 8B bench: 128 (default) vs 64 vs 32 keys
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "k128|LOQA_LLM_ATTN_SPLIT_KEYS=128" "k64|LOQA_LLM_ATTN_SPLIT_KEYS=64" "k32|LOQA_LLM_ATTN_SPLIT_KEYS=32" "k128b|LOQA_LLM_ATTN_SPLIT_KEYS=128"; do
  label="${v%%|*}"; envs="${v#*|}"
  env $envs timeout -k 10 400 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g23_c5_${label}.json 2> gpurun_out/g23_c5_${label}.err || exit 12
  echo "$label $(cut -c1-330 gpurun_out/g23_c5_${label}.json)"
done
echo done
