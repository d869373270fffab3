# config 5 rank step with the decode-grid cap raised (a TP rank's GPU runs no
# Whisper decoder beside it in the projection)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "cap2048|LOQA_LLM_MAX_WGS=2048" "cap4096|LOQA_LLM_MAX_WGS=4096"; do
  label="${v%%|*}"; envs="${v#*|}"
  env $envs timeout -k 10 400 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g15_c5_${label}.json 2> gpurun_out/g15_c5_${label}.err || exit 12
  echo "$label $(cut -c1-330 gpurun_out/g15_c5_${label}.json)"
done
echo done
