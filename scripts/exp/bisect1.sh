set -u
cd "${GRAFT_REPO_ROOT}"
bash scripts/exp/bench_old.sh || exit $?
AB='nov2|LOQA_PREFILL_O_SPLITS=0 LOQA_ENC_O_SPLITS=0;nostager|LOQA_PCM_STAGER=0' bash scripts/exp/bench_ab.sh
