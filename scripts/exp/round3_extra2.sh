set -u
cd "${GRAFT_REPO_ROOT}"
bash scripts/tp_gpu_check.sh || exit $?
bash scripts/exp/round3_extra.sh
