# bench of the worktree at _old (an older commit) next to the current tree, same box
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd _old && timeout -k 10 300 python bench.py > ../gpurun_out/ab_old.log 2>&1)
rc=$?; grep '^{"metric"' gpurun_out/ab_old.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/ab_new.log 2>&1
rc=$?; grep '^{"metric"' gpurun_out/ab_new.log | cut -c1-300; exit $rc
