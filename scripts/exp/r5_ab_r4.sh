# same-box A/B: the round-4 tree (ab_r4/, a git worktree of 0271e56) vs this tree
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  (cd ab_r4 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > ../gpurun_out/ab_old_$i.json 2>/dev/null) || exit 11
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_new_$i.json 2>/dev/null || exit 12
done
echo done
