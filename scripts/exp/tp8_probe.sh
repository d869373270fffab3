set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 280 python -u scripts/exp/tp8_probe.py --world 8 --layers 4 --stall 90 --serve-timeout 200 > gpurun_out/tp8_probe_default.log 2>&1
rc=$?
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/tp8_probe_default.log | tail -40 | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 280 python -u scripts/exp/tp8_probe.py --world 8 --layers 4 --hwq 1 --stall 90 --serve-timeout 200 > gpurun_out/tp8_probe_hwq1.log 2>&1
rc=$?
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/tp8_probe_hwq1.log | tail -20 | cut -c1-400
exit $rc
