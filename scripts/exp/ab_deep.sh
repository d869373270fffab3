set -u
mkdir -p gpurun_out
LOQA_FUSED_DEEP=4 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_fused_decode.py > gpurun_out/deep_tests.log 2>&1 || { tail -20 gpurun_out/deep_tests.log; exit 1; }
tail -1 gpurun_out/deep_tests.log
for v in 0 4 0 4; do
  LOQA_FUSED_DEEP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_deep_$v.log 2>&1 || { tail -5 gpurun_out/ab_deep_$v.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_deep_$v.log') if l.startswith('{')][-1])
print('deep=$v', d['value'], d['phase_ms_per_step']['llm_decode'], d['phase_ms_per_step']['llm_decode_steps'], d['phase_ms_per_step']['stt'])"
done
