# STT decode-GEMM workgroup cap A/B (20-step benches, ABCABC)
set -u
mkdir -p gpurun_out
for v in none 128 192 none 128 192; do
  if [ $v = none ]; then e=""; else e="LOQA_STT_MAX_WGS=$v"; fi
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_cap_$v.log 2>&1 || { tail -5 gpurun_out/ab_cap_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_cap_$v.log') if l.startswith('{')][-1])
p=d['phase_ms_per_step']
print('cap=$v', d['value'], round(p['llm_decode']/p['llm_decode_steps'],3), p['stt'], p['stt_decode'])"
done
