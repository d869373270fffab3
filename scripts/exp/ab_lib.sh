# Same-box A/B of two builds of the kernels library (ab_kernels/old.so vs
# new.so, copied over the in-tree library between 20-step benches)
set -u
mkdir -p gpurun_out
L=loqa_hub_amd/_native/libloqa_kernels.so
for v in new old new old; do
  cp ab_kernels/$v.so $L
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_lib_$v.log 2>&1 || { tail -5 gpurun_out/ab_lib_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_lib_$v.log') if l.startswith('{')][-1])
p=d['phase_ms_per_step']
print('$v', d['value'], round(p['llm_decode']/p['llm_decode_steps'],3), p['stt'], p['llm_prefill'])"
done
cp ab_kernels/new.so $L
