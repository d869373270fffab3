# prologue launches v2 (longer poll sleep, 32 solo all-reduce blocks), sc1
# loads vs acquire + plain loads; config 5 one stream with the decode-step slope
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tp_gpu.py -m gpu -k "prologue" > gpurun_out/g6_t1.txt 2>&1 || { tail -30 gpurun_out/g6_t1.txt; exit 11; }
LOQA_PRO_ACQ=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tp_gpu.py -m gpu -k "prologue" > gpurun_out/g6_t2.txt 2>&1 || { tail -30 gpurun_out/g6_t2.txt; exit 12; }
tail -1 gpurun_out/g6_t1.txt gpurun_out/g6_t2.txt
run() {
  label=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g6_c5_$label.json 2> gpurun_out/g6_c5_$label.err || { tail -5 gpurun_out/g6_c5_$label.err; exit 13; }
  python - "$label" gpurun_out/g6_c5_$label.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:>14}: step {d['rank_step_ms_local_collectives']:.3f} ms, projected {d['projected_ms_per_added_command']}")
PY
}
run pro X=1
run pro_acq LOQA_PRO_ACQ=1
run nopro LOQA_TP_PROLOGUE=0
run pro_b X=2
run pro_acq_b LOQA_PRO_ACQ=1
run nopro_b LOQA_TP_PROLOGUE=0
for v in pro "pro_acq LOQA_PRO_ACQ=1"; do
  set -- $v; label=$1; shift
  rm -rf gpurun_out/g6_prof
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g6_prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --prefill-rows 0 > gpurun_out/g6_prof.log 2>&1 || { tail -20 gpurun_out/g6_prof.log; exit 14; }
  f=$(ls gpurun_out/g6_prof/c5_kernel_trace.csv gpurun_out/g6_prof/*/c5_kernel_trace.csv 2>/dev/null | head -1)
  python scripts/decode_steps.py "$f" tp > gpurun_out/g6_anat_$label.txt 2>&1; head -8 gpurun_out/g6_anat_$label.txt
done
rm -rf gpurun_out/g6_prof
timeout -k 10 900 python -u scripts/bench_configs.py --config 5 --streams 1 --no-tts --per-stream 6 --warmup 1 > gpurun_out/g6_c5_1stream.log 2>&1 || { tail -20 gpurun_out/g6_c5_1stream.log; exit 15; }
grep '^{' gpurun_out/g6_c5_1stream.log | cut -c1-700
echo done
