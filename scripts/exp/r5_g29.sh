# served hub (gRPC relays -> front end -> GPU worker, single-relay bypass) with
# the on-GPU voice loaded from an MMS-TTS-shaped checkpoint (16 kHz, SDP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
python scripts/exp/make_mms_ckpt.py /tmp/mms_ckpt > gpurun_out/g29_ckpt.log 2>&1 || { tail -5 gpurun_out/g29_ckpt.log; exit 1; }
HUB_TTS_CHECKPOINT=/tmp/mms_ckpt timeout -k 10 600 python -u bench.py --mode hub --served-dp --tts --steps 20 --warmup 3 --bypass > gpurun_out/g29_hub_tts_mms.log 2>&1 || { tail -20 gpurun_out/g29_hub_tts_mms.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g29_hub_tts_mms.log | tail -1 | cut -c1-1500
