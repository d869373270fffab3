#!/bin/bash
# VITS checkpoint loader on the GPU: parity tests through the HIP kernels plus
# the existing VITS GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_vits_checkpoint.py tests/test_engine_gpu.py -k "vits or checkpoint" -m gpu \
  > gpurun_out/r5_vits_ckpt_gpu.txt 2>&1
rc=$?; tail -25 gpurun_out/r5_vits_ckpt_gpu.txt; exit $rc
