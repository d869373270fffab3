# MI355X hub image (the reference's Dockerfile:1-63 builds a static Go binary;
# here: a ROCm + PyTorch base, the in-tree gfx950 kernels built at image build).
FROM rocm/pytorch:latest
WORKDIR /opt/loqa-hub
COPY . .
RUN python -m loqa_hub_amd._native.build && pip install --no-deps -e .
ENV LOQA_PORT=3000 \
    LOQA_GRPC_PORT=50051 \
    HSA_ENABLE_IPC_MODE_LEGACY=0
EXPOSE 3000 50051
# one GPU: loqa-hub; 8 GPUs DP: HUB_NUM_GPUS=8; 70B TP=8: torchrun (parallel/tp_serving.py)
CMD ["loqa-hub"]
