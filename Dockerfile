# iit-amd on AMD Instinct MI355X (gfx950): ROCm PyTorch base, the gfx950 kernel library built in the image.
#   docker build -t iit-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host --shm-size 16g iit-amd python bench.py
# (the reference's image, /root/reference/Dockerfile, is CUDA PyTorch + dev tooling; this one targets ROCm only)
ARG BASE=rocm/pytorch:latest
FROM ${BASE} AS base
ENV DEBIAN_FRONTEND=noninteractive \
    PYTORCH_ROCM_ARCH=gfx950 \
    IIT_OFFLOAD_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /workspace/iit-amd

FROM base AS prod
COPY . .
# hipcc cross-compiles csrc/*.hip for gfx950 into iit_amd/_native (no GPU needed at build time), then the package
RUN python3 -c "import __graft_entry__ as g; g.build()" && python3 -m pip install --no-deps .

FROM prod AS test
RUN python3 -m pip install pytest pytest-timeout pytest-xdist hypothesis
CMD ["python3", "-m", "pytest", "tests", "-q", "-m", "not gpu"]
