# MI355X node labeller image: ghcr.io/mi355x/k8s-device-plugin:labeller-<appVersion>
# (Makefile `images`). Drop-in: ./k8s-node-labeller in /root is the native
# labeller (in-cluster or -kubeconfig, HTTPS through OpenSSL; libdrm_amdgpu and
# libamd_smi dlopen()ed for the family / firmware labels). No interpreter and
# no ROCm toolchain: plain Ubuntu, the binary, libamd_smi and the distro
# libraries (checked by tests/test_image_layout.py).
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
FROM ${ROCM_IMAGE} AS build
ARG GIT_DESCRIBE=dev
RUN apt-get update && apt-get install -y --no-install-recommends \
        cmake ninja-build g++ python3-dev python3-pip libdrm-dev libssl-dev && \
    pip3 install --no-cache-dir pybind11 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN GIT_DESCRIBE=${GIT_DESCRIBE} python3 rocm_k8s_device_plugin_amd/_build.py --no-hip && \
    rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller -h >/dev/null

FROM ubuntu:22.04
RUN apt-get update && apt-get install -y --no-install-recommends libdrm2 libdrm-amdgpu1 libssl3 && \
    rm -rf /var/lib/apt/lists/*
COPY --from=build /opt/rocm/lib/libamd_smi.so* /opt/rocm/lib/
ENV LD_LIBRARY_PATH=/opt/rocm/lib
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller /opt/mi355x/bin/mi355x-node-labeller
WORKDIR /root
RUN ln -s /opt/mi355x/bin/mi355x-node-labeller /root/k8s-node-labeller && \
    ln -s /opt/mi355x/bin/mi355x-node-labeller /root/mi355x-node-labeller
CMD ["./k8s-node-labeller"]
