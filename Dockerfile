# MI355X device plugin image: ghcr.io/mi355x/k8s-device-plugin:<appVersion>
# (Makefile `images`). Drop-in for rocm/k8s-device-plugin: ./k8s-device-plugin
# in /root is the native daemon and the default command logs like upstream.
# The runtime stage holds no interpreter: the daemon and the HSA-direct
# liveness probe (gfx950 code object embedded) on the ROCm runtime base,
# which provides libhsa-runtime64 and libamd_smi (both dlopen()ed).
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
FROM ${ROCM_IMAGE} AS build
ARG GIT_DESCRIBE=dev
RUN apt-get update && apt-get install -y --no-install-recommends \
        cmake ninja-build g++ python3-dev python3-pip libdrm-dev && \
    pip3 install --no-cache-dir pybind11 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN GIT_DESCRIBE=${GIT_DESCRIBE} python3 rocm_k8s_device_plugin_amd/_build.py && \
    rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe --help >/dev/null && \
    rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin -h >/dev/null

FROM ${ROCM_IMAGE}
ARG GIT_DESCRIBE=dev
LABEL org.opencontainers.image.title="amdgpu-device-plugin (MI355X)" org.opencontainers.image.version="${GIT_DESCRIBE}"
RUN apt-get update && apt-get install -y --no-install-recommends libdrm-amdgpu1 && rm -rf /var/lib/apt/lists/*
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin /opt/mi355x/bin/mi355x-device-plugin
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe /opt/mi355x/bin/mi355x-liveness-probe
WORKDIR /root
RUN ln -s /opt/mi355x/bin/mi355x-device-plugin /root/k8s-device-plugin && \
    ln -s /opt/mi355x/bin/mi355x-device-plugin /root/mi355x-device-plugin
CMD ["./k8s-device-plugin", "-logtostderr=true", "-stderrthreshold=INFO", "-v=5"]
