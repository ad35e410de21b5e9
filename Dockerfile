# MI355X device plugin image: ghcr.io/mi355x/k8s-device-plugin:<appVersion>
# (Makefile `images`). Drop-in for rocm/k8s-device-plugin: ./k8s-device-plugin
# in /root is the native daemon and the default command logs like upstream.
# The runtime stage holds no interpreter and no ROCm toolchain: plain Ubuntu
# with the daemon, the HSA-direct liveness probe (gfx950 code object
# embedded) and the three ROCm libraries they load (libhsa-runtime64 for the
# probe, libamd_smi for the -smi_* health sources, both dlopen()ed, and
# librocprofiler-register, which libhsa-runtime64 links), plus the distro
# libraries those link. tests/test_image_layout.py checks every DT_NEEDED and
# dlopen() target of what is copied against what this stage provides
# (reference: Dockerfile:23-33, alpine + one binary + libdrm).
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

FROM ubuntu:22.04
ARG GIT_DESCRIBE=dev
LABEL org.opencontainers.image.title="amdgpu-device-plugin (MI355X)" org.opencontainers.image.version="${GIT_DESCRIBE}"
RUN apt-get update && apt-get install -y --no-install-recommends libdrm2 libdrm-amdgpu1 libelf1 libnuma1 && \
    rm -rf /var/lib/apt/lists/*
COPY --from=build /opt/rocm/lib/libhsa-runtime64.so* /opt/rocm/lib/
COPY --from=build /opt/rocm/lib/librocprofiler-register.so* /opt/rocm/lib/
COPY --from=build /opt/rocm/lib/libamd_smi.so* /opt/rocm/lib/
ENV LD_LIBRARY_PATH=/opt/rocm/lib
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin /opt/mi355x/bin/mi355x-device-plugin
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe /opt/mi355x/bin/mi355x-liveness-probe
WORKDIR /root
RUN ln -s /opt/mi355x/bin/mi355x-device-plugin /root/k8s-device-plugin && \
    ln -s /opt/mi355x/bin/mi355x-device-plugin /root/mi355x-device-plugin
CMD ["./k8s-device-plugin", "-logtostderr=true", "-stderrthreshold=INFO", "-v=5"]
