# MI355X device plugin image. Drop-in for rocm/k8s-device-plugin: the binary
# is ./k8s-device-plugin in /root and the default command logs like upstream.
# Build stage compiles the C++ core, the gfx950 code object and the HSA probe.
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
FROM ${ROCM_IMAGE} AS build
RUN apt-get update && apt-get install -y --no-install-recommends \
        cmake ninja-build g++ python3-dev python3-pip libdrm-dev && \
    pip3 install --no-cache-dir pybind11 grpcio protobuf pyyaml && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN python3 rocm_k8s_device_plugin_amd/_build.py && \
    rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe --help >/dev/null && \
    rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin -h >/dev/null && \
    python3 -c "import rocm_k8s_device_plugin_amd.proto.deviceplugin, rocm_k8s_device_plugin_amd.proto.metricssvc"

FROM ${ROCM_IMAGE}
ARG GIT_DESCRIBE=dev
LABEL org.opencontainers.image.title="amdgpu-device-plugin (MI355X)" org.opencontainers.image.version="${GIT_DESCRIBE}"
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip libdrm-amdgpu1 && \
    pip3 install --no-cache-dir grpcio protobuf pyyaml && rm -rf /var/lib/apt/lists/*
WORKDIR /root
COPY --from=build /src/rocm_k8s_device_plugin_amd /opt/mi355x-dp/rocm_k8s_device_plugin_amd
COPY scripts/k8s-device-plugin /root/k8s-device-plugin
# the same plugin as one native process (container driver, no Python in it):
# command: ["./mi355x-device-plugin", "-pulse=30"]   (Helm: dp.native=true)
RUN ln -s /opt/mi355x-dp/rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin /root/mi355x-device-plugin
ENV MI355X_DP_HOME=/opt/mi355x-dp MI355X_DP_NO_AUTOBUILD=1
CMD ["./k8s-device-plugin", "-logtostderr=true", "-stderrthreshold=INFO", "-v=5"]
