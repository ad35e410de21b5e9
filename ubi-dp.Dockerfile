# UBI9-based MI355X device plugin image; default health pulse 30 s like the upstream UBI image.
ARG BUILD_IMAGE=rocm/dev-almalinux-9:7.2
FROM ${BUILD_IMAGE} AS build
RUN dnf install -y cmake ninja-build gcc-c++ python3-devel python3-pip libdrm-devel && \
    pip3 install --no-cache-dir pybind11 && dnf clean all
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN python3 rocm_k8s_device_plugin_amd/_build.py

FROM registry.access.redhat.com/ubi9/ubi-minimal:latest
RUN microdnf install -y python3 python3-pip libdrm && pip3 install --no-cache-dir grpcio protobuf pyyaml && \
    microdnf clean all
# ROCr runtime for the HSA-direct liveness probe
COPY --from=build /opt/rocm/lib/libhsa-runtime64.so* /opt/rocm/lib/librocprofiler-register.so* /opt/rocm/lib/
WORKDIR /root
COPY --from=build /src/rocm_k8s_device_plugin_amd /opt/mi355x-dp/rocm_k8s_device_plugin_amd
COPY scripts/k8s-device-plugin /root/k8s-device-plugin
RUN ln -s /opt/mi355x-dp/rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin /root/mi355x-device-plugin
COPY LICENSE* /licenses/
ENV MI355X_DP_HOME=/opt/mi355x-dp MI355X_DP_NO_AUTOBUILD=1 LD_LIBRARY_PATH=/opt/rocm/lib
CMD ["./k8s-device-plugin", "-logtostderr=true", "-stderrthreshold=INFO", "-v=5", "-pulse=30"]
