# UBI9-based MI355X device plugin image: ghcr.io/mi355x/k8s-device-plugin:<appVersion>-ubi
# (Makefile `images`); default health pulse 30 s like the upstream UBI image.
# ROCr (liveness probe) and amd-smi (-smi_* health sources) come from the
# build stage's ROCm with the system libraries they link.
ARG BUILD_IMAGE=rocm/dev-almalinux-9:7.2
FROM ${BUILD_IMAGE} AS build
ARG GIT_DESCRIBE=dev
RUN dnf install -y cmake ninja-build gcc-c++ python3-devel python3-pip libdrm-devel && \
    pip3 install --no-cache-dir pybind11 && dnf clean all
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN GIT_DESCRIBE=${GIT_DESCRIBE} python3 rocm_k8s_device_plugin_amd/_build.py && \
    rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin -h >/dev/null

FROM registry.access.redhat.com/ubi9/ubi-minimal:latest
RUN microdnf install -y libdrm elfutils-libelf numactl-libs zlib libstdc++ && microdnf clean all
COPY --from=build /opt/rocm/lib/libhsa-runtime64.so* /opt/rocm/lib/librocprofiler-register.so* /opt/rocm/lib/libamd_smi.so* /opt/rocm/lib/
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-device-plugin /opt/mi355x/bin/mi355x-device-plugin
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-liveness-probe /opt/mi355x/bin/mi355x-liveness-probe
WORKDIR /root
RUN ln -s /opt/mi355x/bin/mi355x-device-plugin /root/k8s-device-plugin && \
    ln -s /opt/mi355x/bin/mi355x-device-plugin /root/mi355x-device-plugin
COPY LICENSE* /licenses/
ENV LD_LIBRARY_PATH=/opt/rocm/lib
CMD ["./k8s-device-plugin", "-logtostderr=true", "-stderrthreshold=INFO", "-v=5", "-pulse=30"]
