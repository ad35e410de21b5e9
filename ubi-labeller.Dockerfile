# UBI9-based MI355X node labeller image: ghcr.io/mi355x/k8s-device-plugin:labeller-<appVersion>-ubi
# (Makefile `images`).
ARG BUILD_IMAGE=rocm/dev-almalinux-9:7.2
FROM ${BUILD_IMAGE} AS build
ARG GIT_DESCRIBE=dev
RUN dnf install -y cmake ninja-build gcc-c++ python3-devel python3-pip libdrm-devel openssl-devel && \
    pip3 install --no-cache-dir pybind11 && dnf clean all
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN GIT_DESCRIBE=${GIT_DESCRIBE} python3 rocm_k8s_device_plugin_amd/_build.py --no-hip && \
    rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller -h >/dev/null

FROM registry.access.redhat.com/ubi9/ubi-minimal:latest
RUN microdnf install -y libdrm openssl-libs libstdc++ && microdnf clean all
COPY --from=build /opt/rocm/lib/libamd_smi.so* /opt/rocm/lib/
COPY --from=build /src/rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller /opt/mi355x/bin/mi355x-node-labeller
WORKDIR /root
RUN ln -s /opt/mi355x/bin/mi355x-node-labeller /root/k8s-node-labeller && \
    ln -s /opt/mi355x/bin/mi355x-node-labeller /root/mi355x-node-labeller
COPY LICENSE* /licenses/
ENV LD_LIBRARY_PATH=/opt/rocm/lib
CMD ["./k8s-node-labeller"]
