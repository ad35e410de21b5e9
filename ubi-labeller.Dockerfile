# UBI9-based MI355X node labeller image.
ARG BUILD_IMAGE=rocm/dev-almalinux-9:7.2
FROM ${BUILD_IMAGE} AS build
RUN dnf install -y cmake ninja-build gcc-c++ python3-devel python3-pip libdrm-devel openssl-devel && \
    pip3 install --no-cache-dir pybind11 && dnf clean all
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN python3 rocm_k8s_device_plugin_amd/_build.py --no-hip && \
    rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller -h >/dev/null

FROM registry.access.redhat.com/ubi9/ubi-minimal:latest
RUN microdnf install -y python3 python3-pip libdrm openssl-libs && pip3 install --no-cache-dir grpcio protobuf pyyaml && \
    microdnf clean all
WORKDIR /root
COPY --from=build /src/rocm_k8s_device_plugin_amd /opt/mi355x-dp/rocm_k8s_device_plugin_amd
COPY scripts/k8s-node-labeller /root/k8s-node-labeller
RUN ln -s /opt/mi355x-dp/rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller /root/mi355x-node-labeller
COPY LICENSE* /licenses/
ENV MI355X_DP_HOME=/opt/mi355x-dp MI355X_DP_NO_AUTOBUILD=1
CMD ["./k8s-node-labeller"]
