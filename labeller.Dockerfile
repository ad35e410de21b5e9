# MI355X node labeller image (drop-in: ./k8s-node-labeller in /root).
ARG ROCM_IMAGE=rocm/dev-ubuntu-22.04:7.2
FROM ${ROCM_IMAGE} AS build
RUN apt-get update && apt-get install -y --no-install-recommends \
        cmake ninja-build g++ python3-dev python3-pip libdrm-dev libssl-dev && \
    pip3 install --no-cache-dir pybind11 && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY native native
COPY rocm_k8s_device_plugin_amd rocm_k8s_device_plugin_amd
RUN python3 rocm_k8s_device_plugin_amd/_build.py --no-hip && \
    rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller -h >/dev/null

FROM ${ROCM_IMAGE}
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip libdrm-amdgpu1 libssl3 && \
    pip3 install --no-cache-dir grpcio protobuf pyyaml && rm -rf /var/lib/apt/lists/*
WORKDIR /root
COPY --from=build /src/rocm_k8s_device_plugin_amd /opt/mi355x-dp/rocm_k8s_device_plugin_amd
COPY scripts/k8s-node-labeller /root/k8s-node-labeller
# the same labeller as one native process (in-cluster, no Python in it):
# command: ["./mi355x-node-labeller"]   (Helm: lbl.native=true)
RUN ln -s /opt/mi355x-dp/rocm_k8s_device_plugin_amd/bin/mi355x-node-labeller /root/mi355x-node-labeller
ENV MI355X_DP_HOME=/opt/mi355x-dp MI355X_DP_NO_AUTOBUILD=1
CMD ["./k8s-node-labeller"]
