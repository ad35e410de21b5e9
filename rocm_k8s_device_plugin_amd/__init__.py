"""MI355X-native Kubernetes device plugin and node labeller.

Drop-in replacement for the ROCm k8s-device-plugin / k8s-node-labeller
(reference: bhatnitish/rocm-k8s-device-plugin). Native core (C++/HIP) in
``native/`` is exposed as ``_native`` / ``_hip``; the control plane
(kubelet Device Plugin v1beta1 over grpc.aio, labeller REST client) is Python.
"""
__version__ = "0.1.0"
