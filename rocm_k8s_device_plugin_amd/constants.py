"""Literal values of the drop-in surface.

Source of truth: internal/pkg/types/constants.go:21-93 (reference) and
kubelet v1beta1 constants.go. Changing any of these breaks compatibility with
existing DaemonSets, pod specs and node selectors.
"""
from __future__ import annotations

# label kinds, in the reference's flag order (constants.go:21)
SUPPORTED_LABELS = [
    "mode", "firmware", "family", "driver-version", "driver-src-version", "device-id", "product-name",
    "vram", "simd-count", "cu-count", "compute-memory-partition", "compute-partitioning-supported",
    "memory-partitioning-supported",
]

# command line flag names (constants.go:24-33)
FLAG_PULSE = "pulse"
FLAG_DRIVER_TYPE = "driver_type"
FLAG_RESOURCE_NAMING_STRATEGY = "resource_naming_strategy"

# resource naming strategies (constants.go:36-41)
STRATEGY_SINGLE = "single"
STRATEGY_MIXED = "mixed"

# driver types (constants.go:44-52)
CONTAINER = "container"
VF_PASSTHROUGH = "vf-passthrough"
PF_PASSTHROUGH = "pf-passthrough"
DRIVER_TYPES = (CONTAINER, VF_PASSTHROUGH, PF_PASSTHROUGH)

# sysfs locations, relative to the sysfs root (constants.go:55-74 use absolute /sys paths)
VFIO_DRIVER_REL = "bus/pci/drivers/vfio-pci"
VFIO_DRIVER_NAME = "vfio-pci"
GIM_DRIVER_REL = "bus/pci/drivers/gim"
GIM_MODULE_REL = "module/gim"
GIM_DRIVER_NAME = "gim"
PCI_DEVICES_REL = "bus/pci/devices"
KFD_CLASS_REL = "class/kfd"

PCI_GPU_ENV_PREFIX = "PCI_RESOURCE_AMD_COM"
AMD_VENDOR_ID = "0x1002"

DEVICE_TYPE_GPU = "gpu"
DEVICE_TYPE_GPU_VF = "gpu_vf"
DEVICE_TYPE_GPU_PF = "gpu_pf"

RESOURCE_NAMESPACE = "amd.com"
EXPORTER_HEALTH_TIMEOUT_S = 10.0

# gfx_target_version reported by kfd for CDNA4 / MI355X (gfx950)
GFX950_TARGET_VERSION = 90500
# MI355X device ids seen in kfd device_id (decimal in sysfs properties)
MI355X_HBM_BYTES = 288 * 1000 ** 3

# label prefixes (cmd/k8s-node-labeller/main.go:38-44)
EXPERIMENTAL_PREFIX = "beta.amd.com"
AMD_PREFIX = "amd.com"
LEGACY_COMPUTE_PARTITIONING_SUPPORTED = "amd.com/compute-partitioning-supported"
LEGACY_MEMORY_PARTITIONING_SUPPORTED = "amd.com/memory-partitioning-supported"
LEGACY_PARTITION_TYPE = "amd.com/compute-memory-partition"
