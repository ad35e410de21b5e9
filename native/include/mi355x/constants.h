// Literal values shared with the Python control plane. These are wire/drop-in
// contracts with the reference (internal/pkg/types/constants.go:21-93) and
// with kubelet (vendor/k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/constants.go).
#pragma once

namespace mi355x {

constexpr const char* kAmdVendorId = "0x1002";
constexpr const char* kGimDriverName = "gim";
constexpr const char* kVfioDriverName = "vfio-pci";
constexpr const char* kResourceNamespace = "amd.com";
constexpr const char* kDeviceTypeGpu = "gpu";
constexpr const char* kDeviceTypeGpuVf = "gpu_vf";
constexpr const char* kDeviceTypeGpuPf = "gpu_pf";
constexpr const char* kPciGpuEnvPrefix = "PCI_RESOURCE_AMD_COM";

// gfx_target_version of CDNA4 / MI355X (gfx950) as kfd reports it.
constexpr int kGfx950TargetVersion = 90500;

// Reference pair-weight constants (internal/pkg/allocator/device.go:38-54).
constexpr int kSameDevIdWeight = 10;
constexpr int kDifferentDevIdWeight = 20;
constexpr int kXgmiLinkWeight = 10;
constexpr int kPcieLinkWeight = 40;
constexpr int kOtherLinkWeight = 50;
constexpr int kSameNumaWeight = 10;
constexpr int kDifferentNumaWeight = 20;

}  // namespace mi355x
