// Container Device Interface specs and names for the advertised GPUs (the
// native daemon's -device_list_strategy / -cdi_spec_dir).
//
// The reference returns DeviceSpecs only (internal/pkg/amdgpu/amdgpu.go:255-297).
// Kubernetes >= 1.28 also lets a plugin name CDI devices
// (ContainerAllocateResponse.cdi_devices, field 5 of api.proto), which the CRI
// runtime resolves against spec files in /var/run/cdi. The spec files here are
// byte-for-byte what the Python CLI writes (rocm_k8s_device_plugin_amd/cdi.py:
// json.dump(indent=1, sort_keys=True)): one `amd.com-<resource>.json` per
// resource, kind `amd.com/<resource>`, one device per advertised ID with its
// card and render nodes, /dev/kfd in the spec-wide edits. Written atomically
// (temp file + rename), so a runtime scanning the directory never reads half a
// file.
#pragma once

#include <map>
#include <set>
#include <string>
#include <vector>

#include "mi355x/gpu_discovery.h"

namespace mi355x::cdi {

constexpr const char* kVersion = "0.5.0";
constexpr const char* kDeviceSpecs = "device-specs";
constexpr const char* kCdiCri = "cdi-cri";
constexpr const char* kCdiAnnotations = "cdi-annotations";

struct Strategies {
  bool specs = true, cri = false, annotations = false;
  std::vector<std::string> order = {"device-specs"};  // as given (unique)
  bool cdi() const { return cri || annotations; }
};

// "-device_list_strategy" value (comma-separated) -> strategies; false + err on an unknown one
bool parse_strategies(const std::string& value, Strategies* out, std::string* err);

bool valid_name(const std::string& dev_id);     // letters, digits, _ - . : ; alnum at both ends
bool valid_class(const std::string& resource);  // letters, digits, _ - ; alnum first
std::string kind(const std::string& resource);  // amd.com/<resource>
std::string qualified_name(const std::string& resource, const std::string& dev_id);  // amd.com/gpu=<id>
std::string annotation_key(const std::string& resource);  // cdi.k8s.io/amd.com_<resource>
std::string spec_filename(const std::string& resource);    // amd.com-<resource>.json
// a JSON string literal as Python's json.dumps writes the str (ensure_ascii); bytes that are
// not UTF-8 as os.fsdecode's surrogate escapes
std::string json_str(const std::string& s);

// The spec document of one resource; "" + err when a name is not CDI-valid.
std::string spec_json(const std::string& resource, const std::vector<GpuDevice>& devices, std::string* err);

// Writes (atomically replaces) one spec per resource in `members` and removes
// the files of `stale` resources that are not in `members`. "" on success.
std::string write_specs(const std::string& dir, const std::map<std::string, std::vector<GpuDevice>>& members,
                        const std::set<std::string>& stale, std::vector<std::string>* written = nullptr);

}  // namespace mi355x::cdi
