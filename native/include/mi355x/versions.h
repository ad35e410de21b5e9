// Version banner of the native daemons.
//
// The reference prints "<argv0> version <gitDescribe>" and the libraries it
// depends on (hwloc) in its usage text and logs them at start-up
// (cmd/k8s-device-plugin/main.go:37-48,77-79); the describe string is stamped
// at build time (Dockerfile:21, -ldflags -X main.gitDescribe). Here the build
// stamps MI355X_GIT_DESCRIBE (CMake cache variable, fed by _build.py from
// `git describe` or by the Dockerfiles' GIT_DESCRIBE build argument) and the
// library line names what this build depends on: the ROCm release, the
// loaded amdgpu driver, libdrm_amdgpu and amd-smi (NUMA comes from sysfs, so
// there is no hwloc). Same fields as the Python CLIs' utils/versions.py.
#pragma once

#include <string>
#include <vector>

namespace mi355x::versions {

// the build's describe, or a newer one from <bin>/../VERSION when that file
// names this build's own source digest (_build.py keeps it current); "dev"
// when the build was not stamped
std::string git_describe();
std::string source_digest();                    // first 12 hex of the native sources' content hash, or ""
std::string rocm(const std::string& rocm_path = "");  // <ROCM_PATH or /opt/rocm>/.info/version
std::string amdgpu(const std::string& sysfs_root);    // module version, "in-tree", or ""
std::string libdrm_amdgpu();                    // path of the libdrm_amdgpu the process would load, or ""
std::string amd_smi();                          // amdsmi_get_lib_version(), or ""

// "rocm: 7.2.0, amdgpu: in-tree, libdrm_amdgpu: /usr/lib/..., amd-smi: 26.2.1, numa_source: sysfs"
std::string library_line(const std::string& sysfs_root);

// The banner: `title`, "<argv0> version <describe> (native sources <digest>)", the library line.
std::vector<std::string> banner(const std::string& title, const std::string& argv0, const std::string& sysfs_root);

}  // namespace mi355x::versions
