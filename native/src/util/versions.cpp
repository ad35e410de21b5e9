#include "mi355x/versions.h"

#include <dlfcn.h>
#include <link.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

#ifndef MI355X_GIT_DESCRIBE
#define MI355X_GIT_DESCRIBE "dev"
#endif
#ifndef MI355X_SOURCE_DIGEST
#define MI355X_SOURCE_DIGEST ""
#endif

namespace mi355x::versions {
namespace {

std::string read_trimmed(const std::string& path) {
  std::ifstream f(path);
  if (!f) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ' || s.back() == '\r' || s.back() == '\t')) s.pop_back();
  return s;
}

bool is_dir(const std::string& p) {
  struct stat st {};
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::string rocm_path() {
  const char* e = std::getenv("ROCM_PATH");
  return e && *e ? e : "/opt/rocm";
}

// amdsmi_version_t (amd_smi/amdsmi.h): {uint32 major, minor, release; const char* build}
struct SmiVersion {
  uint32_t major, minor, release;
  const char* build;
};

}  // namespace

std::string source_digest() { return MI355X_SOURCE_DIGEST; }

// <dir of this executable>/../VERSION: "describe=<x>" and "digest=<y>" lines
// that _build.py rewrites whenever HEAD's describe changes while the native
// sources (and so these binaries) stay the same. Used only when its digest is
// this build's own: a commit then names itself without relinking anything.
std::string stamped_describe() {
  const std::string own = source_digest();
  if (own.empty()) return "";
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "";
  buf[n] = 0;
  std::string dir = buf;
  dir = dir.substr(0, dir.rfind('/'));
  std::ifstream f(dir.substr(0, dir.rfind('/')) + "/VERSION");
  std::string line, describe, digest;
  while (std::getline(f, line)) {
    if (line.rfind("describe=", 0) == 0) describe = line.substr(9);
    if (line.rfind("digest=", 0) == 0) digest = line.substr(7);
  }
  return digest == own ? describe : "";
}

std::string git_describe() {
  static const std::string d = [] {
    const std::string s = stamped_describe();
    return s.empty() ? std::string(MI355X_GIT_DESCRIBE) : s;
  }();
  return d;
}

std::string rocm(const std::string& path) { return read_trimmed((path.empty() ? rocm_path() : path) + "/.info/version"); }

std::string amdgpu(const std::string& sysfs_root) {
  // in-tree amdgpu has no module version; DKMS (amdgpu-dkms) exposes one
  const std::string mod = sysfs_root + "/module/amdgpu";
  std::string v = read_trimmed(mod + "/version");
  if (v.empty() && is_dir(mod)) v = "in-tree";
  return v;
}

std::string libdrm_amdgpu() {
  void* h = ::dlopen("libdrm_amdgpu.so.1", RTLD_LAZY | RTLD_LOCAL);
  if (!h) return "";
  std::string out = "libdrm_amdgpu.so.1";
  struct link_map* lm = nullptr;
  if (::dlinfo(h, RTLD_DI_LINKMAP, &lm) == 0 && lm && lm->l_name && *lm->l_name) out = lm->l_name;
  ::dlclose(h);
  return out;
}

std::string amd_smi() {
  void* h = nullptr;
  const std::string own = rocm_path() + "/lib/libamd_smi.so";
  for (const char* so : {"libamd_smi.so", own.c_str()})
    if ((h = ::dlopen(so, RTLD_LAZY | RTLD_LOCAL))) break;
  if (!h) return "";
  std::string out;
  using fn_t = int (*)(SmiVersion*);
  if (auto fn = reinterpret_cast<fn_t>(::dlsym(h, "amdsmi_get_lib_version"))) {
    SmiVersion v{};
    if (fn(&v) == 0) {
      char b[64];
      std::snprintf(b, sizeof(b), "%u.%u.%u", v.major, v.minor, v.release);
      out = b;
    }
  }
  ::dlclose(h);
  return out;
}

std::string library_line(const std::string& sysfs_root) {
  auto or_na = [](const std::string& s) { return s.empty() ? std::string("n/a") : s; };
  return "rocm: " + or_na(rocm()) + ", amdgpu: " + or_na(amdgpu(sysfs_root)) +
         ", libdrm_amdgpu: " + or_na(libdrm_amdgpu()) + ", amd-smi: " + or_na(amd_smi()) + ", numa_source: sysfs";
}

std::vector<std::string> banner(const std::string& title, const std::string& argv0, const std::string& sysfs_root) {
  const std::string dg = source_digest();
  return {title, argv0 + " version " + git_describe() + (dg.empty() ? "" : " (native sources " + dg + ")"),
          library_line(sysfs_root)};
}

}  // namespace mi355x::versions
