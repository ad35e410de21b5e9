// CDI specs and names (mi355x/cdi.h).
#include "mi355x/cdi.h"

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "mi355x/sysfs.h"

namespace mi355x::cdi {

namespace {

bool alnum(char c) { return std::isalnum(static_cast<unsigned char>(c)) != 0; }

}  // namespace

std::string json_str(const std::string& s) {  // json.dumps (ensure_ascii)
  std::string o = "\"";
  auto u16 = [&o](unsigned v) {
    char b[8];
    std::snprintf(b, sizeof(b), "\\u%04x", v);
    o += b;
  };
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (c < 0x20 || c == 0x7F) {  // json.dumps escapes everything outside ' '..'~'
      u16(c);
    } else if (c < 0x80) {
      o += static_cast<char>(c);
    } else {
      // one code point of well-formed UTF-8 -> \uXXXX (a surrogate pair above U+FFFF), as
      // json.dumps writes a str; any other byte -> \udcXX, the str os.fsdecode makes of it
      const int n = c >= 0xF0 && c <= 0xF4 ? 4 : c >= 0xE0 && c <= 0xEF ? 3 : c >= 0xC2 && c <= 0xDF ? 2 : 0;
      unsigned cp = n == 4 ? c & 0x07u : n == 3 ? c & 0x0Fu : c & 0x1Fu;
      bool ok = n > 0 && i + n <= s.size();
      for (int k = 1; ok && k < n; ++k) {
        const unsigned char d = static_cast<unsigned char>(s[i + k]);
        ok = (d & 0xC0) == 0x80;
        cp = (cp << 6) | (d & 0x3Fu);
      }
      // overlong 3/4-byte forms, UTF-16 surrogates and values past U+10FFFF are not UTF-8
      ok = ok && !(n == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) &&
           !(n == 4 && (cp < 0x10000 || cp > 0x10FFFF));
      if (!ok) {
        u16(0xDC00u | c);
      } else {
        if (cp >= 0x10000) {
          u16(0xD800u + ((cp - 0x10000) >> 10));
          u16(0xDC00u + ((cp - 0x10000) & 0x3FF));
        } else {
          u16(cp);
        }
        i += n - 1;
      }
    }
  }
  return o + "\"";
}

namespace {

// {"hostPath": p, "path": p, "permissions": "rw"} at indent level `lvl` (indent=1)
std::string node_json(const std::string& path, int lvl) {
  const std::string in(lvl, ' '), in1(lvl + 1, ' ');
  return in + "{\n" + in1 + "\"hostPath\": " + json_str(path) + ",\n" + in1 + "\"path\": " + json_str(path) + ",\n" +
         in1 + "\"permissions\": \"rw\"\n" + in + "}";
}

// {"deviceNodes": [...]} as the value of a key at level `lvl`
std::string edits_json(const std::vector<std::string>& paths, int lvl) {
  const std::string in(lvl, ' '), in1(lvl + 1, ' ');
  std::string o = "{\n" + in1 + "\"deviceNodes\": ";
  if (paths.empty()) {
    o += "[]";
  } else {
    o += "[\n";
    for (size_t i = 0; i < paths.size(); ++i) o += node_json(paths[i], lvl + 2) + (i + 1 < paths.size() ? ",\n" : "\n");
    o += in1 + "]";
  }
  return o + "\n" + in + "}";
}

}  // namespace

bool parse_strategies(const std::string& value, Strategies* out, std::string* err) {
  Strategies s;
  s.specs = false;
  s.order.clear();
  bool any = false;
  size_t start = 0;
  const std::string v = value.empty() ? kDeviceSpecs : value;
  while (start <= v.size()) {
    size_t end = v.find(',', start);
    if (end == std::string::npos) end = v.size();
    std::string item = v.substr(start, end - start);
    item.erase(0, item.find_first_not_of(" \t"));
    item.erase(item.find_last_not_of(" \t") + 1);
    start = end + 1;
    if (item.empty()) continue;
    if (std::find(s.order.begin(), s.order.end(), item) == s.order.end() &&
        (item == kDeviceSpecs || item == kCdiCri || item == kCdiAnnotations))
      s.order.push_back(item);
    if (item == kDeviceSpecs) s.specs = true;
    else if (item == kCdiCri) s.cri = true;
    else if (item == kCdiAnnotations) s.annotations = true;
    else
      return *err = "invalid device_list_strategy '" + item + "', supported values are device-specs, cdi-cri, " +
                    "cdi-annotations",
             false;
    any = true;
  }
  if (!any) {
    s.specs = true;
    s.order = {kDeviceSpecs};
  }
  *out = s;
  return true;
}

bool valid_name(const std::string& id) {
  if (id.empty() || !alnum(id.front()) || !alnum(id.back())) return false;
  return std::all_of(id.begin(), id.end(), [](char c) { return alnum(c) || c == '_' || c == '-' || c == '.' || c == ':'; });
}

bool valid_class(const std::string& r) {
  if (r.empty() || !alnum(r.front())) return false;
  return std::all_of(r.begin(), r.end(), [](char c) { return alnum(c) || c == '_' || c == '-'; });
}

std::string kind(const std::string& resource) { return "amd.com/" + resource; }
std::string qualified_name(const std::string& resource, const std::string& id) { return kind(resource) + "=" + id; }
std::string annotation_key(const std::string& resource) { return "cdi.k8s.io/amd.com_" + resource; }
std::string spec_filename(const std::string& resource) { return "amd.com-" + resource + ".json"; }

std::string spec_json(const std::string& resource, const std::vector<GpuDevice>& devices, std::string* err) {
  if (!valid_class(resource)) return *err = "resource '" + resource + "' is not a valid CDI class", "";
  std::vector<const GpuDevice*> devs;
  for (const auto& d : devices) {
    if (!valid_name(d.id)) return *err = "device ID '" + d.id + "' is not a valid CDI device name", "";
    devs.push_back(&d);
  }
  std::sort(devs.begin(), devs.end(), [](const GpuDevice* a, const GpuDevice* b) { return a->id < b->id; });
  std::string o = "{\n \"cdiVersion\": " + json_str(kVersion) + ",\n \"containerEdits\": " +
                  edits_json({"/dev/kfd"}, 1) + ",\n \"devices\": ";
  if (devs.empty()) {
    o += "[]";
  } else {
    o += "[\n";
    for (size_t i = 0; i < devs.size(); ++i) {
      std::vector<std::string> paths;  // card then renderD (topology.py dev_paths)
      if (devs[i]->card >= 0) paths.push_back("/dev/dri/card" + std::to_string(devs[i]->card));
      if (devs[i]->render_minor >= 0) paths.push_back("/dev/dri/renderD" + std::to_string(devs[i]->render_minor));
      o += "  {\n   \"containerEdits\": " + edits_json(paths, 3) + ",\n   \"name\": " + json_str(devs[i]->id) +
           "\n  }" + (i + 1 < devs.size() ? ",\n" : "\n");
    }
    o += " ]";
  }
  return o + ",\n \"kind\": " + json_str(kind(resource)) + "\n}\n";
}

std::string write_specs(const std::string& dir, const std::map<std::string, std::vector<GpuDevice>>& members,
                        const std::set<std::string>& stale, std::vector<std::string>* written) {
  // mkdir -p
  for (size_t p = 1; p <= dir.size(); ++p)
    if (p == dir.size() || dir[p] == '/') {
      const std::string sub = dir.substr(0, p);
      if (::mkdir(sub.c_str(), 0755) != 0 && errno != EEXIST) return sub + ": " + std::strerror(errno);
    }
  for (const auto& [res, devs] : members) {
    std::string err;
    const std::string doc = spec_json(res, devs, &err);
    if (!err.empty()) return err;
    // not *.json while being written: runtimes scan the directory for specs
    std::string tmpl = path_join(dir, ".cdi-XXXXXX.tmp");
    std::vector<char> name(tmpl.begin(), tmpl.end());
    name.push_back('\0');
    const int fd = ::mkstemps(name.data(), 4);
    if (fd < 0) return dir + ": " + std::strerror(errno);
    const std::string tmp = name.data();
    size_t off = 0;
    while (off < doc.size()) {
      const ssize_t n = ::write(fd, doc.data() + off, doc.size() - off);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        const std::string e = std::strerror(errno);
        ::close(fd);
        ::unlink(tmp.c_str());
        return tmp + ": " + e;
      }
      off += static_cast<size_t>(n);
    }
    ::fchmod(fd, 0644);
    ::close(fd);
    const std::string path = path_join(dir, spec_filename(res));
    if (::rename(tmp.c_str(), path.c_str()) != 0) {
      const std::string e = std::strerror(errno);
      ::unlink(tmp.c_str());
      return path + ": " + e;
    }
    if (written) written->push_back(path);
  }
  for (const auto& r : stale)
    if (!members.count(r)) ::unlink(path_join(dir, spec_filename(r)).c_str());
  return "";
}

}  // namespace mi355x::cdi
