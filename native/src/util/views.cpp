// Container start-up views (mi355x/views.h); layout of node_view.py / topology_view.py.
#include "mi355x/views.h"

#include <ftw.h>
#include <limits.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>

#include "mi355x/sysfs.h"

namespace mi355x::views {

namespace {

bool digits_after(const std::string& s, const char* prefix) {
  const size_t n = std::strlen(prefix);
  if (s.size() <= n || s.compare(0, n, prefix) != 0) return false;
  return std::all_of(s.begin() + static_cast<long>(n), s.end(), [](char c) { return c >= '0' && c <= '9'; });
}

bool all_digits(const std::string& s) {
  return !s.empty() && std::all_of(s.begin(), s.end(), [](char c) { return c >= '0' && c <= '9'; });
}

std::vector<std::string> sorted_dir(const std::string& p) {
  auto v = list_dir(p);
  std::sort(v.begin(), v.end());
  return v;
}

bool is_link(const std::string& p) {
  struct stat st {};
  return ::lstat(p.c_str(), &st) == 0 && S_ISLNK(st.st_mode);
}

std::string mkdirs(const std::string& dir) {
  for (size_t p = 1; p <= dir.size(); ++p)
    if (p == dir.size() || dir[p] == '/') {
      const std::string sub = dir.substr(0, p);
      if (::mkdir(sub.c_str(), 0755) != 0 && errno != EEXIST) return sub + ": " + std::strerror(errno);
    }
  return "";
}

std::string write_text(const std::string& path, const std::string& data) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return path + ": " + std::strerror(errno);
  const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
  if (std::fclose(f) != 0 || !ok) return path + ": write failed";
  return "";
}

std::string symlink_to(const std::string& target, const std::string& at) {
  if (::symlink(target.c_str(), at.c_str()) != 0) return at + ": " + std::strerror(errno);
  return "";
}

int rm_one(const char* p, const struct stat*, int, struct FTW*) { return ::remove(p); }
void rmtree(const std::string& p) { ::nftw(p.c_str(), rm_one, 16, FTW_DEPTH | FTW_PHYS); }

std::string make_temp_dir(const std::string& parent, const char* prefix) {
  std::string tmpl = path_join(parent, std::string(prefix) + "XXXXXX");
  std::vector<char> b(tmpl.begin(), tmpl.end());
  b.push_back('\0');
  if (!::mkdtemp(b.data())) return "";
  return b.data();
}

// kfd properties text -> (key, value) lines in order
std::vector<std::pair<std::string, std::string>> kv_lines(const std::string& text) {
  std::vector<std::pair<std::string, std::string>> out;
  size_t pos = 0;
  while (pos < text.size()) {
    size_t e = text.find('\n', pos);
    if (e == std::string::npos) e = text.size();
    std::string line = text.substr(pos, e - pos);
    pos = e + 1;
    const size_t a = line.find_first_not_of(" \t\r");
    if (a == std::string::npos) continue;
    const size_t b = line.find_first_of(" \t", a);
    std::string k = line.substr(a, b == std::string::npos ? std::string::npos : b - a), v;
    if (b != std::string::npos) {
      const size_t c = line.find_first_not_of(" \t", b);
      if (c != std::string::npos) {
        v = line.substr(c);
        while (!v.empty() && (v.back() == ' ' || v.back() == '\t' || v.back() == '\r')) v.pop_back();
      }
    }
    out.emplace_back(std::move(k), std::move(v));
  }
  return out;
}

std::string render(const std::vector<std::pair<std::string, std::string>>& kv) {
  std::string o;
  for (const auto& [k, v] : kv) o += k + " " + v + "\n";
  return o;
}

bool is_cpu_node(const std::string& props) {
  for (const auto& [k, v] : kv_lines(props))
    if (k == "simd_count") return v == "0" || v.empty();
  return true;
}

// sysfs reports every file as 4 KiB: copy contents, not sizes; symlinks skipped
std::string copy_tree(const std::string& src, const std::string& dst) {
  if (auto e = mkdirs(dst); !e.empty()) return e;
  for (const auto& name : sorted_dir(src)) {
    const std::string s = path_join(src, name), d = path_join(dst, name);
    if (is_link(s)) continue;
    if (is_dir(s)) {
      if (auto e = copy_tree(s, d); !e.empty()) return e;
    } else if (auto data = read_file(s)) {
      if (auto e = write_text(d, *data); !e.empty()) return e;
    }
  }
  return "";
}

// rewritten link property texts (links to nodes outside the view dropped)
std::vector<std::string> links(const std::string& dir, const std::map<int, int>& remap) {
  std::vector<std::string> out;
  if (!is_dir(dir)) return out;
  auto names = list_dir(dir);
  std::sort(names.begin(), names.end(), [](const std::string& a, const std::string& b) {
    const long x = all_digits(a) ? std::atol(a.c_str()) : (1L << 30), y = all_digits(b) ? std::atol(b.c_str()) : (1L << 30);
    return x < y;
  });
  for (const auto& n : names) {
    auto text = read_file(path_join(path_join(dir, n), "properties"));
    if (!text) continue;
    auto kv = kv_lines(*text);
    int from = -1, to = -1;
    bool bad = false;
    for (const auto& [k, v] : kv) {
      if (k == "node_from" || k == "node_to") {
        char* end = nullptr;
        const long x = std::strtol(v.c_str(), &end, 10);
        if (v.empty() || *end) bad = true;
        (k == "node_from" ? from : to) = static_cast<int>(x);
      }
    }
    if (bad || !remap.count(from) || !remap.count(to)) continue;
    for (auto& [k, v] : kv) {
      if (k == "node_from") v = std::to_string(remap.at(from));
      else if (k == "node_to") v = std::to_string(remap.at(to));
    }
    out.push_back(render(kv));
  }
  return out;
}

}  // namespace

// ---- node view -----------------------------------------------------------------
std::string build_node_view(const std::string& src, const std::string& dst, const std::string& alias,
                            const std::string& cpu_root, const std::string& src_cpu_root, int* nlinks, int* nhidden) {
  int l = 0, h = 0;
  if (auto e = mkdirs(dst); !e.empty()) return e;
  if (!is_dir(src)) return src + ": not a directory";
  for (const auto& name : sorted_dir(src)) {
    const std::string s = path_join(src, name);
    if (!(digits_after(name, "node") && is_dir(s))) {
      if (auto e = symlink_to(path_join(alias, name), path_join(dst, name)); !e.empty()) return e;
      ++l;
      continue;
    }
    const std::string nd = path_join(dst, name);
    if (auto e = mkdirs(nd); !e.empty()) return e;
    for (const auto& child : sorted_dir(s)) {
      if (digits_after(child, "cpu")) {
        const std::string cd = path_join(nd, child);
        if (auto e = mkdirs(cd); !e.empty()) return e;
        for (const auto& ent : sorted_dir(path_join(src_cpu_root, child))) {
          if (ent == "cache") {
            ++h;
            continue;
          }
          if (auto e = symlink_to(path_join(path_join(cpu_root, child), ent), path_join(cd, ent)); !e.empty()) return e;
          ++l;
        }
      } else {
        if (auto e = symlink_to(path_join(path_join(alias, name), child), path_join(nd, child)); !e.empty()) return e;
        ++l;
      }
    }
  }
  if (nlinks) *nlinks = l;
  if (nhidden) *nhidden = h;
  return "";
}

NodeView::NodeView(std::string root, const std::string& sysfs_root, std::string alias)
    : root_(std::move(root)), alias_(std::move(alias)), src_(path_join(sysfs_root, "devices/system/node")),
      src_cpu_(path_join(sysfs_root, "devices/system/cpu")) {}

std::string NodeView::build() {
  if (!path_.empty()) return "";
  if (auto e = mkdirs(root_); !e.empty()) return e;
  const std::string tmp = make_temp_dir(root_, ".node-");
  if (tmp.empty()) return root_ + ": " + std::strerror(errno);
  const std::string final_path = path_join(root_, "node");
  std::string e = build_node_view(src_, path_join(tmp, "node"), alias_, kCpuContainerPath, src_cpu_, &links, &hidden);
  if (e.empty()) {
    if (path_exists(final_path) || is_link(final_path)) rmtree(final_path);
    if (::rename(path_join(tmp, "node").c_str(), final_path.c_str()) != 0) e = final_path + ": " + std::strerror(errno);
  }
  rmtree(tmp);
  if (e.empty()) path_ = final_path;
  return e;
}

std::vector<std::pair<std::string, std::string>> NodeView::mounts() const {
  std::vector<std::pair<std::string, std::string>> out;
  if (path_.empty()) return out;
  char a[PATH_MAX], b[PATH_MAX];
  const bool same = ::realpath(alias_.c_str(), a) && ::realpath(src_.c_str(), b) ? std::strcmp(a, b) == 0
                                                                                 : alias_ == src_;
  if (!same) out.emplace_back(src_, alias_);
  out.emplace_back(path_, kNodeContainerPath);
  return out;
}

// ---- topology view -------------------------------------------------------------
std::string build_topology_view(const std::string& src_topology, const std::string& dst,
                                const std::vector<int>& gpu_nodes) {
  const std::set<int> keep(gpu_nodes.begin(), gpu_nodes.end());
  const std::string nodes_src = path_join(src_topology, "nodes");
  std::vector<int> ids;
  for (const auto& n : list_dir(nodes_src))
    if (all_digits(n)) ids.push_back(std::atoi(n.c_str()));
  std::sort(ids.begin(), ids.end());
  std::vector<int> kept;
  for (int i : ids) {
    auto props = read_file(path_join(path_join(nodes_src, std::to_string(i)), "properties"));
    if (!props) continue;
    if (is_cpu_node(*props) || keep.count(i)) kept.push_back(i);
  }
  for (int g : keep)
    if (std::find(kept.begin(), kept.end(), g) == kept.end())
      return "kfd node " + std::to_string(g) + " not readable under " + nodes_src;
  std::map<int, int> remap;
  for (size_t k = 0; k < kept.size(); ++k) remap[kept[k]] = static_cast<int>(k);
  if (auto e = mkdirs(path_join(dst, "nodes")); !e.empty()) return e;
  for (const char* name : {"generation_id", "system_properties"})
    if (auto data = read_file(path_join(src_topology, name)))
      if (auto e = write_text(path_join(dst, name), *data); !e.empty()) return e;
  for (const auto& [orig, now] : remap) {
    const std::string s = path_join(nodes_src, std::to_string(orig));
    const std::string d = path_join(path_join(dst, "nodes"), std::to_string(now));
    if (auto e = mkdirs(d); !e.empty()) return e;
    for (const auto& sub : sorted_dir(s)) {
      if (sub == "io_links" || sub == "p2p_links" || sub == "properties") continue;
      const std::string sp = path_join(s, sub);
      if (is_link(sp)) continue;
      if (is_dir(sp)) {
        if (auto e = copy_tree(sp, path_join(d, sub)); !e.empty()) return e;
      } else if (auto data = read_file(sp)) {
        if (auto e = write_text(path_join(d, sub), *data); !e.empty()) return e;
      }
    }
    std::map<std::string, size_t> counts;
    for (const char* kind : {"io_links", "p2p_links"}) {
      const auto texts = links(path_join(s, kind), remap);
      counts[std::string(kind) + "_count"] = texts.size();
      if (auto e = mkdirs(path_join(d, kind)); !e.empty()) return e;
      for (size_t j = 0; j < texts.size(); ++j) {
        const std::string ld = path_join(path_join(d, kind), std::to_string(j));
        if (auto e = mkdirs(ld); !e.empty()) return e;
        if (auto e = write_text(path_join(ld, "properties"), texts[j]); !e.empty()) return e;
      }
    }
    auto props = kv_lines(read_file(path_join(s, "properties")).value_or(""));
    for (auto& [k, v] : props)
      if (auto c = counts.find(k); c != counts.end()) v = std::to_string(c->second);
    if (auto e = write_text(path_join(d, "properties"), render(props)); !e.empty()) return e;
  }
  return "";
}

std::string TopologyViews::get(std::vector<int> gpu_nodes, std::string* err) {
  std::sort(gpu_nodes.begin(), gpu_nodes.end());
  gpu_nodes.erase(std::unique(gpu_nodes.begin(), gpu_nodes.end()), gpu_nodes.end());
  std::string key = read_trimmed(path_join(src_, "generation_id")).value_or("") + ":";
  for (size_t i = 0; i < gpu_nodes.size(); ++i) key += (i ? "," : "") + std::to_string(gpu_nodes[i]);
  uint64_t h = 1469598103934665603ull;  // FNV-1a: one directory per (kfd generation, node set)
  for (unsigned char c : key) h = (h ^ c) * 1099511628211ull;
  char name[24];
  std::snprintf(name, sizeof(name), "%016llx", static_cast<unsigned long long>(h));
  const std::string path = path_join(base_, name);
  if (is_dir(path)) return path;
  std::lock_guard<std::mutex> lk(mu_);
  if (is_dir(path)) return path;
  if (auto e = mkdirs(base_); !e.empty()) return *err = e, "";
  const std::string tmp = make_temp_dir(base_, ".view-");
  if (tmp.empty()) return *err = base_ + ": " + std::strerror(errno), "";
  if (auto e = build_topology_view(src_, tmp, gpu_nodes); !e.empty()) {
    rmtree(tmp);
    return *err = e, "";
  }
  if (::rename(tmp.c_str(), path.c_str()) != 0) {
    const std::string e = std::strerror(errno);
    rmtree(tmp);
    return *err = path + ": " + e, "";
  }
  built_++;
  return path;
}

}  // namespace mi355x::views
