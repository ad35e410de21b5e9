#include "mi355x/kfd_topology.h"

#include <algorithm>

namespace mi355x {

uint64_t KfdNode::local_mem_bytes() const {
  uint64_t total = 0;
  for (const auto& b : mem_banks) total += b.size_in_bytes;
  if (total == 0) total = prop_u64("local_mem_size");
  return total;
}

bool parse_kfd_link(const std::string& properties_path, bool p2p, KfdLink* out) {
  auto kv = parse_kv_file(properties_path);
  if (!kv) return false;
  out->type = static_cast<int>(kv_i64(*kv, "type", kLinkUndefined));
  out->node_from = static_cast<int>(kv_i64(*kv, "node_from", -1));
  out->node_to = static_cast<int>(kv_i64(*kv, "node_to", -1));
  out->weight = static_cast<int>(kv_i64(*kv, "weight", 0));
  out->min_bandwidth = kv_i64(*kv, "min_bandwidth", 0);
  out->max_bandwidth = kv_i64(*kv, "max_bandwidth", 0);
  out->flags = static_cast<int>(kv_i64(*kv, "flags", 0));
  out->p2p = p2p;
  return out->node_from >= 0 && out->node_to >= 0;
}

static void load_links(const std::string& dir, bool p2p, std::vector<KfdLink>* out) {
  auto entries = list_dir(dir);
  // numeric order, so link 10 follows link 9
  std::vector<std::pair<int64_t, std::string>> numbered;
  for (auto& e : entries)
    if (is_all_digits(e)) numbered.emplace_back(parse_i64(e, 0), e);
  std::sort(numbered.begin(), numbered.end());
  for (auto& [n, e] : numbered) {
    KfdLink l;
    if (parse_kfd_link(path_join(path_join(dir, e), "properties"), p2p, &l)) out->push_back(l);
  }
}

KfdTopology KfdTopology::load(const std::string& nodes_dir) {
  KfdTopology t;
  t.nodes_dir_ = nodes_dir;
  std::vector<int> ids;
  for (auto& e : list_dir(nodes_dir))
    if (is_all_digits(e)) ids.push_back(static_cast<int>(parse_i64(e, -1)));
  std::sort(ids.begin(), ids.end());
  for (int id : ids) {
    std::string dir = path_join(nodes_dir, std::to_string(id));
    const std::string props = path_join(dir, "properties");
    auto kv = parse_kv_file(props);
    if (!kv) {
      if (path_exists(props)) t.unreadable_.push_back(id);
      continue;
    }
    KfdNode n;
    n.id = id;
    n.props = std::move(*kv);
    if (auto name = read_trimmed(path_join(dir, "name"))) n.name = *name;
    if (auto g = read_trimmed(path_join(dir, "gpu_id"))) n.gpu_id = parse_i64(*g, 0);
    load_links(path_join(dir, "io_links"), false, &n.io_links);
    load_links(path_join(dir, "p2p_links"), true, &n.p2p_links);
    std::string banks = path_join(dir, "mem_banks");
    std::vector<std::pair<int64_t, std::string>> numbered;
    for (auto& e : list_dir(banks))
      if (is_all_digits(e)) numbered.emplace_back(parse_i64(e, 0), e);
    std::sort(numbered.begin(), numbered.end());
    for (auto& [bn, e] : numbered) {
      auto bkv = parse_kv_file(path_join(path_join(banks, e), "properties"));
      if (!bkv) continue;
      KfdMemBank b;
      b.heap_type = static_cast<int>(kv_i64(*bkv, "heap_type", 0));
      b.size_in_bytes = kv_u64(*bkv, "size_in_bytes", 0);
      b.flags = static_cast<int>(kv_i64(*bkv, "flags", 0));
      b.width = static_cast<int>(kv_i64(*bkv, "width", 0));
      b.mem_clk_max = static_cast<int>(kv_i64(*bkv, "mem_clk_max", 0));
      n.mem_banks.push_back(b);
    }
    t.index_[id] = t.nodes_.size();
    t.nodes_.push_back(std::move(n));
  }
  return t;
}

KfdTopology KfdTopology::load_sysfs(const std::string& sysfs_root) {
  return load(path_join(sysfs_root, "class/kfd/kfd/topology/nodes"));
}

const KfdNode* KfdTopology::node(int id) const {
  auto it = index_.find(id);
  return it == index_.end() ? nullptr : &nodes_[it->second];
}

const KfdNode* KfdTopology::node_by_render_minor(int minor) const {
  for (auto& n : nodes_)
    if (n.drm_render_minor() == minor && minor > 0) return &n;
  return nullptr;
}

std::map<int, std::string> KfdTopology::render_to_unique_id() const {
  std::map<int, std::string> out;
  for (auto& n : nodes_) {
    int m = n.drm_render_minor();
    if (m <= 0) continue;
    // the reference skips nodes without a parseable unique_id (amdgpu.go:435-439)
    auto it = n.props.find("unique_id");
    if (it == n.props.end() || !is_all_digits(it->second)) continue;
    out[m] = it->second;
  }
  return out;
}

std::map<int, int> KfdTopology::render_to_node_id() const {
  std::map<int, int> out;
  for (auto& n : nodes_) {
    int m = n.drm_render_minor();
    if (m > 0) out[m] = n.id;
  }
  return out;
}

std::vector<const KfdNode*> KfdTopology::gpu_nodes() const {
  std::vector<const KfdNode*> out;
  for (auto& n : nodes_)
    if (n.is_gpu()) out.push_back(&n);
  return out;
}

int KfdTopology::count_gpu_nodes() const {
  int c = 0;
  for (auto& n : nodes_)
    if (n.simd_count() > 0) ++c;
  return c;
}

bool KfdTopology::any_live_gpu() const {
  for (auto& n : nodes_)
    if (n.is_live_gpu()) return true;
  return false;
}

std::vector<KfdLink> KfdTopology::all_gpu_links() const {
  std::vector<KfdLink> out;
  for (auto& n : nodes_) {
    if (!n.has_render_node()) continue;
    out.insert(out.end(), n.io_links.begin(), n.io_links.end());
    out.insert(out.end(), n.p2p_links.begin(), n.p2p_links.end());
  }
  return out;
}

}  // namespace mi355x
