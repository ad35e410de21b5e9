#include <algorithm>
#include <deque>
#include <limits>
#include <set>
#include <unordered_set>

#include "mi355x/allocator.h"
#include "mi355x/constants.h"

namespace mi355x {

namespace {

// Error strings are part of the drop-in surface: kubelet logs them verbatim
// (reference besteffort_policy.go:36-43).
constexpr const char* kInvalidSize = "allocation size can not be negative";
constexpr const char* kInvalidAvailable = "available devices count less than allocation size";
constexpr const char* kInvalidRequired = "must_include devices size is more than allocation size";
constexpr const char* kInvalidReqAvailable =
    "must_include length should be less than or equal to avilable device size";
constexpr const char* kInvalidInit = "Init method must be called before Allocate";
constexpr const char* kNoCandidate = "No candidate subset found with matching criteria";

int link_rank(int type) {
  // lower is better: xGMI, then PCIe, then anything else
  if (type == kLinkXgmi) return 0;
  if (type == kLinkPcie) return 1;
  return 2;
}

bool is_xcp_id(const std::string& id) { return id.find("amdgpu_xcp") != std::string::npos; }

}  // namespace

int pair_weight_formula(bool same_gpu, int link_type, bool same_numa, bool cross_hive,
                        const AllocatorOptions& opt, bool has_link) {
  if (!has_link && !opt.missing_pair_is_worst) return 0;  // reference quirk (device.go:266)
  int w = same_gpu ? kSameDevIdWeight : kDifferentDevIdWeight;
  if (!has_link) {
    // Partitions of one package talk over the on-die fabric; anything else
    // without a reported link is treated as the worst link.
    w += same_gpu ? kXgmiLinkWeight : kOtherLinkWeight;
  } else if (link_type == kLinkXgmi) {
    w += kXgmiLinkWeight;
  } else if (link_type == kLinkPcie) {
    w += kPcieLinkWeight;
  } else {
    w += kOtherLinkWeight;
  }
  w += same_numa ? kSameNumaWeight : kDifferentNumaWeight;
  if (cross_hive) w += opt.cross_hive_penalty;
  return w;
}

std::string HiveAllocator::init(const std::vector<AllocDevice>& devs, const KfdTopology& topo,
                                const AllocatorOptions& opt) {
  devs_.clear();
  index_.clear();
  groups_.clear();
  dev_group_.clear();
  w_.clear();
  link_.clear();
  link_kw_.clear();
  link_bw_.clear();
  linked_pairs_ = from_keys_ = inferred_pairs_ = 0;
  opt_ = opt;
  if (devs.empty()) return "Devices list is empty. Unable to calculate pair wise weights";

  devs_ = devs;
  const int n = static_cast<int>(devs_.size());
  std::unordered_map<int, int> node2dev;
  for (int i = 0; i < n; ++i) {
    index_.emplace(devs_[i].id, i);
    node2dev.emplace(devs_[i].node_id, i);
    if (devs_[i].hive_id == 0)
      if (const KfdNode* kn = topo.node(devs_[i].node_id)) devs_[i].hive_id = kn->hive_id();
  }

  link_.assign(static_cast<size_t>(n) * n, 0);
  link_kw_.assign(static_cast<size_t>(n) * n, 0);
  link_bw_.assign(static_cast<size_t>(n) * n, 0);
  for (const KfdLink& l : topo.all_gpu_links()) {
    auto a = node2dev.find(l.node_from), b = node2dev.find(l.node_to);
    if (a == node2dev.end() || b == node2dev.end() || a->second == b->second) continue;
    int i = a->second, j = b->second;
    const size_t ij = static_cast<size_t>(i) * n + j, ji = static_cast<size_t>(j) * n + i;
    int& cur = link_[ij];
    int t = l.type <= 0 ? kLinkOther : l.type;
    const bool better_type = cur == 0 || link_rank(t) < link_rank(cur);
    const bool same_type_better = cur == t && ((l.weight > 0 && (link_kw_[ij] == 0 || l.weight < link_kw_[ij])) ||
                                               (l.weight == link_kw_[ij] && l.max_bandwidth > link_bw_[ij]));
    if (better_type || same_type_better) {
      cur = t;
      link_[ji] = t;
      link_kw_[ij] = link_kw_[ji] = l.weight;
      link_bw_[ij] = link_bw_[ji] = l.max_bandwidth;
    }
  }
  std::unordered_set<int> froms;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (link_[static_cast<size_t>(i) * n + j]) {
        ++linked_pairs_;
        froms.insert(std::min(devs_[i].node_id, devs_[j].node_id));
      }
  from_keys_ = froms.size();

  // Pairs with an endpoint whose kfd node is unreadable have no kfd link.
  // With a recovered identity the link type still follows from the fabric:
  // partitions of one package talk on-die (kfd reports them as xGMI), GPUs of
  // one xGMI hive are one xGMI hop apart (8x MI355X: fully connected), and
  // GPUs outside a common hive go through PCIe.
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const auto& a = devs_[i];
      const auto& b = devs_[j];
      if (!(a.inferred_links || b.inferred_links)) continue;
      if (link_[static_cast<size_t>(i) * n + j]) continue;
      bool a_known = a.inferred_links || a.node_id >= 0;
      bool b_known = b.inferred_links || b.node_id >= 0;
      if (!a_known || !b_known) continue;
      int t;
      if (!a.unique_id.empty() && a.unique_id == b.unique_id)
        t = kLinkXgmi;
      else if (a.hive_id != 0 && a.hive_id == b.hive_id)
        t = kLinkXgmi;
      else
        t = kLinkPcie;
      link_[static_cast<size_t>(i) * n + j] = link_[static_cast<size_t>(j) * n + i] = t;
      ++inferred_pairs_;
    }

  std::set<std::pair<std::string, std::string>> degraded;
  for (const auto& p : opt.degraded_links)
    degraded.insert(p.first < p.second ? p : std::make_pair(p.second, p.first));
  w_.assign(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (i == j) continue;
      const auto& a = devs_[i];
      const auto& b = devs_[j];
      int lt = link_[static_cast<size_t>(i) * n + j];
      if (lt != 0 && !degraded.empty() && a.unique_id != b.unique_id &&
          degraded.count(a.unique_id < b.unique_id ? std::make_pair(a.unique_id, b.unique_id)
                                                   : std::make_pair(b.unique_id, a.unique_id)))
        lt = kLinkOther;
      bool cross_hive = a.hive_id != 0 && b.hive_id != 0 && a.hive_id != b.hive_id;
      w_[static_cast<size_t>(i) * n + j] =
          pair_weight_formula(a.unique_id == b.unique_id, lt, a.numa_node == b.numa_node, cross_hive, opt_, lt != 0);
    }

  // group by physical GPU, in first-seen order; members by kfd node id
  std::unordered_map<std::string, int> gidx;
  dev_group_.assign(n, -1);
  for (int i = 0; i < n; ++i) {
    auto it = gidx.find(devs_[i].unique_id);
    int g;
    if (it == gidx.end()) {
      g = static_cast<int>(groups_.size());
      gidx.emplace(devs_[i].unique_id, g);
      groups_.push_back(Group{devs_[i].unique_id, "", {}});
    } else {
      g = it->second;
    }
    if (!is_xcp_id(devs_[i].id)) groups_[g].parent_id = devs_[i].id;
    groups_[g].members.push_back(i);
    dev_group_[i] = g;
  }
  // members by kfd node id; devices without a readable kfd node keep their
  // input order (the discovery order: the PCI function, then xcp by index)
  for (auto& g : groups_)
    std::stable_sort(g.members.begin(), g.members.end(), [&](int a, int b) {
      int na = devs_[a].node_id < 0 ? std::numeric_limits<int>::max() : devs_[a].node_id;
      int nb = devs_[b].node_id < 0 ? std::numeric_limits<int>::max() : devs_[b].node_id;
      return na < nb;
    });
  if (opt_.extended_search_auto) {
    opt_.extended_search = false;
    for (const auto& g : groups_) opt_.extended_search |= g.members.size() > 1;
  }
  return "";
}

int HiveAllocator::pair_weight(const std::string& a, const std::string& b) const {
  auto ia = index_.find(a), ib = index_.find(b);
  if (ia == index_.end() || ib == index_.end()) return -1;
  return w_[static_cast<size_t>(ia->second) * devs_.size() + ib->second];
}

int HiveAllocator::link_type(const std::string& a, const std::string& b) const {
  auto ia = index_.find(a), ib = index_.find(b);
  if (ia == index_.end() || ib == index_.end()) return -1;
  return link_[static_cast<size_t>(ia->second) * devs_.size() + ib->second];
}

std::string HiveAllocator::validate(const std::vector<std::string>& available,
                                    const std::vector<std::string>& required, int size, AllocResult* out,
                                    std::vector<int>* avail_idx, std::vector<int>* req_idx) const {
  if (size <= 0) return kInvalidSize;
  if (static_cast<int>(available.size()) < size) return kInvalidAvailable;
  if (static_cast<int>(required.size()) > size) return kInvalidRequired;
  if (required.size() > available.size()) return kInvalidReqAvailable;
  if (devs_.empty()) return kInvalidInit;
  if (static_cast<int>(available.size()) == size) {
    out->ids = available;
    out->short_circuit = true;
    return "";
  }
  if (static_cast<int>(required.size()) == size) {
    out->ids = required;
    out->short_circuit = true;
    return "";
  }
  std::unordered_set<std::string> av(available.begin(), available.end());
  for (auto& r : required)
    if (!av.count(r)) return kNoCandidate;
  std::unordered_set<int> seen;
  for (auto& a : available) {
    auto it = index_.find(a);
    if (it == index_.end()) return "unknown device ID: " + a;
    if (seen.insert(it->second).second) avail_idx->push_back(it->second);
  }
  std::unordered_set<int> rseen;
  for (auto& r : required) {
    auto it = index_.find(r);
    if (it == index_.end()) return "unknown device ID: " + r;
    if (rseen.insert(it->second).second) req_idx->push_back(it->second);
  }
  return "";
}

std::vector<std::vector<int>> HiveAllocator::filtered_groups(const std::vector<int>& avail_idx,
                                                             const std::vector<int>& req_idx) const {
  std::vector<char> is_av(devs_.size(), 0), is_req(devs_.size(), 0);
  for (int i : avail_idx) is_av[i] = 1;
  for (int i : req_idx) is_req[i] = 1;
  struct FG {
    const Group* g;
    std::vector<int> m;
  };
  std::vector<FG> fgs;
  for (auto& g : groups_) {
    FG f{&g, {}};
    for (int m : g.members)
      if (is_av[m] && !is_req[m]) f.m.push_back(m);
    if (!f.m.empty()) fgs.push_back(std::move(f));
  }
  // anti-fragmentation order: fewest free partitions first, then parent ID
  // (reference filterPartitions, device.go:339-349); unique_id breaks the
  // remaining ties deterministically.
  std::stable_sort(fgs.begin(), fgs.end(), [](const FG& a, const FG& b) {
    if (a.m.size() != b.m.size()) return a.m.size() < b.m.size();
    if (a.g->parent_id != b.g->parent_id) return a.g->parent_id < b.g->parent_id;
    return a.g->key < b.g->key;
  });
  std::vector<std::vector<int>> out;
  out.reserve(fgs.size());
  for (auto& f : fgs) out.push_back(std::move(f.m));
  return out;
}

AllocResult HiveAllocator::allocate(const std::vector<std::string>& available,
                                    const std::vector<std::string>& required, int size) const {
  AllocResult res;
  std::vector<int> avail_idx, req_idx;
  res.error = validate(available, required, size, &res, &avail_idx, &req_idx);
  if (!res.error.empty() || res.short_circuit) return res;
  if (opt_.extended_search && allocate_extended(avail_idx, req_idx, size, &res)) return res;

  const size_t n = devs_.size();
  auto W = [&](int a, int b) { return static_cast<int64_t>(w_[static_cast<size_t>(a) * n + b]); };
  const auto fg = filtered_groups(avail_idx, req_idx);
  const int G = static_cast<int>(fg.size());
  const int need = size - static_cast<int>(req_idx.size());
  int maxc = 0;
  for (auto& g : fg) maxc = std::max(maxc, static_cast<int>(g.size()));
  const int R = maxc + 1;

  // Aggregates. P[g][r]: internal weight of the first r members of g.
  // Q[p][r]: weight between the first r members of p and the required set.
  // C[(p*G+g)*R + r]: weight between the first r members of p and all of g,
  // filled lazily per (p, g) row: requests that fit inside one GPU never
  // touch it, which keeps small CPX requests at O(partitions^2).
  std::vector<int64_t> P(static_cast<size_t>(G) * R, 0), Q(static_cast<size_t>(G) * R, 0);
  for (int p = 0; p < G; ++p) {
    const auto& mp = fg[p];
    for (int r = 1; r <= static_cast<int>(mp.size()); ++r) {
      int64_t add = 0, radd = 0;
      for (int i = 0; i < r - 1; ++i) add += W(mp[i], mp[r - 1]);
      for (int q : req_idx) radd += W(mp[r - 1], q);
      P[p * R + r] = P[p * R + r - 1] + add;
      Q[p * R + r] = Q[p * R + r - 1] + radd;
    }
  }
  std::vector<int64_t> C;
  std::vector<char> c_ready;
  auto cross = [&](int p, int g, int r) -> int64_t {
    if (C.empty()) {
      C.assign(static_cast<size_t>(G) * G * R, 0);
      c_ready.assign(static_cast<size_t>(G) * G, 0);
    }
    const size_t row = static_cast<size_t>(p) * G + g;
    if (!c_ready[row]) {
      const auto& mp = fg[p];
      for (int rr = 1; rr <= static_cast<int>(mp.size()); ++rr) {
        int64_t c = 0;
        for (int m : fg[g]) c += W(mp[rr - 1], m);
        C[row * R + rr] = C[row * R + rr - 1] + c;
      }
      c_ready[row] = 1;
    }
    return C[row * R + r];
  };
  int64_t RR = 0;
  for (size_t i = 0; i < req_idx.size(); ++i)
    for (size_t j = i + 1; j < req_idx.size(); ++j) RR += W(req_idx[i], req_idx[j]);

  struct Best {
    bool found = false;
    int64_t w = std::numeric_limits<int64_t>::max();
    int level = 0;
    std::vector<int> seq;
    int partial = -1;  // group whose prefix is taken, -1 = all full
    int take = 0;
  } best;

  std::vector<int> S;
  std::vector<int> seq;
  std::vector<char> inS(G, 0);
  uint64_t cands = 0;

  // depth-first over sets of whole GPUs (strictly increasing group index)
  auto dfs = [&](auto&& self, int start, int64_t fw, int cnt) -> void {
    if (best.found && fw + RR > best.w) return;  // all weights are >= 0
    const int r = need - cnt;
    for (int p = 0; p < G; ++p) {
      const int cp = static_cast<int>(fg[p].size());
      if (inS[p] || cp < r) continue;
      int64_t w = fw + RR + P[p * R + r] + Q[p * R + r];
      for (int g : S) w += cross(p, g, r);
      ++cands;
      if (best.found && w > best.w) continue;
      const int level = static_cast<int>(S.size()) + 1;
      seq.assign(S.begin(), S.end());
      bool exact = (cp == r);
      if (exact) {
        seq.insert(std::upper_bound(seq.begin(), seq.end(), p), p);
      } else {
        seq.push_back(p);
      }
      bool better = !best.found || w < best.w || (w == best.w && level < best.level) ||
                    (w == best.w && level == best.level && seq < best.seq);
      if (better) {
        best.found = true;
        best.w = w;
        best.level = level;
        best.seq = seq;
        best.partial = exact ? -1 : p;
        best.take = r;
      }
    }
    for (int g = start; g < G; ++g) {
      const int cg = static_cast<int>(fg[g].size());
      if (cnt + cg >= need) continue;
      int64_t nfw = fw + P[g * R + cg] + Q[g * R + cg];
      for (int h : S) nfw += cross(g, h, cg);
      S.push_back(g);
      inS[g] = 1;
      self(self, g + 1, nfw, cnt + cg);
      inS[g] = 0;
      S.pop_back();
    }
  };
  dfs(dfs, 0, 0, 0);
  res.candidates = cands;
  if (!best.found) {
    res.error = kNoCandidate;
    return res;
  }
  res.weight = best.w;
  for (int g : best.seq) {
    int take = (g == best.partial) ? best.take : static_cast<int>(fg[g].size());
    for (int i = 0; i < take; ++i) res.ids.push_back(devs_[fg[g][i]].id);
  }
  for (int q : req_idx) res.ids.push_back(devs_[q].id);
  return res;
}

bool HiveAllocator::allocate_extended(const std::vector<int>& avail_idx, const std::vector<int>& req_idx, int size,
                                      AllocResult* out) const {
  const size_t n = devs_.size();
  auto at = [&](int a, int b) { return static_cast<size_t>(a) * n + b; };
  const auto fg = filtered_groups(avail_idx, req_idx);
  const int need = size - static_cast<int>(req_idx.size());
  // the free devices in anti-fragmentation order (fg: fewest free first)
  std::vector<int> pool, pool_group;
  for (size_t g = 0; g < fg.size(); ++g)
    for (int m : fg[g]) {
      pool.push_back(m);
      pool_group.push_back(dev_group_[m]);  // physical GPU
    }
  std::vector<int> cand = pool;  // every device a chosen set can contain
  cand.insert(cand.end(), req_idx.begin(), req_idx.end());

  // classes of interchangeable free devices: same GPU and identical weights
  // and kfd link figures to every other device a set can contain
  auto same_row = [&](int a, int b) {
    for (int x : cand) {
      if (x == a || x == b) continue;
      if (w_[at(a, x)] != w_[at(b, x)] || link_kw_[at(a, x)] != link_kw_[at(b, x)] ||
          link_bw_[at(a, x)] != link_bw_[at(b, x)])
        return false;
    }
    return true;
  };
  struct Class {
    int group;
    std::vector<int> members;  // pool order
  };
  // equal figures of a and b towards x (one of the columns same_row compares)
  auto same_col = [&](int a, int b, int x) {
    return w_[at(a, x)] == w_[at(b, x)] && link_kw_[at(a, x)] == link_kw_[at(b, x)] &&
           link_bw_[at(a, x)] == link_bw_[at(b, x)];
  };
  std::vector<Class> cls;
  for (size_t i = 0; i < pool.size(); ++i) {
    int found = -1;
    for (size_t c = 0; c < cls.size() && found < 0; ++c)
      if (cls[c].group == pool_group[i] && same_row(cls[c].members[0], pool[i])) {
        // the new device matches every member m: rows of m and of the first member
        // agree off {first, m}, the new row agrees with the first off {first, new},
        // so only the first member's own column is left to compare
        const int f = cls[c].members[0];
        bool all = true;
        for (size_t k2 = 1; k2 < cls[c].members.size() && all; ++k2) all = same_col(cls[c].members[k2], pool[i], f);
        if (all) found = static_cast<int>(c);
      }
    if (found < 0) {
      cls.push_back(Class{pool_group[i], {pool[i]}});
    } else {
      cls[found].members.push_back(pool[i]);
    }
  }
  // Explore the largest classes first: sets that keep to few, full GPUs have the
  // most cheap intra-GPU pairs, so the first leaves are near the optimum and the
  // bound prunes early; classes of one size also become neighbours for the
  // symmetry rule below. (The order of exploration decides nothing: ties are
  // broken on the chosen devices' pool positions, fewest-free GPUs first.)
  std::stable_sort(cls.begin(), cls.end(),
                   [](const Class& a, const Class& b) { return a.members.size() > b.members.size(); });
  const int K = static_cast<int>(cls.size());
  // class-level aggregates
  std::vector<int64_t> wi(K, 0), wr(K, 0), kwr(K, 0), bwr(K, 0);
  std::vector<int64_t> wc(static_cast<size_t>(K) * K, 0), kwc(static_cast<size_t>(K) * K, 0),
      bwc(static_cast<size_t>(K) * K, 0);
  for (int c = 0; c < K; ++c) {
    const int a = cls[c].members[0];
    if (cls[c].members.size() > 1) wi[c] = w_[at(a, cls[c].members[1])];
    for (int q : req_idx) {
      wr[c] += w_[at(a, q)];
      kwr[c] += link_kw_[at(a, q)];
      bwr[c] += link_bw_[at(a, q)];
    }
    for (int d = 0; d < K; ++d) {
      if (d == c) continue;
      const int b = cls[d].members[0];
      wc[static_cast<size_t>(c) * K + d] = w_[at(a, b)];
      kwc[static_cast<size_t>(c) * K + d] = link_kw_[at(a, b)];
      bwc[static_cast<size_t>(c) * K + d] = link_bw_[at(a, b)];
    }
  }
  int64_t RR = 0;
  std::vector<char> req_group(groups_.size(), 0);
  for (size_t i = 0; i < req_idx.size(); ++i) {
    req_group[dev_group_[req_idx[i]]] = 1;
    for (size_t j = i + 1; j < req_idx.size(); ++j) RR += w_[at(req_idx[i], req_idx[j])];
  }
  std::vector<int> suffix_cap(K + 1, 0);
  for (int c = K - 1; c >= 0; --c) suffix_cap[c] = suffix_cap[c + 1] + static_cast<int>(cls[c].members.size());
  // For the lower bound on the pairs among the devices still to choose from
  // classes c..: the smallest weight of a pair inside one class and of a pair
  // across two classes, and the class sizes largest first. With intra-class
  // pairs the cheaper kind (partitions of one GPU), m devices have at most
  // P(m) = sum t_i (t_i - 1) / 2 intra pairs, t_i filling the largest classes
  // first; the rest of the m (m - 1) / 2 pairs cross classes.
  constexpr int64_t kInf = std::numeric_limits<int64_t>::max() / 4;
  std::vector<int64_t> wmin_intra(K + 1, kInf), wmin_cross(K + 1, kInf);
  for (int c = K - 1; c >= 0; --c) {
    wmin_intra[c] = wmin_intra[c + 1];
    if (cls[c].members.size() > 1) wmin_intra[c] = std::min(wmin_intra[c], wi[c]);
    wmin_cross[c] = wmin_cross[c + 1];
    for (int d = c + 1; d < K; ++d) wmin_cross[c] = std::min(wmin_cross[c], wc[static_cast<size_t>(c) * K + d]);
  }
  auto pair_bound = [&](int c, int m) -> int64_t {
    const int64_t pairs = static_cast<int64_t>(m) * (m - 1) / 2;
    if (pairs == 0) return 0;
    const int64_t wa = wmin_intra[c], wx = wmin_cross[c];
    if (wa >= wx) return pairs * wx;  // crossing is never dearer: every pair at the cross minimum
    int64_t intra = 0;
    int left = m;
    for (int d = c; d < K && left; ++d) {  // classes are in size order, largest first
      const int t = std::min<int>(left, static_cast<int>(cls[d].members.size()));
      intra += static_cast<int64_t>(t) * (t - 1) / 2;
      left -= t;
    }
    return intra * wa + (pairs - intra) * (wx >= kInf ? wa : wx);
  };
  // symmetry: class c is interchangeable with c-1 (same size, same weights and
  // link figures to everything else). Taking no more from c than from c-1
  // loses no optimum: the tie-break prefers earlier pool positions anyway.
  std::vector<char> sym_prev(K, 0);
  for (int c = 1; c < K; ++c) {
    const int b = c - 1;
    bool same = cls[c].members.size() == cls[b].members.size() && wi[c] == wi[b] && wr[c] == wr[b] &&
                kwr[c] == kwr[b] && bwr[c] == bwr[b];
    for (int d = 0; d < K && same; ++d) {
      if (d == b || d == c) continue;
      same = wc[static_cast<size_t>(c) * K + d] == wc[static_cast<size_t>(b) * K + d] &&
             kwc[static_cast<size_t>(c) * K + d] == kwc[static_cast<size_t>(b) * K + d] &&
             bwc[static_cast<size_t>(c) * K + d] == bwc[static_cast<size_t>(b) * K + d];
    }
    sym_prev[c] = same;
  }
  std::vector<std::pair<int64_t, int>> unit;  // scratch for the bound
  unit.reserve(K);
  // fewest GPUs not yet in the set that classes c.. must add to supply m more
  // devices (the GPUs already used supply what they can first)
  std::vector<int> group_uses(groups_.size(), 0);
  std::vector<int> new_cap(groups_.size(), 0), caps;
  caps.reserve(groups_.size());
  auto new_gpus_needed = [&](int c, int m) -> int {
    int left = m;
    std::fill(new_cap.begin(), new_cap.end(), 0);
    for (int d = c; d < K; ++d) {
      const int g = cls[d].group, sz = static_cast<int>(cls[d].members.size());
      if (group_uses[g]) left -= sz;
      else new_cap[g] += sz;
    }
    if (left <= 0) return 0;
    caps.clear();
    for (int v : new_cap)
      if (v) caps.push_back(v);
    std::sort(caps.rbegin(), caps.rend());
    int t = 0;
    for (int v : caps) {
      ++t;
      if ((left -= v) <= 0) break;
    }
    return t;
  };

  struct Key {
    int64_t w = std::numeric_limits<int64_t>::max();
    int gpus = 0;
    int64_t kw = 0;   // lower better
    int64_t bw = 0;   // higher better
    std::vector<int> picks;  // pool positions of the chosen devices (sorted): anti-fragmentation order
  } best;
  bool found = false;
  std::vector<int> k(K, 0);
  for (int q : req_idx) group_uses[dev_group_[q]]++;
  uint64_t nodes = 0, leaves = 0;
  bool aborted = false;
  std::vector<int> pos_in_pool(n, -1);
  for (size_t i = 0; i < pool.size(); ++i) pos_in_pool[pool[i]] = static_cast<int>(i);

  // w: weight of the chosen free devices among themselves and with the required set
  auto dfs = [&](auto&& self, int c, int cnt, int64_t w, int64_t kw, int64_t bw, int gpus) -> void {
    if (aborted) return;
    if (++nodes > opt_.extended_node_limit) {
      aborted = true;
      return;
    }
    const int m = need - cnt;
    if (m == 0) {
      ++leaves;
      const int64_t total = w + RR;
      Key key;
      key.w = total;
      key.gpus = gpus;
      key.kw = kw;
      key.bw = bw;
      for (int d = 0; d < K; ++d)
        for (int i = 0; i < k[d]; ++i) key.picks.push_back(pos_in_pool[cls[d].members[i]]);
      std::sort(key.picks.begin(), key.picks.end());
      bool better = !found || key.w < best.w ||
                    (key.w == best.w &&
                     (key.gpus < best.gpus ||
                      (key.gpus == best.gpus &&
                       (key.kw < best.kw || (key.kw == best.kw && (key.bw > best.bw ||
                                                                  (key.bw == best.bw && key.picks < best.picks)))))));
      if (better) {
        best = std::move(key);
        found = true;
      }
      return;
    }
    if (c >= K || suffix_cap[c] < m) return;
    if (found) {
      // lower bound: the m cheapest attachments to what is chosen (per class,
      // up to its size) plus the pairs among the m new devices (pair_bound)
      unit.clear();
      for (int d = c; d < K; ++d) {
        int64_t a = wr[d];
        for (int e = 0; e < c; ++e)
          if (k[e]) a += static_cast<int64_t>(k[e]) * wc[static_cast<size_t>(d) * K + e];
        unit.emplace_back(a, static_cast<int>(cls[d].members.size()));
      }
      std::sort(unit.begin(), unit.end());
      int64_t lb = 0;
      int left = m;
      for (auto& [a, cap] : unit) {
        const int t = std::min(left, cap);
        lb += a * t;
        left -= t;
        if (!left) break;
      }
      lb += pair_bound(c, m);
      if (w + RR + lb > best.w) return;
      if (w + RR + lb == best.w && gpus + new_gpus_needed(c, m) > best.gpus) return;  // can only tie, on more GPUs
    }
    int cap = std::min<int>(m, static_cast<int>(cls[c].members.size()));
    if (c > 0 && sym_prev[c]) cap = std::min(cap, k[c - 1]);
    for (int take = cap; take >= 0; --take) {
      int64_t dw = static_cast<int64_t>(take) * (take - 1) / 2 * wi[c] + take * wr[c];
      int64_t dkw = take * kwr[c], dbw = take * bwr[c];
      for (int d = 0; d < c; ++d) {
        if (!k[d]) continue;
        dw += static_cast<int64_t>(take) * k[d] * wc[static_cast<size_t>(c) * K + d];
        if (cls[d].group != cls[c].group) {
          dkw += static_cast<int64_t>(take) * k[d] * kwc[static_cast<size_t>(c) * K + d];
          dbw += static_cast<int64_t>(take) * k[d] * bwc[static_cast<size_t>(c) * K + d];
        }
      }
      const int g = cls[c].group;
      const bool new_gpu = take > 0 && group_uses[g] == 0;
      k[c] = take;
      group_uses[g] += take;
      self(self, c + 1, cnt + take, w + dw, kw + dkw, bw + dbw, gpus + (new_gpu ? 1 : 0));
      group_uses[g] -= take;
      k[c] = 0;
      if (aborted) return;
    }
  };
  int req_gpus = 0;
  for (char r : req_group) req_gpus += r;
  dfs(dfs, 0, 0, 0, 0, 0, req_gpus);
  if (aborted) return false;
  out->candidates = leaves;
  if (!found) {
    out->error = kNoCandidate;
    return true;
  }
  out->weight = best.w;
  for (int p : best.picks) out->ids.push_back(devs_[pool[p]].id);
  for (int q : req_idx) out->ids.push_back(devs_[q].id);
  return true;
}

AllocResult HiveAllocator::reference_allocate(const std::vector<std::string>& available,
                                              const std::vector<std::string>& required, int size) const {
  AllocResult res;
  std::vector<int> avail_idx, req_idx;
  res.error = validate(available, required, size, &res, &avail_idx, &req_idx);
  if (!res.error.empty() || res.short_circuit) return res;

  const size_t n = devs_.size();
  const auto fg = filtered_groups(avail_idx, req_idx);
  const int G = static_cast<int>(fg.size());
  const int need = size - static_cast<int>(req_idx.size());

  struct Cand {
    std::vector<int> ids;
    std::vector<int> parents;
    int64_t w = 0;
  };
  auto add = [&](Cand& c, int dev) {
    for (int d : c.ids) c.w += w_[static_cast<size_t>(d) * n + dev];
    c.ids.push_back(dev);
  };
  auto finish = [&](Cand& c) {
    for (int q : req_idx) add(c, q);
  };

  std::vector<Cand> finals;
  std::deque<Cand> temp;
  for (int idx = 0; idx < G; ++idx) {
    Cand c;
    c.parents = {idx};
    add(c, fg[idx][0]);
    if (need == 1) {
      finish(c);
      finals.push_back(std::move(c));
      continue;
    }
    bool done = false;
    for (size_t i = 1; i < fg[idx].size(); ++i) {
      add(c, fg[idx][i]);
      if (static_cast<int>(i) == need - 1) {
        done = true;
        break;
      }
    }
    if (done) {
      finish(c);
      finals.push_back(std::move(c));
    } else {
      temp.push_back(std::move(c));
    }
  }
  while (!temp.empty()) {
    Cand cur = std::move(temp.front());
    temp.pop_front();
    if (static_cast<int>(cur.parents.size()) == G) continue;
    for (int idx = 0; idx < G; ++idx) {
      if (std::find(cur.parents.begin(), cur.parents.end(), idx) != cur.parents.end()) continue;
      Cand c = cur;
      c.parents.push_back(idx);
      bool done = false;
      for (int d : fg[idx]) {
        add(c, d);
        if (static_cast<int>(c.ids.size()) == need) {
          finish(c);
          finals.push_back(c);
          done = true;
          break;
        }
      }
      if (!done && static_cast<int>(c.ids.size()) < need) temp.push_back(std::move(c));
    }
  }
  res.candidates = finals.size();
  const Cand* best = nullptr;
  for (auto& c : finals)
    if (!best || c.w < best->w) best = &c;
  if (!best) {
    res.error = kNoCandidate;
    return res;
  }
  res.weight = best->w;
  for (int d : best->ids) res.ids.push_back(devs_[d].id);
  return res;
}

}  // namespace mi355x
