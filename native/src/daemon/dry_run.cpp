#include "dry_run.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <set>

#include "mi355x/constants.h"
#include "../kube/json.h"

namespace mi355x::daemon {
namespace {

json::Value jnum(double v) {
  json::Value x;
  x.kind = json::Value::Number;
  char b[64];
  if (v == static_cast<double>(static_cast<long long>(v)) && std::fabs(v) < 1e15)
    std::snprintf(b, sizeof(b), "%lld", static_cast<long long>(v));
  else
    std::snprintf(b, sizeof(b), "%.17g", v);
  x.s = b;
  return x;
}
json::Value jbool(bool v) {
  json::Value x;
  x.kind = json::Value::Bool;
  x.b = v;
  return x;
}
json::Value jarr() {
  json::Value x;
  x.kind = json::Value::Array;
  return x;
}
json::Value jnull() { return json::Value{}; }

int model_xgmi_link_mbps(int device_id, int gfx) {  // models/gpu.py xgmi_link_mbps
  switch (device_id) {
    case 0x75a3: case 0x75b3: return 76000;  // MI355X (measured)
    case 0x74a1: case 0x74a2: return 64000;  // MI300X / MI308X
    case 0x740f: return 50000;               // MI210
  }
  switch (gfx) {
    case 90500: return 76000;
    case 90402: return 64000;
    case 90010: return 50000;
  }
  return 0;
}

}  // namespace

FabricReport fabric_report(const std::vector<const GpuDevice*>& devs, const KfdTopology& topo) {
  std::map<std::pair<int, int>, std::pair<int, int64_t>> links;  // io_links win over p2p_links
  for (const KfdNode* n : topo.gpu_nodes()) {
    for (const auto& l : n->p2p_links) links[{l.node_from, l.node_to}] = {l.type, l.max_bandwidth};
    for (const auto& l : n->io_links) links[{l.node_from, l.node_to}] = {l.type, l.max_bandwidth};
  }
  auto link = [&](const GpuDevice* a, const GpuDevice* b) -> std::pair<std::string, int64_t> {
    if (!a->unique_id.empty() && a->unique_id == b->unique_id) return {"same_gpu", 0};
    auto it = links.find({a->node_id, b->node_id});
    if (it == links.end()) it = links.find({b->node_id, a->node_id});
    if (it == links.end()) return {"unknown", 0};
    int64_t bw = it->second.second;
    if (it->second.first == kLinkXgmi) {
      if (bw <= 0) bw = model_xgmi_link_mbps(a->pci_device_id, a->gfx_target_version);
      return {"xgmi", bw};
    }
    if (it->second.first == kLinkPcie) return {"pcie", bw};
    return {"unknown", bw};
  };
  FabricReport rep;
  std::vector<const GpuDevice*> reps;
  std::set<std::string> seen;
  std::set<uint64_t> hives;
  for (const GpuDevice* d : devs) {
    hives.insert(d->hive_id);
    if (seen.insert(!d->unique_id.empty() ? d->unique_id : d->bdf).second) reps.push_back(d);
  }
  rep.one_hive = hives.size() == 1 && !hives.count(0);
  if (reps.size() <= 1) return rep;
  int64_t egress_min = -1;
  std::vector<std::pair<std::string, int64_t>> slow;
  for (const GpuDevice* a : reps) {
    int64_t eg = 0;
    for (const GpuDevice* b : reps) {
      if (a == b) continue;
      const auto [cls, bw] = link(a, b);
      if (cls == "xgmi") eg += bw;
      else slow.emplace_back(cls, bw);
    }
    egress_min = egress_min < 0 ? eg : std::min(egress_min, eg);
  }
  if (slow.empty() && egress_min > 0) {
    rep.has_bound = true;
    rep.bound_gbs = static_cast<double>(egress_min) / 1000.0;
  } else if (std::any_of(slow.begin(), slow.end(), [](const auto& x) { return x.first == "unknown"; })) {
    // no bound without kfd links
  } else if (!slow.empty()) {
    int64_t mn = -1;
    for (const auto& [c, bw] : slow)
      if (bw > 0) mn = mn < 0 ? bw : std::min(mn, bw);
    if (mn > 0) {
      rep.has_bound = true;
      rep.bound_gbs = static_cast<double>(mn) / 1000.0;
    }
  }
  return rep;
}

std::string dry_run_report(const Flags& f, bool impl_ok, Driver driver, const std::vector<Resource>& resources,
                           const KfdTopology& topo, const std::vector<std::string>& warnings,
                           const health::Engine* engine) {
  json::Value out = json::Value::object();
  out.set("implementation", impl_ok ? json::Value::string(driver_name(driver)) : jnull());
  json::Value res = json::Value::object();
  for (const auto& r : resources) {
    json::Value rv = json::Value::object();
    json::Value devs = jarr();
    std::vector<std::string> ids;
    auto health_of = [&](const std::string& id) {
      auto it = r.health.find(id);
      return json::Value::string(it == r.health.end() || it->second ? "Healthy" : "Unhealthy");
    };
    for (const auto& g : r.group_ids) {
      json::Value d = json::Value::object();
      d.set("id", json::Value::string(g));
      d.set("health", health_of(g));
      d.set("numa", jarr());
      devs.arr.push_back(d);
      ids.push_back(g);
    }
    std::map<std::string, const GpuDevice*> by_id;
    for (const auto& gd : r.devices) {
      json::Value d = json::Value::object();
      d.set("id", json::Value::string(gd.id));
      d.set("health", health_of(gd.id));
      json::Value numa = jarr();
      if (gd.numa_node >= 0) numa.arr.push_back(jnum(gd.numa_node));
      d.set("numa", numa);
      devs.arr.push_back(d);
      ids.push_back(gd.id);
      by_id[gd.id] = &gd;
    }
    rv.set("devices", devs);
    rv.set("preferred_allocation", jbool(r.allocator != nullptr));
    if (r.allocator && !ids.empty()) {
      json::Value prefs = json::Value::object();
      std::set<int> ks = {1, 2, 4, 8, static_cast<int>(ids.size())};
      for (int k : ks) {
        if (k < 1 || k > static_cast<int>(ids.size())) continue;
        const AllocResult a = r.allocator->allocate(ids, {}, k);
        json::Value pv = json::Value::object();
        json::Value chosen = jarr();
        std::vector<const GpuDevice*> set;
        for (const auto& id : a.ids) {
          chosen.arr.push_back(json::Value::string(id));
          if (by_id.count(id)) set.push_back(by_id[id]);
        }
        pv.set("ids", chosen);
        if (driver == Driver::Container) {
          const FabricReport fr = fabric_report(set, topo);
          pv.set("one_hive", jbool(fr.one_hive));
          pv.set("allreduce_bound_gbs", fr.has_bound ? jnum(fr.bound_gbs) : jnull());
        }
        prefs.set(std::to_string(k), pv);
      }
      rv.set("allocations", prefs);
    }
    res.set(std::string(kResourceNamespace) + "/" + r.name, rv);
  }
  out.set("resources", res);
  if (driver == Driver::Container && impl_ok) {
    json::Value w = jarr();
    for (const auto& x : warnings) w.arr.push_back(json::Value::string(x));
    out.set("warnings", w);
    json::Value ls = jarr();
    for (const auto& x : f.lists.order) ls.arr.push_back(json::Value::string(x));
    out.set("device_list_strategy", ls);
    if (f.lists.cdi()) out.set("cdi_spec_dir", json::Value::string(f.cdi_spec_dir));
  }
  if (engine && f.smi_xgmi) {
    json::Value x = json::Value::object();
    x.set("readings", jnum(static_cast<double>(engine->xgmi_readings())));
    x.set("error", json::Value::string(engine->xgmi_error()));
    json::Value pairs = jarr();
    for (const auto& [a, b] : engine->degraded_links()) {
      json::Value pr = jarr();
      pr.arr.push_back(json::Value::string(a));
      pr.arr.push_back(json::Value::string(b));
      pairs.arr.push_back(pr);
    }
    x.set("degraded_pairs", pairs);
    json::Value down = json::Value::object();
    for (const auto& [bdf, n] : engine->links_down()) down.set(bdf, jnum(n));
    x.set("links_down", down);
    out.set("xgmi", x);
  }
  if (engine && !engine->perf_last().empty()) {
    const auto verdicts = engine->perf_verdicts();
    json::Value thr = json::Value::object();
    for (const auto& [dev, o] : engine->perf_last()) {
      json::Value t = json::Value::object();
      auto v = verdicts.find(dev);
      t.set("state", json::Value::string(v == verdicts.end() ? "ok" : v->second.first));
      t.set("reason", json::Value::string(v == verdicts.end() ? "" : v->second.second));
      for (const char* k : {"hbm_write_gbps", "hbm_read_gbps", "hbm_bad_words", "mfma_tflops", "clock_mhz_median"})
        if (auto d = o.detail.find(k); d != o.detail.end()) t.set(k, jnum(d->second));
      if (!o.xcd_clock_mhz.empty()) {
        json::Value xs = jarr();
        for (double c : o.xcd_clock_mhz) xs.arr.push_back(jnum(c));
        t.set("xcd_clock_mhz", xs);
      }
      if (auto d = o.detail.find("total_us"); d != o.detail.end()) t.set("total_us", jnum(d->second));
      thr.set(dev, t);
    }
    out.set("throughput", thr);
  }
  return json::serialize(out);
}

}  // namespace mi355x::daemon
