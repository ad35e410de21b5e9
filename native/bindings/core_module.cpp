// pybind11 bindings for the native core (_native).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "mi355x/allocator.h"
#include "mi355x/constants.h"
#include "mi355x/dir_watch.h"
#include "mi355x/drm_query.h"
#include "mi355x/gpu_discovery.h"
#include "mi355x/kfd_topology.h"
#include "mi355x/pci_scan.h"
#include "mi355x/smi_query.h"
#include "mi355x/sysfs.h"
#include "../src/kube/json.h"
#include "../src/kube/yaml.h"

namespace py = pybind11;
using namespace mi355x;

void bind_rpc(py::module_& m);     // rpc_module.cpp
void bind_health(py::module_& m);  // health_module.cpp

namespace {

py::dict link_to_dict(const KfdLink& l) {
  py::dict d;
  d["type"] = l.type;
  d["node_from"] = l.node_from;
  d["node_to"] = l.node_to;
  d["weight"] = l.weight;
  d["min_bandwidth"] = l.min_bandwidth;
  d["max_bandwidth"] = l.max_bandwidth;
  d["flags"] = l.flags;
  d["p2p"] = l.p2p;
  return d;
}

py::dict alloc_result(const AllocResult& r) {
  py::dict d;
  d["ids"] = r.ids;
  d["error"] = r.error;
  d["weight"] = r.weight;
  d["candidates"] = r.candidates;
  d["short_circuit"] = r.short_circuit;
  return d;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X device-plugin native core: kfd topology, discovery, allocator, PCI, drm, amd-smi";
  m.attr("GFX950_TARGET_VERSION") = kGfx950TargetVersion;
  m.attr("LINK_XGMI") = static_cast<int>(kLinkXgmi);
  m.attr("LINK_PCIE") = static_cast<int>(kLinkPcie);

  m.def("parse_kv_file", [](const std::string& p) -> py::object {
    auto kv = parse_kv_file(p);
    if (!kv) return py::none();
    py::dict d;
    for (auto& [k, v] : *kv) d[py::str(k)] = v;
    return d;
  });

  py::class_<KfdNode>(m, "KfdNode")
      .def_readonly("id", &KfdNode::id)
      .def_readonly("name", &KfdNode::name)
      .def_readonly("gpu_id", &KfdNode::gpu_id)
      .def_property_readonly("props", [](const KfdNode& n) {
        py::dict d;
        for (auto& [k, v] : n.props) d[py::str(k)] = v;
        return d;
      })
      .def("prop", &KfdNode::prop, py::arg("key"), py::arg("fallback") = 0)
      .def("prop_str", &KfdNode::prop_str)
      .def_property_readonly("io_links", [](const KfdNode& n) {
        py::list l;
        for (auto& x : n.io_links) l.append(link_to_dict(x));
        return l;
      })
      .def_property_readonly("p2p_links", [](const KfdNode& n) {
        py::list l;
        for (auto& x : n.p2p_links) l.append(link_to_dict(x));
        return l;
      })
      .def_property_readonly("mem_bank_sizes", [](const KfdNode& n) {
        std::vector<uint64_t> v;
        for (auto& b : n.mem_banks) v.push_back(b.size_in_bytes);
        return v;
      })
      .def_property_readonly("cpu_cores_count", &KfdNode::cpu_cores_count)
      .def_property_readonly("simd_count", &KfdNode::simd_count)
      .def_property_readonly("simd_per_cu", &KfdNode::simd_per_cu)
      .def_property_readonly("gfx_target_version", &KfdNode::gfx_target_version)
      .def_property_readonly("drm_render_minor", &KfdNode::drm_render_minor)
      .def_property_readonly("num_xcc", &KfdNode::num_xcc)
      .def_property_readonly("device_id", &KfdNode::device_id)
      .def_property_readonly("location_id", &KfdNode::location_id)
      .def_property_readonly("domain", &KfdNode::domain)
      .def_property_readonly("hive_id", &KfdNode::hive_id)
      .def_property_readonly("unique_id", &KfdNode::unique_id)
      .def_property_readonly("local_mem_bytes", &KfdNode::local_mem_bytes)
      .def_property_readonly("is_gpu", &KfdNode::is_gpu)
      .def_property_readonly("is_live_gpu", &KfdNode::is_live_gpu);

  py::class_<KfdTopology>(m, "KfdTopology")
      .def_static("load", &KfdTopology::load, py::arg("nodes_dir"))
      .def_static("load_sysfs", &KfdTopology::load_sysfs, py::arg("sysfs_root") = "/sys")
      .def_property_readonly("nodes", [](const KfdTopology& t) { return t.nodes(); })
      .def_property_readonly("nodes_dir", &KfdTopology::nodes_dir)
      .def("node", [](const KfdTopology& t, int id) -> py::object {
        const KfdNode* n = t.node(id);
        return n ? py::cast(*n) : py::none();
      })
      .def("render_to_unique_id", &KfdTopology::render_to_unique_id)
      .def("render_to_node_id", &KfdTopology::render_to_node_id)
      .def("gpu_node_ids", [](const KfdTopology& t) {
        std::vector<int> ids;
        for (auto* n : t.gpu_nodes()) ids.push_back(n->id);
        return ids;
      })
      .def("count_gpu_nodes", &KfdTopology::count_gpu_nodes)
      .def("unreadable_node_ids", &KfdTopology::unreadable_node_ids)
      .def("any_live_gpu", &KfdTopology::any_live_gpu)
      .def("all_gpu_links", [](const KfdTopology& t) {
        py::list l;
        for (auto& x : t.all_gpu_links()) l.append(link_to_dict(x));
        return l;
      });

  py::class_<GpuDevice>(m, "GpuDevice")
      .def(py::init<>())
      .def_readwrite("id", &GpuDevice::id)
      .def_readwrite("bdf", &GpuDevice::bdf)
      .def_readwrite("is_partition", &GpuDevice::is_partition)
      .def_readwrite("xcp_index", &GpuDevice::xcp_index)
      .def_readwrite("card", &GpuDevice::card)
      .def_readwrite("render_minor", &GpuDevice::render_minor)
      .def_readwrite("unique_id", &GpuDevice::unique_id)
      .def_readwrite("compute_partition", &GpuDevice::compute_partition)
      .def_readwrite("memory_partition", &GpuDevice::memory_partition)
      .def_readwrite("numa_node", &GpuDevice::numa_node)
      .def_readwrite("node_id", &GpuDevice::node_id)
      .def_readwrite("gfx_target_version", &GpuDevice::gfx_target_version)
      .def_readwrite("simd_count", &GpuDevice::simd_count)
      .def_readwrite("simd_per_cu", &GpuDevice::simd_per_cu)
      .def_readwrite("num_xcc", &GpuDevice::num_xcc)
      .def_readwrite("pci_device_id", &GpuDevice::pci_device_id)
      .def_readwrite("location_id", &GpuDevice::location_id)
      .def_readwrite("domain", &GpuDevice::domain)
      .def_readwrite("hive_id", &GpuDevice::hive_id)
      .def_readwrite("vram_bytes", &GpuDevice::vram_bytes)
      .def_readwrite("identity", &GpuDevice::identity)
      .def_property_readonly("partition_type", &GpuDevice::partition_type)
      .def_property_readonly("cu_count", &GpuDevice::cu_count);

  py::class_<DiscoveryResult>(m, "DiscoveryResult")
      .def_readonly("devices", &DiscoveryResult::devices)
      .def_readonly("driver_loaded", &DiscoveryResult::driver_loaded)
      .def_readonly("kfd_present", &DiscoveryResult::kfd_present)
      .def_readonly("warnings", &DiscoveryResult::warnings)
      .def_readonly("kfd_unreadable_nodes", &DiscoveryResult::kfd_unreadable_nodes)
      .def_readonly("recovered_devices", &DiscoveryResult::recovered_devices)
      .def_readonly("unresolved", &DiscoveryResult::unresolved);
  m.def("partitions_for_mode", &partitions_for_mode, py::arg("mode"), py::arg("total_xcc"));
  m.def("xcc_count_for_device_id", &xcc_count_for_device_id, py::arg("pci_device_id"));

  m.def("discover_gpus", py::overload_cast<const std::string&>(&discover_gpus), py::arg("sysfs_root") = "/sys");
  m.def("discover_gpus_with", py::overload_cast<const std::string&, const KfdTopology&>(&discover_gpus),
        py::arg("sysfs_root"), py::arg("topology"));
  m.def("partition_config_count", &partition_config_count);
  m.def("is_homogeneous", &is_homogeneous);
  m.def("compute_partition_supported", &compute_partition_supported, py::arg("sysfs_root") = "/sys");
  m.def("memory_partition_supported", &memory_partition_supported, py::arg("sysfs_root") = "/sys");
  m.def("parse_debugfs_firmware_info", [](const std::string& p) {
    auto fi = parse_debugfs_firmware_info(p);
    return py::make_tuple(fi.feature, fi.firmware);
  });

  py::class_<AllocDevice>(m, "AllocDevice")
      .def(py::init([](std::string id, int node_id, int numa_node, std::string unique_id, uint64_t hive_id,
                       bool inferred_links) {
             return AllocDevice{std::move(id), node_id, numa_node, std::move(unique_id), hive_id, inferred_links};
           }),
           py::arg("id"), py::arg("node_id"), py::arg("numa_node"), py::arg("unique_id"), py::arg("hive_id") = 0,
           py::arg("inferred_links") = false)
      .def_readwrite("inferred_links", &AllocDevice::inferred_links)
      .def_readwrite("id", &AllocDevice::id)
      .def_readwrite("node_id", &AllocDevice::node_id)
      .def_readwrite("numa_node", &AllocDevice::numa_node)
      .def_readwrite("unique_id", &AllocDevice::unique_id)
      .def_readwrite("hive_id", &AllocDevice::hive_id);

  py::class_<AllocatorOptions>(m, "AllocatorOptions")
      .def(py::init([](bool missing_pair_is_worst, int cross_hive_penalty) {
             AllocatorOptions o;
             o.missing_pair_is_worst = missing_pair_is_worst;
             o.cross_hive_penalty = cross_hive_penalty;
             return o;
           }),
           py::arg("missing_pair_is_worst") = true, py::arg("cross_hive_penalty") = 100)
      .def_readwrite("missing_pair_is_worst", &AllocatorOptions::missing_pair_is_worst)
      .def_readwrite("cross_hive_penalty", &AllocatorOptions::cross_hive_penalty)
      .def_readwrite("degraded_links", &AllocatorOptions::degraded_links)
      .def_readwrite("extended_search", &AllocatorOptions::extended_search)
      .def_readwrite("extended_search_auto", &AllocatorOptions::extended_search_auto)
      .def_readwrite("extended_node_limit", &AllocatorOptions::extended_node_limit);

  // shared: the native gRPC server keeps using an allocator snapshot while
  // Python initialises its replacement
  py::class_<HiveAllocator, std::shared_ptr<HiveAllocator>>(m, "HiveAllocator")
      .def(py::init<>())
      .def("init", &HiveAllocator::init, py::arg("devices"), py::arg("topology"),
           py::arg("options") = AllocatorOptions())
      .def(
          "allocate",
          [](const HiveAllocator& a, const std::vector<std::string>& av, const std::vector<std::string>& req,
             int size) {
            AllocResult r;
            {
              py::gil_scoped_release nogil;
              r = a.allocate(av, req, size);
            }
            return alloc_result(r);
          },
          py::arg("available"), py::arg("required"), py::arg("size"))
      .def(
          "reference_allocate",
          [](const HiveAllocator& a, const std::vector<std::string>& av, const std::vector<std::string>& req,
             int size) {
            AllocResult r;
            {
              py::gil_scoped_release nogil;
              r = a.reference_allocate(av, req, size);
            }
            return alloc_result(r);
          },
          py::arg("available"), py::arg("required"), py::arg("size"))
      .def_property_readonly("initialized", &HiveAllocator::initialized)
      .def_property_readonly("num_devices", &HiveAllocator::num_devices)
      .def_property_readonly("num_groups", &HiveAllocator::num_groups)
      .def_property_readonly("num_linked_pairs", &HiveAllocator::num_linked_pairs)
      .def_property_readonly("num_from_keys", &HiveAllocator::num_from_keys)
      .def_property_readonly("num_inferred_pairs", &HiveAllocator::num_inferred_pairs)
      .def("pair_weight", &HiveAllocator::pair_weight)
      .def_property_readonly("extended", &HiveAllocator::extended)
      .def("link_type", &HiveAllocator::link_type);

  py::class_<PciFunctionInfo>(m, "PciFunctionInfo")
      .def_readonly("pf", &PciFunctionInfo::pf)
      .def_readonly("vf", &PciFunctionInfo::vf)
      .def_readonly("device_id", &PciFunctionInfo::device_id);
  py::class_<PciScanResult>(m, "PciScanResult")
      .def_readonly("groups", &PciScanResult::groups)
      .def_readonly("ok", &PciScanResult::ok)
      .def_readonly("error", &PciScanResult::error);
  m.def("scan_vf_mapping", &scan_vf_mapping, py::arg("sysfs_root") = "/sys");
  m.def("scan_pf_mapping", &scan_pf_mapping, py::arg("sysfs_root") = "/sys");
  m.def("read_gim_versions", [](const std::string& root) -> py::object {
    auto g = read_gim_versions(root);
    if (!g.ok) return py::none();
    return py::make_tuple(g.version, g.srcversion);
  }, py::arg("sysfs_root") = "/sys");

  m.def(
      "yaml_to_json",
      [](const std::string& text) -> py::tuple {
        std::string err;
        auto v = yaml::parse(text, &err);
        if (!v) return py::make_tuple(py::none(), err);
        return py::make_tuple(json::serialize(*v), std::string());
      },
      py::arg("text"), "the config-file YAML reader (kubeconfig, -config): (JSON text, '') or (None, error)");
  m.def(
      "json_roundtrip",
      [](const std::string& text) -> py::tuple {
        std::string err;
        auto v = json::parse(text, &err);
        if (!v) return py::make_tuple(py::none(), err);
        return py::make_tuple(json::serialize(*v), std::string());
      },
      py::arg("text"), "the labeller's JSON reader + writer (Node objects, watch events): (JSON text, '') or (None, error)");
  m.def("family_id_to_string", &family_id_to_string);
  m.def("drm_available", &drm_available);
  m.def("drm_is_amd_card", &drm_is_amd_card);
  m.def("drm_dev_functional", [](const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
    std::string err;
    bool ok = drm_dev_functional(dev_root, sysfs_root, card, &err);
    return py::make_tuple(ok, err);
  });
  m.def("drm_query_gpu_info", [](const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
    auto i = drm_query_gpu_info(dev_root, sysfs_root, card);
    py::dict d;
    d["ok"] = i.ok;
    d["error"] = i.error;
    d["drm_major"] = i.drm_major;
    d["drm_minor"] = i.drm_minor;
    d["family_id"] = i.family_id;
    d["family"] = i.family;
    d["asic_id"] = i.asic_id;
    d["chip_rev"] = i.chip_rev;
    d["chip_external_rev"] = i.chip_external_rev;
    d["marketing_name"] = i.marketing_name;
    return d;
  });
  m.def("drm_query_firmware", [](const std::string& dev_root, const std::string& sysfs_root, const std::string& card) {
    auto f = drm_query_firmware(dev_root, sysfs_root, card);
    py::dict d;
    d["ok"] = f.ok;
    d["error"] = f.error;
    d["feature"] = f.feature;
    d["firmware"] = f.firmware;
    return d;
  });

  m.def("smi_available", &smi_available);
  m.def("smi_hold", [] {
    py::gil_scoped_release nogil;
    return smi_hold();
  });
  m.def("smi_unhold", [] {
    py::gil_scoped_release nogil;
    smi_unhold();
  });
  m.def("smi_event_name", [](int t) { return std::string(smi_event_name(t)); });
  py::class_<SmiEventWatcher>(m, "SmiEventWatcher")
      .def(py::init<>())
      .def("start", [](SmiEventWatcher& w, uint64_t mask) {
        py::gil_scoped_release nogil;
        return w.start(mask);
      }, py::arg("mask"))
      .def("poll", [](SmiEventWatcher& w, int timeout_ms) {
        std::vector<SmiEvent> ev;
        {
          py::gil_scoped_release nogil;
          ev = w.poll(timeout_ms);
        }
        py::list out;
        for (auto& e : ev) {
          py::dict d;
          d["bdf"] = e.bdf;
          d["type"] = e.type;
          d["name"] = e.name;
          d["message"] = e.message;
          out.append(d);
        }
        return out;
      }, py::arg("timeout_ms") = 0)
      .def("stop", [](SmiEventWatcher& w) {
        py::gil_scoped_release nogil;
        w.stop();
      })
      .def_property_readonly("running", &SmiEventWatcher::running)
      .def_property_readonly("devices", &SmiEventWatcher::devices);
  m.def("smi_xgmi_links", [] {
    SmiXgmiSnapshot s;
    {
      py::gil_scoped_release nogil;
      s = smi_xgmi_links();
    }
    py::dict out;
    out["ok"] = s.ok;
    out["error"] = s.error;
    py::list gpus;
    for (auto& g : s.gpus) {
      py::dict d;
      d["bdf"] = g.bdf;
      d["status_ok"] = g.status_ok;
      d["status"] = g.status;
      d["metrics_ok"] = g.metrics_ok;
      py::list peers;
      for (auto& p : g.peers) {
        py::dict pd;
        pd["peer_bdf"] = p.peer_bdf;
        pd["link_type"] = p.link_type;
        pd["bit_rate_gbps"] = p.bit_rate_gbps;
        pd["max_bandwidth_gbps"] = p.max_bandwidth_gbps;
        pd["read_kb"] = p.read_kb;
        pd["write_kb"] = p.write_kb;
        peers.append(pd);
      }
      d["peers"] = peers;
      d["error"] = g.error;
      gpus.append(d);
    }
    out["gpus"] = gpus;
    return out;
  });
  m.def("smi_snapshot", [] {
    SmiSnapshot s;
    {
      py::gil_scoped_release nogil;
      s = smi_snapshot();
    }
    py::dict out;
    out["ok"] = s.ok;
    out["error"] = s.error;
    py::list gpus;
    for (auto& g : s.gpus) {
      py::dict d;
      d["bdf"] = g.bdf;
      d["uuid"] = g.uuid;
      d["market_name"] = g.market_name;
      d["device_id"] = g.device_id;
      d["target_graphics_version"] = g.target_graphics_version;
      d["num_compute_units"] = g.num_compute_units;
      d["kfd_id"] = g.kfd_id;
      d["kfd_node_id"] = g.kfd_node_id;
      d["partition_id"] = g.partition_id;
      d["xgmi_hive_id"] = g.xgmi_hive_id;
      d["compute_partition"] = g.compute_partition;
      d["memory_partition"] = g.memory_partition;
      d["vram_mb"] = g.vram_mb;
      d["ecc_ok"] = g.ecc_ok;
      d["gfx_activity"] = g.gfx_activity;
      d["ecc_correctable"] = g.ecc_correctable;
      d["ecc_uncorrectable"] = g.ecc_uncorrectable;
      d["drm_render"] = g.drm_render;
      d["drm_card"] = g.drm_card;
      d["hsa_id"] = g.hsa_id;
      d["hip_id"] = g.hip_id;
      d["hip_uuid"] = g.hip_uuid;
      d["driver_name"] = g.driver_name;
      d["driver_version"] = g.driver_version;
      gpus.append(d);
    }
    out["gpus"] = gpus;
    return out;
  });
  py::class_<DirWatcher>(m, "DirWatcher")
      .def(py::init<>())
      .def("open", &DirWatcher::open, py::arg("dir"))
      .def("fileno", &DirWatcher::fd)
      .def("read_events", &DirWatcher::read_events)
      .def("close", &DirWatcher::close);
  bind_rpc(m);
  bind_health(m);
}
