"""Topology / discovery parity with the reference's parsers and fixtures
(internal/pkg/amdgpu/amdgpu_test.go) plus MI355X fixture discovery, including
the layout seen on a real MI355X box (56 amdgpu_xcp_* devices in SPX that kfd
does not know, render-only /dev, EPERM'd kfd properties)."""
import os
import shutil

import pytest

from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import Inventory, discover, hip_ordinals


def test_parse_topology_properties(ref_testdata):
    n = core()
    mb = n.parse_kv_file(str(ref_testdata / "topology-parsing/topology/nodes/1/mem_banks/0/properties"))
    assert int(mb["size_in_bytes"]) == 17163091968
    assert int(mb["flags"]) == 0
    props = n.parse_kv_file(str(ref_testdata / "topology-parsing/topology/nodes/2/properties"))
    assert int(props["simd_count"]) == 256
    assert int(props["simd_id_base"]) == 2147487744
    assert "asdf" not in props
    assert n.parse_kv_file(str(ref_testdata / "nope")) is None


def test_unique_id_string(ref_testdata):
    """Reference TestParseTopologyPropertiesString expects unique_id 14073402507705256557 in
    topology-parsing nodes/2 — but that file has no unique_id line, so the reference test
    fails statically. We assert what the fixture actually contains."""
    n = core()
    props = n.parse_kv_file(str(ref_testdata / "topology-parsing/topology/nodes/2/properties"))
    assert "unique_id" not in props
    t = n.KfdTopology.load(str(ref_testdata / "topology-parsing/topology/nodes"))
    assert t.render_to_unique_id() == {}  # nodes without unique_id are skipped, as in the reference


def test_render_dev_ids_mi308(ref_testdata):
    """TestRenderDevIdsFromTopology (amdgpu_test.go:234-278)."""
    t = core().KfdTopology.load(str(ref_testdata / "topology-parsing-mi308/topology/nodes"))
    got = t.render_to_unique_id()
    exp_groups = {
        128: "598046273873802902", 136: "11803749423592941193", 144: "10187445671099294242",
        152: "9604994527082705072", 160: "17466021589395472075", 168: "1044926823201815193",
        176: "13372828617950681944", 184: "6576958293045616595"}
    exp = {base + i: uid for base, uid in exp_groups.items() for i in range(4)}
    assert got == exp


def test_count_gpu_nodes(ref_testdata):
    """TestCountGPUDevFromTopology expects 2."""
    assert core().KfdTopology.load(str(ref_testdata / "topology-parsing/topology/nodes")).count_gpu_nodes() == 2


def test_debugfs_firmware(ref_testdata):
    """TestParseDebugFSFirmwareInfo (amdgpu_test.go:179-232)."""
    feat, fw = core().parse_debugfs_firmware_info(str(ref_testdata / "debugfs-parsing/amdgpu_firmware_info"))
    exp_feat = {"VCE": 0, "UVD": 0, "MC": 0, "ME": 35, "PFP": 35, "CE": 35, "RLC": 0, "MEC": 33, "MEC2": 33,
                "SOS": 0, "ASD": 0, "SMC": 0, "SDMA0": 40, "SDMA1": 40}
    exp_fw = {"VCE": 0x352d0400, "UVD": 0x01571100, "MC": 0, "ME": 0x94, "PFP": 0xa4, "CE": 0x4a, "RLC": 0x58,
              "MEC": 0x160, "MEC2": 0x160, "SOS": 0x00161a92, "ASD": 0x0016129a, "SMC": 0x001c2800,
              "SDMA0": 0x197, "SDMA1": 0x197}
    assert feat == exp_feat and fw == exp_fw


def test_reference_links_and_hives(ref_testdata):
    t = core().KfdTopology.load(str(ref_testdata / "topo-mi210-xgmi-pcie/nodes"))
    hives = {t.node(i).hive_id for i in range(2, 10)}
    assert len(hives) == 2
    n2 = t.node(2)
    assert {l["node_to"] for l in n2.io_links if l["type"] == 11} == {3, 4, 5}
    assert {l["node_to"] for l in n2.p2p_links} >= {6, 7, 8, 9}
    cpx = core().KfdTopology.load(str(ref_testdata / "topo-mi300-cpx/topology/nodes"))
    assert cpx.count_gpu_nodes() == 63
    assert cpx.node(2).location_id == 1280 and cpx.node(9).location_id == 1287


@pytest.mark.parametrize("mode,parts", [("spx", 1), ("dpx", 2), ("qpx", 4), ("cpx", 8)])
@pytest.mark.parametrize("nps", ["nps1", "nps2"])
def test_discover_mi355x_modes(tmp_path, mode, parts, nps):
    fi = make_mi355x_node(tmp_path, compute_partition=mode, memory_partition=nps)
    inv = discover(str(fi.sysfs))
    assert len(inv) == 8 * parts
    assert inv.partition_counts() == {f"{mode}_{nps}": 8 * parts}
    assert [d.id for d in inv.devices[:8]] == fi.bdfs
    for d in inv.devices:
        assert d.gfx_target_version == 90500 and d.is_gfx950
        assert d.cu_count == 256 // parts and d.num_xcc == 8 // parts
        assert d.hive_id == fi.hive_ids[0]
        assert d.node_id == fi.node_ids[d.id] and d.render_minor == fi.render_minors[d.id]
        assert d.bdf in fi.bdfs
    # partitions share their parent's unique_id, NUMA node and partition mode
    for uid, devs in inv.physical_gpus().items():
        assert len(devs) == parts
        assert len({d.numa_node for d in devs}) == 1 and len({d.bdf for d in devs}) == 1
    assert inv.compute_partition_supported() and inv.memory_partition_supported()


def test_real_box_layout_quirks(tmp_path):
    """What the MI355X box showed (profiles/archive/measurements_r1_r3.md §5): SPX, yet 7 amdgpu_xcp_*
    platform devices per GPU with drm nodes that kfd does not know; those must not
    become kubelet devices."""
    fi = make_mi355x_node(tmp_path)
    plat = fi.sysfs / "devices/platform"
    minor = 500
    for i in range(56):
        d = plat / f"amdgpu_xcp_{i}" / "drm"
        (d / f"card{100 + i}").mkdir(parents=True)
        (d / f"renderD{minor + i}").mkdir(parents=True)
    inv = discover(str(fi.sysfs))
    assert len(inv) == 8 and not any(d.is_partition for d in inv.devices)


def test_unreadable_kfd_nodes(tmp_path):
    """kfd EPERMs the properties of cgroup-denied GPUs inside containers: the device
    stays (from PCI sysfs) with its identity recovered from sysfs, but carries no
    kfd node and no HIP ordinal (tests/test_kfd_denied.py covers whole nodes)."""
    fi = make_mi355x_node(tmp_path)
    victim = fi.node_ids[fi.bdfs[2]]
    os.remove(fi.sysfs / "class/kfd/kfd/topology/nodes" / str(victim) / "properties")
    inv = discover(str(fi.sysfs))
    d = inv.by_id[fi.bdfs[2]]
    assert d.node_id == -1 and d.identity == "sysfs"
    assert d.unique_id == fi.unique_ids[2] and d.hive_id == fi.hive_ids[2]
    assert d.gfx_target_version == 90500       # from a readable sibling of the same part
    assert fi.bdfs[2] not in hip_ordinals(inv, str(fi.dev))
    from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy
    pol = BestEffortPolicy()
    pol.init(inv.devices, inv.topology)
    assert pol.native.num_groups == 8
    assert pol.native.link_type(fi.bdfs[2], fi.bdfs[3]) == 11   # same hive -> xGMI, inferred


def test_device_without_drm_does_not_inherit(tmp_path):
    """Reference Appendix B #8: card/renderD leaked from the previous loop iteration."""
    fi = make_mi355x_node(tmp_path)
    drm = fi.sysfs / "devices/pci0000:00" / fi.bdfs[3] / "drm"
    shutil.rmtree(drm)
    inv = discover(str(fi.sysfs))
    d = inv.by_id[fi.bdfs[3]]
    # no drm node: nothing kfd-side; the identity is its own (sysfs), not its neighbour's
    assert d.card == -1 and d.render_minor == -1 and d.unique_id == fi.unique_ids[3]
    assert inv.by_id[fi.bdfs[2]].card != -1


def test_missing_numa_skips_device(tmp_path):
    fi = make_mi355x_node(tmp_path)
    os.remove(fi.sysfs / "devices/pci0000:00" / fi.bdfs[0] / "numa_node")
    inv = discover(str(fi.sysfs))
    assert fi.bdfs[0] not in inv.by_id and len(inv) == 7
    assert any("numa_node" in w for w in inv.warnings)


def test_no_driver(tmp_path):
    inv = discover(str(tmp_path))
    assert len(inv) == 0 and not inv.driver_loaded


def test_hip_ordinals_follow_kfd_node_order(tmp_path):
    fi = make_mi355x_node(tmp_path, compute_partition="dpx")
    inv = discover(str(fi.sysfs))
    ords = hip_ordinals(inv, str(fi.dev))
    by_node = sorted(inv.devices, key=lambda d: d.node_id)
    assert [ords[d.id] for d in by_node] == list(range(16))
    # a render node the process cannot open is skipped by ROCr -> ordinals shift
    os.chmod(fi.dev / "dri" / f"renderD{by_node[0].render_minor}", 0)
    if os.getuid() != 0:  # root ignores permission bits
        ords2 = hip_ordinals(inv, str(fi.dev))
        assert by_node[0].id not in ords2 and ords2[by_node[1].id] == 0
