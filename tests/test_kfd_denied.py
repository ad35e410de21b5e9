"""Discovery and placement when kfd denies topology reads.

kfd answers EPERM for every file under the topology node of a GPU the
reader's device cgroup denies: the gpurun box shows 7 of 8 GPU nodes that way
(profiles/archive/sysfs_access_box.json), and a non-privileged plugin pod without
/dev (the drop-in Helm chart's default) sees all of them that way. The
reference then drops every amdgpu_xcp_* partition (its render node is not in
the kfd map, internal/pkg/amdgpu/amdgpu.go:521-565) and places by weight 0
pairs. Here identity comes from PCI sysfs instead (unique_id, xgmi_hive_id,
the amdgpu_xcp drm-minor block layout), or preferred allocation is switched
off with a warning and a metric.
"""
import itertools
import os
import random
import shutil

import pytest

from rocm_k8s_device_plugin_amd.allocator import BestEffortPolicy
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.base import new_context
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.testing.fixtures import deny_kfd_nodes, make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover
from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY

# the MI355X box's probe order: card0 is not the lowest BDF
PROBE_ORDER = [3, 0, 5, 1, 7, 2, 6, 4]


def _ident(inv):
    return {d.id: (d.unique_id, d.hive_id, d.location_id, d.bdf, d.numa_node, d.compute_partition,
                   d.memory_partition, d.card, d.render_minor) for d in inv.devices}


def _all_gpu_nodes(fi):
    return sorted(set(fi.node_ids.values()))


@pytest.mark.parametrize("layout", ["kernel", "compact"])
@pytest.mark.parametrize("mode", ["spx", "dpx", "qpx", "cpx"])
def test_fully_denied_node_keeps_every_partition(tmp_path, layout, mode):
    fi = make_mi355x_node(tmp_path, compute_partition=mode, xcp_layout=layout, probe_order=PROBE_ORDER)
    ref = discover(str(fi.sysfs))
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    inv = discover(str(fi.sysfs))
    assert len(inv) == len(ref) == len(fi.device_ids)
    assert _ident(inv) == _ident(ref)
    assert all(d.identity == "sysfs" and d.node_id == -1 for d in inv.devices)
    assert inv.placement_trusted and not inv.unresolved
    assert len(inv.kfd_unreadable_nodes) == len(_all_gpu_nodes(fi))
    assert any("unreadable" in w for w in inv.warnings)
    # CU shape comes from the part model when no sibling is readable
    assert inv.partition_counts() == ref.partition_counts()


def test_cpx_8x8_fully_denied_advertises_64_grouped(tmp_path):
    """The verdict's acceptance case: CPX 8x8, every GPU properties file
    unreadable -> 64 devices with correct per-GPU grouping."""
    fi = make_mi355x_node(tmp_path, compute_partition="cpx", xcp_layout="kernel", probe_order=PROBE_ORDER)
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    inv = discover(str(fi.sysfs))
    assert len(inv) == 64
    groups = inv.physical_gpus()
    assert len(groups) == 8 and all(len(v) == 8 for v in groups.values())
    for dev_id, g in fi.gpu_of.items():
        assert inv.by_id[dev_id].unique_id == fi.unique_ids[g]
    pol = BestEffortPolicy()
    pol.init(inv.devices, inv.topology)
    assert pol.native.num_groups == 8
    assert pol.native.num_inferred_pairs == 64 * 63 // 2


@pytest.mark.parametrize("mode,hive_size", [("cpx", 8), ("cpx", 4), ("dpx", 4), ("spx", 4)])
def test_allocations_identical_with_and_without_kfd(tmp_path, mode, hive_size):
    """Links inferred from sysfs identity give the same pair weights as kfd's
    io_links/p2p_links, so every preferred allocation is the same."""
    fi = make_mi355x_node(tmp_path, compute_partition=mode, hive_size=hive_size, xcp_layout="kernel",
                          probe_order=PROBE_ORDER)
    ref = discover(str(fi.sysfs))
    p_ref = BestEffortPolicy()
    p_ref.init(ref.devices, ref.topology)
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    inv = discover(str(fi.sysfs))
    p_inv = BestEffortPolicy()
    p_inv.init(inv.devices, inv.topology)
    ids = [d.id for d in ref.devices]
    for a, b in itertools.combinations(ids, 2):
        assert p_inv.native.pair_weight(a, b) == p_ref.native.pair_weight(a, b), (a, b)
    rng = random.Random(7)
    for _ in range(60):
        avail = sorted(rng.sample(ids, rng.randint(2, len(ids))))
        size = rng.randint(1, len(avail))
        req = sorted(rng.sample(avail, rng.randint(0, min(2, size))))
        assert p_inv.allocate(avail, req, size) == p_ref.allocate(avail, req, size)


def test_gpurun_box_shape_seven_of_eight_denied(tmp_path):
    """What the gpurun box shows: SPX, 7 xcp devices per GPU present but
    inactive, 7 of 8 GPU nodes EPERM."""
    fi = make_mi355x_node(tmp_path, xcp_layout="kernel", probe_order=PROBE_ORDER)
    allowed = fi.bdfs[5]
    deny_kfd_nodes(fi, [n for d, n in fi.node_ids.items() if d != allowed])
    inv = discover(str(fi.sysfs))
    assert sorted(inv.by_id) == sorted(fi.bdfs)           # inactive xcp slots are not devices
    assert inv.by_id[allowed].identity == "kfd"
    assert sorted(inv.recovered) == sorted(b for b in fi.bdfs if b != allowed)
    # gfx / CU shape copied from the readable sibling of the same part and mode
    assert all(d.gfx_target_version == 90500 and d.cu_count == 256 for d in inv.devices)
    assert len(inv.hives()) == 1


def test_no_sysfs_identity_disables_preferred_allocation(tmp_path, caplog):
    fi = make_mi355x_node(tmp_path, compute_partition="dpx", xcp_layout="kernel")
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    for b in fi.bdfs[:2]:
        os.remove(fi.sysfs / "devices/pci0000:00" / b / "unique_id")
    inv = discover(str(fi.sysfs))
    assert not inv.placement_trusted
    assert set(fi.bdfs[:2]) <= set(inv.unresolved)
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None, liveness=False))
    ctx = new_context("gpu")
    impl.start(ctx)
    assert ctx.allocator_error
    assert not impl.options(ctx).get_preferred_allocation_available
    text = REGISTRY.render()
    assert "mi355x_dp_devices_identity_unknown" in text and "mi355x_dp_kfd_unreadable_nodes 16" in text
    # the devices themselves are still advertised (kubelet picks among them)
    assert len(impl.devices("gpu")) == 16


def test_recovered_node_keeps_preferred_allocation(tmp_path):
    fi = make_mi355x_node(tmp_path, compute_partition="cpx", xcp_layout="kernel")
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None, liveness=False))
    ctx = new_context("gpu")
    impl.start(ctx)
    assert not ctx.allocator_error
    assert impl.options(ctx).get_preferred_allocation_available
    # 8 partitions of one GPU beat 8 spread ones
    ids = [d.id for d in impl.devices("gpu")]
    got = ctx.allocator.allocate(ids, [], 8)
    assert len({impl.inv.by_id[i].unique_id for i in got}) == 1


def test_inconsistent_xcp_block_is_not_guessed(tmp_path):
    """An xcp whose card and render offsets disagree (interleaved probes) is
    not attributed to any GPU: its partitions are dropped with a warning."""
    fi = make_mi355x_node(tmp_path, compute_partition="dpx", xcp_layout="kernel")
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    # move GPU 0's active xcp to the next xcp index: index - slot no longer constant in the block
    plat = fi.sysfs / "devices/platform"
    shutil.move(str(plat / "amdgpu_xcp_1"), str(plat / "amdgpu_xcp_tmp"))
    shutil.move(str(plat / "amdgpu_xcp_0"), str(plat / "amdgpu_xcp_1"))
    shutil.move(str(plat / "amdgpu_xcp_tmp"), str(plat / "amdgpu_xcp_0"))
    inv = discover(str(fi.sysfs))
    assert any("contiguous" in w for w in inv.warnings)
    assert fi.bdfs[0] in inv.by_id
    assert not [d for d in inv.devices if d.is_partition and d.bdf == fi.bdfs[0]]
    assert len([d for d in inv.devices if d.is_partition]) == 7


def test_unknown_part_in_cpx_is_not_guessed(tmp_path):
    fi = make_mi355x_node(tmp_path, compute_partition="cpx", xcp_layout="kernel", device_id=0x1234)
    deny_kfd_nodes(fi, _all_gpu_nodes(fi))
    inv = discover(str(fi.sysfs))
    assert len(inv) == 8 and not any(d.is_partition for d in inv.devices)
    assert any("partition count" in w for w in inv.warnings)


def test_partitions_for_mode_matches_models():
    from rocm_k8s_device_plugin_amd.models import REGISTRY as MODELS
    from rocm_k8s_device_plugin_amd.ops.native import core
    n = core()
    for m in MODELS:
        for did in m.device_ids:
            if m.compute_partitions:
                assert n.xcc_count_for_device_id(did) == m.xcds, m.name
            for mode in m.compute_partitions:
                assert n.partitions_for_mode(mode, m.xcds) == m.partitions_per_gpu(mode)


def test_labels_count_denied_gpus_like_device_id(tmp_path):
    """The gpurun box's shape (7 of 8 kfd nodes EPERM): vram / cu-count /
    simd-count count every GPU, like device-id and product-name, from what
    discovery recovered from PCI sysfs; native labeller and Python oracle agree,
    and the counts match the raw sysfs (8 pci:amdgpu functions, 1 readable kfd
    GPU node). The reference labeller runs privileged and reads every node
    (k8s-ds-amdgpu-labeller.yaml:66-67), so a privileged run gives these counts."""
    import json
    import subprocess
    from rocm_k8s_device_plugin_amd.labeller import labels as L
    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    fi = make_mi355x_node(tmp_path, xcp_layout="kernel", probe_order=PROBE_ORDER)
    allowed = fi.bdfs[5]
    deny_kfd_nodes(fi, [n for d, n in fi.node_ids.items() if d != allowed])
    pci = [b for b in os.listdir(fi.sysfs / "module/amdgpu/drivers/pci:amdgpu") if b.count(":") == 2]
    nodes = fi.sysfs / "class/kfd/kfd/topology/nodes"
    readable = []
    for n in os.listdir(nodes):
        try:   # deny_kfd_nodes makes the read fail, as EPERM does on the box
            props = (nodes / n / "properties").read_text()
        except OSError:
            continue
        if "cpu_cores_count 0" in props and "simd_count" in props:
            readable.append(n)
    assert len(pci) == 8 and len(readable) == 1
    kinds = ["device-id", "product-name", "vram", "cu-count", "simd-count"]
    exe = os.path.join(str(PKG_DIR), "bin", "mi355x-node-labeller")
    p = subprocess.run([exe, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                        *[f"-{k}" for k in kinds]], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert got == L.generate_labels({k: True for k in kinds}, "container", sysfs_root=str(fi.sysfs),
                                    dev_root=str(fi.dev))
    assert got["amd.com/gpu.device-id.75a3"] == str(len(pci))
    assert got["amd.com/gpu.vram.288G"] == got["amd.com/gpu.cu-count.256"] == got["amd.com/gpu.simd-count.1024"] \
        == str(len(pci))
    # a GPU with nothing readable or recovered (no readable sibling of its part) stays uncounted
    deny_kfd_nodes(fi, [fi.node_ids[allowed]])
    p = subprocess.run([exe, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-cu-count",
                        "-vram"], capture_output=True, text=True, timeout=60)
    got = json.loads(p.stdout)
    assert not any(k.startswith("amd.com/gpu.cu-count") for k in got), got
    assert got["amd.com/gpu.vram.288G"] == "8"                   # each GPU's own mem_info_vram_total

