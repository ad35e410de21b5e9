"""Per-allocation kfd topology views (experimental -topology_view)."""
import asyncio
import os

import pytest

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.plugin.base import PluginContext
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology_view import KFD_TOPOLOGY_CONTAINER_PATH, TopologyViews, build_view


def test_view_contents(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="dpx")
    src = str(fi.sysfs / "class/kfd/kfd/topology")
    keep = [fi.node_ids["0000:65:00.0"], fi.node_ids["0000:f5:00.0"]]
    remap = build_view(src, str(tmp_path / "v"), keep)
    assert remap == {0: 0, 1: 1, keep[0]: 2, keep[1]: 3}
    t = core().KfdTopology.load(str(tmp_path / "v/nodes"))
    assert [n.id for n in t.nodes] == [0, 1, 2, 3]
    assert t.count_gpu_nodes() == 2
    orig = core().KfdTopology.load(str(fi.sysfs / "class/kfd/kfd/topology/nodes"))
    for old, new in remap.items():
        a, b = orig.node(old), t.node(new)
        assert a.unique_id == b.unique_id and a.hive_id == b.hive_id and a.drm_render_minor == b.drm_render_minor
        # links only inside the view, retargeted, counts fixed
        links = b.io_links + b.p2p_links
        assert all(l["node_from"] == new and l["node_to"] in (0, 1, 2, 3) for l in links)
        assert b.prop("io_links_count") == len(b.io_links) and b.prop("p2p_links_count") == len(b.p2p_links)
    # the xGMI link between the two kept GPUs survives (RCCL topology detection needs it)
    assert {(l["node_to"], l["type"]) for l in t.node(2).io_links} >= {(3, 11)}
    # gpu_id copied verbatim (kfd ioctls address GPUs by gpu_id)
    assert (tmp_path / "v/nodes/2/gpu_id").read_text() == (fi.sysfs / f"class/kfd/kfd/topology/nodes/{keep[0]}/gpu_id").read_text()
    assert (tmp_path / "v/generation_id").exists()
    assert sum(len(f) for _, _, f in os.walk(tmp_path / "v")) < sum(len(f) for _, _, f in os.walk(src))


def test_view_cache_and_missing_node(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    views = TopologyViews(str(tmp_path / "views"), str(fi.sysfs / "class/kfd/kfd/topology"))
    a = views.get([fi.node_ids[fi.bdfs[0]]])
    b = views.get([fi.node_ids[fi.bdfs[0]]])
    c = views.get([fi.node_ids[fi.bdfs[1]], fi.node_ids[fi.bdfs[0]]])
    assert a == b != c and views.built == 2
    with pytest.raises(FileNotFoundError):
        views.get([999])


def test_allocate_returns_topology_mount(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None),
                         topology_view_dir=str(tmp_path / "views"))
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=[fi.bdfs[2], fi.bdfs[3]])
    resp = impl.allocate(PluginContext("gpu"), req)
    (m,) = resp.container_responses[0].mounts
    assert m.container_path == KFD_TOPOLOGY_CONTAINER_PATH and m.read_only
    t = core().KfdTopology.load(os.path.join(m.host_path, "nodes"))
    assert t.count_gpu_nodes() == 2
    # default: no mounts (upstream behaviour)
    plain = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None))
    assert not plain.allocate(PluginContext("gpu"), req).container_responses[0].mounts
