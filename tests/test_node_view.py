"""NUMA-node sysfs view without per-CPU cache descriptors (-node_view)."""
import os

from rocm_k8s_device_plugin_amd.node_view import NODE_ALIAS, NODE_CONTAINER_PATH, NodeView, build_node_view


def _sysfs(tmp_path, nodes=2, cpus_per_node=3):
    root = tmp_path / "sys"
    node_root = root / "devices/system/node"
    cpu_root = root / "devices/system/cpu"
    (node_root).mkdir(parents=True)
    (node_root / "online").write_text(f"0-{nodes - 1}\n")
    (node_root / "possible").write_text(f"0-{nodes - 1}\n")
    for n in range(nodes):
        nd = node_root / f"node{n}"
        nd.mkdir()
        (nd / "meminfo").write_text(f"Node {n} MemTotal: 1 kB\n")
        (nd / "distance").write_text("10 32\n")
        (nd / "hugepages").mkdir()
        for c in range(n * cpus_per_node, (n + 1) * cpus_per_node):
            cd = cpu_root / f"cpu{c}"
            (cd / "cache/index0").mkdir(parents=True)
            (cd / "cache/index0/size").write_text("48K\n")
            (cd / "topology").mkdir()
            (cd / "online").write_text("1\n")
            os.symlink(f"../../cpu/cpu{c}", nd / f"cpu{c}")
    return root


def test_view_hides_only_node_relative_cpu_caches(tmp_path):
    root = _sysfs(tmp_path)
    src = root / "devices/system/node"
    dst = tmp_path / "view"
    # alias = the real directory itself, as in tools/archive/experiments/view_emulation.py
    links, hidden = build_node_view(str(src), str(dst), alias=str(src), cpu_root=str(root / "devices/system/cpu"))
    assert hidden == 6
    # live files through symlinks, CPU entries except the cache directory
    assert (dst / "online").read_text() == "0-1\n"
    assert (dst / "node1/meminfo").read_text().startswith("Node 1")
    assert (dst / "node1/hugepages").is_dir()
    assert sorted(os.listdir(dst / "node0/cpu1")) == ["online", "topology"]
    assert (dst / "node0/cpu1/online").read_text() == "1\n"
    assert not (dst / "node0/cpu1/cache").exists()
    # the real cpu directory still has its caches
    assert (root / "devices/system/cpu/cpu1/cache/index0/size").exists()
    # what ROCr's walk sees: no cache index files under the view
    walked = [f for d, _, fs in os.walk(dst, followlinks=False) for f in fs if "cache" in d]
    assert walked == []


def test_view_symlinks_point_at_container_paths(tmp_path):
    root = _sysfs(tmp_path, nodes=1, cpus_per_node=1)
    dst = tmp_path / "view"
    build_node_view(str(root / "devices/system/node"), str(dst))
    assert os.readlink(dst / "node0/meminfo") == f"{NODE_ALIAS}/node0/meminfo"
    assert os.readlink(dst / "online") == f"{NODE_ALIAS}/online"
    assert os.readlink(dst / "node0/cpu0/online") == "/sys/devices/system/cpu/cpu0/online"


def test_nodeview_builds_once_and_mounts(tmp_path):
    root = _sysfs(tmp_path)
    nv = NodeView(str(tmp_path / "views"), sysfs_root=str(root))
    m = nv.mounts()
    assert m[0] == (str(root / "devices/system/node"), NODE_ALIAS)
    assert m[1][1] == NODE_CONTAINER_PATH and os.path.isdir(m[1][0])
    assert nv.mounts() == m and nv.hidden == 6


def test_allocate_returns_node_view_mounts(tmp_path):
    from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
    from rocm_k8s_device_plugin_amd.plugin.base import PluginContext
    from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
    from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    fi = make_mi355x_node(tmp_path / "n")
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None),
                         node_view_dir=str(tmp_path / "nv"))
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=[fi.bdfs[0]])
    mounts = list(impl.allocate(PluginContext("gpu"), req).container_responses[0].mounts)
    assert [(m.container_path, m.read_only) for m in mounts] == [(NODE_ALIAS, True), (NODE_CONTAINER_PATH, True)]
    assert os.path.isdir(mounts[1].host_path)


def test_nodeview_alias_equal_to_host_path_needs_one_mount(tmp_path):
    root = _sysfs(tmp_path)
    src = str(root / "devices/system/node")
    nv = NodeView(str(tmp_path / "views"), sysfs_root=str(root), alias=src)
    (m,) = nv.mounts()
    assert m[1] == NODE_CONTAINER_PATH
    # symlinks resolve directly on the host
    assert open(os.path.join(m[0], "node0/meminfo")).read().startswith("Node 0")
