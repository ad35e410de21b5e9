"""Container start-up views in the native daemon (`-node_view`,
`-topology_view`, experimental). The Allocate mounts and the view trees they
point at equal the Python plugin's (node_view.py, topology_view.py): the same
files with the same contents, the same symlink targets, the same container
paths. Views are built once per node and once per allocated GPU set."""
import asyncio
import os
import random

import pytest

from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
from rocm_k8s_device_plugin_amd.plugin.base import PluginContext
from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
from rocm_k8s_device_plugin_amd.proto import deviceplugin as pb
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

from test_native_cdi import _daemon
from test_native_health import _stop


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _tree(root):
    out = {}
    for d, dirs, files in os.walk(root):
        for name in dirs + files:
            p = os.path.join(d, name)
            rel = os.path.relpath(p, root)
            if os.path.islink(p):
                out[rel] = ("link", os.readlink(p))
            elif os.path.isdir(p):
                out[rel] = ("dir",)
            else:
                with open(p) as f:
                    out[rel] = ("file", f.read())
    return out


def _add_cpu_tree(fi, nodes=2, cpus_per_node=3):
    """A small NUMA tree with per-CPU caches (whatever the fixture has is replaced)."""
    import shutil
    shutil.rmtree(fi.sysfs / "devices/system/node", ignore_errors=True)
    shutil.rmtree(fi.sysfs / "devices/system/cpu", ignore_errors=True)
    root = fi.sysfs
    node_root = root / "devices/system/node"
    cpu_root = root / "devices/system/cpu"
    node_root.mkdir(parents=True, exist_ok=True)
    (node_root / "online").write_text(f"0-{nodes - 1}\n")
    for n in range(nodes):
        nd = node_root / f"node{n}"
        nd.mkdir(exist_ok=True)
        (nd / "meminfo").write_text(f"Node {n} MemTotal: 1 kB\n")
        for c in range(n * cpus_per_node, (n + 1) * cpus_per_node):
            cd = cpu_root / f"cpu{c}"
            (cd / "cache/index0").mkdir(parents=True, exist_ok=True)
            (cd / "cache/index0/size").write_text("48K\n")
            (cd / "online").write_text("1\n")
            if not os.path.lexists(nd / f"cpu{c}"):
                os.symlink(f"../../cpu/cpu{c}", nd / f"cpu{c}")


@pytest.mark.parametrize("partition", ["spx", "dpx"])
def test_view_mounts_and_trees_equal_the_python_plugin(tmp_path, partition):
    fi = make_mi355x_node(tmp_path / "n", compute_partition=partition)
    _add_cpu_tree(fi)
    impl = ContainerImpl("single", str(fi.sysfs), HealthConfig(exporter_socket=None),
                         topology_view_dir=str(tmp_path / "py-topo"), node_view_dir=str(tmp_path / "py-node"))
    ctx = PluginContext("gpu")
    kdir = str(tmp_path / "dp")
    rng = random.Random(11)

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-node_view", "-topology_view")
        try:
            st = await k.wait_for_resource("amd.com/gpu", len(impl.devices("gpu")), timeout=20)
            ids = sorted(st.devices)
            for _ in range(6):
                chosen = sorted(rng.sample(ids, rng.randint(1, min(4, len(ids)))))
                areq = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=chosen),
                                                              pb.ContainerAllocateRequest(devices_ids=[])])
                got = await k._call(st, "Allocate", areq, pb.AllocateResponse)
                want = impl.allocate(ctx, areq)
                g, w = got.container_responses[0], want.container_responses[0]
                assert list(g.devices) == list(w.devices)
                assert [(m.container_path, m.read_only) for m in g.mounts] == \
                       [(m.container_path, m.read_only) for m in w.mounts]
                assert len(g.mounts) == 3                       # topology view, node alias, node view
                for gm, wm in zip(g.mounts, w.mounts):
                    if gm.container_path == "/run/mi355x/sys-node":
                        assert gm.host_path == wm.host_path      # the real node directory
                    else:
                        assert _tree(gm.host_path) == _tree(wm.host_path), gm.container_path
                assert got.container_responses[1] == want.container_responses[1]
                assert not got.container_responses[1].mounts          # views only for containers with devices
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "node view: " in err and "per-CPU cache directories left out" in err

    asyncio.run(asyncio.wait_for(go(), 60))
    # one topology view per distinct node set, none rebuilt
    assert len([d for d in os.listdir(os.path.join(kdir, "mi355x-topology")) if not d.startswith(".")]) <= 6


def test_views_off_by_default_and_unbuildable_node_view_is_not_fatal(tmp_path):
    import shutil
    fi = make_mi355x_node(tmp_path / "n")
    shutil.rmtree(fi.sysfs / "devices/system/node", ignore_errors=True)   # nothing to build the view from

    async def go():
        kdir = str(tmp_path / "dp")
        k = FakeKubelet(kdir)
        await k.start()
        p = _daemon(kdir, fi, "-node_view")
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            adm = await k.admit("amd.com/gpu", 1)
            assert not adm.response.container_responses[0].mounts
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0 and "node view unavailable" in err, err[-2000:]

    asyncio.run(asyncio.wait_for(go(), 60))
