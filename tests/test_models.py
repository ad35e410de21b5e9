"""GPU hardware models and the discovery consistency check (CPU)."""
import shutil

import pytest

from rocm_k8s_device_plugin_amd.models import MI210, MI300X, MI308X, MI355X, check_inventory, model_for
from rocm_k8s_device_plugin_amd.topology import Gpu, discover


def test_registry_lookup():
    assert model_for(0x75A3) is MI355X
    assert model_for(0x75B3) is MI355X            # VF id maps to its PF's model
    assert model_for(0x74A1) is MI300X
    assert model_for(0x74A2) is MI308X
    assert model_for(0x740F) is MI210
    assert model_for(0, 90500) is MI355X          # by gfx target when the device id is unknown
    assert model_for(0x1234) is None and model_for() is None


def test_mi355x_partition_layout():
    assert MI355X.gfx == "gfx950" and MI355X.gfx_target_version == 90500
    assert [MI355X.partitions_per_gpu(m) for m in ("spx", "dpx", "qpx", "cpx")] == [1, 2, 4, 8]
    assert [MI355X.cus_per_partition(m) for m in ("spx", "dpx", "qpx", "cpx")] == [256, 128, 64, 32]
    assert MI355X.partitions_per_gpu("CPX") == 8
    assert MI355X.partitions_per_gpu("nps1") is None
    assert MI355X.supports("cpx", "nps2") and not MI355X.supports("cpx", "nps4")
    assert MI308X.partitions_per_gpu("cpx") == 4      # 4 XCDs (reference fixture: 8 GPUs x 4)
    assert MI210.partitions_per_gpu("spx") is None


@pytest.mark.parametrize("cp,mp", [("spx", "nps1"), ("dpx", "nps2"), ("qpx", "nps1"), ("cpx", "nps2")])
def test_fixture_nodes_are_consistent(tmp_path, cp, mp):
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    fi = make_mi355x_node(tmp_path / "n", compute_partition=cp, memory_partition=mp)
    inv = discover(str(fi.sysfs))
    assert len(inv) == 8 * MI355X.partitions_per_gpu(cp)
    assert check_inventory(inv.devices) == []
    assert not [w for w in inv.warnings if "partitions discovered" in w]


def test_missing_partition_is_flagged(tmp_path):
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    xcps = sorted((fi.sysfs / "devices/platform").glob("amdgpu_xcp_*"), key=lambda p: int(p.name.rsplit("_", 1)[1]))
    shutil.rmtree(xcps[0])     # a partition of the first GPU disappears (half-applied reconfiguration)
    inv = discover(str(fi.sysfs))
    assert len(inv) == 63
    assert any("7 cpx partitions discovered" in w and "MI355X has 8" in w for w in inv.warnings)


def _gpu(i, uid, cp, simd=1024, dev=0x75A3, gfx=90500):
    return Gpu(id=f"d{i}", bdf=f"0000:{i:02x}:00.0", is_partition=False, xcp_index=-1, card=i, render_minor=128 + i,
               unique_id=uid, compute_partition=cp, memory_partition="nps1", numa_node=0, node_id=i,
               gfx_target_version=gfx, simd_count=simd, simd_per_cu=4, pci_device_id=dev)


def test_check_inventory_rules():
    # consistent SPX GPU
    assert check_inventory([_gpu(0, "u0", "spx")]) == []
    # mixed modes on one physical GPU
    w = check_inventory([_gpu(0, "u0", "dpx", simd=512), _gpu(1, "u0", "spx", simd=512)])
    assert any("different compute modes" in x for x in w)
    # wrong CU count for the mode
    w = check_inventory([_gpu(0, "u0", "dpx", simd=256), _gpu(1, "u0", "dpx", simd=512)])
    assert any("64 CUs" in x and "128" in x for x in w)
    # unsupported mode
    assert any("does not support" in x for x in check_inventory([_gpu(0, "u0", "xpx")]))
    # devices without kfd data (EPERM'd nodes in a restricted container) and unknown parts are skipped
    assert check_inventory([_gpu(0, "u0", "dpx", gfx=0)]) == []
    assert check_inventory([_gpu(0, "u0", "dpx", dev=0x1234, gfx=11)]) == []


def test_reference_fixture_models(ref_testdata):
    """The reference's captured trees name the parts the registry models."""
    from rocm_k8s_device_plugin_amd.ops.native import core
    cases = {"topo-mi300-cpx/topology/nodes": MI300X, "topology-parsing-mi308/topology/nodes": MI308X,
             "topo-mi210-xgmi-pcie/nodes": MI210}
    for rel, model in cases.items():
        topo = core().KfdTopology.load(str(ref_testdata / rel))
        gpus = [topo.node(i) for i in topo.gpu_node_ids()]
        assert gpus
        for n in gpus:
            assert model_for(n.device_id, n.gfx_target_version) is model, (rel, n.device_id)
            assert n.gfx_target_version == model.gfx_target_version
