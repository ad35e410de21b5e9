"""Version banner and NUMA locality (the reference's hwloc role, C18)."""
import pytest

from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.utils.versions import _cpulist, banner_line, numa_locality, versions


def test_cpulist_parser():
    assert _cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert _cpulist("") == []


def test_numa_locality_from_pci_sysfs(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")            # 8 GPUs over 2 NUMA nodes
    locs = [numa_locality(b, str(fi.sysfs)) for b in fi.bdfs]
    assert [l["numa_nodes"] for l in locs] == [[0]] * 4 + [[1]] * 4
    assert locs[0]["cpus"] == list(range(64)) and locs[7]["cpus"] == list(range(64, 128))
    with pytest.raises(FileNotFoundError):
        numa_locality("0000:ff:1f.7", str(fi.sysfs))


def test_numa_locality_without_affinity(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    (fi.sysfs / "bus/pci/devices" / fi.bdfs[0] / "numa_node").write_text("-1\n")
    for n in (0, 1):
        (fi.sysfs / f"devices/system/node/node{n}").mkdir(parents=True, exist_ok=True)
    assert numa_locality(fi.bdfs[0], str(fi.sysfs))["numa_nodes"] == [0, 1]


def test_banner(tmp_path):
    v = versions(str(tmp_path))
    assert v["numa_source"] == "sysfs" and v["amdgpu"] is None
    line = banner_line(str(tmp_path))
    assert line.startswith("rocm: ") and "amdgpu: n/a" in line
