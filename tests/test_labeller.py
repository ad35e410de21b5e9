"""Node labeller label schema: parity with cmd/k8s-node-labeller/main.go.

labeller/labels.py is the oracle the native labeller's labels are compared
with (tests/test_native_labeller.py); the apiserver loop exists only in the
native labeller and is tested there."""
import json
import os
import time

import pytest

from rocm_k8s_device_plugin_amd import constants as C
from rocm_k8s_device_plugin_amd.labeller import labels as L
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

ALL = {k: True for k in C.SUPPORTED_LABELS}


def test_create_labels_single_and_multi():
    one = L.create_labels("family", {"AI": 8})
    assert one == {"beta.amd.com/gpu.family.AI": "8", "beta.amd.com/gpu.family": "AI",
                   "amd.com/gpu.family.AI": "8", "amd.com/gpu.family": "AI"}
    two = L.create_labels("vram", {"288G": 4, "144G": 4})
    assert "amd.com/gpu.vram" not in two and two["amd.com/gpu.vram.288G"] == "4"
    assert L.create_labels("x", {}) == {}


def test_all_label_keys_reference_lists():
    keys = set(L.all_label_keys())
    # every generator of the reference + the three un-prefixed legacy keys (main.go:50-62)
    for k in C.SUPPORTED_LABELS:
        assert f"amd.com/gpu.{k}" in keys
    for k in ("amd.com/compute-partitioning-supported", "amd.com/memory-partitioning-supported",
              "amd.com/compute-memory-partition"):
        assert k in keys
    exp = set(L.all_experimental_label_keys())
    assert "beta.amd.com/gpu.family" in exp and "beta.amd.com/gpu.mode" in exp


def test_remove_old_node_labels_reference_cases():
    """The two cases of TestRemoveOldNodeLabels (main_test.go:59-125)."""
    labels = {
        "amd.com/gpu.cu-count": "104", "amd.com/gpu.device-id": "740f", "amd.com/gpu.driver-version": "6.10.5",
        "amd.com/gpu.family": "AI", "amd.com/gpu.product-name": "Instinct_MI210", "amd.com/gpu.simd-count": "416",
        "amd.com/gpu.vram": "64G", "beta.amd.com/gpu.cu-count": "104", "beta.amd.com/gpu.cu-count.104": "1",
        "beta.amd.com/gpu.device-id": "740f", "beta.amd.com/gpu.device-id.740f": "1",
        "beta.amd.com/gpu.family": "HPC", "beta.amd.com/gpu.family.HPC": "1",
        "beta.amd.com/gpu.product-name": "Instinct_MI300X", "beta.amd.com/gpu.product-name.Instinct_MI300X": "1",
        "beta.amd.com/gpu.simd-count": "416", "beta.amd.com/gpu.simd-count.416": "1",
        "beta.amd.com/gpu.vram": "64G", "beta.amd.com/gpu.vram.64G": "1", "dummyLabel1": "1", "dummyLabel2": "2",
    }
    assert L.remove_old_node_labels(labels) == {"dummyLabel1": "1", "dummyLabel2": "2"}
    keep = {"amd.com/cpu": "true", "amd.com/gpu": "true", "amd.com/mi300x": "true", "dummyLabel1": "1",
            "dummyLabel2": "2"}
    assert L.remove_old_node_labels(keep) == keep
    # improvement: orphaned beta counters are removed too
    assert L.remove_old_node_labels({"beta.amd.com/gpu.family.AI": "8"}) == {}
    assert L.remove_old_node_labels(None) == {}


@pytest.mark.parametrize("mode,parts", [("spx", 1), ("cpx", 8), ("qpx", 4)])
def test_container_labels_mi355x(tmp_path, mode, parts):
    fi = make_mi355x_node(tmp_path, compute_partition=mode)
    lab = L.generate_labels({**ALL, "firmware": False, "family": False}, "container", str(fi.sysfs), str(fi.dev))
    n = 8 * parts
    assert lab["amd.com/gpu.device-id"] == "75a3"
    assert lab["amd.com/gpu.device-id.75a3"] == str(n)
    assert lab["amd.com/gpu.product-name"] == "AMD_Instinct_MI355X"
    assert lab["amd.com/gpu.cu-count"] == str(256 // parts)
    assert lab["amd.com/gpu.simd-count"] == str(1024 // parts)
    assert lab["amd.com/gpu.vram"] == f"{288 // parts}G"
    assert lab["amd.com/gpu.compute-memory-partition"] == f"{mode}_nps1"
    assert lab["amd.com/gpu.compute-partitioning-supported"] == "true"
    assert lab["amd.com/gpu.memory-partitioning-supported"] == "true"
    assert lab["amd.com/gpu.mode"] == "container" and lab["beta.amd.com/gpu.mode"] == "container"
    assert lab["amd.com/gpu.driver-version"] == "6.12.12"
    assert lab["amd.com/gpu.driver-src-version"] == "A1B2C3D4E5F60718293A4B5"
    # beta + amd.com for counted kinds only; driver versions are amd.com only
    assert "beta.amd.com/gpu.driver-version" not in lab
    # firmware/family need a real GPU (libdrm ioctl); off here
    assert not any("firmware" in k or "family" in k for k in lab)
    # the opt-in additions stay off unless enabled
    assert not any("gfx-target" in k for k in lab)


def test_extra_labels(tmp_path):
    fi = make_mi355x_node(tmp_path, hive_size=4)
    lab = L.generate_labels({"gfx-target": True, "xgmi-hive-count": True}, "container", str(fi.sysfs),
                            str(fi.dev))
    assert lab["amd.com/gpu.gfx-target"] == "gfx950"
    assert lab["amd.com/gpu.xgmi-hive-count"] == "2"
    assert L.gfx_name(90402) == "gfx942" and L.gfx_name(90010) == "gfx90a" and L.gfx_name(90500) == "gfx950"


def test_xgmi_links_down_label(tmp_path):
    """Counts links amd-smi reports down (status 0) on this node's GPUs; disabled
    slots (2) and other nodes' GPUs do not count; no label without amd-smi."""
    fi = make_mi355x_node(tmp_path)

    def reading(down_on_first=0):
        gpus = [{"bdf": b, "status_ok": True, "status": [2] + [1] * 7, "peers": [], "metrics_ok": False}
                for b in fi.bdfs]
        gpus[0]["status"] = [2] + [0] * down_on_first + [1] * (7 - down_on_first)
        gpus.append({"bdf": "0000:ee:00.0", "status_ok": True, "status": [0] * 8})    # not ours
        return {"ok": True, "error": "", "gpus": gpus}

    on = {"xgmi-links-down": True}
    lab = L.generate_labels(on, "container", str(fi.sysfs), str(fi.dev), xgmi_source=lambda: reading(0))
    assert lab == {"amd.com/gpu.xgmi-links-down": "0"}
    lab = L.generate_labels(on, "container", str(fi.sysfs), str(fi.dev), xgmi_source=lambda: reading(2))
    assert lab == {"amd.com/gpu.xgmi-links-down": "2"}
    lab = L.generate_labels(on, "container", str(fi.sysfs), str(fi.dev),
                            xgmi_source=lambda: {"ok": False, "error": "no amd-smi", "gpus": []})
    assert lab == {}
    assert "amd.com/gpu.xgmi-links-down" in L.all_label_keys()


def test_heterogeneous_no_partition_label(tmp_path):
    fi = make_mi355x_node(tmp_path, per_gpu_compute=["spx"] * 4 + ["cpx"] * 4)
    lab = L.generate_labels({"compute-memory-partition": True}, "container", str(fi.sysfs), str(fi.dev))
    assert lab == {}


def test_no_partition_support(tmp_path):
    fi = make_mi355x_node(tmp_path, partition_support=False)
    lab = L.generate_labels({"compute-partitioning-supported": True, "memory-partitioning-supported": True},
                            "container", str(fi.sysfs), str(fi.dev))
    assert lab == {"amd.com/gpu.compute-partitioning-supported": "false",
                   "amd.com/gpu.memory-partitioning-supported": "false"}


def test_vf_labels(tmp_path):
    fi = make_mi355x_node(tmp_path, mode="vf", vfs_per_gpu=2)
    lab = L.generate_labels(ALL, "", str(fi.sysfs), str(fi.dev))
    assert lab["amd.com/gpu.mode"] == "vf-passthrough" and lab["beta.amd.com/gpu.mode"] == "vf-passthrough"
    assert lab["amd.com/gpu.driver-version"] == "8.1.0.K"      # cut at '+'
    assert lab["amd.com/gpu.driver-src-version"] == "F00DFACE0123456789ABCDE"
    assert lab["amd.com/gpu.device-id.0x75b3"] == "16"         # raw VF ids, as the reference emits them


def test_pf_labels(tmp_path):
    fi = make_mi355x_node(tmp_path, mode="pf")
    lab = L.generate_labels(ALL, "", str(fi.sysfs), str(fi.dev))
    assert lab["amd.com/gpu.mode"] == "pf-passthrough"
    assert "beta.amd.com/gpu.mode" not in lab
    assert lab["amd.com/gpu.device-id.0x75a3"] == "8"


def test_no_gpus_no_labels(tmp_path):
    (tmp_path / "sys").mkdir()
    assert L.generate_labels(ALL, "", str(tmp_path / "sys"), str(tmp_path / "dev")) == {}


def test_labeller_cli_dry_run(tmp_path, capsys):
    from rocm_k8s_device_plugin_amd.cli import node_labeller
    fi = make_mi355x_node(tmp_path)
    rc = node_labeller.main(["-dry_run", "-vram", "-cu-count=true", "-simd-count=false",
                             "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)])
    assert rc == 0
    out = json.loads(capsys.readouterr().out)
    assert out["amd.com/gpu.vram"] == "288G" and out["amd.com/gpu.cu-count"] == "256"
    assert not any("simd" in k for k in out)


def test_driver_version_fallback_when_card_has_no_module_version(tmp_path):
    """amdgpu built in / without a version under the card's driver/module: the
    reference labels "" (main.go:166-181); here /sys/module/amdgpu/version."""
    import os
    fi = make_mi355x_node(tmp_path)
    os.unlink(fi.sysfs / "bus/pci/drivers/amdgpu/module")
    lab = L.generate_labels({"driver-version": True}, "container", str(fi.sysfs), str(fi.dev))
    assert lab["amd.com/gpu.driver-version"] == "6.12.12"
    (fi.sysfs / "module/amdgpu/version").unlink()
    lab = L.generate_labels({"driver-version": True}, "container", str(fi.sysfs), str(fi.dev))
    assert lab["amd.com/gpu.driver-version"] == ""      # nothing left to read (no amd-smi here)


def test_label_values_are_valid_kubernetes_values():
    """One invalid value makes the apiserver reject the whole node patch."""
    import re
    ok = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")
    banner = "Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0,GNUld(GNUBinutils)2.46)#1-ant-ociSMP"
    assert L._driver_version_value(banner) == "6.18.54-ant.1"
    assert L._driver_version_value("6.12.12") == "6.12.12"
    for v in (banner, "a b", "(x)", "-lead", "trail-", "x" * 80, "", "6.12.12", "AMD_Instinct_MI355_OAM"):
        s = L.sanitize_label_value(v)
        assert len(s) <= 63 and ok.match(s), (v, s)
    assert L.sanitize_label_value("6.12.12") == "6.12.12"
