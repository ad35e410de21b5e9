"""`mi355x-device-plugin -dry_run`: the node report (what kubelet would be
told, the preferred sets for 1/2/4/8/all devices with their xGMI fabric, CDI
settings, health) equals the Python CLI's `-dry_run` on the same node; with
the health engine on, it carries the throughput check and xGMI sections."""
import json
import os
import subprocess
import sys

import pytest

from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

from test_native_health import EXE, STUB

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _norm(doc):
    for r in doc["resources"].values():
        r["devices"] = sorted(r["devices"], key=lambda d: d["id"])
    return doc


def _both(fi, tmp_path, *args):
    common = ["-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", "",
              "-kubelet_dir", str(tmp_path / "dp"), *args]
    nat = subprocess.run([EXE, *common], capture_output=True, text=True, timeout=60)
    assert nat.returncode == 0, nat.stderr[-2000:]
    py = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", *common],
                        capture_output=True, text=True, timeout=120, env=dict(os.environ, PYTHONPATH=REPO))
    assert py.returncode == 0, py.stderr[-2000:]
    return _norm(json.loads(nat.stdout)), _norm(json.loads(py.stdout))


@pytest.mark.parametrize("partition,args", [
    ("spx", []),
    ("cpx", []),
    ("cpx", ["-resource_naming_strategy", "mixed", "-device_list_strategy", "cdi-cri,device-specs"]),
    ("dpx", ["-pulse", "1"]),
])
def test_report_equals_the_python_cli(tmp_path, partition, args):
    fi = make_mi355x_node(tmp_path / "n", compute_partition=partition)
    extra = list(args)
    if "-device_list_strategy" in extra:
        extra += ["-cdi_spec_dir", str(tmp_path / "cdi")]
    nat, py = _both(fi, tmp_path, *extra)
    assert nat == py
    assert nat["implementation"] == "container" and nat["resources"]
    for r in nat["resources"].values():
        assert r["preferred_allocation"] and "1" in r["allocations"]


def test_whole_node_allocation_reports_the_ring_bound(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    nat, _ = _both(fi, tmp_path)
    a8 = nat["resources"]["amd.com/gpu"]["allocations"]["8"]
    assert len(a8["ids"]) == 8 and a8["one_hive"] and a8["allreduce_bound_gbs"] == 7 * 76.0


def test_report_with_health_engine_sections(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"perf": {"2": "slow_hbm"}}))
    xg = tmp_path / "xgmi.json"
    xg.write_text(json.dumps({"ok": True, "error": "", "gpus": []}))
    p = subprocess.run([EXE, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                        "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe", STUB,
                        "-perf_check_every", "1", "-smi_xgmi"], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, MI355X_STUB_PROBE_CONTROL=str(ctl), MI355X_SMI_XGMI_FILE=str(xg)))
    assert p.returncode == 0, p.stderr[-2000:]
    doc = json.loads(p.stdout)
    thr = doc["throughput"]
    assert len(thr) == 8 and sorted(s["state"] for s in thr.values()).count("degraded") == 1
    slow = [d for d, s in thr.items() if s["state"] == "degraded"][0]
    assert "HBM read 1500" in thr[slow]["reason"] and thr[slow]["hbm_read_gbps"] == 1500
    ok = [s for s in thr.values() if s["state"] == "ok"][0]
    assert ok["hbm_read_gbps"] == 6000 and len(ok["xcd_clock_mhz"]) == 8
    assert doc["xgmi"] == {"readings": 1, "error": "", "degraded_pairs": [], "links_down": {}}
    assert all(d["health"] == "Healthy" for d in doc["resources"]["amd.com/gpu"]["devices"])


def test_trace_file_spans(tmp_path):
    """-trace_file: Chrome-trace spans of the admission path (RPC -> allocator)
    and the health path (sweep -> probe request), written at shutdown."""
    import asyncio
    from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
    from test_native_health import _stop
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    kdir, trace = str(tmp_path / "dp"), tmp_path / "trace.json"

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                              "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe", STUB,
                              "-trace_file", str(trace)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                             text=True, env=dict(os.environ, MI355X_STUB_PROBE_CONTROL=str(ctl)))
        try:
            await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            await k.admit("amd.com/gpu", 3)
            await asyncio.sleep(1.2)
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-2000:]

    asyncio.run(asyncio.wait_for(go(), 60))
    doc = json.loads(trace.read_text())
    ev = doc["traceEvents"]
    names = {e["name"] for e in ev}
    assert {"GetPreferredAllocation", "Allocate", "allocator.allocate", "health.sweep", "liveness.request"} <= names
    alloc = [e for e in ev if e["name"] == "Allocate"][0]
    assert alloc["ph"] == "X" and alloc["cat"] == "rpc" and alloc["args"]["resource"] == "gpu"
    assert len(alloc["args"]["ids"].split(",")) == 3 and alloc["dur"] >= 0
    sweep = [e for e in ev if e["name"] == "health.sweep"][0]
    req = [e for e in ev if e["name"] == "liveness.request"][0]
    assert sweep["ts"] <= req["ts"] and req["ts"] + req["dur"] <= sweep["ts"] + sweep["dur"] + 1   # nested


def test_device_ids_restricts_the_advertised_set(tmp_path):
    fi = make_mi355x_node(tmp_path / "n", compute_partition="cpx")
    keep = ["amdgpu_xcp_1", "amdgpu_xcp_9", fi.bdfs[0]]
    p = subprocess.run([EXE, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket",
                        "", "-device_ids", ",".join(keep + ["bogus"])], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    devs = {d["id"] for d in json.loads(p.stdout)["resources"]["amd.com/gpu"]["devices"]}
    assert devs == set(keep) and "-device_ids: bogus is not a discovered device" in p.stderr


@pytest.mark.parametrize("sub", ["topology-parsing/topology", "topology-parsing-mi308/topology",
                                 "topo-mi300-cpx/topology", "topo-mi210-xgmi-pcie"])
def test_report_on_reference_captures_equals_the_python_cli(tmp_path, ref_testdata, sub):
    """The reference's own kfd captures (wrapped with the PCI / drm entries
    discovery joins them with): same report from both implementations, and on
    the MI210 capture (two xGMI hives of 4, PCIe between them) a pod of 4
    stays in one hive (3 xGMI links of 50 GB/s per GPU: a 150 GB/s ring bound)
    while all 8 span the hives, whose link the capture gives no bandwidth:
    no bound is claimed for it."""
    from rocm_k8s_device_plugin_amd.testing.fixtures import wrap_kfd_topology
    fi = wrap_kfd_topology(ref_testdata / sub, tmp_path / "n")
    nat, py = _both(fi, tmp_path)
    assert nat == py
    if sub == "topo-mi210-xgmi-pcie":
        allocs = nat["resources"]["amd.com/gpu"]["allocations"]
        assert allocs["4"]["one_hive"] and allocs["4"]["allreduce_bound_gbs"] == 150
        assert allocs["2"]["allreduce_bound_gbs"] == 50
        assert not allocs["8"]["one_hive"] and allocs["8"]["allreduce_bound_gbs"] is None


@pytest.mark.parametrize("partition", ["spx", "cpx"])
def test_device_count_limit_equals_the_python_cli(tmp_path, monkeypatch, partition):
    """AMD_GPU_DEVICE_COUNT, else gpu.device_count of -config (documented by the
    reference, docs/user-guide/configuration.md:11,45-91): the first N physical
    GPUs are advertised, every partition of each."""
    fi = make_mi355x_node(tmp_path / "n", compute_partition=partition)
    per_gpu = 8 if partition == "cpx" else 1
    cfg = tmp_path / "config.yaml"
    cfg.write_text("gpu:\n  device_count: 5\n    # five GPUs\n")   # an indented comment ends the scalar

    def advertised(doc):
        return len(doc["resources"]["amd.com/gpu"]["devices"])

    for env, config, gpus in (("2", "", 2), (" 3 ", "", 3), ("x", str(cfg), 5), ("", str(cfg), 5),
                              ("-1", str(cfg), 5), ("1", str(cfg), 1)):
        monkeypatch.setenv("AMD_GPU_DEVICE_COUNT", env)
        nat, py = _both(fi, tmp_path, *(["-config", config] if config else []))
        assert nat == py, (env, config)
        assert advertised(nat) == gpus * per_gpu, (env, config)
    monkeypatch.delenv("AMD_GPU_DEVICE_COUNT")
    common = ["-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", ""]
    bad = tmp_path / "bad.yaml"
    bad.write_text("gpu:\n  device_count: lots\n")
    for path, why in ((bad, "bad gpu.device_count"), (tmp_path / "missing.yaml", "is unreadable")):
        p = subprocess.run([EXE, *common, "-config", str(path)], capture_output=True, text=True, timeout=60)
        assert p.returncode == 1 and why in p.stderr, p.stderr[-500:]
        q = subprocess.run([sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", *common,
                            "-config", str(path)], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, PYTHONPATH=REPO))
        assert q.returncode != 0


@pytest.mark.parametrize("unknown", [0, 2])
def test_kfd_denied_node_report_equals_the_python_cli(tmp_path, unknown):
    """Every kfd GPU node denied (a container's device cgroup): devices are
    identified from PCI sysfs; when some lack even a sysfs unique_id the
    physical-GPU identity is unknown and preferred allocation is switched off
    (kubelet picks), the devices still advertised."""
    from rocm_k8s_device_plugin_amd.testing.fixtures import deny_kfd_nodes
    fi = make_mi355x_node(tmp_path / "n", compute_partition="dpx", xcp_layout="kernel")
    deny_kfd_nodes(fi, sorted(set(fi.node_ids.values())))
    for b in fi.bdfs[:unknown]:
        os.remove(fi.sysfs / "devices/pci0000:00" / b / "unique_id")
    nat, py = _both(fi, tmp_path)
    assert nat == py
    r = nat["resources"]["amd.com/gpu"]
    assert len(r["devices"]) == 16 and r["preferred_allocation"] is (unknown == 0)
    assert any("unreadable" in w for w in nat["warnings"])
    assert bool([w for w in nat["warnings"] if "identity unknown" in w]) is (unknown > 0)
