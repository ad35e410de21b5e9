"""Node labeller: schema parity with cmd/k8s-node-labeller/main.go and the
reconcile loop against a fake apiserver."""
import json
import os
import time

import pytest

from rocm_k8s_device_plugin_amd import constants as C
from rocm_k8s_device_plugin_amd.labeller import labels as L
from rocm_k8s_device_plugin_amd.labeller.controller import NodeLabeller, label_patch
from rocm_k8s_device_plugin_amd.labeller.kube import KubeClient, KubeConfig, KubeError, load_kubeconfig
from rocm_k8s_device_plugin_amd.testing.fake_apiserver import FakeApiServer
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


def test_label_patch_minimal():
    cur = {"amd.com/gpu.vram": "64G", "beta.amd.com/gpu.vram": "64G", "beta.amd.com/gpu.vram.64G": "1",
           "other": "x"}
    want = {"amd.com/gpu.vram": "288G"}
    p = label_patch(cur, want)
    assert p == {"beta.amd.com/gpu.vram": None, "beta.amd.com/gpu.vram.64G": None, "amd.com/gpu.vram": "288G"}
    assert label_patch({"amd.com/gpu.vram": "288G"}, want) == {}


def test_reconcile_against_fake_apiserver(tmp_path):
    fi = make_mi355x_node(tmp_path)
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("node-a", {"amd.com/gpu.family": "stale", "beta.amd.com/gpu.family": "stale",
                                "beta.amd.com/gpu.family.stale": "8", "kubernetes.io/hostname": "node-a"})
        client = KubeClient(KubeConfig(server=srv.url, token="tok"))
        enabled = {**ALL, "firmware": False, "family": False}
        lab = NodeLabeller(client, "node-a",
                           lambda: L.generate_labels(enabled, "container", str(fi.sysfs), str(fi.dev)), resync_s=0)
        lab.run(once=True)
        got = srv.labels("node-a")
        assert got["kubernetes.io/hostname"] == "node-a"
        assert "amd.com/gpu.family" not in got and "beta.amd.com/gpu.family.stale" not in got
        assert got["amd.com/gpu.vram"] == "288G"
        patches = [r for r in srv.requests if r[0] == "PATCH"]
        assert len(patches) == 1
        # second pass: nothing to change -> no PATCH
        assert lab.reconcile_once()
        assert len([r for r in srv.requests if r[0] == "PATCH"]) == 1
        # someone deletes a label -> re-asserted
        srv.nodes["node-a"]["metadata"]["labels"].pop("amd.com/gpu.vram")
        assert lab.reconcile_once()
        assert srv.labels("node-a")["amd.com/gpu.vram"] == "288G"
        # apiserver errors are retried, not fatal
        srv.fail_next = 1
        assert not lab.reconcile_once()
        assert lab.stats.errors == 1
        assert lab.reconcile_once()
    finally:
        srv.stop()


def test_unauthorized_and_missing_node():
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("n")
        with pytest.raises(KubeError) as e:
            KubeClient(KubeConfig(server=srv.url, token="bad")).get_node("n")
        assert e.value.status == 401
        with pytest.raises(KubeError) as e:
            KubeClient(KubeConfig(server=srv.url, token="tok")).get_node("missing")
        assert e.value.status == 404
    finally:
        srv.stop()


def test_kubeconfig_parsing(tmp_path):
    import base64
    ca = base64.b64encode(b"-----BEGIN CERTIFICATE-----\nx\n-----END CERTIFICATE-----\n").decode()
    kc = tmp_path / "kubeconfig"
    kc.write_text(f"""
apiVersion: v1
kind: Config
current-context: c1
clusters:
- name: k1
  cluster: {{server: "https://10.0.0.1:6443/", certificate-authority-data: "{ca}"}}
contexts:
- name: c1
  context: {{cluster: k1, user: u1}}
users:
- name: u1
  user: {{token: abc}}
""")
    cfg = load_kubeconfig(str(kc))
    assert cfg.server == "https://10.0.0.1:6443" and cfg.token == "abc"
    assert cfg.ca_file and os.path.exists(cfg.ca_file)


def test_labeller_cli_dry_run(tmp_path, capsys):
    from rocm_k8s_device_plugin_amd.cli import node_labeller
    fi = make_mi355x_node(tmp_path)
    rc = node_labeller.main(["-dry_run", "-vram", "-cu-count=true", "-simd-count=false",
                             "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)])
    assert rc == 0
    out = json.loads(capsys.readouterr().out)
    assert out["amd.com/gpu.vram"] == "288G" and out["amd.com/gpu.cu-count"] == "256"
    assert not any("simd" in k for k in out)


def test_labeller_cli_against_fake_apiserver(tmp_path):
    from rocm_k8s_device_plugin_amd.cli import node_labeller
    fi = make_mi355x_node(tmp_path)
    srv = FakeApiServer(token=None).start()
    try:
        srv.add_node("worker-7")
        kc = tmp_path / "kc"
        kc.write_text(f"clusters: [{{name: a, cluster: {{server: '{srv.url}'}}}}]\n"
                      "contexts: [{name: a, context: {cluster: a, user: a}}]\ncurrent-context: a\n"
                      "users: [{name: a, user: {}}]\n")
        rc = node_labeller.main(["-kubeconfig", str(kc), "-node_name", "worker-7", "-once",
                                 "-mode", "-vram", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)])
        assert rc == 0
        got = srv.labels("worker-7")
        assert got["amd.com/gpu.mode"] == "container" and got["amd.com/gpu.vram"] == "288G"
    finally:
        srv.stop()


def test_reconcile_falls_back_to_update_without_patch_verb(tmp_path):
    """Upstream RBAC (get/list/watch/update, no patch) keeps working."""
    fi = make_mi355x_node(tmp_path)
    srv = FakeApiServer(token=None).start()
    try:
        srv.add_node("n1", {"beta.amd.com/gpu.vram": "64G", "beta.amd.com/gpu.vram.64G": "1", "x": "y"})
        srv.forbid = {"PATCH"}
        client = KubeClient(KubeConfig(server=srv.url))
        lab = NodeLabeller(client, "n1", lambda: L.generate_labels({"vram": True}, "container", str(fi.sysfs),
                                                                   str(fi.dev)), resync_s=0)
        assert lab.reconcile_once()
        assert lab.stats.updates == 1
        got = srv.labels("n1")
        assert got["amd.com/gpu.vram"] == "288G" and got["x"] == "y"
        assert "beta.amd.com/gpu.vram.64G" not in got
    finally:
        srv.stop()


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


def test_node_name_sources(tmp_path, monkeypatch):
    """-node_name / $DS_NODE_NAME first, else the hostname file the reference's
    README documents (cmd/k8s-node-labeller/README.md:10)."""
    from rocm_k8s_device_plugin_amd.cli import node_labeller as cli
    monkeypatch.delenv("DS_NODE_NAME", raising=False)
    ns = cli.build_parser().parse_args([])
    f = tmp_path / "hostname"
    assert cli.node_name_from(ns, str(f)) == ""
    f.write_text("gpu-node-7\n")
    assert cli.node_name_from(ns, str(f)) == "gpu-node-7"
    ns = cli.build_parser().parse_args(["-node_name", "n1"])
    assert cli.node_name_from(ns, str(f)) == "n1"


def _wait(pred, timeout=30.0):
    import time
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.01)
    return pred()


def _running_labeller(tmp_path, srv, **kw):
    import threading
    fi = make_mi355x_node(tmp_path)
    client = KubeClient(KubeConfig(server=srv.url, token="tok"))
    enabled = {**ALL, "firmware": False, "family": False}
    lab = NodeLabeller(client, "node-w", lambda: L.generate_labels(enabled, "container", str(fi.sysfs), str(fi.dev)),
                       resync_s=300, **kw)
    t = threading.Thread(target=lab.run, daemon=True)
    t.start()
    return lab, t


def _quiet(lab, for_s=0.5, limit_s=10.0):
    """Wait until the labeller has started no pass for `for_s`; its pass count then."""
    import time
    last, since, t0 = lab.stats.passes, time.monotonic(), time.monotonic()
    while time.monotonic() - since < for_s and time.monotonic() - t0 < limit_s:
        time.sleep(0.05)
        if lab.stats.passes != last:
            last, since = lab.stats.passes, time.monotonic()
    return last


def test_watch_restores_a_stripped_label_within_seconds(tmp_path):
    """Labels stripped by someone else come back from the watch event, not
    the 300 s resync (reference: controller-runtime watch, main.go:551-580)."""
    import time
    srv = FakeApiServer(token="tok").start()
    lab = t = None
    try:
        srv.add_node("node-w", {"kubernetes.io/hostname": "node-w"})
        lab, t = _running_labeller(tmp_path, srv)
        assert _wait(lambda: srv.labels("node-w").get("amd.com/gpu.vram") == "288G")
        assert _wait(lambda: srv.watch_starts >= 1)
        # let the passes of the start-up (and of our own first PATCH's event) finish first: a pass
        # counts when it starts, so one still running would restore the label uncounted
        passes = _quiet(lab)
        labels = srv.labels("node-w")
        labels.pop("amd.com/gpu.vram")
        t0 = time.monotonic()
        srv.set_labels("node-w", labels)
        # seconds, not the 300 s resync (bounded loosely: the suite may run on a loaded host or
        # against the -O0 coverage build of the native core)
        assert _wait(lambda: srv.labels("node-w").get("amd.com/gpu.vram") == "288G", 60.0)
        assert time.monotonic() - t0 < 60.0
        assert lab.stats.watch_kicks >= 1 and lab.stats.passes > passes
        # our own PATCH comes back as an event that needs nothing: no reconcile loop. Let a pass
        # that is still running finish, then nothing more may start.
        settled = _quiet(lab)
        time.sleep(0.6)
        assert lab.stats.passes == settled
    finally:
        if lab is not None:
            lab.stop()
            t.join(5)
        srv.stop()


def test_watch_relabels_a_recreated_node_and_survives_watch_expiry(tmp_path):
    srv = FakeApiServer(token="tok").start()
    lab = t = None
    try:
        srv.add_node("node-w")
        lab, t = _running_labeller(tmp_path, srv)
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-w"))
        assert _wait(lambda: srv.watch_starts >= 1)
        srv.expire_watches()                       # apiserver ends the watch: reconnect
        assert _wait(lambda: srv.watch_starts >= 2)
        srv.delete_node("node-w")
        srv.add_node("node-w", {"kubernetes.io/hostname": "node-w"})   # re-created without labels
        assert _wait(lambda: srv.labels("node-w").get("amd.com/gpu.vram") == "288G", 30.0)
        # a watch from a compacted resourceVersion gets 410: re-list, keep going
        starts = srv.watch_starts
        srv.min_rv = 10 ** 6
        srv.expire_watches()
        assert _wait(lambda: srv.watch_starts >= starts + 2)    # 410, then a fresh watch (no resourceVersion)
        srv.min_rv = 0
        assert t.is_alive() and lab.stats.watch_errors == 0
    finally:
        if lab is not None:
            lab.stop()
            t.join(5)
            assert not t.is_alive()
        srv.stop()


def test_watch_failure_backs_off_and_resync_still_applies(tmp_path):
    """Without the watch verb (403) the labeller logs, backs off and keeps its
    periodic resync."""
    srv = FakeApiServer(token="tok").start()
    lab = t = None
    try:
        srv.add_node("node-w")
        srv.forbid = set()
        orig = srv.requests
        lab, t = _running_labeller(tmp_path, srv, watch_backoff_max_s=0.2)
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-w"))
        assert _wait(lambda: srv.watch_starts >= 1)
        srv.token = "other"          # every later request is 401, the watch included
        srv.expire_watches()
        assert _wait(lambda: lab.stats.watch_errors >= 2, 30.0)
        assert orig is srv.requests and t.is_alive()
    finally:
        if lab is not None:
            lab.stop()
            t.join(5)
        srv.stop()


def test_rotated_service_account_token_is_picked_up(tmp_path, monkeypatch):
    """kubelet rewrites the projected token inside its lifetime: requests use
    the new file content (mtime change), and a 401 re-reads the file once."""
    from rocm_k8s_device_plugin_amd.labeller import kube
    srv = FakeApiServer(token="tok-1").start()
    try:
        srv.add_node("n1")
        sa = tmp_path / "sa"
        sa.mkdir()
        (sa / "token").write_text("tok-1\n")
        monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "127.0.0.1")
        cfg = kube.in_cluster_config(str(sa))
        cfg.server = srv.url                       # plain HTTP fake
        c = KubeClient(cfg)
        assert c.get_node("n1")["metadata"]["name"] == "n1"
        # rotation: the server and the file move to tok-2 together
        srv.token = "tok-2"
        (sa / "token").write_text("tok-2\n")
        os.utime(sa / "token", ns=(time.time_ns(), time.time_ns() + 10**9))
        assert c.get_node("n1")["metadata"]["name"] == "n1" and cfg.token == "tok-2"
        # the server moved on first (mtime unchanged): the 401 forces a re-read
        st = os.stat(sa / "token")
        srv.token = "tok-3"
        (sa / "token").write_text("tok-3\n")
        os.utime(sa / "token", ns=(st.st_atime_ns, st.st_mtime_ns))
        assert c.get_node("n1")["metadata"]["name"] == "n1" and cfg.token == "tok-3"
        # a stale file stays a 401 (one retry, no loop)
        srv.token = "tok-4"
        with pytest.raises(KubeError) as ei:
            c.get_node("n1")
        assert ei.value.status == 401
        (sa / "token").unlink()
        with pytest.raises(KubeError):
            kube.in_cluster_config(str(sa))
    finally:
        srv.stop()


def test_watch_cut_right_away_backs_off_instead_of_spinning(tmp_path):
    """A server (or proxy) that ends every watch stream at once is reconnected
    with backoff, not in a tight loop; a stripped label still comes back."""
    srv = FakeApiServer(token="tok").start()
    lab = t = None
    try:
        srv.add_node("node-w")
        srv.watch_max_s = 0.0
        lab, t = _running_labeller(tmp_path, srv, watch_backoff_max_s=0.4)
        assert _wait(lambda: "amd.com/gpu.vram" in srv.labels("node-w"))
        time.sleep(2.0)
        # backoff 0.2, 0.4, 0.4, ...: a handful of reconnects in 2 s (a spin makes hundreds)
        assert 2 <= srv.watch_starts <= 12, srv.watch_starts
        assert lab.stats.watch_errors == 0 and t.is_alive()
    finally:
        if lab is not None:
            lab.stop()
            t.join(5)
        srv.stop()


def _tls_material(d):
    """A CA and a server certificate for 127.0.0.1 signed by it (openssl CLI)."""
    import shutil
    import subprocess
    if not shutil.which("openssl"):
        pytest.skip("openssl not installed")

    def run(*a):
        subprocess.run(["openssl", *a], check=True, capture_output=True, timeout=60)
    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "ca.key"), "-out", str(d / "ca.crt"),
        "-days", "2", "-subj", "/CN=test-ca")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "srv.key"), "-out", str(d / "srv.csr"),
        "-subj", "/CN=kubernetes")
    (d / "ext.cnf").write_text("subjectAltName=IP:127.0.0.1,DNS:kubernetes.default.svc\n")
    run("x509", "-req", "-in", str(d / "srv.csr"), "-CA", str(d / "ca.crt"), "-CAkey", str(d / "ca.key"),
        "-CAcreateserial", "-out", str(d / "srv.crt"), "-days", "2", "-extfile", str(d / "ext.cnf"))
    return str(d / "srv.crt"), str(d / "srv.key"), str(d / "ca.crt")


def test_labeller_in_cluster_over_tls(tmp_path, monkeypatch):
    """The production path: in-cluster service-account token and CA bundle, HTTPS
    with certificate verification (main.go uses controller-runtime's
    GetConfigOrDie, which resolves to the same in-cluster config)."""
    from rocm_k8s_device_plugin_amd.cli import node_labeller
    from rocm_k8s_device_plugin_amd.labeller import kube
    crt, key, ca = _tls_material(tmp_path)
    fi = make_mi355x_node(tmp_path / "n")
    srv = FakeApiServer(token="sa-token", tls=(crt, key)).start()
    try:
        srv.add_node("worker-9")
        sa = tmp_path / "sa"
        sa.mkdir()
        (sa / "token").write_text("sa-token\n")
        (sa / "ca.crt").write_text(open(ca).read())
        monkeypatch.setattr(kube, "SA_DIR", str(sa))
        monkeypatch.delenv("KUBECONFIG", raising=False)
        monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "127.0.0.1")
        monkeypatch.setenv("KUBERNETES_SERVICE_PORT", str(srv.port))
        cfg = kube.in_cluster_config(str(sa))
        assert cfg.server == f"https://127.0.0.1:{srv.port}" and cfg.ca_file == str(sa / "ca.crt")
        rc = node_labeller.main(["-node_name", "worker-9", "-once", "-mode", "-cu-count",
                                 "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev)])
        assert rc == 0
        got = srv.labels("worker-9")
        assert got["amd.com/gpu.mode"] == "container" and got["amd.com/gpu.cu-count"] == "256"
        # a CA that did not sign the server certificate is refused, not ignored
        other = tmp_path / "other"
        other.mkdir()
        _, _, bad_ca = _tls_material(other)
        bad = KubeClient(KubeConfig(server=cfg.server, token="sa-token", ca_file=bad_ca))
        with pytest.raises(Exception) as ei:
            bad.get_node("worker-9")
        assert "CERTIFICATE_VERIFY_FAILED" in str(ei.value) or "certificate verify failed" in str(ei.value)
    finally:
        srv.stop()


def test_partition_switch_relabels_on_the_next_resync(tmp_path):
    """Labels are generated again on every reconcile, so a compute/memory
    partition switch reaches the node on the next pass (the reference computes
    them once at start-up)."""
    import shutil
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    srv = FakeApiServer(token="tok").start()
    try:
        srv.add_node("worker-3")
        client = KubeClient(KubeConfig(server=srv.url, token="tok"))
        enabled = {"compute-memory-partition": True, "cu-count": True, "mode": True}
        lab = NodeLabeller(client, "worker-3",
                           lambda: L.generate_labels(enabled, "container", str(fi.sysfs), str(fi.dev)),
                           resync_s=0, watch=False)
        assert lab.reconcile_once()
        before = srv.labels("worker-3")
        assert before["amd.com/gpu.compute-memory-partition"] == "spx_nps1"
        assert before["amd.com/gpu.cu-count"] == "256"
        # the driver now shows CPX / NPS2 (a fresh tree swapped in, as after a switch)
        new = tmp_path / "n.new"
        make_mi355x_node(new, compute_partition="cpx", memory_partition="nps2")
        shutil.rmtree(root / "sys")
        os.rename(new / "sys", root / "sys")
        assert lab.reconcile_once()
        after = srv.labels("worker-3")
        assert after["amd.com/gpu.compute-memory-partition"] == "cpx_nps2"
        assert after["amd.com/gpu.cu-count"] == "32"
        assert not any(k.startswith("beta.amd.com/gpu.compute-memory-partition.spx") for k in after)
    finally:
        srv.stop()


def test_topology_watch_relabels_within_a_second(tmp_path):
    """-topology_watch: the labeller polls the GPU topology fingerprint and
    relabels on a change without waiting for the (here 1 h) resync."""
    import shutil
    import threading
    import time
    from rocm_k8s_device_plugin_amd.topology import topology_signature
    root = tmp_path / "n"
    fi = make_mi355x_node(root)
    srv = FakeApiServer(token="tok").start()
    lab = None
    try:
        srv.add_node("worker-4")
        client = KubeClient(KubeConfig(server=srv.url, token="tok"))
        enabled = {"compute-memory-partition": True}
        lab = NodeLabeller(client, "worker-4",
                           lambda: L.generate_labels(enabled, "container", str(fi.sysfs), str(fi.dev)),
                           resync_s=3600, watch=False, change_source=lambda: topology_signature(str(fi.sysfs)),
                           change_interval_s=0.1)
        t = threading.Thread(target=lab.run, daemon=True)
        t.start()
        deadline = time.monotonic() + 10
        while srv.labels("worker-4").get("amd.com/gpu.compute-memory-partition") != "spx_nps1":
            assert time.monotonic() < deadline
            time.sleep(0.02)
        # swapped in two renames, as the driver's view changes at once (an rmtree of the old tree
        # first would leave half a tree to poll for as long as the deletion takes on a loaded host)
        from test_reload import repartition
        repartition(root, compute_partition="dpx", generation=2)
        t0 = time.monotonic()
        while srv.labels("worker-4").get("amd.com/gpu.compute-memory-partition") != "dpx_nps1":
            # ~0.2 s when idle (two 0.1 s polls + one relabel); 60 s leaves room for a loaded CI host,
            # still far from the 1 h resync
            assert time.monotonic() - t0 < 60.0, srv.labels("worker-4")
            time.sleep(0.02)
        assert lab.stats.topology_changes == 1
    finally:
        if lab is not None:
            lab.stop()
        srv.stop()
