"""The full-chip sweep and the throughput check in the native health engine
(`mi355x-device-plugin -liveness_chip_sweep_every / -perf_check_every`), over
the stub probe. These are the scenarios of tests/test_perf_check.py for the
Python monitor: verdicts per perf_action, cadence, partition-scaled floors,
spawn mode, metrics and flag validation. The kernels themselves run in
tests/test_gpu.py."""
import asyncio
import json
import os
import subprocess
import sys
import urllib.request

import pytest

from rocm_k8s_device_plugin_amd.ops.native import core
from rocm_k8s_device_plugin_amd.testing.fake_kubelet import FakeKubelet
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node

from test_native_health import EXE, STUB, _by_ordinal, _stop
from test_native_metrics import _free_port, _series


@pytest.fixture(scope="module", autouse=True)
def _built():
    from rocm_k8s_device_plugin_amd import _build
    _build.ensure_built(hip=False)


def _engine(tmp_path, control, **opts):
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps(control))
    o = dict(dev_root=str(fi.dev), liveness=True, probe_exe=STUB, argv_prefix=[sys.executable], probe_timeout_s=3.0,
             extra_env={"MI355X_STUB_PROBE_CONTROL": str(ctl)}, fail_threshold=1, perf_check_every=1)
    o.update(opts)
    eng = core().HealthEngine(str(fi.sysfs), o)
    return fi, ctl, eng, _by_ordinal(eng)


def test_perf_report_mode(tmp_path):
    fi, ctl, eng, dev = _engine(tmp_path, {"perf": {"3": "slow_xcd", "4": "corrupt", "5": "slow_hbm",
                                                    "6": "slow_mfma"}})
    try:
        eng.sweep()
        snap, perf = eng.snapshot(), eng.perf_verdicts()
        assert eng.stats()["perf_checks"] == 1
        # wrong data is a failure whatever perf_action says; slow GPUs are only reported
        assert {d for d, (ok, _) in snap.items() if not ok} == {dev[4]}
        assert "hbm_bad_words=3" in snap[dev[4]][1][0]
        assert perf[dev[3]][0] == "degraded" and "XCD 3 at 510 MHz" in perf[dev[3]][1]
        assert perf[dev[5]][0] == "degraded" and "HBM read 1500" in perf[dev[5]][1]
        assert perf[dev[6]][0] == "degraded" and "bf16 MFMA 400" in perf[dev[6]][1]
        assert perf[dev[0]] == ("ok", "")
        text = core().metrics_render()
        assert f'mi355x_dp_perf_state{{device="{dev[3]}"}} 1.0' in text
        assert f'mi355x_dp_perf_state{{device="{dev[4]}"}} 2.0' in text
        assert f'mi355x_dp_perf_xcd_clock_mhz{{device="{dev[3]}",xcd="3"}} 510.0' in text
        assert f'mi355x_dp_perf_hbm_read_gbps{{device="{dev[0]}"}} 6000.0' in text
        ctl.write_text("{}")
        eng.sweep()
        assert all(ok for ok, _ in eng.snapshot().values())
        assert all(s == "ok" for s, _ in eng.perf_verdicts().values())
    finally:
        eng.close()


def test_perf_unhealthy_mode_and_cadence(tmp_path):
    fi, ctl, eng, dev = _engine(tmp_path, {"perf": {"3": "slow_xcd"}}, perf_action="unhealthy", perf_check_every=3)
    try:
        eng.sweep()                                   # sweep 0: checked
        assert not eng.snapshot()[dev[3]][0]
        ctl.write_text("{}")
        eng.sweep()                                   # sweeps 1, 2: no check, the verdict stands
        eng.sweep()
        assert eng.stats()["perf_checks"] == 1 and not eng.snapshot()[dev[3]][0]
        eng.sweep()                                   # sweep 3: checked again, passes
        assert eng.stats()["perf_checks"] == 2 and eng.snapshot()[dev[3]][0]
    finally:
        eng.close()


def test_perf_floors_scale_with_partition(tmp_path):
    _, _, eng, _ = _engine(tmp_path, {})
    try:
        whole = {"cu_count": 256, "hbm_read_gbps": 2900.0, "hbm_write_gbps": 4000.0, "mfma_tflops": 1500.0,
                 "xcd_clock_mhz": [1500.0] * 8}
        assert eng.perf_problems(whole) == ["HBM read 2900 GB/s < 3000"]
        cpx = {"cu_count": 32, "hbm_read_gbps": 700.0, "hbm_write_gbps": 600.0, "mfma_tflops": 180.0,
               "xcd_clock_mhz": [1500.0]}
        assert eng.perf_problems(cpx) == []
        assert eng.perf_problems(dict(cpx, mfma_tflops=50.0)) == ["bf16 MFMA 50 TFLOP/s < 88"]
    finally:
        eng.close()


def test_perf_spawn_mode(tmp_path):
    """Without the server the check runs per device in a fresh process (--perf)."""
    fi, ctl, eng, dev = _engine(tmp_path, {"perf": {"2": "corrupt", "1": "slow_mfma"}}, persistent=False)
    try:
        eng.sweep()
        perf = eng.perf_verdicts()
        assert perf[dev[2]][0] == "failed" and "hbm_bad_words" in perf[dev[2]][1]
        assert perf[dev[1]][0] == "degraded" and perf[dev[0]] == ("ok", "")
    finally:
        eng.close()


def test_busy_gpu_gets_neither_chip_sweep_nor_perf_check(tmp_path):
    from test_native_health import _busy_gpu
    from rocm_k8s_device_plugin_amd.topology import discover
    fi, ctl, eng, dev = _engine(tmp_path, {"perf": {"2": "corrupt", "5": "corrupt"}}, chip_sweep_every=1)
    try:
        _busy_gpu(fi, discover(str(fi.sysfs)), dev[5])
        eng.sweep()
        st = eng.stats()
        assert st["chip_sweeps"] == 1 and st["perf_checks"] == 1
        perf = eng.perf_verdicts()
        assert perf[dev[2]][0] == "failed" and dev[5] not in perf      # the busy GPU was not checked
    finally:
        eng.close()


def test_chip_sweep_replaces_the_probe_on_its_cadence(tmp_path):
    """A "pending" stub device never completes a one-wave probe but answers
    the chip sweep: on sweep turns it passes, on probe turns it fails."""
    fi, ctl, eng, dev = _engine(tmp_path, {"2": "pending"}, chip_sweep_every=2, perf_check_every=0,
                                keep_queues=False)
    try:
        eng.sweep()                                   # sweep 0: full-chip sweep
        assert eng.snapshot()[dev[2]][0] and eng.stats()["chip_sweeps"] == 1
        eng.sweep()                                   # sweep 1: one-wave probe, stays queued on an idle GPU
        assert not eng.snapshot()[dev[2]][0]
        eng.sweep()                                   # sweep 2: full-chip sweep again
        assert eng.stats()["chip_sweeps"] == 2 and eng.snapshot()[dev[2]][0]
    finally:
        eng.close()


def test_daemon_perf_check_and_validation(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"perf": {"4": "corrupt", "6": "slow_mfma"}}))
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = _by_ordinal(eng)
    eng.close()
    kdir = str(tmp_path / "dp")
    port = _free_port()

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                              "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe", STUB,
                              "-liveness_fail_threshold", "1", "-liveness_timeout", "3", "-perf_check_every", "1",
                              "-perf_action", "unhealthy", "-liveness_chip_sweep_every", "2",
                              "-metrics_port", str(port)],
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=dict(os.environ, MI355X_STUB_PROBE_CONTROL=str(ctl)))
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert {d for d, h in st.devices.items() if h == "Unhealthy"} == {dev[4], dev[6]}
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                s = _series(r.read().decode())
            assert s[f'mi355x_dp_perf_state{{device="{dev[4]}"}}'] == 2.0
            assert s[f'mi355x_dp_perf_state{{device="{dev[6]}"}}'] == 1.0
            assert s["mi355x_dp_perf_checks_total"] >= 1
            ctl.write_text("{}")
            st = await k.wait_for_update("amd.com/gpu", st.updates, timeout=20)
            assert all(h == "Healthy" for h in st.devices.values())
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "throughput check ok -> failed" in err

    asyncio.run(asyncio.wait_for(go(), 60))
    for args, want in ((["-perf_check_every", "5"], "needs -liveness"),
                       (["-pulse", "1", "-liveness", "-perf_check_every", "5", "-perf_action", "drain"],
                        "perf_action")):
        p = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=20)
        assert p.returncode == 1 and want in p.stderr, (args, p.stderr)


def test_daemon_shutdown_during_a_throughput_check_changes_no_verdict(tmp_path):
    """SIGTERM while a throughput check is in flight: the check is cut short,
    which is no verdict. No device flips to Unhealthy on the way out (found in
    an MI355X soak, where the last check of the run logged `ok -> failed ...
    probe interrupted (shutdown)` and `Healthy -> Unhealthy`)."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text("{}")
    eng = core().HealthEngine(str(fi.sysfs), {"dev_root": str(fi.dev)})
    dev = _by_ordinal(eng)
    eng.close()
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                              "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe", STUB,
                              "-liveness_fail_threshold", "1", "-liveness_timeout", "30", "-perf_check_every", "1",
                              "-perf_action", "unhealthy"],
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=dict(os.environ, MI355X_STUB_PROBE_CONTROL=str(ctl)))
        try:
            st = await k.wait_for_resource("amd.com/gpu", 8, timeout=20)
            assert all(h == "Healthy" for h in st.devices.values())
            ctl.write_text(json.dumps({"perf": {"2": "hang"}}))   # the next check never returns
            await asyncio.sleep(3.0)
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        assert "-> Unhealthy" not in err and "-> failed" not in err, err[-3000:]
        assert all(h == "Healthy" for h in k.resources["amd.com/gpu"].devices.values())
        return dev

    asyncio.run(asyncio.wait_for(go(), 60))


def test_daemon_shutdown_while_the_probe_server_starts_spawns_no_fallback(tmp_path):
    """SIGTERM while the probe server is still starting (its hello not yet read):
    that sweep is interrupted, not a failed server start, so the daemon does not
    fall back to one fresh GPU process per device on its way out."""
    fi = make_mi355x_node(tmp_path / "n")
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps({"serve": "slow_start", "serve_start_s": 60}))
    log = tmp_path / "starts.log"
    kdir = str(tmp_path / "dp")

    async def go():
        k = FakeKubelet(kdir)
        await k.start()
        p = subprocess.Popen([EXE, "-kubelet_dir", kdir, "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                              "-exporter_socket", "", "-pulse", "1", "-liveness", "-liveness_probe", STUB,
                              "-liveness_timeout", "30"],
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=dict(os.environ, MI355X_STUB_PROBE_CONTROL=str(ctl), MI355X_STUB_PROBE_LOG=str(log)))
        try:
            # the first sweep (before registration) starts the server and waits for its hello
            for _ in range(400):
                if log.exists() and log.read_text().startswith("serve"):
                    break
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.3)
        finally:
            rc, err = await asyncio.to_thread(_stop, p)
            await k.stop()
        assert rc == 0, err[-3000:]
        starts = log.read_text().split()
        assert starts and all(s.startswith("serve") for s in starts), (starts, err[-3000:])
        assert "re-probing each device in its own process" not in err, err[-3000:]
        assert "-> Unhealthy" not in err, err[-3000:]

    asyncio.run(asyncio.wait_for(go(), 60))
