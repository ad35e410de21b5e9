"""Throughput check (HBM pattern bandwidth, sustained MFMA rate, per-XCD clocks):
the monitor's verdicts and metrics over the stub probe, and the CLI wiring.
The kernels themselves run in tests/test_gpu.py."""
import asyncio
import json
import os
import subprocess
import sys

from rocm_k8s_device_plugin_amd.health.liveness import LivenessProber
from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig, HealthMonitor
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover
from rocm_k8s_device_plugin_amd.utils.metrics import REGISTRY

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(REPO, "rocm_k8s_device_plugin_amd", "testing", "stub_probe.py")


def _monitor(tmp_path, control, **cfg):
    fi = make_mi355x_node(tmp_path / "n")
    inv = discover(str(fi.sysfs))
    ctl = tmp_path / "ctl.json"
    ctl.write_text(json.dumps(control))
    prober = LivenessProber(exe=STUB, argv_prefix=[sys.executable], timeout_s=3.0,
                            extra_env={"MI355X_STUB_PROBE_CONTROL": str(ctl)}, **cfg.pop("prober", {}))
    hc = HealthConfig(exporter_socket=None, liveness=True, fail_threshold=1, perf_check_every=1, **cfg)
    mon = HealthMonitor(inv, hc, prober=prober, ordinal_map={d.id: i for i, d in enumerate(inv.devices)})
    return fi, ctl, mon


def test_perf_report_mode(tmp_path):
    fi, ctl, mon = _monitor(tmp_path, {"perf": {"3": "slow_xcd", "4": "corrupt", "5": "slow_hbm", "6": "slow_mfma"}})

    async def go():
        await mon.check_once()
        snap, perf = mon.snapshot(), mon.perf_verdicts()
        assert mon.perf_checks == 1
        # wrong data is a failure whatever perf_action says; slow GPUs are only reported
        assert {d for d, v in snap.items() if v.health == "Unhealthy"} == {fi.bdfs[4]}
        assert "hbm_bad_words=3" in snap[fi.bdfs[4]].reasons[0]
        assert perf[fi.bdfs[3]][0] == "degraded" and "XCD 3 at 510 MHz" in perf[fi.bdfs[3]][1]
        assert perf[fi.bdfs[5]][0] == "degraded" and "HBM read 1500" in perf[fi.bdfs[5]][1]
        assert perf[fi.bdfs[6]][0] == "degraded" and "bf16 MFMA 400" in perf[fi.bdfs[6]][1]
        assert perf[fi.bdfs[0]] == ("ok", "")
        text = REGISTRY.render()
        assert f'mi355x_dp_perf_state{{device="{fi.bdfs[3]}"}} 1' in text
        assert f'mi355x_dp_perf_state{{device="{fi.bdfs[4]}"}} 2' in text
        assert f'mi355x_dp_perf_xcd_clock_mhz{{device="{fi.bdfs[3]}",xcd="3"}} 510' in text
        assert f'mi355x_dp_perf_hbm_read_gbps{{device="{fi.bdfs[0]}"}} 6000' in text
        ctl.write_text("{}")
        await mon.check_once()
        assert all(v.health == "Healthy" for v in mon.snapshot().values())
        assert all(s == "ok" for s, _ in mon.perf_verdicts().values())
        await mon.close()

    asyncio.run(asyncio.wait_for(go(), 60))


def test_perf_unhealthy_mode_and_cadence(tmp_path):
    fi, ctl, mon = _monitor(tmp_path, {"perf": {"3": "slow_xcd"}}, perf_action="unhealthy")
    mon.cfg.perf_check_every = 3

    async def go():
        await mon.check_once()                        # sweep 0: checked
        assert mon.snapshot()[fi.bdfs[3]].health == "Unhealthy"
        ctl.write_text("{}")
        await mon.check_once()                        # sweeps 1, 2: no check, the verdict stands
        await mon.check_once()
        assert mon.perf_checks == 1 and mon.snapshot()[fi.bdfs[3]].health == "Unhealthy"
        await mon.check_once()                        # sweep 3: checked again, passes
        assert mon.perf_checks == 2 and mon.snapshot()[fi.bdfs[3]].health == "Healthy"
        await mon.close()

    asyncio.run(asyncio.wait_for(go(), 60))


def test_perf_floors_scale_with_partition(tmp_path):
    _, _, mon = _monitor(tmp_path, {})
    whole = {"cu_count": 256, "hbm_read_gbps": 2900.0, "hbm_write_gbps": 4000.0, "mfma_tflops": 1500.0,
             "xcd_clock_mhz": [1500] * 8}
    assert mon.perf_problems(whole) == ["HBM read 2900 GB/s < 3000"]
    # a CPX partition (32 CUs, one XCD) is held to an eighth of the floors
    cpx = {"cu_count": 32, "hbm_read_gbps": 700.0, "hbm_write_gbps": 600.0, "mfma_tflops": 180.0,
           "xcd_clock_mhz": [1500]}
    assert mon.perf_problems(cpx) == []
    assert mon.perf_problems(dict(cpx, mfma_tflops=50.0)) == ["bf16 MFMA 50 TFLOP/s < 88"]


def test_perf_spawn_mode(tmp_path):
    """Without the server the check runs per device in a fresh process (--perf)."""
    fi, ctl, mon = _monitor(tmp_path, {"perf": {"2": "corrupt"}}, liveness_mode="spawn",
                            prober={"mode": "spawn"})

    async def go():
        res = await mon.prober.perf({fi.bdfs[1]: 1, fi.bdfs[2]: 2})
        assert res[fi.bdfs[1]].ok and res[fi.bdfs[1]].detail["mfma_tflops"] == 1550.0
        assert not res[fi.bdfs[2]].ok and "hbm_bad_words" in res[fi.bdfs[2]].reason

    asyncio.run(asyncio.wait_for(go(), 60))


def test_perf_cli_validation(tmp_path):
    fi = make_mi355x_node(tmp_path / "n")
    env = dict(os.environ, PYTHONPATH=REPO)
    base = [sys.executable, "-m", "rocm_k8s_device_plugin_amd.cli.device_plugin", "-dry_run", "-sysfs_root",
            str(fi.sysfs), "-dev_root", str(fi.dev), "-exporter_socket", "", "-kubelet_dir", str(tmp_path / "k")]
    bad = subprocess.run(base + ["-perf_check_every", "5"], capture_output=True, text=True, timeout=120, env=env)
    assert bad.returncode != 0 and "needs -liveness" in bad.stderr
    bad = subprocess.run(base + ["-liveness", "-perf_check_every", "5", "-perf_action", "drain"], capture_output=True,
                         text=True, timeout=120, env=env)
    assert bad.returncode != 0 and "perf_action" in bad.stderr


def test_perf_in_dry_run(tmp_path):
    """-dry_run with -pulse and -perf_check_every reports each idle GPU's throughput."""
    from rocm_k8s_device_plugin_amd.cli.device_plugin import dry_run_report
    from rocm_k8s_device_plugin_amd.plugin.container import ContainerImpl
    fi, ctl, mon = _monitor(tmp_path, {"perf": {"2": "slow_hbm"}})
    impl = ContainerImpl("single", str(fi.sysfs), inventory=mon.inv, monitor=mon)
    doc = asyncio.run(asyncio.wait_for(dry_run_report(impl, sweep=True), 60))
    thr = doc["throughput"]
    assert len(thr) == 8 and thr[fi.bdfs[2]]["state"] == "degraded" and "HBM read 1500" in thr[fi.bdfs[2]]["reason"]
    assert thr[fi.bdfs[0]]["state"] == "ok" and thr[fi.bdfs[0]]["hbm_read_gbps"] == 6000.0
    json.dumps(doc)
