"""Fabric model of allocated sets and the RCCL/gloo collective check (CPU)."""
import json
import os
import socket
import subprocess
import time
import sys

import pytest

from rocm_k8s_device_plugin_amd.models import MI355X
from rocm_k8s_device_plugin_amd.parallel import Fabric
from rocm_k8s_device_plugin_amd.parallel.collectives import BUS_FACTOR, parse_size, summary
from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
from rocm_k8s_device_plugin_amd.topology import discover

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_full_hive_bound(tmp_path):
    inv = discover(str(make_mi355x_node(tmp_path / "n").sysfs))
    fab = Fabric(inv)
    ids = [d.id for d in inv.devices]
    for k in (2, 4, 8):
        r = fab.report(ids[:k])
        assert r.one_hive and r.physical_gpus == k
        assert r.pairs["xgmi"] == k * (k - 1) // 2 and r.pairs["pcie"] == 0
        assert r.min_xgmi_degree == k - 1
        # k-1 links per GPU carry a ring each: the bound grows with the set
        assert r.allreduce_bound_gbs == pytest.approx((k - 1) * MI355X.xgmi_link_mbps / 1000)
    assert fab.report(ids[:1]).allreduce_bound_gbs is None


def test_split_hive_is_bounded_by_pcie(tmp_path):
    inv = discover(str(make_mi355x_node(tmp_path / "n", hive_size=4).sysfs))
    fab = Fabric(inv)
    ids = [d.id for d in inv.devices]
    same = fab.report(ids[:4])
    split = fab.report(ids[2:6])          # 2 GPUs from each hive
    assert same.one_hive and not split.one_hive
    assert split.pairs["pcie"] == 4 and split.pairs["xgmi"] == 2
    assert "crosses PCIe" in split.note
    assert same.allreduce_bound_gbs == pytest.approx(3 * MI355X.xgmi_link_mbps / 1000)
    assert split.allreduce_bound_gbs is None or split.allreduce_bound_gbs < same.allreduce_bound_gbs


def test_partitions_share_their_gpu(tmp_path):
    inv = discover(str(make_mi355x_node(tmp_path / "n", compute_partition="cpx").sysfs))
    fab = Fabric(inv)
    gpus = list(inv.physical_gpus().values())
    one = fab.report([d.id for d in gpus[0][:4]])
    assert one.physical_gpus == 1 and one.pairs["same_gpu"] == 6
    two = fab.report([d.id for d in gpus[0][:2] + gpus[1][:2]])
    assert two.physical_gpus == 2 and two.pairs["same_gpu"] == 2 and two.pairs["xgmi"] == 4
    assert two.allreduce_bound_gbs == pytest.approx(MI355X.xgmi_link_mbps / 1000)


def test_bus_factors_and_sizes():
    assert BUS_FACTOR["all_reduce"](8) == pytest.approx(1.75)
    assert BUS_FACTOR["all_gather"](8) == pytest.approx(0.875)
    assert parse_size("64K") == 65536 and parse_size("1M") == 1 << 20 and parse_size("123") == 123
    s = summary([{"op": "all_reduce", "bytes": 1, "busbw_gbs": 1.0, "ok": True},
                 {"op": "all_reduce", "bytes": 4, "busbw_gbs": 3.0, "ok": True},
                 {"op": "reduce_scatter", "bytes": 4, "ok": None, "unsupported": "gloo"}])
    assert s["ok"] and s["busbw_gbs"] == {"all_reduce": 3.0}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_collectives_gloo_two_ranks():
    """The pod-side CLI, launched the way a pod would (torchrun, one rank per device), on gloo."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "-m", "rocm_k8s_device_plugin_amd.parallel.collectives",
           "--sizes", "4K,64K", "--iters", "2", "--warmup", "1", "--dtype", "float32"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    ops = {r["op"] for r in rows}
    assert {"all_reduce", "all_gather", "all_to_all"} <= ops
    for r in rows:
        assert r["ranks"] == 2
        if not r.get("unsupported"):
            assert r["ok"] is True and r["algbw_gbs"] > 0


def test_bench_fixture_reports_fabric_and_collectives():
    """bench.py at N=2 on the fixture: the timed admissions, then collectives on the 2 ranks."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--fixture", "--steps", "2",
           "--warmup", "1"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["higher_is_better"] is False
    fab, rccl = d["extra"]["fabric"], d["extra"]["rccl"]
    assert fab["one_hive"] and fab["pairs"]["xgmi"] == 1
    assert rccl["ok"] and rccl["backend"] == "gloo" and rccl["busbw_gbs"]["all_reduce"] > 0
    # the containers went through the runtime path: the pod's process saw both GPUs'
    # render nodes, and the per-GPU comparison split them one per rank
    e = d["extra"]
    assert e["container_dev_view"] == "specs" and e["latency_p50_ms_container_mode_per-gpu"] > 0
    # the plugin under test is the primary entrypoint, the native daemon
    assert e["plugin"] == "native-daemon" == d["config"]["plugin"]
    assert set(e["plugin_server_p50_us"]) == {"GetPreferredAllocation", "Allocate"}
    assert len(e["steps_ms"]) == 2
    # gloo carries the step barriers: no rank holds a GPU context or kfd fd in the timed loop
    assert e["launcher"] == "torchrun" and d["config"]["launcher"] == "torchrun"
    assert e["bench_process_gpu"]["clean"] and len(e["bench_process_gpu"]["ranks"]) == 2
    # 2 of the fixture's 8 GPUs from a fragmented availability (second plugin
    # instance, containers split one per rank as in the headline run)
    fr = e["fragmented_n_of_m"]
    assert fr["advertised"] == 8 and fr["requested"] == 2 and fr["short_circuit_steps"] == 0
    assert fr["candidates"] > 0 and fr["same_set_as_reference"] is True


def test_bench_n_of_m_searches_inside_the_timed_step():
    """--gpus 3 --advertise 8: every timed admission's GetPreferredAllocation is
    a real search (no short-circuit, candidates > 0) over a fragmented
    availability, and picks the reference BFS's set."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "bench.py", "--fixture", "--gpus", "3", "--advertise", "8", "--steps", "3",
                        "--warmup", "1"], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    ta = d["extra"]["timed_allocation"]
    assert ta["advertised"] == 8 and ta["requested"] == 3 and len(ta["held"]) == 2 and ta["available"] == 6
    assert ta["preferred_used"] and ta["short_circuit_steps"] == 0 and ta["candidates"] > 0
    assert ta["same_set_as_reference"] is True and len(ta["chosen"]) == 1
    assert "8 GPUs advertised, 1 pod requesting 3, 2 held" in d["config"]["parallelism"]
    assert d["extra"]["fragmented_n_of_m"] is None       # only with M = N
    e = d["extra"]
    assert e["launcher"] == "single-process"
    assert e["bench_process_gpu"] == {"ranks": [{"torch_cuda_initialized": False, "kfd_fds": 0, "render_fds": 0}],
                                      "clean": True}
    ta = e["tail_attribution"]
    assert set(ta["phase_p50_ms"]) == {"plugin_rpc", "runtime_prep", "exec_and_library_load", "gpu_runtime_init",
                                       "device_setup", "launch_and_verify"}
    assert all(s["latency_ms"] > ta["threshold_ms"] for s in ta["slow_steps"])


def test_bench_python_plugin_option():
    """--plugin python: the Python CLI's plugin in the bench process serves the admissions."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "bench.py", "--fixture", "--steps", "2", "--warmup", "1", "--plugin",
                        "python"], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["extra"]["plugin"] == "python" and d["extra"]["plugin_server_p50_us"]


def test_bench_extras_deadline_keeps_the_headline():
    """A secondary measurement that overruns --extras-deadline (standing in for
    a hung RCCL communicator or DMA on a sick node): rank 0 still prints exactly
    one headline line, naming the unfinished stage, every rank exits 0 (rank 1
    sees rank 0 leave mid-collective), and no plugin daemon is left behind."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--fixture", "--steps", "2",
           "--warmup", "1", "--extras-deadline", "0.5"]
    proc = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            start_new_session=True)   # its own process group: whatever it leaves is ours
    try:
        out, err = proc.communicate(timeout=300)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, 9)
    assert proc.returncode == 0, err[-2000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    inc = d["extra"]["extras_incomplete"]
    assert inc["deadline_s"] == 0.5 and inc["stage"] and inc["error"] is None, (inc, err[-3000:])
    # the timed loop's own numbers are all there
    e = d["extra"]
    assert len(e["steps_ms"]) == 2 and e["bench_process_gpu"]["clean"] and e["plugin"] == "native-daemon"
    assert "exceeded --extras-deadline" in err
    # a SIGKILLed daemon may linger for a moment (or as a zombie if PID 1 does not reap)
    for _ in range(40):
        ps = subprocess.run(["ps", "-eo", "pgid=,stat=,cmd="], capture_output=True, text=True).stdout
        left = [l for l in ps.splitlines() if l.split(None, 2)[0] == str(proc.pid) and not l.split()[1].startswith("Z")]
        if not left:
            break
        time.sleep(0.1)
    assert not left, left


# ------------------------------------------------------------------ the driver's multi-GPU run, rehearsed on CPU
def _ps_group(pgid):
    ps = subprocess.run(["ps", "-eo", "pgid=,stat=,cmd="], capture_output=True, text=True).stdout
    return [l for l in ps.splitlines() if l.split(None, 2)[0] == str(pgid) and not l.split()[1].startswith("Z")]


def _bench_ranks(n, *args, torchrun=True, timeout=300):
    """bench.py as the driver launches it at N (torchrun, one rank per GPU) on the
    synthetic 8x MI355X node; returns (the one JSON line, stderr). Fails if
    anything of the run's process group (a plugin daemon, a rank) outlives it."""
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(n), "--master-addr",
               "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(n), "--fixture", *args]
    else:
        cmd = [sys.executable, "bench.py", "--gpus", str(n), "--fixture", *args]
    proc = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            start_new_session=True)
    t0 = time.monotonic()
    try:
        out, err = proc.communicate(timeout=timeout)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, 9)
    assert proc.returncode == 0, err[-3000:]
    assert time.monotonic() - t0 < timeout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    for _ in range(40):            # a SIGKILLed daemon may linger for a moment
        left = _ps_group(proc.pid)
        if not left:
            break
        time.sleep(0.1)
    assert not left, left
    return json.loads(lines[0]), err


@pytest.mark.parametrize("n,mode", [(4, "pod"), (4, "per-gpu"), (8, "pod"), (8, "per-gpu")])
def test_bench_torchrun_n_ranks_on_the_fixture(n, mode):
    """BASELINE configs #3 / #5 at N = 4 and 8 under torchrun, in both container
    modes: one headline line from rank 0 with N ranks' state, gloo
    collectives over N ranks, and the allocated set's fabric (one xGMI hive,
    N(N-1)/2 links)."""
    d, _ = _bench_ranks(n, "--steps", "3", "--warmup", "1", "--container-mode", mode, "--mode-compare", "2",
                        "--fragmented-compare", "2")
    e = d["extra"]
    assert d["n_gpus"] == n and d["steps"] == 3 and d["value"] > 0 and "extras_incomplete" not in e
    assert e["launcher"] == "torchrun" == d["config"]["launcher"] and e["container_mode"] == mode
    assert e["bench_process_gpu"]["clean"] and len(e["bench_process_gpu"]["ranks"]) == n
    assert e["rccl"]["backend"] == "gloo" and e["rccl"]["ok"]
    assert all(r["ranks"] == n for r in e["rccl"]["rows"])
    assert e["fabric"]["one_hive"] and e["fabric"]["pairs"]["xgmi"] == n * (n - 1) // 2
    other = "per-gpu" if mode == "pod" else "pod"
    assert e[f"latency_p50_ms_container_mode_{other}"] > 0
    assert e["timed_allocation"]["advertised"] == n and len(e["steps_ms"]) == 3


def test_bench_torchrun_8_ranks_extras_deadline_fires():
    """At 8 ranks a deadline that fires inside the extras (rank 0 leaves while
    the others wait in a collective): still exactly one headline line, every
    rank exits 0, no daemon left."""
    d, err = _bench_ranks(8, "--steps", "2", "--warmup", "1", "--extras-deadline", "0.5")
    e = d["extra"]
    inc = e["extras_incomplete"]
    assert inc["deadline_s"] == 0.5 and inc["stage"], inc
    assert d["n_gpus"] == 8 and len(e["steps_ms"]) == 2 and e["bench_process_gpu"]["clean"]
    assert len(e["bench_process_gpu"]["ranks"]) == 8
    assert "exceeded --extras-deadline" in err or "failed:" in err


def test_bench_single_process_8_gpus_on_the_fixture():
    """python bench.py --gpus 8 --fixture (no torchrun): the launcher is the
    single process, one pod with 8 GPUs, no collectives."""
    d, _ = _bench_ranks(8, "--steps", "3", "--warmup", "1", torchrun=False)
    e = d["extra"]
    assert d["n_gpus"] == 8 and e["launcher"] == "single-process" and e["rccl"] is None
    assert e["bench_process_gpu"]["clean"] and len(e["bench_process_gpu"]["ranks"]) == 1
    assert e["fabric"]["pairs"]["xgmi"] == 28 and e["timed_allocation"]["advertised"] == 8
    assert e["host"]["git_describe"] and e["host"]["host_cpus"] >= 1 and e["host"]["kernel"]


def test_bench_health_pulse_runs_on_the_native_daemon():
    """--health-pulse (BASELINE config: health-check DaemonSet enabled) drives
    the native daemon with -pulse; its sweeps are counted from the daemon's
    /metrics (on the fixture: the sysfs sources; on a GPU also liveness and
    amd-smi)."""
    d, _ = _bench_ranks(1, "--steps", "30", "--warmup", "1", "--health-pulse", "1", torchrun=False)
    hl = d["extra"]["health_loop"]
    assert d["config"]["plugin"] == "native-daemon" and hl["plugin"] == "native-daemon"
    assert hl["pulse_s"] == 1.0 and hl["sweeps"] >= 1 and hl["sweep_ms_mean"] is not None
    assert hl["sweep_ms_p50_at_most"] is not None and hl["sweep_ms_p50_at_most"] > 0
    assert hl["unhealthy"] == [] and hl["health_changes"] == 0
