#!/usr/bin/env python3
"""Headline benchmark: p50 Allocate->ContainerReady latency at N advertised MI355X GPUs.

Metric and config come from BASELINE.json ("p50 Allocate→ContainerReady latency;
GPUs advertised at 1/2/4/8 MI355X"). One timed step is one pod admission:

  1. (rank 0) the fake kubelet runs kubelet's devicemanager sequence against
     the real device plugin over UDS gRPC: GetPreferredAllocation for a pod
     requesting amd.com/gpu=N out of the N advertised devices, then Allocate;
  2. the DeviceSpecs in the Allocate response are turned into a "container":
     one fresh process (rank 0) whose /dev/dri holds exactly the allocated
     nodes (--dev-view specs: opens of any other render node fail as in a
     container, so ROCr initialises only the pod's GPUs; container_runtime.py)
     (--container-mode pod, what kubelet starts for a
     pod), or one process per allocated GPU, one per rank, like a torchrun
     workload inside the pod would start (--container-mode per-gpu; reported
     as a comparison at N > 1);
  3. the container initialises the GPU runtime and runs the gfx950 MFMA
     liveness kernel on each of its GPUs (parallel host threads); it is
     "ready" when every tile verifies bit-exactly;
  4. latency = (last container ready) - (kubelet starts GetPreferredAllocation),
     both on CLOCK_MONOTONIC;
  5. (untimed in the latency, inside the timed loop) the pod terminates: its
     processes exit and the driver tears down their kfd processes. The next
     admission starts once /sys/class/kfd/kfd/proc no longer lists them
     (--settle kfd); with --settle none it would start inside that teardown and
     block ~100-150 ms in open("/dev/kfd") (profiles/archive/measurements_r1_r3.md §3c) — reported
     as latency_p50_ms_back_to_back.

The plugin is the real one: by default the native daemon mi355x-device-plugin
(the primary entrypoint: real /sys discovery, C++ allocator and gRPC server;
--plugin python runs the Python CLI's plugin instead); only kubelet and the
CRI runtime are stand-ins (see rocm_k8s_device_plugin_amd/testing/
fake_kubelet.py, container_runtime.py).

  python bench.py --gpus N --steps K --warmup W
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "p50 Allocate→ContainerReady latency; GPUs advertised at 1/2/4/8 MI355X"


def make_parser():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sysfs-root", default="/sys")
    ap.add_argument("--dev-root", default="/dev")
    ap.add_argument("--fixture", action="store_true",
                    help="CPU-only: synthetic 8x MI355X sysfs, containers are no-op processes")
    ap.add_argument("--container-timeout", type=float, default=120.0)
    ap.add_argument("--container-runtime", default="hip", choices=["hip", "hsa"],
                    help="how the container entrypoint reaches the GPU: hip = a HIP program (BASELINE.md: the "
                         "container finishes HIP init and one MFMA liveness kernel; the headline), hsa = the "
                         "same kernel launched through ROCr directly (no libamdhip64, no HIP device set-up)")
    ap.add_argument("--runtime-compare", type=int, default=-1,
                    help="admissions with the other --container-runtime after the timed loop, reported for "
                         "comparison (-1 = as many as --steps; 0 = off)")
    ap.add_argument("--settle", default="kfd", choices=["kfd", "none"],
                    help="between admissions wait until the previous containers' kfd processes are torn down "
                         "(the previous pod has terminated) or start the next one immediately")
    ap.add_argument("--container-mode", default="pod", choices=["pod", "per-gpu"],
                    help="pod: ONE container process gets all N allocated GPUs (rank 0 starts it; what kubelet "
                         "does for a pod); per-gpu: each rank starts a process for its GPU (torchrun-style workload)")
    ap.add_argument("--mode-compare", type=int, default=5,
                    help="for N > 1: extra untimed admissions in the other --container-mode, reported for comparison")
    ap.add_argument("--node-view-compare", type=int, default=5,
                    help="extra untimed admissions with the plugin's -node_view mounts applied to the containers "
                         "(by path redirection: no root for bind mounts), reported for comparison")
    ap.add_argument("--dev-view", default="specs", choices=["specs", "visible-devices"],
                    help="container GPU visibility: specs = the container's /dev holds exactly the Allocate "
                         "DeviceSpecs (ROCr skips the other GPUs' render nodes, as in a real container); "
                         "visible-devices = every host GPU openable, restricted with ROCR_VISIBLE_DEVICES")
    ap.add_argument("--visibility-compare", type=int, default=5,
                    help="extra untimed admissions with the other --dev-view, reported for comparison")
    ap.add_argument("--b2b-compare", type=int, default=5,
                    help="extra untimed admissions with --settle none, reported for comparison")
    ap.add_argument("--throughput-check", type=int, default=1,
                    help="after the timed steps, the throughput check (HBM pattern bandwidth, bf16 MFMA rate, "
                         "per-XCD clocks) on the advertised GPUs, reported in extra.gpu_throughput (1 = on)")
    ap.add_argument("--peer-check", type=int, default=1,
                    help="after the timed loop, DMA-copy + verify over every pair of the N GPUs' links (H2); "
                         "reported in extra.peer_probe, never part of the metric")
    ap.add_argument("--collectives", type=int, default=1,
                    help="for N > 1: after the timed loop, verify + time RCCL all-reduce / all-gather / "
                         "reduce-scatter / all-to-all on the N ranks' GPUs (parallel/collectives.py); "
                         "reported in extra.rccl next to the allocated set's xGMI fabric bound, never part of the metric")
    ap.add_argument("--collective-sizes", default="",
                    help="per-rank bytes for --collectives (default 1M,64M,256M on GPUs, 64K on CPU)")
    ap.add_argument("--health-pulse", type=float, default=0.0,
                    help="> 0: run the plugin as the health DaemonSet does (MFMA liveness via the kept-queue probe "
                         "server, amd-smi ECC / events / xGMI link state) with this pulse in seconds, while pods "
                         "are admitted (BASELINE config: health-check DaemonSet enabled)")
    ap.add_argument("--health-liveness-mode", default="persistent", choices=["persistent", "spawn"],
                    help="with --health-pulse on the native daemon: -liveness_mode (one kept-queue probe server, or "
                         "a fresh probe process per device per sweep); extra.health_loop reports the host memory "
                         "of the daemon and its probe processes over the run")
    ap.add_argument("--health-prestart", type=int, default=0,
                    help="with --health-pulse on the native daemon: -prestart_liveness (kubelet's PreStartContainer "
                         "probes the pod's GPUs through the probe server before the container starts; its time is "
                         "part of the latency and reported as extra.prestart_rpc_p50_ms) (1 = on)")
    ap.add_argument("--advertise", type=int, default=0,
                    help="advertise M devices and request --gpus N of them per pod (default M = N: the headline, "
                         "'GPUs advertised at N'). With M > N the timed admissions start from a fragmented "
                         "availability (--hold devices held by other pods), so GetPreferredAllocation searches")
    ap.add_argument("--hold", type=int, default=-1,
                    help="with M > N: devices held by other pods during the run (default (M-N)//2, alternating "
                         "positions so every hive is fragmented)")
    ap.add_argument("--fragmented-compare", type=int, default=5,
                    help="with M = N and more accessible devices than N: extra untimed admissions of N out of "
                         "every accessible device from a fragmented availability (a second plugin instance), "
                         "reported in extra.fragmented_n_of_m (BASELINE config: full-node hive-aware allocation)")
    ap.add_argument("--plugin", default="native", choices=["native", "python"],
                    help="the device plugin under test: native = the mi355x-device-plugin daemon (the primary "
                         "entrypoint, what ./k8s-device-plugin runs); python = the Python oracle plugin in this "
                         "process, on the same C++ gRPC server")
    ap.add_argument("--kubelet-client", default="", choices=["", "native", "native-thread", "aio"],
                    help="the fake kubelet's admission RPC client: native (a native HTTP/2 client, like kubelet's "
                         "grpc-go) or aio (grpc.aio in the bench's event loop); default native with the native server")
    ap.add_argument("--extras-deadline", type=float, default=300.0,
                    help="seconds after the timed loop for every secondary measurement (comparisons, RCCL, peer "
                         "probe, throughput check); past it rank 0 prints the headline line with what it has and "
                         "every rank exits 0, so a hung extra cannot take the measured headline with it (0 = none)")
    ap.add_argument("--json-out", default="")
    return ap


def parse_args(argv=None):
    return make_parser().parse_args(argv)


def host_info(node) -> dict:
    """The tree's git describe, ROCm and amdgpu driver versions, the host's CPU count
    (ROCr's start-up walks every CPU's cache descriptors) and the kernel release."""
    import platform
    from rocm_k8s_device_plugin_amd import _build
    from rocm_k8s_device_plugin_amd.utils import versions
    v = versions.versions(node.sysfs)
    describe = _build.git_describe()
    if not describe:  # a tree without .git (a GPU box's copy): the version the daemon was built with
        import re
        import subprocess
        from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
        try:
            out = subprocess.run([os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin"), "-h"],
                                 capture_output=True, text=True, timeout=10).stdout
            m = re.search(r" version (\S+)", out)
            describe = m.group(1) if m else ""
        except (OSError, subprocess.TimeoutExpired):
            describe = ""
    return {"git_describe": describe or None, "rocm": v["rocm"], "amdgpu": v["amdgpu"],
            "host_cpus": os.cpu_count(), "kernel": platform.release()}


def _safe_host_info(node) -> dict:
    try:
        return host_info(node)
    except Exception as e:  # noqa: BLE001 - context only: never at the headline's expense
        return {"error": f"{type(e).__name__}: {e}"[:200]}


def result_line(args, d, n, m_adv, held, plugin_kind, elapsed, latency_ms, extra: dict) -> str:
    """The one JSON line the driver reads (value = p50 of the timed admissions)."""
    from rocm_k8s_device_plugin_amd.benchmark.stats import pct
    return json.dumps({
        "metric": METRIC,
        "value": round(pct(latency_ms, .5), 3),
        "unit": "ms",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 3),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic pod specs requesting amd.com/gpu=N; real /sys discovery, fake kubelet over UDS, "
                 "container = fresh process whose /dev is the Allocate DeviceSpecs running the MFMA liveness "
                 "kernel" if not args.fixture else
                 "synthetic 8xMI355X sysfs fixture; stub-probe containers (CPU only)"),
        "config": {"model": "example/pod/alexnet-gpu.yaml-style pod, amd.com/gpu=N",
                   "global_batch": n, "seq_len": None,
                   "parallelism": (f"{m_adv} GPUs advertised, 1 pod requesting {n}, " +
                                   (f"{len(held)} held by other pods, " if held else "") +
                                   ("1 container process with all N GPUs" if args.container_mode == "pod"
                                    else "1 container process per GPU")),
                   "between_admissions": ("previous pod's kfd teardown complete" if args.settle == "kfd"
                                          else "back-to-back"),
                   "launcher": d.launcher, "plugin": plugin_kind},
        "extra": extra,
    })


def main():
    args = parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from rocm_k8s_device_plugin_amd.benchmark.admission import Admissions
    from rocm_k8s_device_plugin_amd.benchmark.coord import Dist, ExtrasGuard
    from rocm_k8s_device_plugin_amd.benchmark.extras import Extras
    from rocm_k8s_device_plugin_amd.benchmark.stats import fragment

    d = Dist()
    n = args.gpus
    if d.world > 1 and d.world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE {d.world}: launch one rank per GPU")
    from rocm_k8s_device_plugin_amd import _build
    if d.rank == 0:
        _build.ensure_built(hip=not args.fixture)
    d.sync()

    m_adv = args.advertise or n
    if m_adv < n:
        raise SystemExit(f"--advertise {m_adv} < --gpus {n}")
    node = plug = None
    if d.rank == 0:
        from rocm_k8s_device_plugin_amd.benchmark.node import BenchNode
        node = BenchNode(args, n, m_adv)
        plug = node.make_plugin("device-plugins", node.adv)
        if m_adv > n:
            plug.hold(fragment([dv.id for dv in node.adv], n, args.hold))
    adm = Admissions(args, d, n, loop=node.loop if node else None, plug=plug)

    for _ in range(args.warmup):
        adm.step(False)
    if d.rank == 0:
        plug.server_ms(reset=True)
    d.sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        adm.step(True)
    d.sync()
    elapsed = time.perf_counter() - t_start
    server_ms = plug.server_ms() if d.rank == 0 else {}
    elapsed = d.max(elapsed)
    rank_gpu_state = d.gather(adm.gpu_state)

    # the headline is measured: from here on everything is bounded by the guard
    guard = ExtrasGuard(d.rank, args.extras_deadline)
    if d.rank == 0:
        from rocm_k8s_device_plugin_amd.benchmark.stats import pct
        guard.kill_on_fire(plug)
        guard.tmp = node.tmp
        core = dict(adm.timed_report(), **{
            "plugin": node.plugin_kind,
            "grpc_server": "native",
            "kubelet_client": node.kclient,
            # breakdown of plugin_rpc (kubelet's GetPreferredAllocation + Allocate round trips): the
            # plugin's own time per RPC, measured inside the native server (the daemon's from its
            # per-RPC log records)
            "plugin_server_p50_us": {rpc: round(pct(v, .5) * 1e3, 1) for rpc, v in sorted(server_ms.items())
                                     if rpc in ("GetPreferredAllocation", "Allocate")},
            # the node under test must look like a kubelet node: no GPU context in the bench /
            # plugin process(es) while the timed containers initialise (worst over the timed steps)
            "launcher": d.launcher,
            "bench_process_gpu": {"ranks": rank_gpu_state,
                                  "clean": not any(s["torch_cuda_initialized"] or s["kfd_fds"]
                                                   for s in rank_gpu_state)},
            "gpus": node.gpu_info(),
            # what produced the number: the build, the host's ROCm / amdgpu, the daemon's own banner
            "host": _safe_host_info(node)})
        held = list(plug.held)

        def line(extra):
            return result_line(args, d, n, m_adv, held, node.plugin_kind, elapsed, adm.rec.latency_ms, extra)

        def partial_line(error):
            """(line, json_out) for the guard: the headline without the unfinished extras."""
            return (line(dict(core, extras_incomplete={"deadline_s": args.extras_deadline, "stage": guard.stage,
                                                       "error": error})), args.json_out)

        guard.fallback = partial_line

    try:
        extra = Extras(args, d, n, adm, guard, node).run()
        if d.rank == 0:
            guard.enter("plugin_stop")
            plug.stop()
            node.close()
            guard.emit(line(dict(core, **extra)), args.json_out)
    except (Exception, SystemExit) as e:  # noqa: BLE001
        # a failed extra (or a peer rank that left) is reported, never fatal to the measured headline
        guard.abandon(f"{type(e).__name__}: {e}"[:300])
    d.close()
    guard.cancel()


if __name__ == "__main__":
    main()
