"""The Python oracle plugin's command line (``python -m
rocm_k8s_device_plugin_amd.cli.device_plugin``).

Not a product: ``k8s-device-plugin`` is the native daemon everywhere (the
images, ``scripts/``, the installed console script). This CLI drives the
Python model the daemon is checked against, with the daemon's flag names.

Reference: cmd/k8s-device-plugin/main.go:34-120. Same flag names and
semantics (``-pulse``, ``-driver_type``, ``-resource_naming_strategy`` plus
glog flags), same validation messages and exit codes, same implementation
auto-selection order (container -> vf-passthrough -> pf-passthrough; an
explicit type that fails exits 1; if every strategy fails the manager still
starts and idles).

Additions (documented by the reference but never implemented there, or new):
``AMD_GPU_DEVICE_COUNT`` / ``CONFIG_FILE_PATH`` (``gpu.device_count``),
``--kubelet-url`` (accepted; registration is always over the UDS),
``-sysfs_root`` / ``-dev_root`` / ``-kubelet_dir`` for fixture-driven runs,
the MFMA liveness probe (``-liveness``), ``-metrics_port`` and JSON logs.
"""
from __future__ import annotations

import asyncio
import os
import sys
from typing import List, Optional


from .. import __version__
from .. import constants as C
from ..health.monitor import HealthConfig
from ..plugin.base import DeviceImpl, DeviceImplError
from ..plugin.manager import ManagerConfig, PluginManager
from ..proto import deviceplugin as pb
from ..topology import device_count_limit_from_env
from ..utils import flags, log

BANNER = ["AMD GPU device plugin for Kubernetes (MI355X-native)",
          f"{os.path.basename(sys.argv[0] if sys.argv else 'k8s-device-plugin')} version {__version__}"]


def build_parser() -> flags.GoFlagParser:
    p = flags.GoFlagParser(prog="k8s-device-plugin", description="\n".join(BANNER))
    p.add_int(C.FLAG_PULSE, 0, "time between health check polling in seconds.  Set to 0 to disable.")
    p.add_str(C.FLAG_DRIVER_TYPE, "", "Driver type to use: container, vf-passthrough, or pf-passthrough")
    p.add_str(C.FLAG_RESOURCE_NAMING_STRATEGY, C.STRATEGY_SINGLE, "Resource strategy to be used: single or mixed")
    flags.add_glog_flags(p)
    p.add_str("kubelet-url", "http://localhost:10250", "accepted for compatibility; registration uses the UDS")
    p.add_str("kubelet_dir", pb.DEVICE_PLUGIN_PATH, "kubelet device-plugin socket directory")
    p.add_str("sysfs_root", "/sys", "sysfs mount to read (fixtures: a generated tree)")
    p.add_str("dev_root", "/dev", "device node directory")
    p.add_str("exporter_socket", pb_exporter_socket(), "AMD metrics-exporter health socket ('' disables)")
    p.add_bool("liveness", False, "run the gfx950 MFMA liveness probe on every device each pulse")
    p.add_str("liveness_mode", "persistent", "persistent: one long-lived probe server per node; spawn: a fresh "
                                             "probe process per device per pulse")
    p.add_bool("liveness_keep_queues", True, "persistent mode: keep each device's probe queue between pulses, so a "
                                             "pulse creates no kfd queue (no HWS runlist update that preempts the "
                                             "pods on that GPU); false: create and destroy it every pulse")
    p.add_int("liveness_chip_sweep_every", 0, "every N-th pulse (and the first) run the full-chip MFMA/LDS sweep "
                                             "(every CU of every XCD) on GPUs with no running work; 0 = off")
    p.add_float("liveness_timeout", 10.0, "per-device liveness probe deadline (s)")
    p.add_int("liveness_fail_threshold", 2, "consecutive probe failures before a device turns Unhealthy")
    p.add_float("liveness_busy_grace", 300.0, "seconds a probe may stay queued behind other processes' work on "
                                              "its GPU (a tenant kernel holding every CU) before it counts as a "
                                              "failure; applies in every liveness mode (kept queues: the queued "
                                              "dispatch's late verdict is awaited; otherwise a deadline miss on "
                                              "a busy GPU is inconclusive)")
    p.add_bool("liveness_corroborate", True, "a probe pending on a busy GPU stays inconclusive only while amd-smi "
                                             "reports GFX activity; 0%% on 2 consecutive sweeps ends the busy grace")
    p.add_int("liveness_crowded_procs", 7, "with this many other processes holding queues on a GPU (or too few "
                                           "free kfd queues) the probe server steps off it, so it adds no process or "
                                           "queue to an oversubscribed HWS runlist; 0 = off")
    p.add_float("liveness_unknown_busy_grace", 30.0, "the busy grace while busy GPUs cannot be told from idle ones "
                                                     "(kfd process list unreadable): every GPU counts as busy, "
                                                     "so the grace is shorter")
    p.add_int("perf_check_every", 0, "every N-th pulse (and the first) run the throughput check on GPUs with no "
                                      "running work: HBM write/read bandwidth over a verified pattern, sustained "
                                      "bf16 MFMA rate, per-XCD clocks (~40 ms of the chip); 0 = off")
    p.add_int("perf_mib", 4096, "throughput check: HBM buffer (MiB)")
    p.add_str("perf_action", "report", "a GPU under the throughput floors is logged and exported (report) or also "
                                       "withdrawn until a check passes (unhealthy); wrong data is always a failure")
    p.add_float("perf_min_hbm_read_gbps", 3000.0, "throughput floor: HBM read GB/s per whole MI355X")
    p.add_float("perf_min_mfma_tflops", 700.0, "throughput floor: dense bf16 MFMA TFLOP/s per whole MI355X")
    p.add_float("perf_min_xcd_clock_ratio", 0.6, "throughput floor: slowest XCD's clock over the median XCD's")
    p.add_bool("smi_ecc", False, "mark a device Unhealthy when its amd-smi uncorrectable ECC count rises")
    p.add_bool("smi_events", False, "subscribe to amd-smi GPU events; a device is Unhealthy between a "
                                    "gpu_pre_reset and its gpu_post_reset, other events are counted")
    p.add_bool("smi_xgmi", False, "watch amd-smi xGMI link state every pulse; a GPU pair whose link goes down "
                                  "stops counting as xGMI-connected in preferred allocation (devices stay Healthy)")
    p.add_bool("send_every_pulse", False, "re-send the full device list on every pulse (reference behaviour)")
    p.add_int("metrics_port", 0, "serve Prometheus /metrics on this port (0 = off)")
    p.add_str("allocator_search", "auto", "GetPreferredAllocation search: auto (extended on nodes with partitioned "
                                          "GPUs, the reference's candidates on whole-GPU nodes), reference, extended")
    p.add_bool("allocator_extended_search", False, "force the extended search: every split of a request over "
                                                   "interchangeable devices (several partial GPUs), ties broken by "
                                                   "fewer GPUs, then kfd link weight/bandwidth")
    p.add_bool("dry_run", False, "print what this node would advertise (implementation, resources, devices, "
                                 "health after one sweep, preferred allocations per size) as JSON and exit")
    p.add_float("topology_watch", 5.0, "seconds between checks for a GPU topology change (kfd generation, "
                                       "partition modes); on a change the devices are re-discovered and "
                                       "re-advertised (0 = off: devices fixed at start-up, as upstream)")
    p.add_bool("topology_view", False, "experimental: bind-mount a kfd topology filtered to the allocated "
                                       "GPUs into each container (faster ROCr start-up, GPU isolation)")
    p.add_bool("node_view", False, "experimental: bind-mount /sys/devices/system/node without the per-CPU cache "
                                   "descriptors ROCr walks at start-up (3x faster hsa_init on 256-CPU hosts)")
    p.add_str("device_list_strategy", "device-specs", "what Allocate returns: device-specs (the /dev nodes, as "
                                                       "upstream), cdi-cri (CDI device names, the runtime applies "
                                                       "the specs in -cdi_spec_dir), cdi-annotations; comma-separated "
                                                       "to combine")
    p.add_str("cdi_spec_dir", "/var/run/cdi", "where the CDI specs of the advertised devices are written "
                                              "(cdi-* device list strategies)")
    p.add_str("log_format", "glog", "glog | json")
    p.add_str("trace_file", "", "write a Chrome trace of RPC / allocator / health spans to this file on exit")
    p.add_str("config", os.environ.get("CONFIG_FILE_PATH", ""), "YAML config file (gpu.device_count, ...)")
    return p


def pb_exporter_socket() -> str:
    from ..proto.metricssvc import DEFAULT_SOCKET
    return DEFAULT_SOCKET


def validate(ns) -> Optional[str]:
    if ns.pulse < 0:
        return f"pulse must be a non-negative integer, got {ns.pulse}"
    if ns.driver_type not in ("",) + C.DRIVER_TYPES:
        return (f"invalid driver_type provided: {ns.driver_type}, supported values are container, "
                "vf-passthrough, or pf-passthrough")
    if ns.resource_naming_strategy not in (C.STRATEGY_SINGLE, C.STRATEGY_MIXED):
        return (f"invalid resource_naming_strategy provided: {ns.resource_naming_strategy}, supported values "
                "are single or mixed")
    try:
        from .. import cdi
        cdi.parse_strategies(ns.device_list_strategy)
    except ValueError as e:
        return str(e)
    if ns.liveness_mode not in ("persistent", "spawn"):
        return f"invalid liveness_mode provided: {ns.liveness_mode}, supported values are persistent or spawn"
    if ns.perf_action not in ("report", "unhealthy"):
        return f"invalid perf_action provided: {ns.perf_action}, supported values are report or unhealthy"
    if ns.perf_check_every > 0 and not ns.liveness:
        return "perf_check_every needs -liveness (the throughput check runs in the probe server)"
    if ns.allocator_search not in ("auto", "reference", "extended"):
        return f"invalid allocator_search provided: {ns.allocator_search}, supported values are auto, reference, extended"
    return None


def load_config(path: str) -> dict:
    if not path:
        return {}
    import yaml  # only with -config: keeps ~20 ms of import off plugin start-up
    with open(path) as f:
        return yaml.safe_load(f) or {}


def create_impl(name: str, ns, device_count: Optional[int]) -> DeviceImpl:
    if name == C.CONTAINER:
        from ..plugin.container import ContainerImpl
        hc = HealthConfig(exporter_socket=ns.exporter_socket or None, liveness=ns.liveness,
                          liveness_timeout_s=ns.liveness_timeout, fail_threshold=ns.liveness_fail_threshold,
                          smi_ecc=ns.smi_ecc, smi_events=ns.smi_events, smi_xgmi=ns.smi_xgmi, dev_root=ns.dev_root,
                          liveness_mode=ns.liveness_mode, chip_sweep_every=ns.liveness_chip_sweep_every,
                          liveness_keep_queues=ns.liveness_keep_queues,
                          liveness_busy_grace_s=ns.liveness_busy_grace,
                          liveness_unknown_busy_grace_s=ns.liveness_unknown_busy_grace,
                          liveness_corroborate=ns.liveness_corroborate,
                          liveness_crowded_procs=ns.liveness_crowded_procs,
                          perf_check_every=ns.perf_check_every, perf_mib=ns.perf_mib, perf_action=ns.perf_action,
                          perf_min_hbm_read_gbps=ns.perf_min_hbm_read_gbps,
                          perf_min_mfma_tflops=ns.perf_min_mfma_tflops,
                          perf_min_xcd_clock_ratio=ns.perf_min_xcd_clock_ratio)
        view_dir = os.path.join(ns.kubelet_dir, "mi355x-topology") if ns.topology_view else None
        node_dir = os.path.join(ns.kubelet_dir, "mi355x-node") if ns.node_view else None
        from .. import cdi
        return ContainerImpl(ns.resource_naming_strategy, ns.sysfs_root, hc, device_count,
                             topology_view_dir=view_dir, node_view_dir=node_dir,
                             device_list_strategy=cdi.parse_strategies(ns.device_list_strategy),
                             cdi_spec_dir=ns.cdi_spec_dir)
    if name == C.VF_PASSTHROUGH:
        from ..plugin.passthrough import VfImpl
        return VfImpl(ns.resource_naming_strategy, ns.sysfs_root, ns.exporter_socket or None)
    if name == C.PF_PASSTHROUGH:
        from ..plugin.passthrough import PfImpl
        return PfImpl(ns.resource_naming_strategy, ns.sysfs_root)
    raise DeviceImplError(f"unknown driver type {name}")


def select_impl(ns, device_count: Optional[int], logger) -> Optional[DeviceImpl]:
    if ns.driver_type:
        try:
            return create_impl(ns.driver_type, ns, device_count)
        except Exception as e:
            logger.error("Error instantiating driver type %s: %s", ns.driver_type, e)
            raise SystemExit(1)
    for name in C.DRIVER_TYPES:
        try:
            impl = create_impl(name, ns, device_count)
        except Exception as e:
            logger.warning("%s implementation failed: %s. Trying next...", name, e)
            continue
        if not impl.resource_names():
            # e.g. kfd present but no GPU behind it: let VF/PF detection run
            logger.warning("%s implementation found no devices. Trying next...", name)
            continue
        return impl
    return None


async def dry_run_report(impl: Optional[DeviceImpl], sweep: bool) -> dict:
    """What the plugin would tell kubelet on this node, without registering."""
    from ..plugin.base import new_context
    if impl is None:
        return {"implementation": None, "resources": {}}
    if sweep:
        await impl.refresh_health()
    out = {"implementation": impl.name, "resources": {}}
    for r in impl.resource_names():
        ctx = new_context(r)
        impl.start(ctx)
        devs = impl.enumerate(ctx)
        ids = [d.ID for d in devs]
        res = {"devices": [{"id": d.ID, "health": d.health, "numa": [n.ID for n in d.topology.nodes]}
                           for d in devs],
               "preferred_allocation": not ctx.allocator_error}
        if not ctx.allocator_error and ids:
            from ..parallel.fabric import Fabric
            fab = Fabric(impl.inv) if hasattr(impl, "inv") else None
            prefs = {}
            for k in sorted({1, 2, 4, 8, len(ids)} & set(range(1, len(ids) + 1))):
                chosen = ctx.allocator.allocate(ids, [], k)
                prefs[str(k)] = {"ids": chosen}
                if fab is not None:
                    rep = fab.report(chosen)
                    prefs[str(k)].update(one_hive=rep.one_hive, allreduce_bound_gbs=rep.allreduce_bound_gbs)
            res["allocations"] = prefs
        out["resources"][f"{C.RESOURCE_NAMESPACE}/{r}"] = res
    if hasattr(impl, "inv"):
        out["warnings"] = list(impl.inv.warnings)
    if hasattr(impl, "list_strategies"):
        out["device_list_strategy"] = list(impl.list_strategies)
        if getattr(impl, "_cdi", False):
            out["cdi_spec_dir"] = impl.cdi_spec_dir
    mon = getattr(impl, "monitor", None)
    if mon is not None and getattr(mon, "fabric", None) is not None:
        fab = mon.fabric
        out["xgmi"] = {"readings": fab.readings, "error": fab.error,
                       "degraded_pairs": [list(p) for p in sorted(fab.degraded)], "links_down": fab.links_down}
    if mon is not None and getattr(mon, "perf_last", None):
        # -perf_check_every: the first sweep ran the throughput check on the idle GPUs
        keys = ("hbm_write_gbps", "hbm_read_gbps", "hbm_bad_words", "mfma_tflops", "clock_mhz_median",
                "xcd_clock_mhz", "total_us")
        out["throughput"] = {dev: {"state": mon.perf_verdicts().get(dev, ("ok", ""))[0],
                                   "reason": mon.perf_verdicts().get(dev, ("ok", ""))[1],
                                   **{k: d.get(k) for k in keys if k in d}}
                             for dev, d in sorted(mon.perf_last.items())}
    await impl.close()
    return out


def main(argv: Optional[List[str]] = None) -> int:
    p = build_parser()
    ns = p.parse_args(argv)
    try:
        logger = log.setup_from_flags(ns, program="k8s-device-plugin")
    except ValueError as e:
        print(f"invalid logging flags: {e}", file=sys.stderr)
        return 1
    err = validate(ns)
    if err:
        logger.error("%s", err)
        return 1
    from ..utils.versions import banner_line
    for line in BANNER + [banner_line(ns.sysfs_root)]:
        logger.info("%s", line)
    cfg = load_config(ns.config)
    device_count = device_count_limit_from_env()
    if device_count is None:
        dc = (cfg.get("gpu") or {}).get("device_count")
        device_count = int(dc) if dc is not None else None
    impl = select_impl(ns, device_count, logger)
    if ns.dry_run:
        import json
        print(json.dumps(asyncio.run(dry_run_report(impl, sweep=ns.pulse > 0)), indent=1))
        return 0
    mc = ManagerConfig(pulse_s=float(ns.pulse), plugin_dir=ns.kubelet_dir, send_every_pulse=ns.send_every_pulse,
                       metrics_port=ns.metrics_port, topology_watch_s=ns.topology_watch,
                       allocator_extended_search="extended" if ns.allocator_extended_search else ns.allocator_search)
    from ..utils.trace import TRACER
    TRACER.configure(ns.trace_file or None)
    try:
        asyncio.run(PluginManager(impl, mc).run())
    finally:
        TRACER.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
