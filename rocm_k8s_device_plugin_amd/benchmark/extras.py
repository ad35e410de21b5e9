"""The secondary measurements bench.py takes after the timed loop.

Each stage runs under the ExtrasGuard (coord.py): it names the stage it
enters, so a stage that overruns --extras-deadline or fails is reported in
``extra.extras_incomplete`` instead of costing the headline. Comparison
admissions run on every rank (they are steps of the same pod); the plugin-side
measurements and the report are rank 0's.
"""
from __future__ import annotations

import os
import time

from .admission import StepRecords
from .stats import alloc_summary, fragment, pct


class Extras:
    def __init__(self, args, dist, n: int, adm, guard, node=None):
        """`adm`: the Admissions of the timed loop; `node`: rank 0's BenchNode (None elsewhere)."""
        self.args, self.d, self.n, self.adm, self.guard, self.node = args, dist, n, adm, guard, node
        self.other_runtime = "hsa" if args.container_runtime == "hip" else "hip"
        self.rt_key = "rocr_direct_container" if self.other_runtime == "hsa" else "hip_runtime_container"
        self.other_mode = "per-gpu" if args.container_mode == "pod" else "pod"
        self.other_view = "visible-devices" if args.dev_view == "specs" else "specs"
        self.out = {"comparisons": {}}

    def _p50(self, xs, key, q=.5):
        self.out[key] = round(pct(xs, q), 3) if xs else None

    def _row(self, name: str, rec: StepRecords) -> None:
        """A comparison row in full (p50, p99, phases, tail attribution, container counters)."""
        self.out["comparisons"][name] = rec.row()

    # ------------------------------------------------------------------ comparison admissions
    def container_mode_compare(self):
        rec = StepRecords()
        if self.n > 1:
            self.guard.enter("container_mode_compare")
            for _ in range(self.args.mode_compare):
                self.adm.step(rec, mode=self.other_mode)
        self._p50(rec.latency_ms, f"latency_p50_ms_container_mode_{self.other_mode}")
        self._row(f"container_mode_{self.other_mode}", rec)

    def node_view_compare(self):
        a_, d, node = self.args, self.d, self.node
        rec = StepRecords()
        if not a_.fixture and a_.node_view_compare > 0:
            # the plugin returns -node_view mounts (alias = host path: the fake runtime
            # applies mounts by redirection and cannot add the alias mount)
            nvplug = None
            impl = getattr(self.adm.plug, "impl", None)
            if d.rank == 0:
                node_dir = os.path.join(node.sysfs, "devices/system/node")
                if node.plugin_kind == "native-daemon":
                    nvplug = node.make_plugin("device-plugins-node-view", node.adv,
                                              ["-node_view", "-node_view_alias", node_dir])
                    self.guard.kill_on_fire(nvplug)
                else:
                    from rocm_k8s_device_plugin_amd.node_view import NodeView
                    impl.node_view = NodeView(os.path.join(node.tmp, "node-view"), node.sysfs, alias=node_dir)
                    impl.node_view.path()  # built at plugin start-up in a real deployment
            self.guard.enter("node_view_compare")
            for _ in range(a_.node_view_compare):
                self.adm.step(rec, pl=nvplug)
            if d.rank == 0:
                if nvplug is not None:
                    nvplug.stop()
                else:
                    impl.node_view = None
        self._p50(rec.latency_ms, "latency_p50_ms_node_view_emulated")
        self._p50(rec.runtime_ms, "node_view_emulated_runtime_init_p50_ms")
        self._row("node_view_emulated", rec)

    def dev_view_compare(self):
        rec = StepRecords()
        if not self.args.fixture:
            self.guard.enter("dev_view_compare")
            for _ in range(self.args.visibility_compare):
                self.adm.step(rec, dev_view=self.other_view)
        self._p50(rec.latency_ms, f"latency_p50_ms_dev_view_{self.other_view}")
        self._row(f"dev_view_{self.other_view}", rec)

    def runtime_compare(self):
        """The other container entrypoint, as many admissions as the headline
        (same settle, same view): with the default HIP container, ROCr-direct."""
        a_ = self.args
        steps = a_.steps if a_.runtime_compare < 0 else a_.runtime_compare
        rec = StepRecords()
        if not a_.fixture and steps > 0:
            self.guard.enter(f"{self.other_runtime}_runtime_compare")
            for _ in range(steps):
                self.adm.step(rec, runtime=self.other_runtime)
        self._p50(rec.latency_ms, f"latency_p50_ms_{self.rt_key}")
        self._p50(rec.latency_ms, f"latency_p99_ms_{self.rt_key}", .99)
        self.out[f"{self.rt_key}_steps"] = len(rec.latency_ms)
        self._row(self.rt_key, rec)

    def back_to_back_compare(self):
        rec = StepRecords()
        if not self.args.fixture and self.args.settle == "kfd":
            self.guard.enter("back_to_back_compare")
            for _ in range(self.args.b2b_compare):
                self.adm.step(rec, settle="none")
        self._p50(rec.latency_ms, "latency_p50_ms_back_to_back")
        self._row("back_to_back", rec)

    def fragmented_compare(self):
        """N of every accessible device, from a fragmented availability (a second
        plugin instance; the headline plugin keeps advertising exactly N)."""
        a_, d, n, node = self.args, self.d, self.n, self.node
        frag = None
        rec, alloc = StepRecords(), []
        do = d.bcast(d.rank == 0 and node.m_adv == n and a_.fragmented_compare > 0 and len(node.usable) > n)
        if do:
            fplug = None
            if d.rank == 0:
                fplug = node.make_plugin("device-plugins-all", node.usable)
                fplug.hold(fragment([dv.id for dv in node.usable], n, a_.hold))
                self.guard.kill_on_fire(fplug)
            self.guard.enter("fragmented_compare")
            for _ in range(a_.fragmented_compare):
                self.adm.step(rec, pl=fplug, alloc_sink=alloc)
            if d.rank == 0:
                frag = {"advertised": len(node.usable), "requested": n, "held": fplug.held,
                        "latency_p50_ms": round(pct(rec.latency_ms, .5), 3), **alloc_summary(fplug, alloc)}
                fplug.stop()
        self.out["fragmented_n_of_m"] = frag
        self._row("fragmented_n_of_m", rec)

    # ------------------------------------------------------------------ data plane
    def collectives(self):
        """The pod's GPUs as a torchrun workload sees them: one rank per GPU, RCCL
        over xGMI (gloo on CPU); a failure is reported, never fatal."""
        a_, d = self.args, self.d
        rccl = None
        if a_.collectives and d.world > 1:
            from rocm_k8s_device_plugin_amd.parallel import collectives as coll
            self.guard.enter("collectives")
            try:
                group, on_gpu = d.rccl_group()   # RCCL is created here, after the timed loop
                if on_gpu:
                    sizes = a_.collective_sizes or "1M,64M,256M"
                    ops, iters, dtype = coll.DEFAULT_OPS, 20, d.torch.bfloat16
                else:
                    sizes = a_.collective_sizes or "64K"
                    ops, iters, dtype = ("all_reduce", "all_gather"), 3, d.torch.float32
                rows = coll.run([coll.parse_size(x) for x in sizes.split(",") if x], ops, iters=iters, warmup=3,
                                dtype=dtype, group=group)
                rccl = coll.summary(rows)
                rccl["backend"] = d.dist.get_backend(group)
            except Exception as e:  # noqa: BLE001
                rccl = {"error": f"{type(e).__name__}: {e}"[:300]}
        self.out["rccl"] = rccl

    # ------------------------------------------------------------------ rank 0 only
    def allocator_microbench(self):
        """Our set search vs the reference's ordered BFS, both in C++ on the same
        weights: the bench request and every smaller one on the N advertised GPUs."""
        self.guard.enter("allocator_microbench")
        pol = self.adm.plug.allocator
        avail = [dv.id for dv in self.node.adv]
        n = self.n
        t = time.perf_counter()
        for _ in range(200):  # both sides called straight into C++ (no trace/stats wrapper)
            pol.native.allocate(avail, [], n)
        ours = (time.perf_counter() - t) / 200 * 1e6
        t = time.perf_counter()
        for _ in range(20):
            ref = pol.reference_allocate(avail, [], n)
        refu = (time.perf_counter() - t) / 20 * 1e6
        sweep = {}
        for k in range(1, n):
            t = time.perf_counter()
            for _ in range(50):
                mine = pol.native.allocate(avail, [], k)
            mine_us = (time.perf_counter() - t) / 50 * 1e6
            t = time.perf_counter()
            for _ in range(3):
                refk = pol.reference_allocate(avail, [], k)
            sweep[str(k)] = {"ours_us": round(mine_us, 2), "reference_us": round((time.perf_counter() - t) / 3 * 1e6, 2),
                             "reference_candidates": refk["candidates"], "ours_candidates": mine["candidates"],
                             "same_set": sorted(mine["ids"]) == sorted(refk["ids"])}
        self.out.update({"allocator_us": round(ours, 2), "reference_algorithm_us": round(refu, 2),
                         "reference_algorithm_candidates": ref["candidates"], "allocator_sweep": sweep})

    def health_loop_report(self):
        a_, node, plug = self.args, self.node, self.adm.plug
        if a_.health_pulse <= 0 or (a_.fixture and node.plugin_kind != "native-daemon"):
            self.out["health_loop"] = None
        elif node.plugin_kind == "native-daemon":
            self.out["health_loop"] = plug.health_report(float(node.health_flags[1]))
        else:
            mon = plug.impl.monitor
            self.out["health_loop"] = {"plugin": "python", "pulse_s": a_.health_pulse, "sweeps": mon.sweeps,
                                       "sweep_ms_last": round(mon.last_sweep_ms, 3),
                                       "unhealthy": sorted(k for k, v in mon.snapshot().items()
                                                           if v.health != "Healthy")}

    def fabric_and_allocation(self):
        from rocm_k8s_device_plugin_amd.parallel.fabric import Fabric
        node, plug = self.node, self.adm.plug
        inv = getattr(plug, "inv", None) or node.full
        try:
            self.out["fabric"] = Fabric(inv).report([dv.id for dv in node.adv]).as_dict()
        except Exception as e:  # noqa: BLE001
            self.out["fabric"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        # the timed admissions' GetPreferredAllocation (with M > N: a real search
        # over the fragmented availability)
        self.out["timed_allocation"] = dict({"advertised": node.m_adv, "requested": self.n, "held": plug.held},
                                           **alloc_summary(plug, self.adm.rec.alloc))

    def gpu_checks(self):
        from .plugins import throughput_check
        a_, node = self.args, self.node
        if a_.throughput_check and not a_.fixture:
            self.guard.enter("throughput_check")
            self.out["gpu_throughput"] = throughput_check(node.adv_ordinals)
        if a_.peer_check and not a_.fixture:
            from rocm_k8s_device_plugin_amd.health.peer import probe_peers
            self.guard.enter("peer_probe")
            try:
                rep = probe_peers(node.adv_ordinals, nbytes=64 << 20, reps=3, timeout_s=120)
                self.out["peer_probe"] = dict(rep.summary(), wall_ms=round(rep.wall_ms, 1))
            except Exception as e:  # noqa: BLE001
                self.out["peer_probe"] = {"error": f"{type(e).__name__}: {e}"[:300]}

    def run(self) -> dict:
        """Every stage in order; rank 0 returns the extra fields (others {})."""
        self.container_mode_compare()
        self.node_view_compare()
        self.dev_view_compare()
        self.runtime_compare()
        self.back_to_back_compare()
        self.fragmented_compare()
        self.collectives()
        if self.d.rank != 0:
            return {}
        self.allocator_microbench()
        self.health_loop_report()
        self.fabric_and_allocation()
        self.gpu_checks()
        return self.out
