"""Rank 0's node under test in bench.py: the sysfs it discovers (the real
/sys, or a synthetic 8x MI355X tree with --fixture), the accessible GPUs, the
advertised set, and the plugin instances behind fake kubelets."""
from __future__ import annotations

import asyncio
import logging
import os
import shutil
import tempfile

from .plugins import NativePluginUnderTest, PluginUnderTest, free_port


class BenchNode:
    def __init__(self, args, n: int, m_adv: int):
        from rocm_k8s_device_plugin_amd.health.monitor import HealthConfig
        from rocm_k8s_device_plugin_amd.topology import discover, hip_ordinals
        from rocm_k8s_device_plugin_amd.utils import log as ulog
        ulog.setup(0)
        logging.getLogger("mi355x").setLevel(logging.WARNING)
        self.args, self.n, self.m_adv = args, n, m_adv
        self.tmp = tempfile.mkdtemp(prefix="mi355x-bench-")
        self.sysfs, self.devroot = args.sysfs_root, args.dev_root
        if args.fixture:
            from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
            fi = make_mi355x_node(os.path.join(self.tmp, "node"))
            self.sysfs, self.devroot = str(fi.sysfs), str(fi.dev)
        self.full = discover(self.sysfs)
        self.ords = hip_ordinals(self.full, self.devroot, check_access=not args.fixture)
        self.usable = sorted((dv for dv in self.full.devices if dv.id in self.ords), key=lambda dv: self.ords[dv.id])
        if len(self.usable) < m_adv:
            raise SystemExit(f"only {len(self.usable)} accessible GPU devices on this node, need {m_adv}")
        self.adv = tuple(self.usable[:m_adv])     # "GPUs advertised at N" (or M with --advertise)
        self.adv_ordinals = [self.ords[dv.id] for dv in self.adv]
        # the Python plugin's health loop needs a GPU; the daemon's runs on the fixture with its sysfs sources
        hp = args.health_pulse if not args.fixture or args.plugin == "native" else 0.0
        self.health_pulse = hp
        self.hcfg = (HealthConfig(exporter_socket=None, liveness=True, smi_ecc=True, smi_events=True, smi_xgmi=True)
                     if hp > 0 else HealthConfig(exporter_socket=None))
        self.idle_hcfg = HealthConfig(exporter_socket=None)
        self.loop = asyncio.new_event_loop()
        self.plugin_kind = "native-daemon" if args.plugin == "native" else "python"
        # the health DaemonSet variant (k8s-ds-amdgpu-dp-health.yaml: -pulse=2 plus the MFMA liveness
        # probe server and amd-smi ECC / events / xGMI) on the daemon; -pulse is whole seconds
        self.health_flags = ()
        if hp > 0 and self.plugin_kind == "native-daemon":
            self.health_flags = ("-pulse", str(max(1, int(round(hp)))),
                                 *(() if args.fixture else ("-liveness", "-liveness_mode", args.health_liveness_mode,
                                                            "-smi_ecc", "-smi_events", "-smi_xgmi",
                                                            *(("-prestart_liveness",) if args.health_prestart
                                                              else ()))))
        # the daemon and the oracle plugin serve on the same C++ server, off the bench's event loop
        self.kclient = args.kubelet_client or "native"

    def make_plugin(self, name, devs, extra=()):
        """A plugin instance advertising `devs` behind its own fake kubelet;
        "device-plugins" is the headline one (it runs the health loop)."""
        main = name == "device-plugins"
        if self.plugin_kind == "native-daemon":
            return NativePluginUnderTest(self.loop, self.tmp, name, self.sysfs, self.devroot, devs, self.full,
                                         self.ords, kubelet_client=self.kclient,
                                         extra=(*extra, *(self.health_flags if main else ())),
                                         metrics_port=free_port() if main and self.health_flags else 0)
        return PluginUnderTest(self.loop, self.tmp, name, self.sysfs, devs, self.full, self.ords,
                               self.hcfg if main else self.idle_hcfg, self.health_pulse if main else 0.0,
                               kubelet_client=self.kclient)

    def gpu_info(self) -> dict:
        adv = self.adv
        return {"ids": [dv.id for dv in adv], "gfx_target_version": sorted({dv.gfx_target_version for dv in adv}),
                "hive_ids": sorted({str(dv.hive_id) for dv in adv}),
                "partition": sorted({dv.partition_type for dv in adv})}

    def close(self) -> None:
        """Tasks still parked (watchers, event waits) are cancelled before the loop goes."""
        loop = self.loop
        rest = [t for t in asyncio.all_tasks(loop) if not t.done()]
        for t in rest:
            t.cancel()
        if rest:
            loop.run_until_complete(asyncio.gather(*rest, return_exceptions=True))
        loop.close()
        shutil.rmtree(self.tmp, ignore_errors=True)
