"""Per-device MFMA liveness probing in isolated child processes.

Each device is probed by its own ``mi355x-liveness-probe`` child with
``ROCR_VISIBLE_DEVICES`` narrowed to that device, under a hard deadline:

* a wedged GPU can only stall its own child, which is killed at the deadline
  and reported Unhealthy — ListAndWatch never blocks on the GPU;
* the plugin process itself never initialises HIP, so it holds no context on
  devices that pods own exclusively;
* the verdict lands on the exact kubelet device ID (partition-accurate in CPX),
  unlike the reference's node-global sysfs check (amdgpu.go:865-910).
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import time
from dataclasses import dataclass, field
from typing import Dict, Mapping, Optional, Sequence

from ..ops.native import probe_executable
from ..utils import log
from ..utils.trace import TRACER

_log = log.get("liveness")

_VISIBILITY_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


@dataclass
class ProbeOutcome:
    ok: bool
    reason: str = ""
    latency_ms: float = 0.0
    detail: dict = field(default_factory=dict)


class LivenessProber:
    def __init__(self, exe: Optional[str] = None, timeout_s: float = 10.0, iters: int = 4, max_parallel: int = 8,
                 extra_env: Optional[Mapping[str, str]] = None, argv_prefix: Sequence[str] = ()):
        self.exe = str(exe) if exe else None
        self.timeout_s = timeout_s
        self.iters = iters
        self.max_parallel = max(1, max_parallel)
        self.extra_env = dict(extra_env or {})
        self.argv_prefix = list(argv_prefix)
        self.sweeps = 0

    def _exe(self) -> str:
        if self.exe is None:
            self.exe = str(probe_executable())
        return self.exe

    def _env(self, ordinal: int) -> Dict[str, str]:
        env = {k: v for k, v in os.environ.items() if k not in _VISIBILITY_VARS}
        env.update(self.extra_env)
        env["ROCR_VISIBLE_DEVICES"] = str(ordinal)
        return env

    async def probe_ordinal(self, ordinal: int, nonce: Optional[int] = None) -> ProbeOutcome:
        nonce = (int(time.monotonic_ns()) ^ (ordinal * 0x9E3779B1)) & 0xFFFFFFFF if nonce is None else nonce
        argv = [*self.argv_prefix, self._exe(), "--devices", "0", "--iters", str(self.iters), "--nonce", str(nonce),
                "--timeout", f"{max(0.5, self.timeout_s - 0.5):.2f}"]
        t0 = time.perf_counter()
        try:
            proc = await asyncio.create_subprocess_exec(
                *argv, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE, env=self._env(ordinal),
                start_new_session=True)
        except OSError as e:
            return ProbeOutcome(False, f"spawn failed: {e}")
        try:
            out, err = await asyncio.wait_for(proc.communicate(), timeout=self.timeout_s)
        except asyncio.TimeoutError:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            await proc.wait()
            return ProbeOutcome(False, f"deadline exceeded ({self.timeout_s:.1f}s)",
                                (time.perf_counter() - t0) * 1e3)
        dt = (time.perf_counter() - t0) * 1e3
        try:
            doc = json.loads(out.decode().strip().splitlines()[-1])
        except (ValueError, IndexError):
            return ProbeOutcome(False, f"unparseable probe output (rc={proc.returncode}): "
                                       f"{(err or out).decode(errors='replace')[-200:]}", dt)
        devs = doc.get("devices") or []
        d = devs[0] if devs else {}
        if proc.returncode != 0 or not doc.get("ok") or not d.get("ok"):
            reason = d.get("error") or doc.get("error") or f"probe exit {proc.returncode}"
            return ProbeOutcome(False, reason, dt, d)
        if d.get("nonce") != nonce:
            return ProbeOutcome(False, f"stale probe result (nonce {d.get('nonce')} != {nonce})", dt, d)
        return ProbeOutcome(True, "", dt, d)

    async def probe(self, ordinals: Mapping[str, int]) -> Dict[str, ProbeOutcome]:
        """device ID -> outcome; devices sharing an ordinal are probed once."""
        sem = asyncio.Semaphore(self.max_parallel)
        uniq = sorted(set(ordinals.values()))

        async def one(o: int):
            async with sem:
                with TRACER.span("liveness.probe", "health", ordinal=o):
                    return o, await self.probe_ordinal(o)

        results = dict(await asyncio.gather(*(one(o) for o in uniq)))
        self.sweeps += 1
        return {dev: results[o] for dev, o in ordinals.items()}
