"""Per-device MFMA liveness probing out of process.

Two modes, both under a hard deadline enforced from here:

``persistent`` (default): one long-lived ``mi355x-liveness-probe --serve``
child keeps the GPU runtime initialised and answers one request per sweep,
probing every device in parallel. Measured on MI355X (profiles/archive/measurements_r1_r3.md §3c):
each GPU process that exits leaves ~150 ms of kfd teardown in the kernel, and a
GPU process that starts meanwhile (a pod's runtime init) blocks in
``open("/dev/kfd")`` for it. A prober that spawned a process per device per
pulse would inject exactly that stall into pod start-up; the server creates
its kfd process once. Per-sweep cost drops from ~150 ms to ~10 ms.

``spawn``: each device probed by its own child with ``ROCR_VISIBLE_DEVICES``
narrowed to that device. Used for isolation whenever the server misses its
deadline or dies: the sweep is re-run per device so that one wedged GPU is
reported Unhealthy on its own rather than taking the whole node with it.

Either way ListAndWatch never blocks on a GPU, the plugin process itself never
initialises a GPU runtime, and the verdict lands on the exact kubelet device
ID (partition-accurate in CPX), unlike the reference's node-global sysfs check
(amdgpu.go:865-910).
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import time
from dataclasses import dataclass, field
from typing import Collection, Dict, Mapping, Optional, Sequence

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
    # kept-queue server: the dispatch has not completed yet and stays queued
    # (e.g. behind a tenant kernel that holds every CU); the next probe waits
    # for it instead of submitting another
    pending: bool = False


class ProbeServerError(RuntimeError):
    pass


class _ProbeServer:
    """One ``--serve`` child: JSON lines on stdout, requests on stdin."""

    def __init__(self, proc: asyncio.subprocess.Process, hello: dict):
        self.proc = proc
        self.hello = hello
        self.requests = 0

    @classmethod
    async def start(cls, argv, env, timeout_s: float) -> "_ProbeServer":
        proc = await asyncio.create_subprocess_exec(
            *argv, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            stderr=asyncio.subprocess.DEVNULL, env=env, start_new_session=True)
        srv = cls(proc, {})
        try:
            srv.hello = await srv._read(timeout_s)
        except BaseException:
            await srv.kill()
            raise
        if not srv.hello.get("serve") or not srv.hello.get("ok"):
            await srv.kill()
            raise ProbeServerError(f"probe server failed to start: {srv.hello}")
        return srv

    async def _read(self, timeout_s: float) -> dict:
        line = await asyncio.wait_for(self.proc.stdout.readline(), timeout=timeout_s)
        if not line:
            raise ProbeServerError(f"probe server exited (rc={self.proc.returncode})")
        try:
            return json.loads(line)
        except ValueError as e:
            raise ProbeServerError(f"unparseable probe server output: {line[-200:]!r}") from e

    async def request(self, line: str, timeout_s: float) -> dict:
        try:
            self.proc.stdin.write(line.encode() + b"\n")
            await self.proc.stdin.drain()
        except (BrokenPipeError, ConnectionResetError) as e:
            raise ProbeServerError(f"probe server gone: {e}") from e
        self.requests += 1
        return await self._read(timeout_s)

    @property
    def alive(self) -> bool:
        return self.proc.returncode is None

    async def kill(self) -> None:
        if self.proc.returncode is None:
            try:
                os.killpg(self.proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        await self.proc.wait()


class LivenessProber:
    MODES = ("persistent", "spawn")
    SERVER_BACKOFF_SWEEPS = 4

    def __init__(self, exe: Optional[str] = None, timeout_s: float = 10.0, iters: int = 4, max_parallel: int = 8,
                 extra_env: Optional[Mapping[str, str]] = None, argv_prefix: Sequence[str] = (),
                 mode: str = "persistent", keep_queues: bool = True,
                 kfd_proc_dir: str = "/sys/class/kfd/kfd/proc"):
        if mode not in self.MODES:
            raise ValueError(f"liveness mode must be one of {self.MODES}, got {mode!r}")
        self.exe = str(exe) if exe else None
        self.timeout_s = timeout_s
        self.iters = iters
        self.max_parallel = max(1, max_parallel)
        self.extra_env = dict(extra_env or {})
        self.argv_prefix = list(argv_prefix)
        self.mode = mode
        # persistent mode only: the server keeps each device's queue, executable
        # and buffers between sweeps (`--serve --keep`), so a sweep creates no
        # kfd queue and causes no HWS runlist update on the tenants' GPUs
        self.keep_queues = keep_queues
        # the server's own kfd process entry (its queues must not make a GPU
        # look busy to the chip-sweep scheduler); found by listing
        # <kfd_proc_dir> around the server's start-up, since the entry is
        # named by the host PID, which a containerised plugin cannot see
        self.kfd_proc_dir = kfd_proc_dir
        self._own_kfd: frozenset = frozenset()
        self.sweeps = 0
        self.server_starts = 0
        self.server_restarts = 0   # restarted after failing a device a fresh process found healthy
        self.fallbacks = 0
        self._server: Optional[_ProbeServer] = None
        self._server_backoff = 0  # sweeps to run in spawn mode after a server failure
        self._pending_nonce: Dict[int, int] = {}   # ordinal -> nonce of the server's outstanding dispatch
        # host ordinals the server may touch (None = every GPU). A GPU left out
        # gets no queue, no ROCr state and no runlist slot from the server.
        self._visible: Optional[tuple] = None
        self._server_visible: Optional[tuple] = None
        # throughput check (kind "perf"): HBM buffer size and MFMA pairs per wave
        self.perf_mib = 4096
        self.perf_iters = 1 << 16

    @property
    def server_running(self) -> bool:
        return self._server is not None and self._server.alive

    def set_visible(self, ordinals: Optional[Collection[int]]) -> None:
        """Restrict the persistent server to these host ordinals (None = all).
        A change restarts the server on its next request (rare: the health
        monitor changes it when a GPU gets or stops being crowded)."""
        self._visible = None if ordinals is None else tuple(sorted(set(int(o) for o in ordinals)))

    def _kfd_entries(self) -> set:
        try:
            return set(os.listdir(self.kfd_proc_dir))
        except OSError:
            return set()

    @property
    def own_kfd_entries(self) -> frozenset:
        """kfd proc entries of the running probe server (empty when unknown).

        Several entries can appear while the server starts if another GPU
        process starts at the same moment; the ambiguity resolves once the
        others have exited (the server's entry lives as long as it does).
        Unresolved, nothing is claimed, so GPUs look busy: the safe side.
        """
        if self._server is None or not self._server.alive:
            return frozenset()
        if len(self._own_kfd) > 1:
            self._own_kfd = frozenset(self._own_kfd & self._kfd_entries())
        return self._own_kfd if len(self._own_kfd) == 1 else frozenset()

    def own_kfd_entries_for(self, gpu_ids) -> frozenset:
        """own_kfd_entries, resolving a start-up ambiguity by queue coverage: a
        kept-queue server holds a queue on every GPU it probed, while a pod's
        process only sees (and queues on) the pod's GPUs. The one candidate
        whose queues cover all of `gpu_ids` is the server."""
        own = self.own_kfd_entries
        want = {int(g) for g in gpu_ids if g}
        if own or len(self._own_kfd) <= 1 or not want or not self.keep_queues:
            return own
        match = []
        for e in sorted(self._own_kfd):
            qdir = os.path.join(self.kfd_proc_dir, e, "queues")
            have = set()
            try:
                for q in os.listdir(qdir):
                    with open(os.path.join(qdir, q, "gpuid")) as f:
                        have.add(int(f.read().strip() or 0))
            except (OSError, ValueError):
                continue
            if want <= have:
                match.append(e)
        if len(match) == 1:
            self._own_kfd = frozenset(match)
            return self._own_kfd
        return frozenset()

    def _exe(self) -> str:
        if self.exe is None:
            self.exe = str(probe_executable())
        return self.exe

    def _env(self, ordinal: Optional[int]) -> Dict[str, str]:
        env = {k: v for k, v in os.environ.items() if k not in _VISIBILITY_VARS}
        env.update(self.extra_env)
        if ordinal is not None:  # the server sees every device: its ordinals are host ROCr ordinals
            env["ROCR_VISIBLE_DEVICES"] = str(ordinal)
        return env

    @staticmethod
    def _nonce(ordinal: int) -> int:
        return (int(time.monotonic_ns()) ^ (ordinal * 0x9E3779B1)) & 0xFFFFFFFF

    @staticmethod
    def _judge(doc_ok: bool, d: dict, nonce: int, dt: float, rc: int = 0) -> ProbeOutcome:
        if rc != 0 or not doc_ok or not d.get("ok"):
            reason = d.get("error") or f"probe exit {rc}"
            return ProbeOutcome(False, reason, dt, d)
        if d.get("nonce") != nonce:
            return ProbeOutcome(False, f"stale probe result (nonce {d.get('nonce')} != {nonce})", dt, d)
        return ProbeOutcome(True, "", dt, d)

    async def probe_ordinal(self, ordinal: int, nonce: Optional[int] = None, kind: str = "probe") -> ProbeOutcome:
        nonce = self._nonce(ordinal) if nonce is None else nonce
        argv = [*self.argv_prefix, self._exe(), "--devices", "0", "--iters", str(self.iters), "--nonce", str(nonce),
                "--timeout", f"{max(0.5, self.timeout_s - 0.5):.2f}"]
        if kind == "sweep":
            argv.append("--sweep")
        elif kind == "perf":
            argv += ["--perf", "--perf-mib", str(self.perf_mib), "--perf-iters", str(self.perf_iters)]
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
            # the dispatch did not complete: on a GPU that runs a tenant's kernels
            # this is inconclusive (HealthMonitor applies the busy grace), as in
            # the kept-queue server
            return ProbeOutcome(False, f"deadline exceeded ({self.timeout_s:.1f}s)",
                                (time.perf_counter() - t0) * 1e3, pending=kind == "probe")
        dt = (time.perf_counter() - t0) * 1e3
        try:
            doc = json.loads(out.decode().strip().splitlines()[-1])
        except (ValueError, IndexError):
            return ProbeOutcome(False, f"unparseable probe output (rc={proc.returncode}): "
                                       f"{(err or out).decode(errors='replace')[-200:]}", dt)
        devs = doc.get("devices") or []
        d = devs[0] if devs else {}
        if not d and doc.get("error"):
            d = {"error": doc["error"]}
        return self._judge(bool(doc.get("ok")), d, nonce, dt, proc.returncode)

    # ------------------------------------------------------------ persistent
    async def _probe_server(self, uniq, kind: str = "probe") -> Dict[int, ProbeOutcome]:
        t0 = time.perf_counter()
        visible = self._visible
        if visible is not None and not set(uniq) <= set(visible):
            visible = tuple(sorted(set(visible) | set(uniq)))
        if self._server is not None and self._server.alive and visible != self._server_visible:
            await self.close()          # the GPUs the server may touch changed
        if self._server is None or not self._server.alive:
            argv = [*self.argv_prefix, self._exe(), "--serve", *(["--keep"] if self.keep_queues else [])]
            env = self._env(None)
            if visible is not None:
                env["ROCR_VISIBLE_DEVICES"] = ",".join(str(o) for o in visible)
            before = self._kfd_entries()
            self._server = await _ProbeServer.start(argv, env, self.timeout_s)
            self._server_visible = visible
            self._own_kfd = frozenset(self._kfd_entries() - before)
            self.server_starts += 1
        # the server numbers the GPUs it sees; with a visibility list those are its positions
        local = {o: (self._server_visible.index(o) if self._server_visible is not None else o) for o in uniq}
        host = {v: k for k, v in local.items()}
        nonces = {o: self._nonce(o) for o in uniq}
        # the server's own dispatch wait ends before our deadline for the reply
        inner = self.timeout_s - min(0.5, 0.25 * self.timeout_s)
        head = f"perf {self.perf_iters} {inner:.2f} {self.perf_mib}" if kind == "perf" else \
            f"{kind} {self.iters} {inner:.2f}"
        line = head + " " + " ".join(f"{local[o]}:{nonces[o]}" for o in uniq)
        doc = await self._server.request(line, self.timeout_s)
        dt = (time.perf_counter() - t0) * 1e3
        by_ord = {}
        for d in doc.get("devices") or []:
            if d.get("ordinal") in host:
                d = dict(d, ordinal=host[d.get("ordinal")])
                by_ord[d["ordinal"]] = d
        out = {}
        for o in uniq:
            d = by_ord.get(o)
            if d is None:
                out[o] = ProbeOutcome(False, "device missing from probe server reply", dt)
                continue
            if kind in ("sweep", "perf"):
                # sweeps and throughput checks run on their own queue: the kept
                # probe slot (and its pending dispatch, if any) is untouched by them
                out[o] = self._judge(bool(d.get("ok")), d, nonces[o], dt)
                continue
            # a late verdict answers the dispatch (and nonce) of the probe that left it pending
            expect = self._pending_nonce.pop(o, nonces[o]) if d.get("late") else nonces[o]
            r = self._judge(bool(d.get("ok")), d, expect, dt)
            if not r.ok and float(d.get("pending_s") or 0) > 0:
                r.pending = True
                self._pending_nonce.setdefault(o, nonces[o])
            elif not r.ok and d.get("hip_error") == -1 and not self.keep_queues:
                r.pending = True     # timed out without a kept slot: no late verdict will follow
            elif not d.get("late"):
                self._pending_nonce.pop(o, None)
            out[o] = r
        return out

    async def close(self) -> None:
        self._pending_nonce.clear()   # a new server starts without outstanding dispatches
        if self._server is not None:
            await self._server.kill()
            self._server = None
            self._server_visible = None

    async def sweep(self, ordinals: Mapping[str, int]) -> Dict[str, ProbeOutcome]:
        """The full-chip sweep (every CU of every XCD) instead of the one-wave probe.

        It holds each CU's whole LDS for ~50 us and waits for the entire grid to
        be resident, so callers run it only on GPUs without foreign work."""
        return await self.probe(ordinals, kind="sweep")

    async def perf(self, ordinals: Mapping[str, int]) -> Dict[str, ProbeOutcome]:
        """The throughput check (HBM pattern write/read bandwidth, sustained bf16
        MFMA rate, per-XCD shader clocks; liveness_kernel.h). `ok` covers
        correctness only (every word read back exact, identical MFMA checksums,
        every XCD ran); the rates are in `detail` for the caller's thresholds.
        It owns the chip for tens of ms: idle GPUs only."""
        return await self.probe(ordinals, kind="perf")

    async def _confirm_failures(self, failed, results, kind: str) -> Dict[int, ProbeOutcome]:
        """Re-probe the devices the server failed, each in a fresh process.

        The server's runtime lives across sweeps (and with kept queues so do its
        queues): after a GPU reset, or anything else that leaves that runtime
        stale, it could keep failing a device that a fresh process finds
        healthy. A failure is therefore only reported when a fresh process
        confirms it; if one does not, the server is restarted for the next sweep.
        """
        sem = asyncio.Semaphore(self.max_parallel)

        async def one(o: int):
            async with sem:
                return o, await self.probe_ordinal(o, kind=kind)

        fresh = dict(await asyncio.gather(*(one(o) for o in failed)))
        out = {}
        stale = False
        for o, r in fresh.items():
            if r.ok:
                stale = True
                out[o] = r
            else:
                out[o] = ProbeOutcome(False, f"{r.reason} (server: {results[o].reason})", r.latency_ms, r.detail)
        if stale:
            self.server_restarts += 1
            _log.warning("probe server failed ordinals %s that a fresh process found healthy; restarting it",
                         sorted(o for o, r in fresh.items() if r.ok))
            await self.close()
        return out

    async def probe(self, ordinals: Mapping[str, int], kind: str = "probe",
                    busy: Collection[int] = ()) -> Dict[str, ProbeOutcome]:
        """device ID -> outcome; devices sharing an ordinal are probed once.

        `busy`: ordinals whose GPU runs other processes' queues. A pending
        dispatch there is a tenant holding the GPU, not evidence of a fault, so
        it is not re-probed in a fresh process (which would only wait too)."""
        uniq = sorted(set(ordinals.values()))
        use_server = self.mode == "persistent" and uniq and self._server_backoff == 0
        self._server_backoff = max(0, self._server_backoff - 1)
        if use_server:
            try:
                with TRACER.span("liveness.request", "health", ordinals=len(uniq), kind=kind):
                    results = await self._probe_server(uniq, kind)
                failed = [o for o in uniq if not results[o].ok and not (results[o].pending and o in busy)]
                if not self.keep_queues and any(r.detail.get("hip_error") == -1 or r.detail.get("hsa_error") == -1
                                                for r in results.values()):
                    # without kept queues a timed-out dispatch's queue (and its 181 MB
                    # save area) can never be freed by the server: restart it. (A timed-out
                    # chip sweep is held by the server, one per device, and freed once it
                    # completes; a restart frees it at once.)
                    await self.close()
                if failed:
                    results.update(await self._confirm_failures(failed, results, kind))
                self.sweeps += 1
                return {dev: results[o] for dev, o in ordinals.items()}
            except (asyncio.TimeoutError, ProbeServerError, OSError) as e:
                # a wedged device stalls the whole server: drop it and isolate per device
                _log.warning("probe server failed (%s); re-probing each device in its own process",
                             e if str(e) else type(e).__name__)
                self.fallbacks += 1
                self._server_backoff = self.SERVER_BACKOFF_SWEEPS
                await self.close()
        sem = asyncio.Semaphore(self.max_parallel)

        async def one(o: int):
            async with sem:
                with TRACER.span("liveness.probe", "health", ordinal=o, kind=kind):
                    return o, await self.probe_ordinal(o, kind=kind)

        results = dict(await asyncio.gather(*(one(o) for o in uniq)))
        self.sweeps += 1
        return {dev: results[o] for dev, o in ordinals.items()}
