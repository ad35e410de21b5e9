"""A minimal stand-in for the CRI runtime step of pod admission.

Real admission: kubelet -> GetPreferredAllocation -> Allocate -> CRI creates
the container with the returned DeviceSpecs -> ROCr in the container sees
exactly the injected render nodes -> the app starts. We cannot create real
containers here, so the runtime step is emulated faithfully where it matters
for latency: a fresh process is started whose GPU visibility is restricted to
the allocated devices, and "ready" is the moment that process has
initialised the GPU runtime and executed the MFMA liveness kernel on its
device(s).

Visibility: a real container's /dev holds exactly the DeviceSpecs (``/dev/kfd``
and each allocated GPU's card / render node), and ROCr's thunk skips every
GPU whose render node it cannot open. Given the specs (``device_paths``), the
HSA entrypoint runs in its path-interposing build with the same view: opens
under ``/dev/dri/`` outside the specs fail with ENOENT (native/tools/
path_interpose.h, ``MI355X_DEV_ALLOW``), so ROCr initialises only the pod's
GPUs, numbered 0..N-1 as inside the container (the HIP entrypoint has the
same build). Without the specs the process sees every GPU the host lets it open and is
restricted with ``ROCR_VISIBLE_DEVICES`` = the host ROCr ordinals instead —
on a node whose GPUs are all accessible that still initialises (and later
tears down) a VM on every GPU, which a container never does.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import time
from dataclasses import dataclass
from typing import FrozenSet, Iterable, List, Optional, Sequence, Set

from .health.liveness import _VISIBILITY_VARS
from .ops.native import probe_executable

_RENDER_RE = re.compile(r"/dev/dri/renderD(\d+)$")


def render_minors_from_specs(container_response) -> List[int]:
    """renderD minors named in a ContainerAllocateResponse's device specs, in order."""
    out = []
    for d in container_response.devices:
        m = _RENDER_RE.search(d.host_path)
        if m:
            out.append(int(m.group(1)))
    return out


@dataclass
class ContainerResult:
    ok: bool
    t_start_ns: int          # parent-side spawn time (CLOCK_MONOTONIC)
    t_ready_ns: int          # child-reported ready time (CLOCK_MONOTONIC)
    wall_ms: float
    doc: dict
    error: str = ""
    # kfd processes that appeared while the container ran and were still being
    # torn down by the driver when it exited (see wait_kfd_released)
    kfd_lingering: FrozenSet[str] = frozenset()
    # kfd processes of other programs on the host that went away while the container
    # started: their driver teardown is what a container's open("/dev/kfd") waits behind
    kfd_foreign_exits: int = 0


KFD_PROC_DIR = "/sys/class/kfd/kfd/proc"


def kfd_processes(proc_dir: str = KFD_PROC_DIR) -> Set[str]:
    """Host PIDs that currently own a kfd process (one directory each)."""
    try:
        return set(os.listdir(proc_dir))
    except OSError:
        return set()


def wait_kfd_released(entries: Iterable[str], timeout_s: float = 0.5, proc_dir: str = KFD_PROC_DIR) -> float:
    """Block until the driver has finished tearing down `entries`; returns ms waited.

    A GPU process's kfd teardown continues for ~150 ms after the process has
    exited, and any GPU process that starts meanwhile blocks in
    open("/dev/kfd") until it is done (measured on MI355X,
    profiles/archive/measurements_r1_r3.md §3c). The procfs entry disappears exactly when the
    teardown completes, so this is the point at which the previous pod has
    really terminated — what kubelet waits for before reusing its devices.
    The entries are host PIDs that appeared while our container ran, so another
    tenant's GPU process started meanwhile can be among them: the wait is
    capped (default 0.5 s, ~3x a teardown) rather than unbounded. What it cannot
    wait for is the teardown of other programs' kfd processes on a shared host:
    a container's open("/dev/kfd") still waits 25-170 ms behind those in ~7 % of
    starts, after a 500 ms settle too (profiles/r5/settle_study_box.json), and
    ContainerResult.kfd_foreign_exits counts them per start.
    """
    left = set(entries)
    t0 = time.monotonic()
    while left and time.monotonic() - t0 < timeout_s:
        time.sleep(0.002)
        left &= kfd_processes(proc_dir)
    return (time.monotonic() - t0) * 1e3


def mount_redirects(mounts: Iterable) -> str:
    """Allocate-response mounts (pb.Mount or (container_path, host_path) tuples)
    -> MI355X_INITPROF_REDIRECT spec (container_path=host_path;...).

    A real runtime bind-mounts these; without root the fake runtime runs the
    path-interposing probe build, which rewrites opens under container_path to
    host_path (native/tools/path_interpose.h). Identity mounts are dropped.
    """
    out = []
    for m in mounts:
        cp, hp = (m.container_path, m.host_path) if hasattr(m, "container_path") else m
        if os.path.abspath(cp) != os.path.abspath(hp):
            out.append(f"{cp}={hp}")
    return ";".join(out)


def start_container(ordinals: Sequence[int], timeout_s: float = 60.0, iters: int = 4,
                    exe: Optional[str] = None, runtime: str = "hsa", mounts: Iterable = (),
                    device_paths: Optional[Sequence[str]] = None,
                    argv_prefix: Sequence[str] = ()) -> ContainerResult:
    """Run the container entrypoint restricted to `ordinals`; block until ready/exit.

    runtime "hsa": the entrypoint launches the MFMA kernel straight through ROCr
    (one AQL dispatch); "hip": the same kernel through the HIP runtime, i.e. what a
    typical HIP/PyTorch application pays before its first kernel.
    device_paths: the container's device nodes from the Allocate DeviceSpecs;
    the process then sees only those GPUs (module docstring).
    exe / argv_prefix: another entrypoint (CPU rehearsals run the stub probe).
    """
    env = {k: v for k, v in os.environ.items() if k not in _VISIBILITY_VARS}
    dev_view = device_paths is not None and runtime in ("hsa", "hip")
    if dev_view:
        dri = [p for p in device_paths if p.startswith("/dev/dri/")]
        if not dri:
            raise ValueError("device_paths name no /dev/dri node")
        env["MI355X_DEV_ALLOW"] = ";".join(dri)
        env["MI355X_INITPROF_COUNT"] = "0"
        runtime = "mountemu" if runtime == "hsa" else "hip-devemu"
    else:
        env["ROCR_VISIBLE_DEVICES"] = ",".join(str(o) for o in ordinals)
    redirect = mount_redirects(mounts)
    if redirect:
        # both interposing builds (HSA mountemu, HIP devemu) apply mounts by redirection
        runtime = {"hsa": "mountemu", "hip": "hip-devemu"}.get(runtime, runtime)
        if runtime not in ("mountemu", "hip-devemu"):
            raise ValueError(f"mounts cannot be applied to the {runtime!r} entrypoint (no path interposition)")
        env["MI355X_INITPROF_REDIRECT"] = redirect
    if runtime in ("mountemu", "hip-devemu"):
        # an emulated container pays only the path checks of its view, never the
        # measurement build's per-path counting (a lock and a map insert per open)
        env.setdefault("MI355X_INITPROF_COUNT", "0")
    argv = [*argv_prefix, exe or str(probe_executable(runtime)), "--devices", ",".join(str(i) for i in range(len(ordinals))),
            "--iters", str(iters), "--timeout", str(min(timeout_s, 30.0))]
    before = kfd_processes()
    t0 = time.monotonic_ns()
    try:
        p = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return ContainerResult(False, t0, 0, (time.monotonic_ns() - t0) / 1e6, {}, "container start timed out")
    wall = (time.monotonic_ns() - t0) / 1e6
    try:
        doc = json.loads(p.stdout.decode().strip().splitlines()[-1])
    except (ValueError, IndexError):
        return ContainerResult(False, t0, 0, wall, {}, f"bad output rc={p.returncode}: {p.stderr.decode()[-300:]}")
    ok = p.returncode == 0 and bool(doc.get("ok"))
    err = "" if ok else "; ".join(d.get("error", "") for d in doc.get("devices", [])) or doc.get("error", "")
    if ok and dev_view and doc.get("hip_device_count") != len(ordinals):
        ok, err = False, (f"container /dev view: ROCr saw {doc.get('hip_device_count')} GPUs, "
                          f"the pod was given {len(ordinals)}")
    after = kfd_processes()
    return ContainerResult(ok, t0, int(doc.get("t_ready_ns", 0)), wall, doc, err, frozenset(after - before),
                           len(before - after))

