"""Loader for the native extensions.

``core()`` returns the host-only ``_native`` module (kfd/sysfs parsing,
allocator, PCI scan, drm, amd-smi); ``hip()`` returns the in-process gfx950
liveness probe. Both build in-tree on first use if the sources are newer than
the binaries. Neither silently falls back to Python: a missing extension is
an ImportError with the build log, because a "healthy" verdict or an
allocation computed without the native core would be a lie.
"""
from __future__ import annotations

import importlib
import os
import threading
from pathlib import Path

_lock = threading.Lock()
_core = None
_hip = None

PKG_DIR = Path(__file__).resolve().parent.parent
PROBE_EXE = PKG_DIR / "bin" / "mi355x-liveness-probe"
PROBE_EXE_HIP = PKG_DIR / "bin" / "mi355x-liveness-probe-hip"
MOUNTEMU_EXE = PKG_DIR / "bin" / "mi355x-probe-mountemu"
HIP_DEVEMU_EXE = PKG_DIR / "bin" / "mi355x-probe-hip-devemu"
HSACO = PKG_DIR / "kernels" / "liveness_gfx950.hsaco"


def _auto_build_allowed() -> bool:
    return os.environ.get("MI355X_DP_NO_AUTOBUILD", "") not in ("1", "true", "yes")


def _load_from(path: str):
    """The same extension from another build (MI355X_NATIVE_CORE_SO: e.g. the gcov
    build tools/native_coverage.py measures the test suite with)."""
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location("rocm_k8s_device_plugin_amd._native", path)
    if spec is None or spec.loader is None:
        raise ImportError(f"cannot load {path}")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


def core():
    """The `_native` host extension."""
    global _core
    if _core is not None:
        return _core
    with _lock:
        if _core is None:
            try:
                if os.environ.get("MI355X_NATIVE_CORE_SO"):
                    _core = _load_from(os.environ["MI355X_NATIVE_CORE_SO"])
                    return _core
                if _auto_build_allowed():
                    from .. import _build
                    _build.ensure_built(hip=None)
                _core = importlib.import_module("rocm_k8s_device_plugin_amd._native")
            except Exception as e:  # pragma: no cover - surfaced loudly
                raise ImportError(f"native core (_native) unavailable: {e}") from e
    return _core


def hip():
    """The `_hip` in-process probe extension (loads the HIP runtime)."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            try:
                if _auto_build_allowed():
                    from .. import _build
                    _build.ensure_built(hip=True)
                _hip = importlib.import_module("rocm_k8s_device_plugin_amd._hip")
            except Exception as e:  # pragma: no cover
                raise ImportError(f"HIP probe extension (_hip) unavailable: {e}") from e
    return _hip


def probe_executable(runtime: str = "hsa") -> Path:
    """The liveness probe: "hsa" (ROCr-direct, default), "hip", or the container
    entrypoint builds with path interposition that the fake container runtime
    uses to give a process the container's view without root (its /dev and the
    Allocate mounts): "mountemu" (HSA) and "hip-devemu" (HIP runtime)."""
    exe = {"hsa": PROBE_EXE, "hip": PROBE_EXE_HIP, "mountemu": MOUNTEMU_EXE, "hip-devemu": HIP_DEVEMU_EXE}[runtime]
    if _auto_build_allowed():
        from .. import _build
        _build.ensure_built(hip=True)
    if not exe.exists():
        raise FileNotFoundError(f"liveness probe executable missing: {exe}")
    return exe
