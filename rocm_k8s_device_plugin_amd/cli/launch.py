"""Installed console scripts: ``k8s-device-plugin`` and ``k8s-node-labeller``
run the native daemons, as ``./k8s-device-plugin`` does in the images and
``scripts/`` does in a checkout (one program per command name, like the
reference's cmd/k8s-device-plugin/main.go:34-120 and
cmd/k8s-node-labeller/main.go:507-590).

The launcher replaces itself with the binary (``os.execv``) before anything in
this process touches a GPU: it imports nothing but the package path.
"""
from __future__ import annotations

import os
import sys

_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin")


def _exec(name: str) -> int:
    exe = os.path.join(_BIN, name)
    if not os.access(exe, os.X_OK):
        sys.stderr.write(f"{exe} is not built (python -m rocm_k8s_device_plugin_amd._build)\n")
        return 127
    os.execv(exe, [sys.argv[0] if sys.argv else name, *sys.argv[1:]])
    return 127  # not reached


def device_plugin() -> int:
    return _exec("mi355x-device-plugin")


def node_labeller() -> int:
    return _exec("mi355x-node-labeller")
