"""NUMA-node sysfs view without per-CPU cache descriptors (opt-in: ``-node_view``).

Measured on an 8x MI355X host with 256 CPUs (profiles/archive/measurements_r1_r3.md §3e): ROCr's
``hsa_init`` opens 9,486 sysfs files, and 7,650 of them are the CPU cache
descriptors it reaches through ``/sys/devices/system/node/node<N>/cpu<M>/cache/
index<K>/*`` — for every CPU of the host, whatever the container's cpuset.
Refusing just those directories (in-process emulation) takes ``hsa_init``
from 48 ms to 14-16 ms; ROCr handles the missing directories (the CPU agent
then reports no cache sizes, which HIP does not use).

The view keeps everything else *live*: the plugin builds, once, a directory
that mirrors ``/sys/devices/system/node`` where

* every top-level file and every ``node<N>/<file>`` is a symlink into the real
  node directory, bind-mounted read-only at ``NODE_ALIAS`` inside the
  container (``meminfo``, ``distance``, ``cpumap``, ``hugepages/`` ... stay
  current);
* each ``node<N>/cpu<M>`` is a real directory whose entries are symlinks to
  ``/sys/devices/system/cpu/cpu<M>/<entry>`` for every entry except
  ``cache``.

``/sys/devices/system/cpu`` itself is untouched, so anything that reads CPU
caches there (lscpu, PyTorch's cpuinfo) sees them as before; only the
node-relative walk that ROCr's thunk does is shortened. The Allocate response
mounts the real directory at ``NODE_ALIAS`` and the view over
``/sys/devices/system/node`` (both read-only).
"""
from __future__ import annotations

import os
import re
import shutil
import tempfile
import threading
from typing import List, Optional, Tuple

NODE_CONTAINER_PATH = "/sys/devices/system/node"
NODE_ALIAS = "/run/mi355x/sys-node"
CPU_CONTAINER_PATH = "/sys/devices/system/cpu"

_NODE = re.compile(r"^node\d+$")
_CPU = re.compile(r"^cpu\d+$")


def build_node_view(src: str, dst: str, alias: str = NODE_ALIAS, cpu_root: str = CPU_CONTAINER_PATH,
                    src_cpu_root: Optional[str] = None) -> Tuple[int, int]:
    """Write the view of `src` (a node directory) into `dst`.

    `alias` is where the real node directory is visible inside the container,
    `cpu_root` where the real cpu directory is; `src_cpu_root` is the host path
    used to list each CPU's entries (defaults to ``<src>/../cpu``). Returns
    (symlinks, hidden cache directories).
    """
    src_cpu_root = src_cpu_root or os.path.join(os.path.dirname(os.path.abspath(src)), "cpu")
    links = hidden = 0
    os.makedirs(dst, exist_ok=True)
    for name in sorted(os.listdir(src)):
        s = os.path.join(src, name)
        if not (_NODE.match(name) and os.path.isdir(s)):
            os.symlink(os.path.join(alias, name), os.path.join(dst, name))
            links += 1
            continue
        nd = os.path.join(dst, name)
        os.makedirs(nd, exist_ok=True)
        for child in sorted(os.listdir(s)):
            if _CPU.match(child):
                cd = os.path.join(nd, child)
                os.makedirs(cd, exist_ok=True)
                try:
                    entries = sorted(os.listdir(os.path.join(src_cpu_root, child)))
                except OSError:
                    entries = []
                for e in entries:
                    if e == "cache":
                        hidden += 1
                        continue
                    os.symlink(os.path.join(cpu_root, child, e), os.path.join(cd, e))
                    links += 1
            else:
                os.symlink(os.path.join(alias, name, child), os.path.join(nd, child))
                links += 1
    return links, hidden


class NodeView:
    """Builds the view once (lazily) and hands out the Allocate mounts."""

    def __init__(self, root: str, sysfs_root: str = "/sys", alias: str = NODE_ALIAS):
        """`alias`: where the real node directory is visible in the container. A
        runtime that cannot mount (bench.py's fake one) passes the host path
        itself, and the view's symlinks then resolve without the alias mount."""
        self.root = root
        self.alias = alias
        self.src = os.path.join(sysfs_root, "devices/system/node")
        self.src_cpu = os.path.join(sysfs_root, "devices/system/cpu")
        self._lock = threading.Lock()
        self._path: Optional[str] = None
        self.links = self.hidden = 0

    def path(self) -> str:
        with self._lock:
            if self._path is None:
                os.makedirs(self.root, exist_ok=True)
                final = os.path.join(self.root, "node")
                tmp = tempfile.mkdtemp(prefix=".node-", dir=self.root)
                try:
                    self.links, self.hidden = build_node_view(self.src, os.path.join(tmp, "node"),
                                                              alias=self.alias, src_cpu_root=self.src_cpu)
                    if os.path.exists(final):
                        shutil.rmtree(final)
                    os.rename(os.path.join(tmp, "node"), final)
                finally:
                    shutil.rmtree(tmp, ignore_errors=True)
                self._path = final
            return self._path

    def mounts(self) -> List[Tuple[str, str]]:
        """(host_path, container_path) pairs, in mount order."""
        view = self.path()
        alias = [] if os.path.abspath(self.alias) == os.path.abspath(self.src) else [(self.src, self.alias)]
        return alias + [(view, NODE_CONTAINER_PATH)]
