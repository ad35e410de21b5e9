"""Per-allocation kfd topology views (opt-in: ``-topology_view``).

Every HIP/ROCr process starts by snapshotting the kfd topology: on an 8x
MI355X node that is ~4,400 sysfs files (about 550 per GPU node, mostly cache
descriptors), and it happens inside every container at start-up, for all
eight GPUs, although the container can only use the ones it was allocated.

With ``-topology_view`` the plugin materialises, once per distinct device set,
a copy of the topology that contains only the CPU nodes and the allocated GPU
nodes (renumbered contiguously, io/p2p links re-targeted and filtered,
``*_links_count`` fixed up), and returns it in the Allocate response as a
read-only bind mount over ``/sys/devices/virtual/kfd/kfd/topology``. ROCr in the
container then reads ~1/8 of the files for a 1-GPU pod and sees exactly its
own GPUs (and the xGMI links between them, which is what RCCL's topology
detection needs). ``gpu_id`` files are copied verbatim, so kfd ioctls, which
address GPUs by gpu_id, are unaffected.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import tempfile
import threading
from typing import Dict, Iterable, List, Optional, Tuple

KFD_TOPOLOGY_CONTAINER_PATH = "/sys/devices/virtual/kfd/kfd/topology"

_lock = threading.Lock()


def _read(p: str) -> Optional[str]:
    try:
        with open(p) as f:
            return f.read()
    except OSError:
        return None


def _kv_lines(text: str) -> List[Tuple[str, str]]:
    out = []
    for line in text.splitlines():
        parts = line.split(None, 1)
        if len(parts) == 2:
            out.append((parts[0], parts[1].strip()))
        elif len(parts) == 1:
            out.append((parts[0], ""))
    return out


def _render(kv: List[Tuple[str, str]]) -> str:
    return "".join(f"{k} {v}\n" for k, v in kv)


def _is_cpu_node(props: str) -> bool:
    for k, v in _kv_lines(props):
        if k == "simd_count":
            return v.strip() in ("0", "")
    return True


def _copy_tree(src: str, dst: str) -> None:
    """Copy a sysfs subtree as regular files (sysfs reports every file as 4 KiB, so
    read/write the content instead of copying by size)."""
    os.makedirs(dst, exist_ok=True)
    for name in sorted(os.listdir(src)):
        s = os.path.join(src, name)
        d = os.path.join(dst, name)
        if os.path.islink(s):
            continue
        if os.path.isdir(s):
            _copy_tree(s, d)
        else:
            data = _read(s)
            if data is not None:
                with open(d, "w") as f:
                    f.write(data)


def _links(src_dir: str, remap: Dict[int, int]) -> List[str]:
    """Rewritten link property texts (links to nodes outside the view are dropped)."""
    out = []
    if not os.path.isdir(src_dir):
        return out
    for name in sorted(os.listdir(src_dir), key=lambda x: int(x) if x.isdigit() else 1 << 30):
        text = _read(os.path.join(src_dir, name, "properties"))
        if text is None:
            continue
        kv = _kv_lines(text)
        d = dict(kv)
        try:
            f, t = int(d.get("node_from", "-1")), int(d.get("node_to", "-1"))
        except ValueError:
            continue
        if f not in remap or t not in remap:
            continue
        kv = [(k, str(remap[f]) if k == "node_from" else str(remap[t]) if k == "node_to" else v) for k, v in kv]
        out.append(_render(kv))
    return out


def build_view(src_topology: str, dst: str, gpu_node_ids: Iterable[int]) -> Dict[int, int]:
    """Write the filtered topology to `dst`. Returns {original node id: view node id}."""
    keep_gpus = set(int(x) for x in gpu_node_ids)
    nodes_src = os.path.join(src_topology, "nodes")
    ids = sorted(int(n) for n in os.listdir(nodes_src) if n.isdigit())
    kept: List[int] = []
    for i in ids:
        props = _read(os.path.join(nodes_src, str(i), "properties"))
        if props is None:
            continue
        if _is_cpu_node(props) or i in keep_gpus:
            kept.append(i)
    missing = keep_gpus - set(kept)
    if missing:
        raise FileNotFoundError(f"kfd nodes {sorted(missing)} not readable under {nodes_src}")
    remap = {orig: new for new, orig in enumerate(kept)}
    os.makedirs(os.path.join(dst, "nodes"), exist_ok=True)
    for name in ("generation_id", "system_properties"):
        data = _read(os.path.join(src_topology, name))
        if data is not None:
            with open(os.path.join(dst, name), "w") as f:
                f.write(data)
    for orig, new in remap.items():
        s = os.path.join(nodes_src, str(orig))
        d = os.path.join(dst, "nodes", str(new))
        os.makedirs(d, exist_ok=True)
        for sub in sorted(os.listdir(s)):
            if sub in ("io_links", "p2p_links", "properties"):
                continue
            sp = os.path.join(s, sub)
            if os.path.isdir(sp) and not os.path.islink(sp):
                _copy_tree(sp, os.path.join(d, sub))
            elif not os.path.islink(sp):
                data = _read(sp)
                if data is not None:
                    with open(os.path.join(d, sub), "w") as f:
                        f.write(data)
        counts = {}
        for kind in ("io_links", "p2p_links"):
            texts = _links(os.path.join(s, kind), remap)
            counts[kind + "_count"] = len(texts)
            os.makedirs(os.path.join(d, kind), exist_ok=True)
            for j, text in enumerate(texts):
                os.makedirs(os.path.join(d, kind, str(j)), exist_ok=True)
                with open(os.path.join(d, kind, str(j), "properties"), "w") as f:
                    f.write(text)
        props = _kv_lines(_read(os.path.join(s, "properties")) or "")
        props = [(k, str(counts[k]) if k in counts else v) for k, v in props]
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(_render(props))
    return remap


class TopologyViews:
    """Cache of views under `base_dir`, one directory per distinct GPU node set."""

    def __init__(self, base_dir: str, src_topology: str):
        self.base_dir = base_dir
        self.src = src_topology
        self.built = 0

    def key(self, gpu_node_ids: Iterable[int]) -> str:
        ids = ",".join(str(i) for i in sorted(set(gpu_node_ids)))
        gen = (_read(os.path.join(self.src, "generation_id")) or "").strip()
        return hashlib.sha1(f"{gen}:{ids}".encode()).hexdigest()[:16]

    def get(self, gpu_node_ids: Iterable[int]) -> str:
        ids = sorted(set(gpu_node_ids))
        path = os.path.join(self.base_dir, self.key(ids))
        if os.path.isdir(path):
            return path
        with _lock:
            if os.path.isdir(path):
                return path
            os.makedirs(self.base_dir, exist_ok=True)
            tmp = tempfile.mkdtemp(prefix=".view-", dir=self.base_dir)
            try:
                build_view(self.src, tmp, ids)
                os.replace(tmp, path)
            except BaseException:
                shutil.rmtree(tmp, ignore_errors=True)
                raise
            self.built += 1
        return path

    def purge(self) -> None:
        shutil.rmtree(self.base_dir, ignore_errors=True)
