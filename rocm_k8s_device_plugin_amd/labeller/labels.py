"""Node label generators — the drop-in label schema.

Reference: cmd/k8s-node-labeller/main.go:31-505. Every generator, prefix,
value transformation and the removal sets are kept identical:

* ``createLabels`` writes, for both ``beta.amd.com/gpu.<kind>`` and
  ``amd.com/gpu.<kind>``: ``<prefix>.<value>=<count>`` plus ``<prefix>=<value>``
  when exactly one distinct value exists (main.go:96-116);
* ``firmware`` labels are beta-only (main.go:132-155);
* ``vram`` is round(size_in_bytes / MiB / 1024) + "G" from kfd mem_banks/0
  (main.go:236-272);
* a GPU whose kfd node this process may not read (a device cgroup denies it)
  is still counted in ``vram``, ``simd-count`` and ``cu-count`` from what
  discovery recovered from PCI sysfs (its own mem_info_vram_total; the SIMD
  shape of a readable GPU of the same part and partition mode), so those
  counts agree with ``device-id``. The reference's labeller runs privileged
  and reads every node (k8s-ds-amdgpu-labeller.yaml:66-67); unprivileged it
  would drop such GPUs from these counts (main.go:237-277);
* ``product-name`` replaces spaces by ``_`` and drops parentheses (main.go:213-233);
* VF mode: gim driver versions, ``vf-passthrough`` mode on both prefixes and
  raw VF device ids; PF mode: only ``amd.com/gpu.mode=pf-passthrough`` and
  raw PF device ids (main.go:438-505).

Data sources are the native core: kfd topology (parsed once, not once per
GPU per label as in the reference), sysfs, libdrm_amdgpu (family/firmware,
via the card node or — inside containers that only get render nodes — the
render node).

Additions (off by default, never emitted unless enabled):
``amd.com/gpu.gfx-target`` (e.g. ``gfx950``), ``amd.com/gpu.xgmi-hive-count`` and
``amd.com/gpu.xgmi-links-down`` (xGMI links amd-smi reports down across the
node's GPUs, disabled slots not counted: a scheduler can keep multi-GPU jobs
off a node whose fabric is degraded; re-asserted every ``-resync``).
"""
from __future__ import annotations

import math
import os
import re
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from .. import constants as C
from ..ops.native import core
from ..topology import Gpu, Inventory, discover
from ..utils import log

_log = log.get("labeller")

EXTRA_LABELS = ["gfx-target", "xgmi-hive-count", "xgmi-links-down"]


def create_label_prefix(name: str, experimental: bool) -> str:
    return f"{C.EXPERIMENTAL_PREFIX if experimental else C.AMD_PREFIX}/gpu.{name}"


def create_labels(kind: str, entries: Dict[str, int]) -> Dict[str, str]:
    labels: Dict[str, str] = {}
    for experimental in (True, False):
        prefix = create_label_prefix(kind, experimental)
        for k, v in entries.items():
            labels[f"{prefix}.{k}"] = str(v)
            if len(entries) == 1:
                labels[prefix] = k
    return labels


@dataclass
class LabelContext:
    sysfs_root: str = "/sys"
    dev_root: str = "/dev"
    inventory: Optional[Inventory] = None
    _fw_cache: dict = field(default_factory=dict)
    _drm_cache: dict = field(default_factory=dict)
    xgmi_source: Optional[Callable[[], dict]] = None   # amd-smi link state (tests inject a fake)

    @property
    def gpus(self) -> List[Gpu]:
        return list(self.inventory.devices) if self.inventory else []

    def drm_node(self, g: Gpu) -> Optional[str]:
        """card<N> if its /dev node exists, else renderD<N> (libdrm works on both)."""
        if g.card >= 0 and os.path.exists(os.path.join(self.dev_root, "dri", f"card{g.card}")):
            return f"card{g.card}"
        if g.render_minor >= 0 and os.path.exists(os.path.join(self.dev_root, "dri", f"renderD{g.render_minor}")):
            return f"renderD{g.render_minor}"
        return f"card{g.card}" if g.card >= 0 else None

    def drm_info(self, g: Gpu) -> dict:
        node = self.drm_node(g)
        if node is None:
            return {"ok": False, "error": "no drm node"}
        if node not in self._drm_cache:
            self._drm_cache[node] = core().drm_query_gpu_info(self.dev_root, self.sysfs_root, node)
        return self._drm_cache[node]

    def drm_firmware(self, g: Gpu) -> dict:
        node = self.drm_node(g)
        if node is None:
            return {"ok": False, "error": "no drm node"}
        if node not in self._fw_cache:
            self._fw_cache[node] = core().drm_query_firmware(self.dev_root, self.sysfs_root, node)
        return self._fw_cache[node]

    def card_attr(self, g: Gpu, attr: str) -> Optional[str]:
        p = os.path.join(self.sysfs_root, "class/drm", f"card{g.card}", "device", attr)
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError as e:
            if log.V(4):
                _log.debug("%s: %s", p, e)
            return None

    def kfd_node(self, g: Gpu):
        if self.inventory is None or g.node_id < 0:
            return None
        return self.inventory.topology.node(g.node_id)


# ----------------------------------------------------------------- generators

def _firmware(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        fw = ctx.drm_firmware(g)
        if not fw["ok"]:
            _log.error("Fail to get firmware versions: %s", fw["error"])
            continue
        for name, ver in fw["feature"].items():
            k = f"{name}.feat.{ver}"
            counts[k] = counts.get(k, 0) + 1
        for name, ver in fw["firmware"].items():
            k = f"{name}.fw.{ver}"
            counts[k] = counts.get(k, 0) + 1
    pfx = create_label_prefix("firmware", True)
    return {f"{pfx}.{k}": str(v) for k, v in counts.items()}


def _family(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        info = ctx.drm_info(g)
        if not info["ok"]:
            _log.error("Fail to get card family name: %s", info["error"])
            continue
        counts[info["family"]] = counts.get(info["family"], 0) + 1
    return create_labels("family", counts)


def _module_attr(ctx: LabelContext, attr: str) -> str:
    for g in ctx.gpus:
        v = ctx.card_attr(g, f"driver/module/{attr}")
        if v is not None:
            return v
    return ""


# Kubernetes label values: <= 63 chars, [A-Za-z0-9] at both ends, [-_.A-Za-z0-9]
# between (apimachinery validation.IsValidLabelValue). The apiserver rejects a
# whole patch with one bad value, which would leave the node with no labels.
_LABEL_VALUE_RE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")


def sanitize_label_value(v: str) -> str:
    if len(v) <= 63 and _LABEL_VALUE_RE.match(v):
        return v
    out = re.sub(r"[^-A-Za-z0-9_.]", "_", v)[:63]
    return re.sub(r"^[^A-Za-z0-9]+|[^A-Za-z0-9]+$", "", out)


_DNS_LABEL_RE = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


def valid_label_key(k: str) -> bool:
    """apimachinery IsQualifiedName: an optional DNS-subdomain prefix and '/',
    then a name of <= 63 characters shaped like a label value (non-empty)."""
    prefix, _, name = k.rpartition("/") if "/" in k else ("", "", k)
    if not name or len(name) > 63 or not _LABEL_VALUE_RE.match(name):
        return False
    if "/" in k:
        if not prefix or len(prefix) > 253:
            return False
        if not all(len(part) <= 63 and _DNS_LABEL_RE.match(part) for part in prefix.split(".")):
            return False
    return True


def clean_labels(labels: Dict[str, str]) -> Dict[str, str]:
    """Values sanitised; a label whose key is invalid (a value that went into
    the key: product name, firmware name) is dropped with a warning, since the
    apiserver would reject the whole patch."""
    out = {}
    for k, v in labels.items():
        if not valid_label_key(k):
            _log.warning("dropping label %s: not a valid Kubernetes label key", k)
            continue
        out[k] = sanitize_label_value(v)
    return out


def _driver_version_value(raw: str) -> str:
    # amd-smi reports an in-tree amdgpu's version as the kernel banner with the
    # spaces removed ("Linuxversion6.18.54-ant.1(nixbld@...)..." on the MI355X
    # host): the kernel release is the driver version then
    m = re.match(r"^Linux\s*version\s*([0-9][^\s(]*)", raw)
    return m.group(1) if m else raw


def _amdgpu_version_fallback(ctx: LabelContext) -> str:
    """The card's ``driver/module/version`` is absent when amdgpu is built into
    the kernel or loaded without a version string (the MI355X test host): the
    reference then labels an empty string (main.go:166-181). Fall back to
    ``/sys/module/amdgpu/version``, then to amd-smi's driver info."""
    try:
        with open(os.path.join(ctx.sysfs_root, "module/amdgpu/version")) as f:
            v = f.read().strip()
            if v:
                return v
    except OSError:
        pass
    n = core()
    if ctx.gpus and n.smi_available():
        snap = n.smi_snapshot()
        mine = {g.bdf.lower() for g in ctx.gpus}
        for g in snap.get("gpus", []) if snap.get("ok") else []:
            if g["bdf"].lower() in mine and g.get("driver_version"):
                return _driver_version_value(g["driver_version"])
    return ""


def _driver_version(ctx: LabelContext) -> Dict[str, str]:
    v = _module_attr(ctx, "version") or _amdgpu_version_fallback(ctx)
    return {create_label_prefix("driver-version", False): v}


def _driver_src_version(ctx: LabelContext) -> Dict[str, str]:
    return {create_label_prefix("driver-src-version", False): _module_attr(ctx, "srcversion")}


def _device_id(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        v = ctx.card_attr(g, "device")
        if v is None:
            continue
        if v[:2] == "0x":
            v = v[2:]
        counts[v] = counts.get(v, 0) + 1
    return create_labels("device-id", counts)


def _product_name(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        v = ctx.card_attr(g, "product_name")
        if v is None:
            continue
        v = v.strip().replace(" ", "_").replace("(", "").replace(")", "")
        if not v:
            continue
        counts[v] = counts.get(v, 0) + 1
    return create_labels("product-name", counts)


def _recovered(g) -> bool:
    """Identity recovered from PCI sysfs: kfd denied this GPU's node."""
    return getattr(g, "identity", "") == "sysfs"


def _vram(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        node = ctx.kfd_node(g)
        if node is not None and node.mem_bank_sizes:
            size = node.mem_bank_sizes[0]
        elif node is None and _recovered(g) and g.vram_bytes > 0:
            size = g.vram_bytes
        else:
            continue
        mib = size // (1024 * 1024)
        # Go's math.Round: half away from zero
        s = int(math.floor(mib / 1024 + 0.5))
        k = f"{s}G"
        counts[k] = counts.get(k, 0) + 1
    return create_labels("vram", counts)


def _simd_count(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        node = ctx.kfd_node(g)
        if node is not None and "simd_count" in node.props:
            k = str(node.simd_count)
        elif node is None and _recovered(g) and g.simd_count > 0:
            k = str(g.simd_count)
        else:
            continue
        counts[k] = counts.get(k, 0) + 1
    return create_labels("simd-count", counts)


def _cu_count(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        node = ctx.kfd_node(g)
        if node is not None and node.simd_per_cu != 0:
            k = str(node.simd_count // node.simd_per_cu)
        elif node is None and _recovered(g) and g.simd_per_cu > 0 and g.simd_count > 0:
            k = str(g.simd_count // g.simd_per_cu)
        else:
            continue
        counts[k] = counts.get(k, 0) + 1
    return create_labels("cu-count", counts)


def _compute_memory_partition(ctx: LabelContext) -> Dict[str, str]:
    inv = ctx.inventory
    if inv is None or not inv.homogeneous:
        return {}
    for t, c in inv.partition_counts().items():
        if c > 0:
            return {create_label_prefix("compute-memory-partition", False): t}
    return {}


def _compute_partitioning_supported(ctx: LabelContext) -> Dict[str, str]:
    v = core().compute_partition_supported(ctx.sysfs_root)
    return {create_label_prefix("compute-partitioning-supported", False): "true" if v else "false"}


def _memory_partitioning_supported(ctx: LabelContext) -> Dict[str, str]:
    v = core().memory_partition_supported(ctx.sysfs_root)
    return {create_label_prefix("memory-partitioning-supported", False): "true" if v else "false"}


def _mode(ctx: LabelContext) -> Dict[str, str]:
    return {create_label_prefix("mode", True): C.CONTAINER, create_label_prefix("mode", False): C.CONTAINER}


def gfx_name(gfx_target_version: int) -> str:
    """kfd gfx_target_version (e.g. 90500) -> LLVM target name (gfx950)."""
    major = gfx_target_version // 10000
    minor = (gfx_target_version // 100) % 100
    step = gfx_target_version % 100
    return f"gfx{major}{minor:x}{step:x}"


def _gfx_target(ctx: LabelContext) -> Dict[str, str]:
    counts: Dict[str, int] = {}
    for g in ctx.gpus:
        if g.gfx_target_version > 0:
            k = gfx_name(g.gfx_target_version)
            counts[k] = counts.get(k, 0) + 1
    return create_labels("gfx-target", counts)


def _xgmi_hive_count(ctx: LabelContext) -> Dict[str, str]:
    hives = {g.hive_id for g in ctx.gpus if g.hive_id}
    if not ctx.gpus:
        return {}
    return {create_label_prefix("xgmi-hive-count", False): str(len(hives))}


def _xgmi_links_down(ctx: LabelContext) -> Dict[str, str]:
    snap = ctx.xgmi_source() if ctx.xgmi_source is not None else core().smi_xgmi_links()
    if not snap.get("ok") or not ctx.gpus:
        return {}
    mine = {g.bdf.lower() for g in ctx.gpus}
    seen = [g for g in snap.get("gpus", []) if g.get("bdf", "").lower() in mine and g.get("status_ok")]
    if not seen:
        return {}
    down = sum(1 for g in seen for st in g.get("status", []) if st == 0)
    return {create_label_prefix("xgmi-links-down", False): str(down)}


LABEL_GENERATORS: Dict[str, Callable[[LabelContext], Dict[str, str]]] = {
    "firmware": _firmware,
    "family": _family,
    "driver-version": _driver_version,
    "driver-src-version": _driver_src_version,
    "device-id": _device_id,
    "product-name": _product_name,
    "vram": _vram,
    "simd-count": _simd_count,
    "cu-count": _cu_count,
    "compute-memory-partition": _compute_memory_partition,
    "compute-partitioning-supported": _compute_partitioning_supported,
    "memory-partitioning-supported": _memory_partitioning_supported,
    "mode": _mode,
    "gfx-target": _gfx_target,
    "xgmi-hive-count": _xgmi_hive_count,
    "xgmi-links-down": _xgmi_links_down,
}


# ------------------------------------------------------------------ key lists

def all_label_keys() -> List[str]:
    """amd.com keys removed before applying (reference initLabelLists, main.go:50-62)."""
    keys = [create_label_prefix(n, False) for n in C.SUPPORTED_LABELS + EXTRA_LABELS]
    keys += [C.LEGACY_COMPUTE_PARTITIONING_SUPPORTED, C.LEGACY_MEMORY_PARTITIONING_SUPPORTED,
             C.LEGACY_PARTITION_TYPE]
    return keys


def all_experimental_label_keys() -> List[str]:
    return [create_label_prefix(n, True) for n in C.SUPPORTED_LABELS + EXTRA_LABELS]


def remove_old_node_labels(labels: Optional[Dict[str, str]]) -> Dict[str, str]:
    """Reference removeOldNodeLabels (main.go:64-83), plus: beta counters
    ``<key>.<value>`` are removed even when the base key is already gone (a
    half-cleaned node would otherwise keep stale counters forever)."""
    if labels is None:
        return {}
    out = dict(labels)
    for k in all_label_keys():
        out.pop(k, None)
    for k in all_experimental_label_keys():
        v = out.pop(k, None)
        if v is not None:
            out.pop(f"{k}.{v}", None)
        for key in [x for x in out if x.startswith(k + ".")]:
            del out[key]
    return out


# --------------------------------------------------------------- per mode

def generate_container_labels(enabled: Dict[str, bool], ctx: LabelContext) -> Dict[str, str]:
    results: Dict[str, str] = {}
    if not ctx.gpus:
        _log.info("No AMD GPUs found, skipping label generation")
        return results
    for name, gen in LABEL_GENERATORS.items():
        if not enabled.get(name):
            continue
        results.update(gen(ctx))
    return clean_labels(results)


def generate_vf_labels(enabled: Dict[str, bool], sysfs_root: str) -> Dict[str, str]:
    n = core()
    results: Dict[str, str] = {}
    res = n.scan_vf_mapping(sysfs_root)
    if not res.ok or not res.groups:
        return results
    gim = n.read_gim_versions(sysfs_root)
    if gim is None:
        return results
    version, srcversion = gim
    if enabled.get("driver-version"):
        results[create_label_prefix("driver-version", False)] = version
    if enabled.get("driver-src-version"):
        results[create_label_prefix("driver-src-version", False)] = srcversion
    if enabled.get("mode"):
        results[create_label_prefix("mode", False)] = C.VF_PASSTHROUGH
        results[create_label_prefix("mode", True)] = C.VF_PASSTHROUGH
    if enabled.get("device-id"):
        counts: Dict[str, int] = {}
        for fns in res.groups.values():
            for f in fns:
                counts[f.device_id] = counts.get(f.device_id, 0) + 1
        results.update(create_labels("device-id", counts))
    return results


def generate_pf_labels(enabled: Dict[str, bool], sysfs_root: str) -> Dict[str, str]:
    n = core()
    results: Dict[str, str] = {}
    res = n.scan_pf_mapping(sysfs_root)
    if not res.ok or not res.groups:
        return results
    if enabled.get("mode"):
        results["amd.com/gpu.mode"] = C.PF_PASSTHROUGH
    if enabled.get("device-id"):
        counts: Dict[str, int] = {}
        for fns in res.groups.values():
            for f in fns:
                counts[f.device_id] = counts.get(f.device_id, 0) + 1
        results.update(create_labels("device-id", counts))
    return results


def generate_labels(enabled: Dict[str, bool], driver_type: str = "", sysfs_root: str = "/sys",
                    dev_root: str = "/dev", inventory: Optional[Inventory] = None,
                    xgmi_source: Optional[Callable[[], dict]] = None) -> Dict[str, str]:
    """Reference generateLabels (main.go:389-408): explicit mode, else container -> VF -> PF."""

    def container():
        inv = inventory
        if inv is None:
            inv = discover(sysfs_root) if os.path.exists(os.path.join(sysfs_root, "module/amdgpu/drivers")) \
                else None
        return generate_container_labels(enabled, LabelContext(sysfs_root, dev_root, inv, xgmi_source=xgmi_source))

    if driver_type == C.CONTAINER:
        return container()
    clean = clean_labels

    if driver_type == C.VF_PASSTHROUGH:
        return clean(generate_vf_labels(enabled, sysfs_root))
    if driver_type == C.PF_PASSTHROUGH:
        return clean(generate_pf_labels(enabled, sysfs_root))
    labels = container()
    if not labels:
        labels = generate_vf_labels(enabled, sysfs_root)
    if not labels:
        labels = generate_pf_labels(enabled, sysfs_root)
    return clean(labels)
