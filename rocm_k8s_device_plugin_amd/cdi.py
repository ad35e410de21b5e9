"""Container Device Interface (CDI) specs for the advertised GPUs.

The reference only returns raw DeviceSpecs in Allocate
(internal/pkg/amdgpu/amdgpu.go:255-297): ``/dev/kfd`` plus each device's
``/dev/dri/card<N>`` and ``/dev/dri/renderD<N>``. Kubernetes >= 1.28 also
lets a device plugin name CDI devices (``ContainerAllocateResponse.cdi_devices``,
field 5, api.proto) which the CRI runtime (containerd >= 1.7, CRI-O >= 1.23)
resolves against spec files in ``/var/run/cdi``. This module writes those
specs and names the devices; ``-device_list_strategy`` selects what Allocate
returns:

* ``device-specs`` (default, reference behaviour): DeviceSpecs only;
* ``cdi-cri``: ``cdi_devices`` entries ``amd.com/<resource>=<device id>``;
* ``cdi-annotations``: the same names in ``cdi.k8s.io/...`` annotations, for
  runtimes that read CDI requests from annotations only.

Several strategies can be combined (comma-separated). A spec file per
resource (``amd.com-<resource>.json``, kind ``amd.com/<resource>``) holds
one CDI device per advertised device ID, the same IDs ListAndWatch reports
(PCI BDF / ``amdgpu_xcp_N``), with its card and render nodes; ``/dev/kfd``
is in the spec-wide edits since every container that gets any GPU needs it
once. Specs are written atomically (temp file + rename: a runtime never
reads half a file) at start-up and after a topology reload.
"""
from __future__ import annotations

import json
import os
import re
import tempfile
from typing import Dict, Iterable, List, Sequence

from . import constants as C

CDI_VERSION = "0.5.0"
DEFAULT_SPEC_DIR = "/var/run/cdi"
VENDOR = C.RESOURCE_NAMESPACE
ANNOTATION_PREFIX = "cdi.k8s.io/"

DEVICE_SPECS = "device-specs"
CDI_CRI = "cdi-cri"
CDI_ANNOTATIONS = "cdi-annotations"
STRATEGIES = (DEVICE_SPECS, CDI_CRI, CDI_ANNOTATIONS)

# CDI name rules (container-device-interface, pkg/parser): a device name is
# letters, digits, '_', '-', '.', ':' and starts / ends with a letter or digit;
# a class is letters, digits, '_', '-' and starts with a letter or digit.
_NAME_RE = re.compile(r"^[A-Za-z0-9](?:[A-Za-z0-9_.:-]*[A-Za-z0-9])?$")
_CLASS_RE = re.compile(r"^[A-Za-z0-9][A-Za-z0-9_-]*$")


def parse_strategies(value: str) -> List[str]:
    """``-device_list_strategy`` value -> ordered unique strategy list."""
    out: List[str] = []
    for s in (value or DEVICE_SPECS).split(","):
        s = s.strip()
        if not s:
            continue
        if s not in STRATEGIES:
            raise ValueError(f"invalid device_list_strategy {s!r}, supported values are {', '.join(STRATEGIES)}")
        if s not in out:
            out.append(s)
    return out or [DEVICE_SPECS]


def kind(resource: str) -> str:
    if not _CLASS_RE.match(resource):
        raise ValueError(f"resource {resource!r} is not a valid CDI class")
    return f"{VENDOR}/{resource}"


def qualified_name(resource: str, dev_id: str) -> str:
    """Fully qualified CDI device name: ``amd.com/gpu=0000:23:00.0``."""
    if not _NAME_RE.match(dev_id):
        raise ValueError(f"device ID {dev_id!r} is not a valid CDI device name")
    return f"{kind(resource)}={dev_id}"


def spec_filename(resource: str) -> str:
    return f"{VENDOR}-{resource}.json"


def _node(path: str) -> dict:
    return {"path": path, "hostPath": path, "permissions": "rw"}


def build_spec(resource: str, devices: Iterable) -> dict:
    """CDI spec for one resource. ``devices`` are topology.Gpu-like objects
    (``id`` and ``dev_paths()``)."""
    devs = []
    for d in sorted(devices, key=lambda g: g.id):
        if not _NAME_RE.match(d.id):
            raise ValueError(f"device ID {d.id!r} is not a valid CDI device name")
        devs.append({"name": d.id, "containerEdits": {"deviceNodes": [_node(p) for p in d.dev_paths()]}})
    return {"cdiVersion": CDI_VERSION, "kind": kind(resource), "devices": devs,
            "containerEdits": {"deviceNodes": [_node("/dev/kfd")]}}


def write_spec(spec_dir: str, resource: str, devices: Iterable) -> str:
    """Write (atomically replace) the spec file of ``resource``; returns its path."""
    spec = build_spec(resource, devices)
    os.makedirs(spec_dir, exist_ok=True)
    path = os.path.join(spec_dir, spec_filename(resource))
    # not *.json: runtimes scan the directory for specs while we write
    fd, tmp = tempfile.mkstemp(prefix=".", suffix=".tmp", dir=spec_dir)
    try:
        with os.fdopen(fd, "w") as f:
            json.dump(spec, f, indent=1, sort_keys=True)
            f.write("\n")
        os.chmod(tmp, 0o644)
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    return path


def write_specs(spec_dir: str, members: Dict[str, Sequence], stale: Iterable[str] = ()) -> List[str]:
    """Write one spec per resource in ``members``; remove the spec files of
    ``stale`` resources (no longer advertised after a topology reload)."""
    paths = [write_spec(spec_dir, r, devs) for r, devs in sorted(members.items())]
    for r in stale:
        if r in members:
            continue
        try:
            os.unlink(os.path.join(spec_dir, spec_filename(r)))
        except OSError:
            pass
    return paths


def annotation_key(resource: str) -> str:
    # one key per plugin resource; the value lists every device of the request
    return f"{ANNOTATION_PREFIX}{VENDOR}_{resource}"


def annotation_value(resource: str, dev_ids: Sequence[str]) -> str:
    return ",".join(qualified_name(resource, i) for i in dev_ids)
