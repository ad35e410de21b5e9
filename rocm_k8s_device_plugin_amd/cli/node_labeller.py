"""The Python oracle labeller's command line: ``python -m
rocm_k8s_device_plugin_amd.cli.node_labeller -dry_run -vram ...`` prints the
labels labeller/labels.py generates for this node, as JSON.

Not a product: ``k8s-node-labeller`` is the native labeller everywhere (the
images, ``scripts/``, the installed console script), and only it talks to the
apiserver. This CLI takes the reference's label flags (one boolean per kind,
cmd/k8s-node-labeller/main.go:518-520, and ``-driver_type``, :516) so the
native labeller's ``-dry_run`` output can be compared with it byte for byte.
"""
from __future__ import annotations

import json
import sys
from typing import List, Optional

from .. import __version__
from .. import constants as C
from ..labeller.labels import EXTRA_LABELS, generate_labels
from ..utils import flags, log


def build_parser() -> flags.GoFlagParser:
    p = flags.GoFlagParser(prog="k8s-node-labeller (Python oracle)",
                           description=f"AMD GPU Node Labeller label oracle (MI355X-native) version {__version__}")
    p.add_str("driver_type", "", "Driver type to use: container, vf-passthrough, or pf-passthrough")
    for k in C.SUPPORTED_LABELS + EXTRA_LABELS:
        p.add_bool(k, False, f"Set this to label nodes with {k} properties", dest=f"label_{k}")
    flags.add_glog_flags(p)
    p.add_bool("dry_run", False, "print the generated labels as JSON and exit (the only mode of this oracle)")
    p.add_str("sysfs_root", "/sys", "sysfs mount to read")
    p.add_str("dev_root", "/dev", "device node directory")
    p.add_str("log_format", "glog", "glog | json")
    return p


def enabled_labels(ns) -> dict:
    return {k: bool(getattr(ns, f"label_{k}")) for k in C.SUPPORTED_LABELS + EXTRA_LABELS}


def main(argv: Optional[List[str]] = None) -> int:
    ns = build_parser().parse_args(argv)
    try:
        logger = log.setup_from_flags(ns, program="k8s-node-labeller")
    except ValueError as e:
        print(f"invalid logging flags: {e}", file=sys.stderr)
        return 1
    if ns.driver_type not in ("",) + C.DRIVER_TYPES:
        logger.error("invalid driver_type %s", ns.driver_type)
        return 1
    if not ns.dry_run:
        logger.error("the Python labeller only prints labels (-dry_run); ./k8s-node-labeller (the native "
                     "labeller) labels the node")
        return 1
    print(json.dumps(generate_labels(enabled_labels(ns), ns.driver_type, ns.sysfs_root, ns.dev_root),
                     indent=1, sort_keys=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())
