"""``k8s-node-labeller`` entry point.

Reference: cmd/k8s-node-labeller/main.go:507-590 — one boolean flag per
label kind (``-vram``, ``-cu-count``, ...), ``-driver_type``, ``-kubeconfig``,
node name from ``$DS_NODE_NAME``. Same flags here; additions: ``-resync``
(periodic re-assert; 0 = as the reference: at start and on Node re-creation), ``-once``, ``-dry_run`` (print
the labels as JSON and exit), ``-sysfs_root`` / ``-dev_root``, and the opt-in
extra kinds ``-gfx-target`` / ``-xgmi-hive-count`` / ``-xgmi-links-down``.
"""
from __future__ import annotations

import json
import os
import signal
import sys
from typing import List, Optional

from .. import __version__
from .. import constants as C
from ..labeller.controller import NodeLabeller
from ..labeller.kube import KubeClient, get_config
from ..labeller.labels import EXTRA_LABELS, generate_labels
from ..utils import flags, log


def build_parser() -> flags.GoFlagParser:
    p = flags.GoFlagParser(prog="k8s-node-labeller",
                           description=f"AMD GPU Node Labeller for Kubernetes (MI355X-native) version {__version__}")
    p.add_str("driver_type", "", "Driver type to use: container, vf-passthrough, or pf-passthrough")
    for k in C.SUPPORTED_LABELS + EXTRA_LABELS:
        p.add_bool(k, False, f"Set this to label nodes with {k} properties", dest=f"label_{k}")
    p.add_str("kubeconfig", "", "Paths to a kubeconfig. Only required if out-of-cluster.")
    flags.add_glog_flags(p)
    p.add_str("node_name", os.environ.get("DS_NODE_NAME", ""), "node to label (default $DS_NODE_NAME)")
    p.add_float("resync", 300.0, "seconds between label re-asserts (0 = as upstream: label at start and whenever "
                                 "the Node object is re-created, no periodic re-assert)")
    p.add_bool("watch", True, "watch the node and re-apply labels as soon as they are stripped or the node is "
                              "re-created (needs the 'watch' verb on nodes, as in the upstream ClusterRole)")
    p.add_float("topology_watch", 5.0, "seconds between checks of the GPU topology (kfd generation_id, partition "
                                       "modes); a change relabels the node at once (0 = off: next resync)")
    p.add_bool("dry_run", False, "print the generated labels as JSON and exit")
    p.add_bool("once", False, "apply the labels once and exit (e.g. from a Job instead of the DaemonSet)")
    p.add_str("sysfs_root", "/sys", "sysfs mount to read")
    p.add_str("dev_root", "/dev", "device node directory")
    p.add_str("log_format", "glog", "glog | json")
    return p


HOSTNAME_FILE = "/labeller/hostname"


def node_name_from(ns, hostname_file: str = HOSTNAME_FILE) -> str:
    """-node_name / $DS_NODE_NAME (what the reference's code reads,
    cmd/k8s-node-labeller/main.go:551), else the file its README documents
    (cmd/k8s-node-labeller/README.md:10) but the code never read."""
    if ns.node_name:
        return ns.node_name
    try:
        with open(hostname_file) as f:
            return f.read().strip()
    except OSError:
        return ""


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
    enabled = enabled_labels(ns)

    def gen():
        return generate_labels(enabled, ns.driver_type, ns.sysfs_root, ns.dev_root)

    if ns.dry_run:
        print(json.dumps(gen(), indent=1, sort_keys=True))
        return 0
    node = node_name_from(ns)
    if not node:
        logger.error("node name unknown: set DS_NODE_NAME or -node_name (or mount %s)", HOSTNAME_FILE)
        return 1
    try:
        client = KubeClient(get_config(ns.kubeconfig))
    except Exception as e:
        logger.error("unable to set up kubernetes client: %s", e)
        return 1
    from ..topology import topology_signature
    lab = NodeLabeller(client, node, gen, resync_s=ns.resync, watch=ns.watch,
                       change_source=lambda: topology_signature(ns.sysfs_root), change_interval_s=ns.topology_watch)
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, lambda *_: lab.stop())
    lab.run(once=ns.once, created_only=not ns.once and ns.resync <= 0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
