"""Node-label reconciler.

Reference: reconcileNodeLabels (cmd/k8s-node-labeller/controller.go:23-58)
driven by a Create-only predicate on the node named ``$DS_NODE_NAME``
(main.go:551-577) — labels are computed once at startup and applied once.

Here the desired labels are recomputed on every pass (hardware state such as
partition mode can change under a running DaemonSet) and re-asserted every
``resync_s`` seconds, so labels removed or edited by someone else come back
(SURVEY Appendix B #11). Each pass: GET node -> diff against
(labels - known AMD keys) + desired -> merge PATCH only if something changed.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

from ..utils import log
from .kube import KubeClient, KubeError
from .labels import remove_old_node_labels

_log = log.get("labeller")


def label_patch(current: Dict[str, str], desired: Dict[str, str]) -> Dict[str, Optional[str]]:
    """Merge-patch body turning `current` into remove_old(current) + desired."""
    target = remove_old_node_labels(current)
    target.update(desired)
    patch: Dict[str, Optional[str]] = {}
    for k in current:
        if k not in target:
            patch[k] = None
    for k, v in target.items():
        if current.get(k) != v:
            patch[k] = v
    return patch


@dataclass
class ReconcileStats:
    passes: int = 0
    patches: int = 0
    updates: int = 0
    errors: int = 0
    last_error: str = ""
    last_patch: Dict[str, Optional[str]] = field(default_factory=dict)


class NodeLabeller:
    def __init__(self, client: KubeClient, node_name: str, generate: Callable[[], Dict[str, str]],
                 resync_s: float = 300.0, retry_s: float = 5.0):
        self.client = client
        self.node = node_name
        self.generate = generate
        self.resync_s = resync_s
        self.retry_s = retry_s
        self.stats = ReconcileStats()
        self._stop = threading.Event()

    def reconcile_once(self) -> bool:
        """Returns True on success (whether or not a patch was needed)."""
        self.stats.passes += 1
        try:
            desired = self.generate()
            node = self.client.get_node(self.node)
            current = (node.get("metadata") or {}).get("labels") or {}
            patch = label_patch(current, desired)
            if patch:
                try:
                    self.client.patch_node_labels(self.node, patch)
                except KubeError as e:
                    if e.status != 403:
                        raise
                    # RBAC from the upstream manifests grants "update" but not
                    # "patch": fall back to the reference's GET + Update
                    self._update_with_retry(desired)
                self.stats.patches += 1
                self.stats.last_patch = patch
                log.info_fields(_log, "node labels updated", node=self.node, changed=len(patch))
            return True
        except (KubeError, OSError) as e:
            self.stats.errors += 1
            self.stats.last_error = str(e)
            _log.error("reconcile of node %s failed: %s", self.node, e)
            return False

    def _update_with_retry(self, desired: Dict[str, str], attempts: int = 5) -> None:
        for i in range(attempts):
            node = self.client.get_node(self.node)
            meta = node.setdefault("metadata", {})
            labels = remove_old_node_labels(meta.get("labels") or {})
            labels.update(desired)
            meta["labels"] = labels
            try:
                self.client.update_node(self.node, node)
                self.stats.updates += 1
                return
            except KubeError as e:
                if e.status != 409 or i == attempts - 1:
                    raise

    def stop(self) -> None:
        self._stop.set()

    def run(self, once: bool = False) -> None:
        while not self._stop.is_set():
            ok = self.reconcile_once()
            if once and ok:
                return
            wait = self.resync_s if ok else self.retry_s
            if wait <= 0:
                if ok:
                    return
                wait = self.retry_s
            self._stop.wait(wait)
