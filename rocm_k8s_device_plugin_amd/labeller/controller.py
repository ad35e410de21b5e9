"""Node-label reconciler.

Reference: reconcileNodeLabels (cmd/k8s-node-labeller/controller.go:23-58)
driven by a Create-only predicate on the node named ``$DS_NODE_NAME``
(main.go:551-577) — labels are computed once at startup and applied once
(and again when the Node object is re-created).

Here the node is watched (``watch=1`` with a fieldSelector on its name,
reconnected with backoff, re-listed after 410 Gone): any event whose labels
differ from the desired ones — the node re-created, a label stripped or edited
by someone else — triggers a reconcile at once. The
desired labels are also recomputed and re-asserted every ``resync_s`` seconds
(hardware state such as partition mode can change under a running
DaemonSet). Each pass: GET node -> diff against (labels - known AMD keys) +
desired -> merge PATCH only if something changed.
"""
from __future__ import annotations

import http.client
import threading
import time
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
    watch_events: int = 0
    watch_kicks: int = 0      # events that triggered a reconcile
    watch_errors: int = 0
    watch_restarts: int = 0
    topology_changes: int = 0  # GPU topology fingerprint changes seen (each relabels at once)


class NodeLabeller:
    def __init__(self, client: KubeClient, node_name: str, generate: Callable[[], Dict[str, str]],
                 resync_s: float = 300.0, retry_s: float = 5.0, watch: bool = True, watch_timeout_s: int = 300,
                 watch_backoff_max_s: float = 30.0, change_source: Optional[Callable[[], object]] = None,
                 change_interval_s: float = 5.0):
        self.client = client
        self.node = node_name
        self.generate = generate
        self.resync_s = resync_s
        self.retry_s = retry_s
        self.watch = watch
        self.watch_timeout_s = watch_timeout_s
        self.watch_backoff_max_s = watch_backoff_max_s
        self.stats = ReconcileStats()
        self._stop = threading.Event()
        self._kick = threading.Event()
        self._desired: Optional[Dict[str, str]] = None
        self._rv = ""
        self._stream = None
        self._watch_thread: Optional[threading.Thread] = None
        # GPU topology fingerprint (kfd generation_id + partition modes): a
        # change -- a partition switch -- relabels at once instead of at the
        # next resync
        self.change_source = change_source
        self.change_interval_s = change_interval_s
        self._change_thread: Optional[threading.Thread] = None
        self._created_only = False

    def reconcile_once(self) -> bool:
        """Returns True on success (whether or not a patch was needed)."""
        self.stats.passes += 1
        try:
            desired = self.generate()
            self._desired = desired
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

    # ------------------------------------------------------------ watch
    def _needs_reconcile(self, node: dict) -> bool:
        if self._desired is None:
            return True
        labels = (node.get("metadata") or {}).get("labels") or {}
        return bool(label_patch(labels, self._desired))

    def _watch_loop(self) -> None:
        backoff = 0.2
        while not self._stop.is_set():
            try:
                stream = self.client.watch_node(self.node, self._rv, timeout_s=self.watch_timeout_s)
                self._stream = stream
                if self._stop.is_set():
                    stream.close()
                    return
                self.stats.watch_restarts += 1
                opened = time.monotonic()
                for ev in stream:
                    self.stats.watch_events += 1
                    typ, obj = ev.get("type"), ev.get("object") or {}
                    if typ == "ERROR":
                        if obj.get("code") == 410:      # resourceVersion too old: re-list
                            self._rv = ""
                            self._kick.set()
                        break
                    rv = (obj.get("metadata") or {}).get("resourceVersion")
                    if rv:
                        self._rv = rv
                    kinds = ("ADDED",) if self._created_only else ("ADDED", "MODIFIED")
                    if typ in kinds and self._needs_reconcile(obj):
                        self.stats.watch_kicks += 1
                        self._kick.set()
                # a stream that lived its timeout reconnects at once; one the
                # server ends right away (proxy, overloaded apiserver) backs off
                # like an error instead of spinning on reconnects
                if time.monotonic() - opened >= 1.0:
                    backoff = 0.2
                elif not self._stop.is_set():
                    self._stop.wait(backoff)
                    backoff = min(backoff * 2, self.watch_backoff_max_s)
            except (KubeError, OSError, ValueError, http.client.HTTPException) as e:
                if self._stop.is_set():
                    return
                if isinstance(e, KubeError) and e.status == 410:
                    self._rv = ""
                self.stats.watch_errors += 1
                _log.warning("watch of node %s failed (%s); retrying in %.1fs", self.node, e, backoff)
                self._stop.wait(backoff)
                backoff = min(backoff * 2, self.watch_backoff_max_s)
            finally:
                self._stream = None

    def stop(self) -> None:
        self._stop.set()
        self._kick.set()
        s = self._stream
        if s is not None:
            s.close()
        if self._watch_thread is not None and self._watch_thread is not threading.current_thread():
            self._watch_thread.join(5)

    def _change_loop(self) -> None:
        try:
            last = self.change_source()
        except Exception:  # noqa: BLE001
            last = None
        seen = last
        while not self._stop.wait(self.change_interval_s):
            try:
                cur = self.change_source()
            except Exception:  # noqa: BLE001
                continue
            # act once the new fingerprint has held for one interval: a switch
            # passes through states with devices half gone
            if cur != last and cur == seen:
                last = cur
                self.stats.topology_changes += 1
                _log.info("GPU topology changed (partition switch?): relabelling node %s", self.node)
                self._kick.set()
            seen = cur

    def run(self, once: bool = False, created_only: bool = False) -> None:
        """once: apply the labels and return. created_only: the reference's
        controller (cmd/k8s-node-labeller/main.go:553-586) -- label at start,
        then again only when the Node object is (re-)created (a watch ADDED
        event whose labels differ); no periodic re-assert, never exits."""
        self._created_only = created_only
        if self.watch and not once and self._watch_thread is None:
            self._watch_thread = threading.Thread(target=self._watch_loop, name="node-watch", daemon=True)
            self._watch_thread.start()
        if self.change_source is not None and self.change_interval_s > 0 and not once and \
                self._change_thread is None:
            self._change_thread = threading.Thread(target=self._change_loop, name="topology-watch", daemon=True)
            self._change_thread.start()
        while not self._stop.is_set():
            self._kick.clear()
            ok = self.reconcile_once()
            if once and ok:
                return
            wait = self.resync_s if ok else self.retry_s
            if created_only and ok:
                wait = 3600.0   # until a watch event kicks
            if wait <= 0:
                if ok and not self.watch:
                    return
                wait = self.retry_s if not ok else 3600.0
            self._kick.wait(wait)
