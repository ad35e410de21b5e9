"""Minimal Kubernetes API client for the node labeller (no client library).

The reference uses controller-runtime (cmd/k8s-node-labeller/main.go:529-586,
controller.go:23-58): GET the Node, strip old labels, overlay new ones, full
``Update`` of the object. Here: GET + a JSON merge patch of
``metadata.labels`` (``null`` deletes a key), which cannot lose concurrent
changes to other fields and needs no resourceVersion retry loop.

Config sources, in order: ``--kubeconfig`` (token or client-certificate auth,
embedded or file CA), ``$KUBECONFIG``, in-cluster service account
(KUBERNETES_SERVICE_HOST/PORT + /var/run/secrets/kubernetes.io/serviceaccount).

Token files (the service account's projected token, a kubeconfig
``tokenFile``) are re-read when they change: kubelet rotates projected tokens
well inside their lifetime, and client-go -- which the reference's
controller-runtime uses -- reloads them the same way. A 401 re-reads the file
at once and retries the request one time.
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import socket
import ssl
import tempfile
import urllib.error
import urllib.parse
import urllib.request
from dataclasses import dataclass
from typing import Dict, Optional


SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(f"HTTP {status}: {msg}")
        self.status = status


@dataclass
class KubeConfig:
    server: str
    token: Optional[str] = None
    ca_file: Optional[str] = None
    cert_file: Optional[str] = None
    key_file: Optional[str] = None
    insecure: bool = False
    token_file: Optional[str] = None
    _token_mtime: int = -1

    def bearer(self, force: bool = False) -> Optional[str]:
        """The current token: re-read from token_file when its mtime changed
        (or when forced after a 401); the last good value if the read fails."""
        if self.token_file:
            try:
                mt = os.stat(self.token_file).st_mtime_ns
                if force or mt != self._token_mtime:
                    with open(self.token_file) as f:
                        tok = f.read().strip()
                    if tok:
                        self.token, self._token_mtime = tok, mt
            except OSError:
                pass
        return self.token

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.server.startswith("https"):
            return None
        ctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        if self.cert_file and self.key_file:
            ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx


def _materialise(data_b64: Optional[str], suffix: str) -> Optional[str]:
    if not data_b64:
        return None
    f = tempfile.NamedTemporaryFile(prefix="labeller-", suffix=suffix, delete=False)
    f.write(base64.b64decode(data_b64))
    f.close()
    os.chmod(f.name, 0o600)
    return f.name


def load_kubeconfig(path: str) -> KubeConfig:
    import yaml  # out-of-cluster only
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    ctx_name = doc.get("current-context")
    contexts = {c["name"]: c.get("context", {}) for c in doc.get("contexts", [])}
    ctx = contexts.get(ctx_name) or (next(iter(contexts.values())) if contexts else {})
    clusters = {c["name"]: c.get("cluster", {}) for c in doc.get("clusters", [])}
    users = {u["name"]: u.get("user", {}) for u in doc.get("users", [])}
    cluster = clusters.get(ctx.get("cluster")) or (next(iter(clusters.values())) if clusters else {})
    user = users.get(ctx.get("user")) or (next(iter(users.values())) if users else {})
    base = os.path.dirname(os.path.abspath(path))

    def rel(p):
        return p if not p or os.path.isabs(p) else os.path.join(base, p)

    token = user.get("token")
    token_file = rel(user["tokenFile"]) if not token and user.get("tokenFile") else None
    cfg = KubeConfig(
        server=cluster.get("server", "").rstrip("/"),
        token=token,
        token_file=token_file,
        ca_file=rel(cluster.get("certificate-authority")) or _materialise(cluster.get("certificate-authority-data"),
                                                                          ".crt"),
        cert_file=rel(user.get("client-certificate")) or _materialise(user.get("client-certificate-data"), ".crt"),
        key_file=rel(user.get("client-key")) or _materialise(user.get("client-key-data"), ".key"),
        insecure=bool(cluster.get("insecure-skip-tls-verify")),
    )
    if token_file and not cfg.bearer():
        raise KubeError(0, f"kubeconfig tokenFile {token_file} is unreadable or empty")
    return cfg


def in_cluster_config(sa_dir: Optional[str] = None) -> KubeConfig:
    sa_dir = sa_dir or SA_DIR
    host = os.environ.get("KUBERNETES_SERVICE_HOST")
    port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
    if not host:
        raise KubeError(0, "not running in a cluster (KUBERNETES_SERVICE_HOST unset) and no kubeconfig given")
    if ":" in host and not host.startswith("["):
        host = f"[{host}]"
    ca = os.path.join(sa_dir, "ca.crt")
    cfg = KubeConfig(server=f"https://{host}:{port}", token_file=os.path.join(sa_dir, "token"),
                     ca_file=ca if os.path.exists(ca) else None)
    if not cfg.bearer():
        raise KubeError(0, f"service-account token {cfg.token_file} is unreadable or empty")
    return cfg


def get_config(kubeconfig: str = "") -> KubeConfig:
    """controller-runtime GetConfigOrDie order: flag, $KUBECONFIG, in-cluster."""
    path = kubeconfig or os.environ.get("KUBECONFIG", "")
    if path:
        return load_kubeconfig(path)
    return in_cluster_config()


class WatchStream:
    """Newline-delimited JSON watch events of one HTTP response; close() from
    another thread ends a blocked read (the socket is shut down)."""

    def __init__(self, resp):
        self._resp = resp
        self.closed = False

    def __iter__(self):
        try:
            while not self.closed:
                line = self._resp.readline()
                if not line:
                    return
                line = line.strip()
                if line:
                    yield json.loads(line)
        except (OSError, ValueError, http.client.HTTPException):
            if not self.closed:
                raise
        finally:
            self.closed = True
            try:
                self._resp.close()   # by the reading thread only: http.client is not thread-safe
            except OSError:
                pass

    def close(self) -> None:
        """Ends the stream from any thread: the socket is shut down, so a
        blocked read returns and the reading thread releases the response."""
        if self.closed:
            return
        self.closed = True
        try:
            sock = self._resp.fp.raw._sock   # http.client internals
            sock.shutdown(socket.SHUT_RDWR)
        except (AttributeError, OSError):
            pass


class KubeClient:
    def __init__(self, cfg: KubeConfig, timeout_s: float = 15.0):
        self.cfg = cfg
        self.timeout_s = timeout_s
        self._ssl = cfg.ssl_context()

    def _request(self, method: str, path: str, body: Optional[dict] = None,
                 content_type: str = "application/json", _retry: bool = True) -> dict:
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.cfg.server + path, data=data, method=method)
        req.add_header("Accept", "application/json")
        req.add_header("User-Agent", "mi355x-node-labeller")
        if data is not None:
            req.add_header("Content-Type", content_type)
        tok = self.cfg.bearer()
        if tok:
            req.add_header("Authorization", f"Bearer {tok}")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s, context=self._ssl) as resp:
                raw = resp.read()
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")[:500]
            if e.code == 401 and _retry and self.cfg.token_file and self.cfg.bearer(force=True) != tok:
                return self._request(method, path, body, content_type, _retry=False)   # rotated token
            raise KubeError(e.code, msg) from e
        except urllib.error.URLError as e:
            raise KubeError(0, str(e.reason)) from e
        return json.loads(raw) if raw else {}

    def get_node(self, name: str) -> dict:
        return self._request("GET", f"/api/v1/nodes/{name}")

    def patch_node_labels(self, name: str, labels: Dict[str, Optional[str]]) -> dict:
        return self._request("PATCH", f"/api/v1/nodes/{name}", {"metadata": {"labels": labels}},
                             "application/merge-patch+json")

    def watch_node(self, name: str, resource_version: str = "", timeout_s: int = 300) -> "WatchStream":
        """Watch one node (``GET /api/v1/nodes?watch=1&fieldSelector=metadata.name=<name>``):
        an iterator of ``{"type": ADDED|MODIFIED|DELETED|BOOKMARK|ERROR, "object": {...}}``
        until the server ends the watch (``timeoutSeconds``) or close() is called."""
        q = {"watch": "1", "fieldSelector": f"metadata.name={name}", "timeoutSeconds": str(int(timeout_s)),
             "allowWatchBookmarks": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        req = urllib.request.Request(self.cfg.server + "/api/v1/nodes?" + urllib.parse.urlencode(q), method="GET")
        req.add_header("Accept", "application/json")
        req.add_header("User-Agent", "mi355x-node-labeller")
        tok = self.cfg.bearer()
        if tok:
            req.add_header("Authorization", f"Bearer {tok}")
        try:
            resp = urllib.request.urlopen(req, timeout=timeout_s + 30, context=self._ssl)
        except urllib.error.HTTPError as e:
            raise KubeError(e.code, e.read().decode(errors="replace")[:500]) from e
        except urllib.error.URLError as e:
            raise KubeError(0, str(e.reason)) from e
        return WatchStream(resp)

    def update_node(self, name: str, node: dict) -> dict:
        """Full-object update (PUT); fails with 409 if resourceVersion is stale."""
        return self._request("PUT", f"/api/v1/nodes/{name}", node)
