"""A tiny fake kube-apiserver for labeller tests: GET / PATCH (JSON merge
patch) / PUT of ``/api/v1/nodes/<name>`` and node watches
(``GET /api/v1/nodes?watch=1&fieldSelector=metadata.name=<n>``, chunked
newline-delimited JSON events, ``timeoutSeconds``, 410 ERROR events for a
resourceVersion older than ``min_rv``) over plain HTTP/1.1, bearer-token
check, request log. Runs in a background thread (stdlib only)."""
from __future__ import annotations

import copy
import json
import queue
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional, Tuple


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class FakeApiServer:
    def __init__(self, token: Optional[str] = "test-token", tls: Optional[Tuple[str, str]] = None,
                 client_ca: Optional[str] = None, host: str = "127.0.0.1", prefix: str = ""):
        """tls: (cert chain PEM, key PEM) to serve HTTPS; client_ca: also require
        a client certificate signed by this CA (kubeconfig client-certificate auth);
        host: the listen address ("::1" for an IPv6 cluster); prefix: the API is
        served below this path only (an apiserver behind a proxy, e.g.
        /k8s/clusters/c-1), which ``url`` includes."""
        self.host = host
        self.prefix = prefix.rstrip("/")
        self.host_headers: List[str] = []
        self.token = token
        self.nodes: Dict[str, dict] = {}
        self.requests: List[Tuple[str, str, Optional[dict]]] = []
        self.fail_next: int = 0          # respond 500 to the next N requests
        self.forbid: set = set()         # HTTP methods answered with 403 (RBAC without that verb)
        self.min_rv = 0                  # watches from an older resourceVersion get a 410 ERROR event
        self.watchers: List[Tuple[str, "queue.Queue"]] = []
        self.watch_starts = 0
        self.watch_max_s: Optional[float] = None   # end every watch after this long (a proxy that cuts streams)
        self._lock = threading.Lock()
        srv = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # quiet
                pass

            def _chunk(self, obj) -> None:
                # bytes: sent as they are (malformed-event tests)
                raw = obj if isinstance(obj, bytes) else (json.dumps(obj) + "\n").encode()
                self.wfile.write(f"{len(raw):x}\r\n".encode() + raw + b"\r\n")
                self.wfile.flush()

            def _watch(self, q):
                name = (q.get("fieldSelector", [""])[0].partition("metadata.name=")[2])
                rv = q.get("resourceVersion", [""])[0]
                timeout = float(q.get("timeoutSeconds", ["300"])[0])
                if srv.watch_max_s is not None:
                    timeout = min(timeout, srv.watch_max_s)
                events: "queue.Queue" = queue.Queue()
                with srv._lock:
                    node = copy.deepcopy(srv.nodes.get(name))
                    srv.watchers.append((name, events))
                    srv.watch_starts += 1
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                try:
                    if rv and int(rv) < srv.min_rv:
                        self._chunk({"type": "ERROR", "object": {"kind": "Status", "code": 410,
                                                                 "message": "too old resource version"}})
                    else:
                        if node is not None and (not rv or node["metadata"]["resourceVersion"] != rv):
                            self._chunk({"type": "ADDED" if not rv else "MODIFIED", "object": node})
                        end = time.monotonic() + timeout
                        while time.monotonic() < end:
                            try:
                                ev = events.get(timeout=min(0.05, max(0.0, end - time.monotonic())))
                            except queue.Empty:
                                continue
                            if ev is None:        # expire_watches()
                                break
                            self._chunk(ev)
                    self.wfile.write(b"0\r\n\r\n")
                    self.wfile.flush()
                except OSError:
                    pass
                finally:
                    with srv._lock:
                        srv.watchers = [w for w in srv.watchers if w[1] is not events]
                self.close_connection = True

            def _auth(self) -> bool:
                if srv.token and self.headers.get("Authorization") != f"Bearer {srv.token}":
                    self._send(401, {"kind": "Status", "message": "Unauthorized"})
                    return False
                return True

            def _send(self, code, body):
                raw = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def _node(self):
                parts = self.path.split("?")[0].strip("/").split("/")
                if len(parts) == 4 and parts[:3] == ["api", "v1", "nodes"]:
                    return parts[3]
                return None

            def _handle(self, method):
                with srv._lock:
                    srv.host_headers.append(self.headers.get("Host", ""))
                if srv.prefix:
                    if not self.path.startswith(srv.prefix + "/"):
                        return self._send(404, {"kind": "Status", "message": f"{self.path} is outside {srv.prefix}"})
                    self.path = self.path[len(srv.prefix):]
                url = urllib.parse.urlparse(self.path)
                q = urllib.parse.parse_qs(url.query)
                if method == "GET" and url.path.rstrip("/") == "/api/v1/nodes" and q.get("watch") == ["1"]:
                    with srv._lock:
                        srv.requests.append(("WATCH", self.path, None))
                    if not self._auth():
                        return
                    return self._watch(q)
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n)) if n else None
                with srv._lock:
                    srv.requests.append((method, self.path, body))
                    if srv.fail_next > 0:
                        srv.fail_next -= 1
                        return self._send(500, {"kind": "Status", "message": "injected failure"})
                if not self._auth():
                    return
                if method in srv.forbid:
                    return self._send(403, {"kind": "Status", "message": f"{method} forbidden"})
                name = self._node()
                with srv._lock:
                    node = srv.nodes.get(name) if name else None
                    if node is None:
                        return self._send(404, {"kind": "Status", "message": f"node {name} not found"})
                    if method == "GET":
                        return self._send(200, node)
                    if method == "PATCH":
                        if self.headers.get("Content-Type") != "application/merge-patch+json":
                            return self._send(415, {"message": "unsupported patch type"})
                        node = merge_patch(node, body)
                    elif method == "PUT":
                        if body["metadata"].get("resourceVersion") != node["metadata"].get("resourceVersion"):
                            return self._send(409, {"kind": "Status", "message": "conflict"})
                        node = body
                    srv._store(name, node, "MODIFIED")
                    return self._send(200, node)

            def do_GET(self):  # noqa: N802
                self._handle("GET")

            def do_PATCH(self):  # noqa: N802
                self._handle("PATCH")

            def do_PUT(self):  # noqa: N802
                self._handle("PUT")

        server_cls = ThreadingHTTPServer
        if ":" in host:
            import socket

            class _V6(ThreadingHTTPServer):
                address_family = socket.AF_INET6
            server_cls = _V6
        self.httpd = server_cls((host, 0), Handler)
        self.scheme = "http"
        if tls is not None:   # (cert chain PEM, key PEM): serve HTTPS like a real apiserver
            import ssl
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(*tls)
            if client_ca:
                ctx.verify_mode = ssl.CERT_REQUIRED
                ctx.load_verify_locations(client_ca)
            self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True)
            self.scheme = "https"
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    @property
    def url(self) -> str:
        host = f"[{self.host}]" if ":" in self.host else self.host
        return f"{self.scheme}://{host}:{self.port}{self.prefix}"

    def _store(self, name: str, node: dict, event: str) -> None:
        """(lock held) bump the resourceVersion, store, notify watchers."""
        self._rv_counter = max(getattr(self, "_rv_counter", 1), int(node["metadata"].get("resourceVersion", "1"))) + 1
        node["metadata"]["resourceVersion"] = str(self._rv_counter)
        self.nodes[name] = node
        for n, q in self.watchers:
            if n == name:
                q.put({"type": event, "object": copy.deepcopy(node)})

    def add_node(self, name: str, labels: Optional[Dict[str, str]] = None) -> None:
        with self._lock:
            self._store(name, {"apiVersion": "v1", "kind": "Node",
                               "metadata": {"name": name, "labels": dict(labels or {}), "resourceVersion": "1"}},
                        "ADDED")

    def send_raw_event(self, name: str, raw: bytes) -> None:
        """Write raw bytes into the watch streams of a node (garbage, truncated JSON)."""
        with self._lock:
            for n, q in self.watchers:
                if n == name:
                    q.put(raw)

    def set_labels(self, name: str, labels: Dict[str, str]) -> None:
        """Replace a node's labels (someone else editing the node)."""
        with self._lock:
            node = copy.deepcopy(self.nodes[name])
            node["metadata"]["labels"] = dict(labels)
            self._store(name, node, "MODIFIED")

    def delete_node(self, name: str) -> None:
        with self._lock:
            node = self.nodes.pop(name)
            for n, q in self.watchers:
                if n == name:
                    q.put({"type": "DELETED", "object": node})

    def expire_watches(self) -> None:
        """End every open watch (as the apiserver does at timeoutSeconds)."""
        with self._lock:
            for _, q in self.watchers:
                q.put(None)

    def labels(self, name: str) -> Dict[str, str]:
        return dict(self.nodes[name]["metadata"].get("labels") or {})

    def start(self) -> "FakeApiServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def tls_material(d):
    """A CA and a server certificate for 127.0.0.1 and ::1 signed by it (openssl CLI):
    (server cert, server key, CA cert) paths under directory `d`."""
    import shutil
    import subprocess
    if not shutil.which("openssl"):
        import pytest
        pytest.skip("openssl not installed")

    def run(*a):
        subprocess.run(["openssl", *a], check=True, capture_output=True, timeout=60)
    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "ca.key"), "-out", str(d / "ca.crt"),
        "-days", "2", "-subj", "/CN=test-ca")
    run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "srv.key"), "-out", str(d / "srv.csr"),
        "-subj", "/CN=kubernetes")
    (d / "ext.cnf").write_text("subjectAltName=IP:127.0.0.1,IP:::1,DNS:kubernetes.default.svc\n")
    run("x509", "-req", "-in", str(d / "srv.csr"), "-CA", str(d / "ca.crt"), "-CAkey", str(d / "ca.key"),
        "-CAcreateserial", "-out", str(d / "srv.crt"), "-days", "2", "-extfile", str(d / "ext.cnf"))
    return str(d / "srv.crt"), str(d / "srv.key"), str(d / "ca.crt")

