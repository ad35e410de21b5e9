"""A tiny fake kube-apiserver for labeller tests: GET / PATCH (JSON merge
patch) / PUT of ``/api/v1/nodes/<name>`` over plain HTTP, bearer-token check,
request log. Runs in a background thread (stdlib only)."""
from __future__ import annotations

import copy
import json
import threading
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
    def __init__(self, token: Optional[str] = "test-token"):
        self.token = token
        self.nodes: Dict[str, dict] = {}
        self.requests: List[Tuple[str, str, Optional[dict]]] = []
        self.fail_next: int = 0          # respond 500 to the next N requests
        self.forbid: set = set()         # HTTP methods answered with 403 (RBAC without that verb)
        self._lock = threading.Lock()
        srv = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

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
                    rv = int(node["metadata"].get("resourceVersion", "1")) + 1
                    node["metadata"]["resourceVersion"] = str(rv)
                    srv.nodes[name] = node
                    return self._send(200, node)

            def do_GET(self):  # noqa: N802
                self._handle("GET")

            def do_PATCH(self):  # noqa: N802
                self._handle("PATCH")

            def do_PUT(self):  # noqa: N802
                self._handle("PUT")

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def add_node(self, name: str, labels: Optional[Dict[str, str]] = None) -> None:
        self.nodes[name] = {"apiVersion": "v1", "kind": "Node",
                            "metadata": {"name": name, "labels": dict(labels or {}), "resourceVersion": "1"}}

    def labels(self, name: str) -> Dict[str, str]:
        return dict(self.nodes[name]["metadata"].get("labels") or {})

    def start(self) -> "FakeApiServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
