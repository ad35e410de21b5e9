"""kubelet's device-manager side as grpc-go runs it, over the frame-level peer
(testing/gopeer.py): a Registration server on ``<dir>/kubelet.sock`` that,
like kubelet, connects back to the plugin *inside* its Register handler.

kubelet's order (pkg/kubelet/cm/devicemanager/plugin/v1beta1/server.go
Register -> connectClient -> client.Connect: dial, GetDevicePluginOptions;
then ``go s.runClient`` -> ListAndWatch) means the ListAndWatch stream is
often open before the Register answer reaches the plugin. ``eager=True``
forces exactly that: the stream is opened before Register returns.
``eager=False`` opens it after the answer was sent (what testing/
fake_kubelet.py does); ``list_and_watch=False`` never opens it (a kubelet that
cannot complete calls on the plugin's transport).

The stream is read on a thread of its own: ``lists`` holds every
ListAndWatchResponse as {device id: health}.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Dict, List, Optional

from ..proto import deviceplugin as pb
from . import gopeer as gp

REGISTER = "/v1beta1.Registration/Register"
DP = "/v1beta1.DevicePlugin/"


class GoKubelet:
    def __init__(self, kdir: str, eager: bool = True, list_and_watch: bool = True,
                 config: Optional[gp.GoServerConfig] = None):
        os.makedirs(kdir, exist_ok=True)
        self.kdir = kdir
        self.eager = eager
        self.list_and_watch = list_and_watch
        self.registrations: List[object] = []
        self.lists: List[Dict[str, str]] = []
        self.stream_ended = threading.Event()
        self.errors: List[str] = []
        self._lock = threading.Lock()
        self._conn: Optional[gp.GoClientConn] = None
        self._sid = 0
        self._stop = threading.Event()
        self._reader: Optional[threading.Thread] = None
        self.srv = gp.GoServer(os.path.join(kdir, "kubelet.sock"), {REGISTER: self._register}, config)

    # Register handler (the GoServer's connection thread)
    def _register(self, msg: bytes):
        req = pb.RegisterRequest.FromString(msg)
        with self._lock:
            self.registrations.append(req)
        self._drop()
        if self.list_and_watch and self.eager:
            self._connect(req.endpoint)
        elif self.list_and_watch:
            threading.Thread(target=self._connect_later, args=(req.endpoint,), daemon=True).start()
        return 0, "", b""

    def _connect_later(self, endpoint: str) -> None:
        time.sleep(0.05)   # the Register answer is out first
        self._connect(endpoint)

    def _connect(self, endpoint: str) -> None:
        try:
            conn = gp.GoClientConn(os.path.join(self.kdir, endpoint))
            code, message, _ = conn.unary(DP + "GetDevicePluginOptions", b"", 10.0)
            if code != 0:
                raise RuntimeError(f"GetDevicePluginOptions: {code} {message}")
            sid = conn.start_call(DP + "ListAndWatch", b"")
        except Exception as e:  # noqa: BLE001 -- recorded, the test asserts on it
            self.errors.append(f"{type(e).__name__}: {e}")
            return
        self._conn, self._sid = conn, sid
        self.stream_ended.clear()
        self._stop.clear()
        self._reader = threading.Thread(target=self._read, args=(conn, sid), daemon=True)
        self._reader.start()

    def _read(self, conn: gp.GoClientConn, sid: int) -> None:
        st = conn.streams[sid]
        try:
            while not self._stop.is_set():
                conn.pump(0.1)
                while st.messages:
                    resp = pb.ListAndWatchResponse.FromString(st.messages.pop(0))
                    with self._lock:
                        self.lists.append({d.ID: d.health for d in resp.devices})
                if st.ended:
                    break
        except (EOFError, OSError):
            pass
        self.stream_ended.set()

    def _drop(self) -> None:
        """A re-registration replaces the previous endpoint (kubelet closes it)."""
        self._stop.set()
        if self._reader is not None:
            self._reader.join(timeout=5)
            self._reader = None
        if self._conn is not None:
            self._conn.close()
            self._conn = None

    def end_stream(self) -> None:
        """kubelet drops the plugin: its ListAndWatch stream is cancelled, the connection closed."""
        conn, sid = self._conn, self._sid
        if conn is not None:
            try:
                conn.cancel(sid)
            except OSError:
                pass
        self._drop()

    def updates(self) -> int:
        with self._lock:
            return len(self.lists)

    def close(self) -> None:
        self._drop()
        self.srv.close()
