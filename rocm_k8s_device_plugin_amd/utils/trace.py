"""Chrome-trace (chrome://tracing / Perfetto) span recorder.

Off by default; ``-trace_file=<path>`` turns it on. Spans cover the admission
path (RPC -> allocator) and the health path (sweep -> per-device probe), so a
slow Allocate or a stuck probe shows up on one timeline. Events are kept in a
bounded ring and written as a JSON array on flush / shutdown.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import deque
from typing import Any, Deque, Dict, Optional


class Tracer:
    def __init__(self, path: Optional[str] = None, max_events: int = 200000):
        self.path = path
        self.enabled = bool(path)
        self._events: Deque[Dict[str, Any]] = deque(maxlen=max_events)
        self._lock = threading.Lock()
        self._pid = os.getpid()

    def configure(self, path: Optional[str]) -> None:
        self.path = path
        self.enabled = bool(path)

    @contextlib.contextmanager
    def span(self, name: str, cat: str = "plugin", **args: Any):
        if not self.enabled:
            yield
            return
        t0 = time.perf_counter_ns()
        try:
            yield
        finally:
            dur = time.perf_counter_ns() - t0
            ev = {"name": name, "cat": cat, "ph": "X", "ts": t0 / 1e3, "dur": dur / 1e3, "pid": self._pid,
                  "tid": threading.get_ident() & 0xFFFF, "args": {k: str(v) for k, v in args.items()}}
            with self._lock:
                self._events.append(ev)

    def complete(self, name: str, cat: str, t0_ns: int, dur_ns: int, **args: Any) -> None:
        """A span recorded elsewhere (the native gRPC server): CLOCK_MONOTONIC ns,
        the same clock as perf_counter_ns on Linux."""
        if not self.enabled:
            return
        ev = {"name": name, "cat": cat, "ph": "X", "ts": t0_ns / 1e3, "dur": dur_ns / 1e3, "pid": self._pid,
              "tid": 0, "args": {k: str(v) for k, v in args.items()}}
        with self._lock:
            self._events.append(ev)

    def instant(self, name: str, cat: str = "plugin", **args: Any) -> None:
        if not self.enabled:
            return
        ev = {"name": name, "cat": cat, "ph": "i", "s": "p", "ts": time.perf_counter_ns() / 1e3, "pid": self._pid,
              "tid": threading.get_ident() & 0xFFFF, "args": {k: str(v) for k, v in args.items()}}
        with self._lock:
            self._events.append(ev)

    def events(self):
        with self._lock:
            return list(self._events)

    def flush(self) -> None:
        if not self.enabled or not self.path:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"traceEvents": self.events(), "displayTimeUnit": "ms"}, f)
        os.replace(tmp, self.path)


TRACER = Tracer()
