"""In-process metrics: latency histograms + counters, Prometheus text format.

The reference exposes no metrics (the labeller even disables
controller-runtime's server, cmd/k8s-node-labeller/main.go:529-532). This
registry backs the optional ``/metrics`` endpoint and the benchmark's
per-RPC p50/p99 numbers.
"""
from __future__ import annotations

import asyncio
import bisect
from collections import deque
import threading
from typing import Deque, Dict, List, Optional, Tuple

_BUCKETS_MS = [0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 25, 50, 100, 250, 500, 1000, 2500, 5000, 10000]


class Histogram:
    # quantile() looks at the most recent samples only: a daemon that runs for
    # months must not keep every observation (the buckets keep the totals)
    def __init__(self, name: str, help: str, keep_samples: int = 4096):
        self.name, self.help = name, help
        self.counts = [0] * (len(_BUCKETS_MS) + 1)
        self.sum = 0.0
        self.n = 0
        self.samples: Deque[float] = deque(maxlen=keep_samples)
        self.keep = keep_samples
        self._lock = threading.Lock()

    def observe(self, ms: float) -> None:
        with self._lock:
            self.counts[bisect.bisect_left(_BUCKETS_MS, ms)] += 1
            self.sum += ms
            self.n += 1
            self.samples.append(ms)

    def quantile(self, q: float) -> float:
        with self._lock:
            s = sorted(self.samples)
        if not s:
            return float("nan")
        i = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
        return s[i]


class Registry:
    def __init__(self) -> None:
        self.hist: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], Histogram] = {}
        self.counters: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], float] = {}
        self.gauges: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], float] = {}
        self.help: Dict[str, str] = {}
        self._lock = threading.Lock()

    def histogram(self, name: str, help: str = "", **labels: str) -> Histogram:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            h = self.hist.get(key)
            if h is None:
                h = self.hist[key] = Histogram(name, help)
                self.help.setdefault(name, help)
        return h

    def inc(self, name: str, v: float = 1.0, help: str = "", **labels: str) -> None:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            self.counters[key] = self.counters.get(key, 0.0) + v
            self.help.setdefault(name, help)

    def set(self, name: str, v: float, help: str = "", **labels: str) -> None:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            self.gauges[key] = v
            self.help.setdefault(name, help)

    @staticmethod
    def _lbl(labels: Tuple[Tuple[str, str], ...], extra: Optional[Tuple[str, str]] = None) -> str:
        items = list(labels) + ([extra] if extra else [])
        if not items:
            return ""
        return "{" + ",".join(f'{k}="{v}"' for k, v in items) + "}"

    def render(self) -> str:
        lines: List[str] = []
        done = set()
        for (name, labels), v in sorted(self.counters.items()):
            if name not in done:
                lines += [f"# HELP {name} {self.help.get(name, '')}", f"# TYPE {name} counter"]
                done.add(name)
            lines.append(f"{name}{self._lbl(labels)} {v}")
        for (name, labels), v in sorted(self.gauges.items()):
            if name not in done:
                lines += [f"# HELP {name} {self.help.get(name, '')}", f"# TYPE {name} gauge"]
                done.add(name)
            lines.append(f"{name}{self._lbl(labels)} {v}")
        for (name, labels), h in sorted(self.hist.items(), key=lambda kv: kv[0]):
            if name not in done:
                lines += [f"# HELP {name} {self.help.get(name, '')}", f"# TYPE {name} histogram"]
                done.add(name)
            cum = 0
            for b, c in zip(_BUCKETS_MS + [float("inf")], h.counts):
                cum += c
                le = "+Inf" if b == float("inf") else f"{b / 1000:g}"
                lines.append(f"{name}_bucket{self._lbl(labels, ('le', le))} {cum}")
            lines.append(f"{name}_sum{self._lbl(labels)} {h.sum / 1000:g}")
            lines.append(f"{name}_count{self._lbl(labels)} {h.n}")
        return "\n".join(lines) + "\n"


REGISTRY = Registry()


async def serve_metrics(port: int, host: str = "0.0.0.0", registry: Registry = REGISTRY):
    """Minimal HTTP/1.0 server for GET /metrics (no threads, no deps)."""

    async def handle(reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        try:
            req = await asyncio.wait_for(reader.readline(), 5)
            while (await asyncio.wait_for(reader.readline(), 5)) not in (b"\r\n", b"\n", b""):
                pass
            path = req.split()[1].decode() if len(req.split()) > 1 else "/"
            if path.startswith("/metrics"):
                body, status = registry.render().encode(), "200 OK"
            elif path.startswith("/healthz"):
                body, status = b"ok\n", "200 OK"
            else:
                body, status = b"not found\n", "404 Not Found"
            writer.write(f"HTTP/1.0 {status}\r\nContent-Type: text/plain; version=0.0.4\r\n"
                         f"Content-Length: {len(body)}\r\n\r\n".encode() + body)
            await writer.drain()
        except (asyncio.TimeoutError, ConnectionError, IndexError):
            pass
        finally:
            writer.close()

    return await asyncio.start_server(handle, host, port)
