"""RCCL collective check for the GPUs a pod was given: one process per GPU,
``torch.distributed`` over RCCL (backend ``"nccl"`` is RCCL on ROCm), xGMI
between the GPUs when the placement kept them in one hive.

For each collective and message size it verifies the result once (exact
small-integer data) and then times ``iters`` back-to-back calls, reporting
rccl-tests style algorithm and bus bandwidth (the slowest rank's time):

    algbw = bytes / t
    busbw = algbw * f(n),  f = 2(n-1)/n all-reduce, (n-1)/n all-gather / reduce-scatter / all-to-all

``bytes`` is the per-rank buffer the collective reduces or exchanges (the full
output for all-gather, the full input for reduce-scatter). Bus bandwidth is
comparable across n and against the fabric bound of ``parallel/fabric.py``.

Used three ways:
* ``bench.py`` at N > 1 runs it on the N ranks after the timed admissions and
  prints it beside the fabric report of the allocated set;
* inside a pod (``example/rccl/allreduce-8gpu.yaml``):
  ``torchrun --nproc-per-node 8 -m rocm_k8s_device_plugin_amd.parallel.collectives``;
* on the CPU with gloo (tests): same code path, no GPU.

The reference has no data-plane code at all; this is the
workload-side evidence for its one performance claim, "XGMI connectivity
offers better performance than PCIE" (docs/user-guide/resource-allocation.md:14).
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional, Sequence

BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
}
DEFAULT_OPS = ("all_reduce", "all_gather", "reduce_scatter", "all_to_all")


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def _sync(torch, device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class _Op:
    """Buffers and the call for one (collective, size) on this rank."""

    def __init__(self, torch, dist, op: str, nbytes: int, dtype, device, group):
        self.torch, self.dist, self.op, self.group = torch, dist, op, group
        self.n = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        es = torch.empty((), dtype=dtype).element_size()
        # element count divisible by n so every chunked collective is well formed
        count = max(self.n, (nbytes // es) // self.n * self.n)
        self.nbytes = count * es
        self.chunk = count // self.n
        mk = lambda k: torch.empty(k, dtype=dtype, device=device)  # noqa: E731
        if op == "all_reduce":
            self.x = mk(count)
        elif op == "all_gather":
            self.x, self.y = mk(self.chunk), mk(count)
        elif op == "reduce_scatter":
            self.x, self.y = mk(count), mk(self.chunk)
        elif op == "all_to_all":
            self.x, self.y = mk(count), mk(count)
        else:
            raise ValueError(f"unknown collective {op!r}")

    def call(self) -> None:
        d, g = self.dist, self.group
        if self.op == "all_reduce":
            d.all_reduce(self.x, group=g)
        elif self.op == "all_gather":
            d.all_gather_into_tensor(self.y, self.x, group=g)
        elif self.op == "reduce_scatter":
            d.reduce_scatter_tensor(self.y, self.x, group=g)
        else:
            d.all_to_all_single(self.y, self.x, group=g)

    def verify(self) -> bool:
        """One call on exact small-integer data; True if this rank's result is right."""
        t, n, r, c = self.torch, self.n, self.rank, self.chunk
        if self.op == "all_reduce":
            self.x.fill_(r + 1)
            self.call()
            return bool((self.x == n * (n + 1) // 2).all().item())
        if self.op == "all_gather":
            self.x.fill_(r)
            self.call()
            want = t.arange(n, device=self.y.device).repeat_interleave(c).to(self.y.dtype)
            return bool(t.equal(self.y, want))
        if self.op == "reduce_scatter":
            self.x.fill_(r + 1)
            self.call()
            return bool((self.y == n * (n + 1) // 2).all().item())
        # all_to_all: rank r sends chunk j = r*n + j to rank j, so it receives j*n + r from rank j
        self.x.copy_((r * n + t.arange(n, device=self.x.device)).repeat_interleave(c).to(self.x.dtype))
        self.call()
        want = (t.arange(n, device=self.y.device) * n + r).repeat_interleave(c).to(self.y.dtype)
        return bool(t.equal(self.y, want))


def measure(op: str, nbytes: int, iters: int = 10, warmup: int = 3, dtype=None, device=None,
            group=None) -> dict:
    """Verify and time one collective on every rank of ``group``; collective call."""
    import torch
    import torch.distributed as dist

    dtype = dtype or torch.bfloat16
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    o = _Op(torch, dist, op, nbytes, dtype, device, group)
    n = o.n
    ok = o.verify()
    for _ in range(warmup):
        o.call()
    _sync(torch, device)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        o.call()
    _sync(torch, device)
    dt = (time.perf_counter() - t0) / max(1, iters)
    # slowest rank's time and every rank's verdict
    agg = torch.tensor([dt, 0.0 if ok else 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(agg, op=dist.ReduceOp.MAX, group=group)
    dt, bad = float(agg[0].item()), bool(agg[1].item())
    algbw = o.nbytes / dt / 1e9
    return {"op": op, "bytes": o.nbytes, "dtype": str(dtype).replace("torch.", ""), "ranks": n,
            "time_us": round(dt * 1e6, 2), "algbw_gbs": round(algbw, 4),
            "busbw_gbs": round(algbw * BUS_FACTOR[op](n), 4), "ok": not bad}


def run(sizes: Sequence[int], ops: Sequence[str] = DEFAULT_OPS, iters: int = 10, warmup: int = 3, dtype=None,
        group=None) -> List[dict]:
    """Every (op, size); a collective the backend lacks (gloo has no
    reduce-scatter) is reported as unsupported instead of failing the run."""
    import torch.distributed as dist

    out: List[dict] = []
    for op in ops:
        for s in sizes:
            try:
                out.append(measure(op, s, iters=iters, warmup=warmup, dtype=dtype, group=group))
            except (RuntimeError, NotImplementedError, ValueError) as e:  # backend lacks the collective
                msg = str(e).splitlines()[0][:160] if str(e) else type(e).__name__
                out.append({"op": op, "bytes": s, "ranks": dist.get_world_size(group), "ok": None,
                            "unsupported": msg})
                break
    return out


def summary(rows: Sequence[dict]) -> Dict[str, object]:
    """Largest-size bus bandwidth per op plus the overall verdict (bench.py extra)."""
    best: Dict[str, dict] = {}
    for r in rows:
        if r.get("unsupported"):
            continue
        if r["op"] not in best or r["bytes"] > best[r["op"]]["bytes"]:
            best[r["op"]] = r
    return {"ok": all(r.get("ok") is not False for r in rows),
            "busbw_gbs": {op: r["busbw_gbs"] for op, r in best.items()},
            "bytes": {op: r["bytes"] for op, r in best.items()},
            "rows": list(rows)}


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--sizes", default="1M,16M,256M", help="per-rank bytes, comma separated (K/M/G suffixes)")
    ap.add_argument("--ops", default=",".join(DEFAULT_OPS))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--backend", default="", help="default: nccl (RCCL) with GPUs, else gloo")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cuda = torch.cuda.is_available()
    backend = a.backend or ("nccl" if cuda else "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if cuda:
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    try:
        rows = run([parse_size(s) for s in a.sizes.split(",") if s], [o for o in a.ops.split(",") if o],
                   iters=a.iters, warmup=a.warmup, dtype=getattr(torch, a.dtype))
        if dist.get_rank() == 0:
            for r in rows:
                print(json.dumps(r), flush=True)
        ok = all(r.get("ok") is not False for r in rows)
    finally:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
