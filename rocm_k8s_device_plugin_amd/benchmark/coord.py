"""Rank coordination (gloo) and the deadline over the secondary measurements
of the admission benchmark (bench.py)."""
from __future__ import annotations

import os
import sys


class Dist:
    """Rank coordination for the bench. The measured thing is a kubelet node
    admitting pods, and a kubelet node has no resident GPU process: the bench
    and plugin processes must not hold a GPU context, kfd queues or an RCCL
    communicator while containers initialise their GPUs. So:

    * step barriers and object exchange run over gloo (CPU, TCP) under torchrun;
      at world = 1 nothing is initialised and torch is not even imported;
    * ``sync()`` synchronises the GPU only if this process already has a HIP
      context (it never creates one); the containers' GPU work is complete by
      construction when a step ends (ready = every MFMA tile verified);
    * RCCL is created only after the timed loop, for the collectives extra
      (``rccl_group()``).
    """

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.launcher = "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or self.world > 1 else "single-process"
        self.torch = None
        self.dist = None
        self.cuda = False   # this process drives a GPU (only ever for the RCCL extra)
        if self.world > 1:
            import torch
            import torch.distributed as dist
            self.torch, self.dist = torch, dist
            dist.init_process_group("gloo")

    def sync(self):
        if self.world > 1:
            self.dist.barrier()
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def rccl_group(self):
        """After the timed loop: (group, on_gpu) for the collectives extra, one
        rank per GPU over RCCL when GPUs are visible, else the gloo group."""
        torch, dist = self.torch, self.dist
        if not torch.cuda.is_available():
            return None, False
        torch.cuda.set_device(self.local_rank)
        self.cuda = True
        return dist.new_group(backend="nccl", device_id=torch.device("cuda", self.local_rank)), True

    def bcast(self, obj):
        if self.world == 1:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def max(self, x: float) -> float:
        return max(self.gather(x))

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


class ExtrasGuard:
    """Bounds the secondary measurements that follow the timed loop.

    Everything after the timed loop (comparison admissions, RCCL collectives,
    the xGMI peer probe, the throughput check) is context, not the metric, and
    some of it runs code that can hang on a sick node (an RCCL communicator, a
    DMA that never completes). The headline is complete when the timed loop
    ends, so a timer armed there bounds the rest: when it fires, or when a
    stage raises (its own failure, or a peer rank that already left), rank 0 prints
    the headline line with ``extra.extras_incomplete`` naming the stage that
    was running, and every rank leaves with status 0 (``os._exit``: a thread
    stuck in a collective cannot be joined). Exactly one line is printed
    whichever path gets there first."""

    def __init__(self, rank: int, deadline_s: float):
        import threading
        self.rank, self.deadline_s = rank, deadline_s
        self.stage = "start"
        self.fallback = None          # rank 0: (error) -> the headline line without the unfinished extras
        self._lock = threading.Lock()
        self._printed = False
        self._abandoning = False
        self._written = threading.Event()   # the printed line (and --json-out) is complete
        self._timer = None
        self._plugins = []            # plugin daemons to SIGKILL when the timer fires (no orphans)
        self.tmp = None               # rank 0's scratch directory (sockets, logs, fixture tree)
        if deadline_s > 0:
            # ranks > 0 leave a little later, so rank 0's line is out first
            self._timer = threading.Timer(deadline_s + (0 if rank == 0 else 5.0), self._fire)
            self._timer.daemon = True
            self._timer.start()

    def enter(self, stage: str) -> None:
        self.stage = stage

    def kill_on_fire(self, plugin) -> None:
        self._plugins.append(plugin)

    def emit(self, line: str, json_out: str = "") -> bool:
        """Print the JSON line (and write it to ``json_out``) unless the other
        path already has; True if written here. Whoever wins writes both, so
        stdout and --json-out always carry the same line."""
        with self._lock:
            if self._printed:
                return False
            self._printed = True
        try:
            data = memoryview((line + "\n").encode())
            while data:   # a blocking pipe can still take a large line in parts
                data = data[os.write(1, data):]
            if json_out:
                with open(json_out, "w") as f:
                    f.write(line + "\n")
        finally:
            self._written.set()
        return True

    def _fire(self) -> None:
        self.abandon(None)

    def abandon(self, error) -> None:
        """Leave now: rank 0 prints the headline line (unless it already has)
        with the unfinished stage, plugin daemons are killed, exit status 0.
        ``error`` is None when the deadline passed, else why the stage failed.
        The first caller leaves; a second one (the main thread failing because
        the timer already killed a plugin daemon) waits for that exit."""
        import time
        with self._lock:
            first = not self._abandoning
            self._abandoning = True
        if not first:
            while True:
                time.sleep(3600)
        why = (f"exceeded --extras-deadline {self.deadline_s:g}s" if error is None else f"failed: {error}")
        msg = f"bench: secondary measurements {why} in stage '{self.stage}'"
        if self.rank == 0 and self.fallback is not None:
            with self._lock:
                printed = self._printed
            if printed:
                # the full line is out or being written by the main thread: let it finish
                self._written.wait(10.0)
                msg = f"bench: {why} in stage '{self.stage}' after the headline line was written"
            else:
                try:
                    self.emit(*self.fallback(error))
                except Exception as e:  # noqa: BLE001
                    msg += f"; headline line failed: {type(e).__name__}: {e}"
        try:
            try:
                sys.stdout.flush()
                os.write(2, (msg + "\n").encode())
            except OSError:
                pass
            for pl in self._plugins:
                proc = getattr(pl, "proc", None)
                if proc is not None and proc.poll() is None:
                    try:
                        proc.kill()
                    except OSError:
                        pass
            if self.tmp:
                import shutil
                shutil.rmtree(self.tmp, ignore_errors=True)
        finally:
            os._exit(0)

    def cancel(self) -> None:
        if self._timer is not None:
            self._timer.cancel()
