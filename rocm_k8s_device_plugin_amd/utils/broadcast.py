"""Generation-counted asyncio broadcast.

The reference drives every plugin's ListAndWatch from ONE unbuffered Go
channel (internal/pkg/manager/manager.go:34,98), so under the ``mixed``
strategy each heartbeat wakes exactly one resource.
A broadcast wakes every waiter once per ``fire()``, and a waiter that was
busy while several fires happened still sees the newest generation.
"""
from __future__ import annotations

import asyncio
from typing import Optional


class Broadcast:
    def __init__(self) -> None:
        self.generation = 0
        self.closed = False
        self._event: Optional[asyncio.Event] = None

    def fire(self) -> None:
        self.generation += 1
        ev, self._event = self._event, None
        if ev is not None:
            ev.set()

    def close(self) -> None:
        self.closed = True
        self.fire()

    async def wait(self, last_generation: int, timeout: Optional[float] = None) -> int:
        """Block until generation != last_generation (or closed / timeout)."""
        while self.generation == last_generation and not self.closed:
            if self._event is None:
                self._event = asyncio.Event()
            ev = self._event
            if timeout is None:
                await ev.wait()
            else:
                try:
                    await asyncio.wait_for(ev.wait(), timeout)
                except asyncio.TimeoutError:
                    break
        return self.generation
