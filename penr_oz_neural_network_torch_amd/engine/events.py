"""Cross-stream ordering events and step timestamps for the fused trainer (csrc/stream_events.cpp).

``torch.cuda.Event`` records with a SYSTEM-scope fence: every XCD's L2 written back and
invalidated each time, ~7 us of idle compute stream per record / wait in the r4 step trace
(profiles/r4_step_timeline_mlp4.txt) plus cold caches for whatever runs next, on either stream.
Ordering two streams of one device needs a device-scope release only, and the per-step timestamps
read back after a synchronize need no fence at all. Inside hipGraph capture the torch events are
kept (capture records them as graph dependencies).
"""
from __future__ import annotations

import os

import torch


class _Native:
    __slots__ = ("h", "dev")

    def __init__(self, h: int, dev: int):
        self.h, self.dev = h, dev

    def record(self, stream) -> None:
        with torch.cuda.stream(stream):
            torch.ops.pz.event_record(self.h, self.dev)

    def wait(self, stream) -> None:
        with torch.cuda.stream(stream):
            torch.ops.pz.event_wait(self.h, self.dev)


class _Torch:
    __slots__ = ("ev",)

    def __init__(self, timing: bool = False):
        self.ev = torch.cuda.Event(enable_timing=timing)

    def record(self, stream) -> None:
        self.ev.record(stream)

    def wait(self, stream) -> None:
        stream.wait_event(self.ev)


class StreamEvents:
    """A ring of device-scope ordering events (re-recorded round robin: every wait on a record is
    enqueued before the ring comes back to it — far fewer than ``ring`` events per step) and
    fence-free timestamp events, one per step until :meth:`release`."""

    def __init__(self, device: torch.device, ring: int = 64):
        self.dev = device.index if device.index is not None else torch.cuda.current_device()
        # PZ_TORCH_EVENTS=1: the system-fenced events of before (A/B)
        self.fenced = os.environ.get("PZ_TORCH_EVENTS", "0") == "1"
        self._ring = [_Native(torch.ops.pz.event_create(self.dev, 0), self.dev) for _ in range(ring)]
        self._next = 0
        self._stamps: list[int] = []

    def sync(self, capture: bool = False):
        """An ordering event: ``.record(stream)`` then ``.wait(other_stream)``."""
        if capture or self.fenced:
            return _Torch()
        ev = self._ring[self._next]
        self._next = (self._next + 1) % len(self._ring)
        return ev

    def stamp(self, stream) -> int:
        """Record a timestamp on ``stream``; returns its handle for :meth:`elapsed`."""
        h = torch.ops.pz.event_create(self.dev, 2 if self.fenced else 1)
        self._stamps.append(h)
        with torch.cuda.stream(stream):
            torch.ops.pz.event_record(h, self.dev)
        return h

    @staticmethod
    def elapsed(start: int, end: int) -> float:
        return float(torch.ops.pz.event_elapsed(start, end))

    def release(self, keep: int | None = None) -> None:
        """Destroy the timestamps recorded so far (after a synchronize), except ``keep``."""
        for h in self._stamps:
            if h != keep:
                torch.ops.pz.event_destroy(h)
        self._stamps = [keep] if keep is not None else []

    def close(self) -> None:
        self.release()
        for ev in self._ring:
            torch.ops.pz.event_destroy(ev.h)
        self._ring = []

    def __del__(self):  # (a trainer dropped without close(); nothing to do at interpreter exit)
        try:
            if self._ring or self._stamps:
                torch.cuda.synchronize(self.dev)
                self.close()
        except Exception:
            pass
