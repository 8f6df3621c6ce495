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


class _Signal:
    """Device-side ordering (csrc/stream_signal.hip): ``record`` launches a one-wave kernel that
    bumps this entry's counter, ``wait`` a one-wave kernel that holds the stream until the counter
    has reached that record's count. The compute stream pays ~1.5 us per record instead of the ~7 us
    of an event with a cross-stream waiter (profiles/r4_packet_gap.txt). Two streams only: a
    re-record of the entry on either stream is ordered after every wait on the previous record.
    Off by default (PZ_DEV_SIG=1): the waiting wave holds a CU for as long as it waits, and the
    256-CU-quantised GEMMs beside it need an extra round (mlp4 1.49 vs 1.09 ms, see
    csrc/stream_signal.hip)."""
    __slots__ = ("ctr", "slot", "n", "timeout_us")

    def __init__(self, ctr: torch.Tensor, slot: int, timeout_us: float):
        self.ctr, self.slot, self.n, self.timeout_us = ctr, slot, 0, timeout_us

    def record(self, stream) -> None:
        self.n += 1
        with torch.cuda.stream(stream):
            torch.ops.pz.signal_set(self.ctr, self.slot)

    def wait(self, stream) -> None:
        with torch.cuda.stream(stream):
            torch.ops.pz.signal_wait(self.ctr, self.slot, self.n, self.timeout_us)


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
        # PZ_DEV_SIG=1: device-side counters instead of events for the ordering ring (A/B)
        self.signals = os.environ.get("PZ_DEV_SIG", "0") == "1" and not self.fenced
        self._ctr = None
        if self.signals:
            self._ctr = torch.zeros(ring * 32, dtype=torch.int32, device=torch.device("cuda", self.dev))
            # a waiter gives up after 5 s and records it (timeouts()): the grid always drains
            self._ring = [_Signal(self._ctr, i, 5e6) for i in range(ring)]
        else:
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

    def timeouts(self) -> int:
        """Signal waits that gave up (read after a synchronize; 0 with events)."""
        if self._ctr is None:
            return 0
        return int(self._ctr.view(-1, 32)[:, 1].sum().item())

    def close(self) -> None:
        self.release()
        for ev in self._ring:
            if isinstance(ev, _Native):
                torch.ops.pz.event_destroy(ev.h)
        self._ring = []

    def __del__(self):  # (a trainer dropped without close(); nothing to do at interpreter exit)
        try:
            if self._ring or self._stamps:
                torch.cuda.synchronize(self.dev)
                self.close()
        except Exception:
            pass
