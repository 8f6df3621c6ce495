"""Cross-stream ordering events and step timestamps for the fused trainer (csrc/stream_events.cpp).

``torch.cuda.Event`` records with a SYSTEM-scope fence: every XCD's L2 written back and
invalidated each time, ~7 us of idle compute stream per record / wait in the r4 step trace
(profiles/r4_step_timeline_mlp4.txt) plus cold caches for whatever runs next, on either stream.
Ordering two streams of one device needs a device-scope release only, and the per-step timestamps
read back after a synchronize need no fence at all. Inside hipGraph capture the torch events are
kept (capture records them as graph dependencies).

(Measured, not kept: the producing kernel's last workgroup storing a flag that the other stream
waits for with hipStreamWaitValue32 — no packet on the producing stream, and the lab's producer idle
fell from 5-9 to ~1 us — but ROCm 7.2 serves that wait with a one-workgroup spin kernel
(__amd_rocclr_streamOpsWait) that holds a CU for as long as it waits, so every 512-tile GEMM of the
step ran a straggler round: mlp4 1.61 vs 1.11 ms, profiles/r5_stream_sig_lab.txt.)
"""
from __future__ import annotations

import torch


class _Native:
    """A device-scope ordering event. ``pending``: recorded, and no wait enqueued on that record
    yet — the ring never re-records such an entry (its waiter would order against the wrong
    stream)."""
    __slots__ = ("h", "dev", "pending")

    def __init__(self, h: int, dev: int):
        self.h, self.dev, self.pending = h, dev, False

    def record(self, stream) -> None:
        with torch.cuda.stream(stream):
            torch.ops.pz.event_record(self.h, self.dev)
        self.pending = True

    def wait(self, stream) -> None:
        with torch.cuda.stream(stream):
            torch.ops.pz.event_wait(self.h, self.dev)
        self.pending = False


class _Torch:
    __slots__ = ("ev",)

    def __init__(self):
        self.ev = torch.cuda.Event()

    def record(self, stream) -> None:
        self.ev.record(stream)

    def wait(self, stream) -> None:
        stream.wait_event(self.ev)


class StreamEvents:
    """A ring of device-scope ordering events, re-recorded round robin, and fence-free timestamp
    events, one per step until :meth:`release`. An entry whose record still has no waiter when the
    ring comes back to it is replaced by a fresh event (the ring grows instead of silently
    re-ordering a waiter against the other stream: a schedule with more records per step than the
    ring, e.g. many GEMM layers, stays correct)."""

    def __init__(self, device: torch.device, ring: int = 64):
        self.dev = device.index if device.index is not None else torch.cuda.current_device()
        self._ring = [_Native(torch.ops.pz.event_create(self.dev, 0), self.dev) for _ in range(ring)]
        self._retired: list[int] = []  # replaced entries, destroyed by release() / close()
        self._next = 0
        self._stamps: list[int] = []

    def sync(self, capture: bool = False):
        """An ordering event: ``.record(stream)`` then ``.wait(other_stream)``."""
        if capture:
            return _Torch()
        ev = self._ring[self._next]
        if ev.pending:  # still awaited: never re-record it
            self._retired.append(ev.h)
            ev = self._ring[self._next] = _Native(torch.ops.pz.event_create(self.dev, 0), self.dev)
        self._next = (self._next + 1) % len(self._ring)
        return ev

    def stamp(self, stream) -> int:
        """Record a timestamp on ``stream``; returns its handle for :meth:`elapsed`."""
        h = torch.ops.pz.event_create(self.dev, 1)
        self._stamps.append(h)
        with torch.cuda.stream(stream):
            torch.ops.pz.event_record(h, self.dev)
        return h

    @staticmethod
    def elapsed(start: int, end: int) -> float:
        return float(torch.ops.pz.event_elapsed(start, end))

    def release(self, keep: int | None = None) -> None:
        """Destroy the timestamps recorded so far and the replaced ring entries (after a
        synchronize), except ``keep``."""
        for h in self._stamps:
            if h != keep:
                torch.ops.pz.event_destroy(h)
        self._stamps = [keep] if keep is not None else []
        for h in self._retired:
            torch.ops.pz.event_destroy(h)
        self._retired = []

    def close(self) -> None:
        """Destroy every event (after a synchronize: nothing may still be recorded or awaited)."""
        self.release()
        for ev in self._ring:
            torch.ops.pz.event_destroy(ev.h)
        self._ring = []

    def abandon(self) -> None:
        """Drop the events WITHOUT synchronizing or destroying them (a failed run whose streams may
        never drain: a device synchronize could hang on a stuck collective). The handles leak."""
        self._ring, self._retired, self._stamps = [], [], []

    # No __del__: a synchronize from the garbage collector could land inside another trainer's
    # hipGraph capture and invalidate it. A trainer dropped without close() leaks its handles.
