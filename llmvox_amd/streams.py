"""Side streams that really run beside another stream.

A process gets GPU_MAX_HW_QUEUES hardware queues per device (4 by default on this ROCm); HIP streams
beyond that share them, and two streams on one hardware queue execute in submission order. torch hands
out streams from a pool round robin, so which pool stream shares the decode stream's queue depends on
how many streams the process created before (a process group's internal streams shift it). A codec
stream on the decode stream's queue silently serialises the codec behind the decode steps: measured,
the idle first chunk then takes 3.6 instead of 1.4 ms (the 10-frame decode waits for the next 30 AR
steps), and the headline's overlap is lost. ``side_stream`` returns a pool stream checked to run
beside the given ones.
"""
from __future__ import annotations

import time
from typing import Iterable, Optional

import torch

_SPIN_CYCLES = 30_000_000  # torch.cuda._sleep: ~15 ms of a spinning wave at the shader clock


def runs_beside(s: "torch.cuda.Stream", other: "torch.cuda.Stream", wait_s: float = 0.004) -> bool:
    """True when work on ``s`` completes while ``other`` is busy: a spin kernel is queued on ``other``
    and an event right after on ``s``; the host polls the event for ``wait_s``. Synchronises both."""
    torch.cuda.synchronize(s.device)
    busy, mark = torch.cuda.Event(), torch.cuda.Event()
    with torch.cuda.stream(other):
        torch.cuda._sleep(_SPIN_CYCLES)
        busy.record(other)
    with torch.cuda.stream(s):
        mark.record(s)
    t_end = time.perf_counter() + wait_s
    ok = False
    while time.perf_counter() < t_end:
        if mark.query():
            ok = not busy.query()
            break
        time.sleep(50e-6)
    torch.cuda.synchronize(s.device)
    return ok


def side_stream(device, beside: Iterable[Optional["torch.cuda.Stream"]], tries: int = 16,
                priority: int = 0) -> "torch.cuda.Stream":
    """A stream of ``device`` that runs concurrently with every stream in ``beside`` (None entries:
    the device's current stream). Tries up to ``tries`` pool streams; returns the last one tried if
    none qualifies (a process whose queues are all shared gets no overlap, as before)."""
    dev = torch.device(device)
    others = [torch.cuda.current_stream(dev) if b is None else b for b in beside]
    s = None
    for _ in range(max(1, tries)):
        s = torch.cuda.Stream(device=dev, priority=priority)
        if all(s != o and runs_beside(s, o) for o in others):
            return s
    return s
