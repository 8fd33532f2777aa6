"""Bounded waits for one-process-per-GPU runs (bench.py at N > 1).

A rank that never delivers its share -- a stalled RCCL send/recv group, a
crashed peer, a gloo gather one rank never joins -- would otherwise leave the
others blocked in torch.cuda.synchronize(), a gloo collective or a stream
wait forever, and an 8-GPU job would end at its outer time limit having
written nothing.  The reference's tile farm-out has no such step (its
goroutines share one process, renderer.go:398-436); this is the guard for
the build's gather.

One daemon thread per process watches a deadline that `guard()` sets before
a blocking call and clears after it (setting it costs two attribute writes,
so guarding the timed region adds nothing measurable).  When a deadline
passes, the thread prints the rank, the phase, its details (step, launch,
partition) on stderr as one line plus JSON, and ends the process with
`os._exit(code)`: no new program is started, no GPU call is made from the
watchdog thread, and the blocked call is simply abandoned.
"""
import json
import os
import sys
import threading
import time
from contextlib import contextmanager

EXIT_CODE = 3  # the process's exit status when the watchdog fires


class Watchdog:
    def __init__(self, seconds, rank, exit_code=EXIT_CODE, poll=0.25, stream=None):
        self.seconds = float(seconds)
        self.rank = rank
        self.exit_code = exit_code
        self.poll = poll
        self.stream = stream or sys.stderr
        self._deadline = None  # (monotonic deadline, phase, info) of the guarded wait, or None
        self._thread = None
        if self.seconds > 0:
            self._thread = threading.Thread(target=self._run, name="rtgo-watchdog", daemon=True)
            self._thread.start()

    @contextmanager
    def guard(self, phase, **info):
        """Bound the block's blocking calls to `seconds` (<= 0: unbounded)."""
        if self._thread is None:
            yield
            return
        prev = self._deadline
        self._deadline = (time.monotonic() + self.seconds, phase, info)
        try:
            yield
        finally:
            self._deadline = prev

    def _run(self):
        while True:
            time.sleep(self.poll)
            d = self._deadline
            if d is None or time.monotonic() < d[0]:
                continue
            _, phase, info = d
            rec = {"watchdog": phase, "rank": self.rank, "seconds": self.seconds, **info}
            try:
                self.stream.write(f"rank {self.rank}: watchdog: {phase} did not complete within {self.seconds:g} s "
                                  f"(step {info.get('step')}, partition {info.get('partition')}); exiting with "
                                  f"status {self.exit_code}: {json.dumps(rec, default=str)}\n")
                self.stream.flush()
            finally:
                os._exit(self.exit_code)


def host_gather(dist, host, rank, world):
    """gloo gather of rank shares (equal-size host tensors) to rank 0: the
    transport of bench.py --host-gather.  Returns the list on rank 0."""
    import torch

    parts = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
    dist.gather(host, parts, dst=0)
    return parts
