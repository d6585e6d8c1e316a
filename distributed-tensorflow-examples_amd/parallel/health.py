"""Liveness: TCPStore heartbeats (SURVEY §5.3 "add a TCPStore heartbeat with timeouts").

The reference has none - a crashed worker never sends its done signal and the
ps waits forever (C07).  With ``--heartbeat_secs > 0`` every task publishes
``dtfe/hb/<job>/<task>`` (wall-clock seconds) from a daemon thread; the ps
counts a worker whose beats stopped for ``--heartbeat_timeout`` seconds as
gone (``ps %d: worker %d lost``) so it can still quit, and workers fail fast
when a ps they need stops beating.  Default off: the reference semantics.
"""
from __future__ import annotations

import os
import sys
import threading
import time


def hb_key(job: str, task: int) -> str:
    return "dtfe/hb/%s/%d" % (job, task)


class Heartbeat:
    def __init__(self, store, job: str, task: int, interval: float):
        self.store, self.key, self.interval = store, hb_key(job, task), interval
        self._stop = threading.Event()
        self._t = None
        if interval > 0:
            self.beat()
            self._t = threading.Thread(target=self._run, daemon=True, name="heartbeat")
            self._t.start()

    def beat(self):
        self.store.set(self.key, "%.3f" % time.time())

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self.beat()
            except Exception:  # noqa: BLE001 - store gone: the job is ending
                return

    def stop(self):
        self._stop.set()


def last_beat(store, job: str, task: int):
    """Seconds since the task's last heartbeat, or None if it never beat."""
    key = hb_key(job, task)
    try:
        if not store.check([key]):
            return None
        return time.time() - float(store.get(key).decode())
    except Exception:  # noqa: BLE001
        return None


class Watchdog:
    """Tracks which peers stopped beating for longer than ``timeout`` (after having beaten)."""

    def __init__(self, store, peers, timeout: float):
        self.store, self.peers, self.timeout = store, list(peers), timeout
        self.lost = set()

    def poll(self):
        newly = []
        for job, task in self.peers:
            if (job, task) in self.lost:
                continue
            age = last_beat(self.store, job, task)
            if age is not None and age > self.timeout:
                self.lost.add((job, task))
                newly.append((job, task, age))
        return newly


class CommWatchdog:
    """Failure detection for the data-parallel collectives ("in sync / all-reduce
    modes a failed rank aborts the job; restart resumes from the checkpoint").

    The gradient all-reduce is a node of the replayed step graph: when a peer dies, the survivors'
    host threads block in the device sync of the next step forever (RCCL has no timeout; the IPC
    kernel gives up after its barrier timeout but the next replay waits again).  This daemon thread
    needs neither the device nor the dead peer: every ``interval`` seconds it reads the peers'
    TCPStore heartbeats (``Heartbeat``) and RCCL's asynchronous error code
    (``RoutedComm.abort`` / ``RcclComm.status``, host-only).  A peer silent for ``timeout`` seconds,
    an unreachable store (its host, rank 0, is gone) or an RCCL error -> it logs the cause, aborts
    the communicators (ncclCommAbort releases the blocked collectives) and ends the process with
    ``exit_code`` (``os._exit``: the main thread may be stuck inside a HIP call)."""

    def __init__(self, store, job: str, rank: int, world: int, comm=None, interval: float = 1.0,
                 timeout: float = 30.0, log=print, exit_fn=None, exit_code: int = 3):
        self.store, self.job, self.rank, self.world = store, job, rank, world
        self.comm, self.interval, self.timeout, self.log = comm, interval, timeout, log
        self.exit_fn = exit_fn or (lambda code: os._exit(code))
        self.exit_code = exit_code
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="comm-watchdog")
        self._t.start()

    def check(self):
        """One poll; returns the failure description, or None while healthy."""
        if self.comm is not None:
            for c in getattr(self.comm, "comms", [self.comm]):
                st = c.status() if hasattr(c, "status") and hasattr(c, "abort") else 0
                if st:
                    return "collective engine error %d (%s)" % (st, type(c).__name__)
        if self.store is None:
            return None
        now = time.time()
        for r in range(self.world):
            if r == self.rank:
                continue
            key = hb_key(self.job, r)
            try:
                if not self.store.check([key]):
                    continue  # never beat yet (still starting)
                age = now - float(self.store.get(key).decode())
            except Exception as e:  # noqa: BLE001 - the store's host (rank 0) is gone
                return "control store unreachable (%s)" % (type(e).__name__,)
            if age > self.timeout:
                return "%s %d silent for %.1f s" % (self.job, r, age)
        return None

    def _run(self):
        while not self._stop.wait(self.interval):
            why = self.check()
            if why is None:
                continue
            if self._stop.is_set():
                return
            self.log("%s %d: %s - aborting the collectives and leaving (the job restarts from the last "
                     "checkpoint)" % (self.job, self.rank, why))
            try:
                sys.stdout.flush()
                if self.comm is not None and hasattr(self.comm, "abort"):
                    self.comm.abort()
            finally:
                self.exit_fn(self.exit_code)
            return

    def stop(self):
        self._stop.set()
