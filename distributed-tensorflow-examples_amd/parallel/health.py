"""Liveness: TCPStore heartbeats (SURVEY §5.3 "add a TCPStore heartbeat with timeouts").

The reference has none - a crashed worker never sends its done signal and the
ps waits forever (C07).  With ``--heartbeat_secs > 0`` every task publishes
``dtfe/hb/<job>/<task>`` from a daemon thread; the ps counts a worker whose beats
stopped for ``--heartbeat_timeout`` seconds as gone (``ps %d: worker %d lost``)
so it can still quit, and in --mode=allreduce (where the heartbeat is on by
default, utils/flags.py resolve_mode) a rank whose peer goes silent aborts the
collectives and exits.  Off by default in --mode=ps: the reference semantics.

A beat is a counter (``"<n> <wall time>"``; the wall time is for people reading
the store).  Readers never compare clocks across hosts: ``BeatTracker`` notes
on its OWN monotonic clock when each peer's counter last changed, so clock
skew between hosts is not silence.
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
        self.n = 0
        self._stop = threading.Event()
        self._t = None
        if interval > 0:
            self.beat()
            self._t = threading.Thread(target=self._run, daemon=True, name="heartbeat")
            self._t.start()

    def beat(self):
        self.n += 1
        self.store.set(self.key, "%d %.3f" % (self.n, time.time()))

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self.beat()
            except Exception:  # noqa: BLE001 - store gone: the job is ending
                return

    def stop(self):
        self._stop.set()


class BeatTracker:
    """Seconds of silence per peer, measured on this process's monotonic clock: the time since
    the peer's beat counter last changed (as seen by ``age`` calls), or - a peer that has not
    beaten yet - since the tracker was created.  ``age`` raises if the store is unreachable."""

    def __init__(self, store):
        self.store = store
        self.t0 = time.monotonic()
        self._seen = {}   # key -> (last value, monotonic time it was first seen)

    def age(self, job: str, task: int):
        """(seconds of silence, has it ever beaten)"""
        key = hb_key(job, task)
        now = time.monotonic()
        if not self.store.check([key]):
            return now - self.t0, False
        v = self.store.get(key)
        last = self._seen.get(key)
        if last is None or last[0] != v:
            self._seen[key] = (v, now)
            return 0.0, True
        return now - last[1], True


def last_beat(store, job: str, task: int):
    """The wall-clock age of the task's last heartbeat as its writer stamped it (for logs and tests
    on one host; failure detection uses BeatTracker), or None if it never beat."""
    key = hb_key(job, task)
    try:
        if not store.check([key]):
            return None
        return time.time() - float(store.get(key).decode().split()[-1])
    except Exception:  # noqa: BLE001
        return None


class Watchdog:
    """Tracks which peers stopped beating for longer than ``timeout`` after having beaten (the ps
    side: a worker that has not started yet may still join, as in the reference)."""

    def __init__(self, store, peers, timeout: float):
        self.store, self.peers, self.timeout = store, list(peers), timeout
        self.lost = set()
        self.tracker = BeatTracker(store)

    def poll(self):
        newly = []
        for job, task in self.peers:
            if (job, task) in self.lost:
                continue
            try:
                age, beaten = self.tracker.age(job, task)
            except Exception:  # noqa: BLE001 - store going away: the job is ending
                return newly
            if beaten and age > self.timeout:
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
    TCPStore heartbeats (``Heartbeat``, ages on this process's clock: ``BeatTracker``) and RCCL's asynchronous error code
    (``RoutedComm.abort`` / ``RcclComm.status``, host-only).  A peer silent for ``timeout`` seconds
    (or that has not beaten at all ``timeout`` seconds after this watchdog started),
    an unreachable store (its host, rank 0, is gone) or an RCCL error -> it logs the cause, aborts
    the communicators (ncclCommAbort releases the blocked collectives) and ends the process with
    ``exit_code`` (``os._exit``: the main thread may be stuck inside a HIP call)."""

    def __init__(self, store, job: str, rank: int, world: int, comm=None, interval: float = 1.0,
                 timeout: float = 30.0, log=print, exit_fn=None, exit_code: int = 3):
        self.store, self.job, self.rank, self.world = store, job, rank, world
        self.comm, self.interval, self.timeout, self.log = comm, interval, timeout, log
        self.exit_fn = exit_fn or (lambda code: os._exit(code))
        self.exit_code = exit_code
        self.tracker = BeatTracker(store) if store is not None else None
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
        for r in range(self.world):
            if r == self.rank:
                continue
            try:
                age, beaten = self.tracker.age(self.job, r)
            except Exception as e:  # noqa: BLE001 - the store's host (rank 0) is gone
                return "control store unreachable (%s)" % (type(e).__name__,)
            if age > self.timeout:
                # (a peer that never beat: it died during setup or its first capture, before its
                # heartbeat thread started - the survivors' next replay would wait for it forever)
                return "%s %d silent for %.1f s%s" % (self.job, r, age, "" if beaten else " (never beat)")
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
