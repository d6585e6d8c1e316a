"""Liveness: TCPStore heartbeats (SURVEY §5.3 "add a TCPStore heartbeat with timeouts").

The reference has none - a crashed worker never sends its done signal and the
ps waits forever (C07).  With ``--heartbeat_secs > 0`` every task publishes
``dtfe/hb/<job>/<task>`` (wall-clock seconds) from a daemon thread; the ps
counts a worker whose beats stopped for ``--heartbeat_timeout`` seconds as
gone (``ps %d: worker %d lost``) so it can still quit, and workers fail fast
when a ps they need stops beating.  Default off: the reference semantics.
"""
from __future__ import annotations

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
