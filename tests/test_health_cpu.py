"""Failure handling of the data-parallel collectives: RoutedComm.check_health on a
fake engine error, and the CommWatchdog thread (heartbeats in a real TCPStore, fake RCCL status)."""
import socket
import threading
import time

import pytest
import torch.distributed as dist

from dtfe.parallel import comm as commmod
from dtfe.parallel.health import BeatTracker, CommWatchdog, Heartbeat, Watchdog, hb_key


class FakeEngine:
    def __init__(self, status=0):
        self._status = status
        self.aborted = False
        self.world = 2

    def status(self):
        return self._status

    def abort(self):
        self.aborted = True

    def close(self):
        pass


def test_check_health_raises_on_engine_error(monkeypatch):
    rc = commmod.RoutedComm(FakeEngine(0))
    monkeypatch.setattr(commmod, "_agree", lambda x, group, device: x)   # one process: agreement = own value
    rc.check_health()                                                    # healthy
    rc.default._status = 5                                               # e.g. ncclRemoteError surfaced async
    with pytest.raises(RuntimeError, match="all-reduce engine failure"):
        rc.check_health()
    rc.abort()
    assert rc.default.aborted


def _store():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return dist.TCPStore("127.0.0.1", port, 1, True, wait_for_workers=False)


def test_watchdog_aborts_when_a_peer_goes_silent():
    store = _store()
    hb0 = Heartbeat(store, "worker", 0, 0.1)
    hb1 = Heartbeat(store, "worker", 1, 0.1)
    eng = FakeEngine(0)
    exited = threading.Event()
    codes = []
    wd = CommWatchdog(store, "worker", 0, 2, comm=commmod.RoutedComm(eng), interval=0.1, timeout=0.6,
                      log=lambda m: None, exit_fn=lambda c: (codes.append(c), exited.set()))
    time.sleep(1.0)
    assert not exited.is_set()          # both beating: healthy
    hb1.stop()                          # worker 1 dies (no more beats)
    assert exited.wait(5.0)
    assert codes == [3] and eng.aborted
    wd.stop()
    hb0.stop()


def test_watchdog_aborts_on_rccl_async_error():
    store = _store()
    eng = FakeEngine(0)
    codes = []
    done = threading.Event()
    wd = CommWatchdog(store, "worker", 0, 1, comm=commmod.RoutedComm(eng), interval=0.05, timeout=10,
                      log=lambda m: None, exit_fn=lambda c: (codes.append(c), done.set()))
    time.sleep(0.3)
    assert not done.is_set()
    eng._status = 6
    assert done.wait(5.0) and eng.aborted
    wd.stop()


def test_watchdog_aborts_when_a_peer_never_beats():
    """A peer that died before its heartbeat thread started (comm setup, first capture) counts as
    silent once the timeout has passed since the watchdog started."""
    store = _store()
    hb0 = Heartbeat(store, "worker", 0, 0.1)
    codes = []
    done = threading.Event()
    wd = CommWatchdog(store, "worker", 0, 2, comm=None, interval=0.1, timeout=0.6, log=lambda m: None,
                      exit_fn=lambda c: (codes.append(c), done.set()))
    assert done.wait(5.0) and codes == [3]
    wd.stop()
    hb0.stop()


def test_beat_ages_use_the_local_clock():
    """A peer whose wall clock is far behind (or ahead) of ours is not silent while its beat
    counter advances: ages come from this process's monotonic clock."""
    store = _store()
    tr = BeatTracker(store)
    age, beaten = tr.age("worker", 1)
    assert not beaten and age < 1.0
    for n in range(1, 4):
        store.set(hb_key("worker", 1), "%d %.3f" % (n, time.time() - 3600.0))   # an hour of clock skew
        age, beaten = tr.age("worker", 1)
        assert beaten and age < 0.5
        time.sleep(0.05)
    time.sleep(0.3)
    age, _ = tr.age("worker", 1)     # no new beat: silence grows on our clock
    assert 0.25 < age < 5.0
    # the ps-side tracker ignores workers that never started (they may still join)
    wd = Watchdog(store, [("worker", 2)], timeout=0.1)
    time.sleep(0.2)
    assert wd.poll() == []


def test_leave_watchdog_counter_survives_store_reuse():
    """train._leave_watchdog on a store reused by a second run: rank 0 waits for ITS run's peers
    (the never-reset counter already holds the first run's tickets)."""
    import threading
    import time

    import torch.distributed as dist

    from dtfe.train import _leave_watchdog

    store = dist.HashStore()
    for r in (1, 0):  # run 1
        _leave_watchdog(store, r, 2, 5.0)
    # run 2: rank 0 arrives first and must wait for rank 1
    t = threading.Thread(target=lambda: (time.sleep(0.5), _leave_watchdog(store, 1, 2, 5.0)))
    t0 = time.time()
    t.start()
    _leave_watchdog(store, 0, 2, 5.0)
    waited = time.time() - t0
    t.join()
    assert 0.4 < waited < 4.0, waited
    assert store.add("dtfe/hb/watchdogs_stopped", 0) == 4
