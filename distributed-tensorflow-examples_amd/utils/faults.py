"""Fault-injection hooks (test T2) driven by the ``DTFE_FAULT`` environment variable.

    DTFE_FAULT="crash@worker:1:step=5;slow@worker:0:ms=20;hang@ps:0:step=3:secs=5"

* ``crash@<job>:<task>:step=N``  the task exits immediately (exit code 17, no cleanup, no done
                                 signal) once its global step reaches N - a killed pod;
* ``slow@<job>:<task>:ms=M``      every step of the task sleeps M ms - a straggler;
* ``hang@<job>:<task>:step=N:secs=S`` the task stalls S seconds once at step N.

Steps are the global step the task observes (workers: after each push; ps: after each
applied update).  Unset: no-op.
"""
from __future__ import annotations

import os
import sys
import time


def _parse(spec: str):
    rules = []
    for part in filter(None, (p.strip() for p in spec.split(";"))):
        kind, _, rest = part.partition("@")
        fields = rest.split(":")
        if len(fields) < 2:
            raise ValueError("DTFE_FAULT: expected kind@job:task[:k=v...], got %r" % part)
        kv = dict(f.split("=", 1) for f in fields[2:])
        rules.append(dict(kind=kind, job=fields[0], task=int(fields[1]), **{k: float(v) for k, v in kv.items()}))
    return rules


class FaultInjector:
    def __init__(self, job: str, task: int, spec: str | None = None, log=print):
        spec = os.environ.get("DTFE_FAULT", "") if spec is None else spec
        self.rules = [r for r in _parse(spec) if r["job"] == job and r["task"] == task]
        self.job, self.task, self.log = job, task, log
        self._hung = False

    def __bool__(self):
        return bool(self.rules)

    def step(self, gs: int):
        for r in self.rules:
            if r["kind"] == "crash" and gs >= r.get("step", 0):
                self.log("fault injection: %s %d crashes at step %d" % (self.job, self.task, gs))
                sys.stdout.flush()
                os._exit(17)
            elif r["kind"] == "slow":
                time.sleep(r.get("ms", 0) / 1000.0)
            elif r["kind"] == "hang" and not self._hung and gs >= r.get("step", 0):
                self._hung = True
                self.log("fault injection: %s %d hangs %.1fs at step %d" % (self.job, self.task, r.get("secs", 0), gs))
                time.sleep(r.get("secs", 0))
