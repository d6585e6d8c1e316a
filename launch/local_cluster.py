#!/usr/bin/env python
"""Single-host cluster launcher: the analog of ``tf.test.create_local_cluster``
and of the K8s pod-per-task deployment the reference implies (README.md:2).

Spawns one process per task with the reference command line
(``--ps_hosts/--worker_hosts/--job_name/--task_index``) on 127.0.0.1 ports,
streams their output with a ``[ps0]``/``[worker1]`` prefix and returns when
every process has exited (non-zero exit if any task failed).

    python launch/local_cluster.py --model gan --ps 1 --workers 2 -- --num_steps=200
    python launch/local_cluster.py --model lstm --ps 2 --workers 3 --gpus 1 -- --device=cuda
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = {m: os.path.join(ROOT, "examples", m, "distributed_%s.py" % m) for m in ("gan", "encoder", "lstm",
                                                                                   "softmax", "cnn")}
SCRIPTS.update({a: os.path.join(ROOT, "examples", "resnet", "distributed_%s.py" % a) for a in ("resnet20", "resnet50")})


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def task_argv(model, ps_hosts, worker_hosts, job, idx, extra):
    return [sys.executable, SCRIPTS[model], "--ps_hosts=" + ps_hosts, "--worker_hosts=" + worker_hosts,
            "--job_name=" + job, "--task_index=%d" % idx] + list(extra)


def _port_clash(codes, outputs):
    """A task failed because another process took one of the probed ports between free_ports()
    and the task's bind (parallel test runs)."""
    return any(c != 0 for c in codes.values()) and any(
        "address already in use" in l.lower() or "eaddrinuse" in l.lower() for ls in outputs.values() for l in ls)


def launch(model, n_ps, n_workers, extra=(), env=None, timeout=None, stream=True, gpus=0, attempts=3):
    for attempt in range(attempts):
        res = _launch_once(model, n_ps, n_workers, extra, env, timeout, stream, gpus)
        if not _port_clash(res[0], res[1]) or attempt == attempts - 1:
            return res
        print("local_cluster: port clash, relaunching on fresh ports", file=sys.stderr, flush=True)


def _launch_once(model, n_ps, n_workers, extra, env, timeout, stream, gpus):
    ports = free_ports(n_ps + n_workers)
    ps_hosts = ",".join("127.0.0.1:%d" % p for p in ports[:n_ps])
    worker_hosts = ",".join("127.0.0.1:%d" % p for p in ports[n_ps:])
    procs = []
    outputs = {}
    base_env = dict(os.environ if env is None else env)
    base_env.setdefault("PYTHONUNBUFFERED", "1")
    tasks = [("ps", i) for i in range(n_ps)] + [("worker", i) for i in range(n_workers)]
    for job, i in tasks:
        e = dict(base_env)
        if gpus:
            e["LOCAL_RANK"] = str(i % gpus if job == "worker" else 0)
        argv = task_argv(model, ps_hosts, worker_hosts, job, i, extra)
        p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e, cwd=ROOT)
        procs.append(((job, i), p))
        outputs[(job, i)] = []

    def pump(key, p):
        for line in p.stdout:
            outputs[key].append(line.rstrip("\n"))
            if stream:
                print("[%s%d] %s" % (key[0], key[1], line.rstrip("\n")), flush=True)

    threads = [threading.Thread(target=pump, args=(k, p), daemon=True) for k, p in procs]
    for t in threads:
        t.start()
    codes = {}
    try:
        for k, p in procs:
            codes[k] = p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        for _, p in procs:
            if p.poll() is None:
                p.kill()
        raise
    finally:
        for t in threads:
            t.join(timeout=5)
    return codes, outputs, (ps_hosts, worker_hosts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=sorted(SCRIPTS), default="softmax")
    ap.add_argument("--ps", type=int, default=1)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=0, help="spread workers over this many local GPUs (LOCAL_RANK)")
    ap.add_argument("extra", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    extra = [x for x in a.extra if x != "--"]
    if not any(x.startswith("--workers") for x in extra):
        extra.append("--workers=%d" % a.workers)
    codes, _, _ = launch(a.model, a.ps, a.workers, extra, gpus=a.gpus)
    bad = {k: c for k, c in codes.items() if c != 0}
    if bad:
        print("failed tasks:", bad, file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
