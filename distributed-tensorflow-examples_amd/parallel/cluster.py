"""Cluster spec, task identity and rendezvous.

The reference builds ``tf.train.ClusterSpec({"ps": [...], "worker": [...]})``
and starts an in-process gRPC server per task (GAN:97-106).  Here the same
``host:port`` lists define:

* a global rank per task: ps tasks first, then workers
  (``rank = task_index`` for ps, ``P + task_index`` for workers);
* the control plane: a c10d ``TCPStore`` served by ``ps:0`` on *its* port
  (``worker:0`` when there is no ps, i.e. all-reduce mode).  It carries the
  rendezvous, readiness flags and heartbeats;
* the data plane: one ``torch.distributed`` world (gloo on CPU, nccl = RCCL
  on MI355X) plus one 2-rank process group per (ps, worker) pair, so every
  worker talks to every ps over its own channel and workers never talk to
  each other (the reference's ``device_filters``, GAN:179).
"""
from __future__ import annotations

import datetime
import socket
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


def parse_hosts(s: str):
    return [h.strip() for h in s.split(",") if h.strip()] if s else []


@dataclass
class ClusterSpec:
    ps: list
    worker: list

    @classmethod
    def from_flags(cls, ps_hosts: str, worker_hosts: str) -> "ClusterSpec":
        return cls(parse_hosts(ps_hosts), parse_hosts(worker_hosts))

    def as_dict(self):
        return {"ps": list(self.ps), "worker": list(self.worker)}

    def num_tasks(self, job: str) -> int:
        return len(self.ps) if job == "ps" else len(self.worker)

    @property
    def world_size(self) -> int:
        return len(self.ps) + len(self.worker)

    def rank_of(self, job: str, task_index: int) -> int:
        if job == "ps":
            if not 0 <= task_index < len(self.ps):
                raise ValueError("ps task_index %d out of range (%d ps tasks)" % (task_index, len(self.ps)))
            return task_index
        if job == "worker":
            if not 0 <= task_index < len(self.worker):
                raise ValueError("worker task_index %d out of range (%d workers)" % (task_index, len(self.worker)))
            return len(self.ps) + task_index
        raise ValueError("job_name must be 'ps' or 'worker', got %r" % job)

    def task_of(self, rank: int):
        if rank < len(self.ps):
            return "ps", rank
        return "worker", rank - len(self.ps)

    def ps_ranks(self):
        return list(range(len(self.ps)))

    def worker_ranks(self):
        return list(range(len(self.ps), self.world_size))

    def store_address(self):
        host = self.ps[0] if self.ps else self.worker[0]
        h, _, p = host.rpartition(":")
        return (h or "127.0.0.1"), int(p)


class Server:
    """Joins the cluster: rendezvous over TCPStore, world process group, pair groups.

    Equivalent of ``tf.train.Server(cluster, job_name, task_index)``.
    ``target`` is kept for API familiarity (``grpc://host:port`` of this task).
    """

    def __init__(self, cluster: ClusterSpec, job_name: str, task_index: int, backend: str = "gloo",
                 timeout_s: float = 1800.0, device=None):
        self.cluster = cluster
        self.job_name = job_name
        self.task_index = task_index
        self.rank = cluster.rank_of(job_name, task_index)
        self.world = cluster.world_size
        self.backend = backend
        host, port = cluster.store_address()
        is_master = self.rank == (0 if cluster.ps else cluster.rank_of("worker", 0))
        timeout = datetime.timedelta(seconds=timeout_s)
        self.store = dist.TCPStore(host, port, self.world, is_master, timeout=timeout, wait_for_workers=False,
                                   use_libuv=True)
        self.target = "grpc://" + (cluster.ps + cluster.worker)[self.rank]
        if not dist.is_initialized():
            # RCCL for device tensors, gloo for the small host-side headers / control tensors
            pg_backend = "cpu:gloo,cuda:nccl" if backend == "nccl" else backend
            dist.init_process_group(pg_backend, store=dist.PrefixStore("pg", self.store), rank=self.rank,
                                    world_size=self.world, timeout=timeout)
        # which GPU every rank drives: a (ps, worker) pair on one GPU cannot share an RCCL
        # communicator (duplicate device), so that pair moves its payloads through host memory
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        ident = "%s/%s" % (socket.gethostname(), self.device)
        self.store.set("dtfe/dev/%d" % self.rank, ident)
        self._dev_ident = {r: self.store.get("dtfe/dev/%d" % r).decode() for r in range(self.world)}
        # one 2-rank group per (ps, worker) pair, created in the same order on every rank
        self.pair_groups = {}
        for p in cluster.ps_ranks():
            for w in cluster.worker_ranks():
                self.pair_groups[(p, w)] = dist.new_group([p, w])
        self.worker_group = dist.new_group(cluster.worker_ranks()) if cluster.worker else None

    def pair(self, ps_rank: int, worker_rank: int):
        return self.pair_groups[(ps_rank, worker_rank)]

    def colocated(self, a: int, b: int) -> bool:
        """True when ranks a and b drive the same GPU of the same host."""
        ia, ib = self._dev_ident[a], self._dev_ident[b]
        return ia == ib and not ia.endswith("/cpu")

    def pair_comm_device(self, ps_rank: int, worker_rank: int, device):
        """Device of the payload tensors a (ps, worker) pair exchanges: the GPU (RCCL
        over xGMI) unless the backend is gloo or both ranks share one GPU (host)."""
        device = torch.device(device)
        if self.backend != "nccl" or device.type != "cuda" or self.colocated(ps_rank, worker_rank):
            return torch.device("cpu")
        return device

    def shutdown(self):
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001 - best effort at exit
                pass


def local_cluster_flags(n_ps: int, n_workers: int, base_port: int):
    """``--ps_hosts/--worker_hosts`` strings for a single-host cluster on 127.0.0.1."""
    ps = ",".join("127.0.0.1:%d" % (base_port + i) for i in range(n_ps))
    wk = ",".join("127.0.0.1:%d" % (base_port + n_ps + i) for i in range(n_workers))
    return ps, wk


def env_flag(name: str, default: str = "") -> str:
    return os.environ.get(name, default)
