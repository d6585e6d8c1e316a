"""Bucketed all-reduce with backward-progress launching (parallel/allreduce.py) on a 2-rank gloo group,
and the ResNet-20 example in all-reduce mode (2 workers, CPU)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dtfe  # noqa: F401
from dtfe.parallel.allreduce import BucketAllReduce

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "launch"))
import local_cluster  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1000
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    buckets = [(600, 1000), (250, 600), (0, 250)]  # back to front, as _buckets builds them
    ar = BucketAllReduce(g, buckets)
    launched = []
    orig = ar.launch
    ar.launch = lambda i, after=None: (launched.append(i), orig(i, after))
    ar.ready(700)   # nothing lies entirely above 700
    a = list(launched)
    ar.ready(600)   # bucket 0
    b = list(launched)
    ar.ready(0)     # the rest
    ar.flush()
    ar.wait()
    q.put((rank, a, b, list(launched), torch.allclose(g, torch.arange(n, dtype=torch.float32) * 3), ar._next))
    dist.destroy_process_group()


def test_bucket_ready_order_and_sum():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, a, b, allb, ok, nxt in res:
        assert a == [] and b == [0] and allb == [0, 1, 2], (rank, a, b, allb)
        assert ok, rank
        assert nxt == 0  # reset for the next step


@pytest.mark.slow
def test_resnet20_allreduce_two_workers(tmp_path):
    md = str(tmp_path / "ck")
    codes, out, _ = local_cluster.launch("resnet20", 0, 2, ["--mode=allreduce", "--device=cpu", "--batch_size=4",
                                                             "--num_steps=3", "--data_dir=/nonexistent",
                                                             "--model_dir=" + md], timeout=300, stream=False)
    assert all(c == 0 for c in codes.values()), out
    for w in (0, 1):
        assert any(l.startswith("Total Time: ") for l in out[("worker", w)])
    assert any(f.startswith("model.ckpt-") for f in os.listdir(md))
