"""dtfe's native RCCL communicator (csrc/bindings/comm_ops.cpp, parallel/rccl.py) and the
bucketed all-reduce on a side stream captured inside a hipGraph.

One GPU box: a 1-rank communicator (RCCL refuses two ranks on one device), which still runs
the real ncclCommInitRank / ncclAllReduce path, the side-stream fork/join and the graph
capture of the collective; the multi-rank sums are covered by the gloo test of
test_allreduce_cpu.py and by the driver's multi-GPU bench."""
import datetime
import socket

import pytest
import torch
import torch.distributed as dist

import dtfe  # noqa: F401
from dtfe import ops
from dtfe.parallel.allreduce import BucketAllReduce
from dtfe.parallel.rccl import AVG, MAX, RcclComm
from dtfe.utils.graphs import StepGraph

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def pg():
    store = dist.TCPStore("127.0.0.1", _port(), 1, True, timeout=datetime.timedelta(seconds=60))
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def test_rccl_comm_ops(pg):
    comm = RcclComm(torch.device("cuda", 0))
    try:
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(100003, device="cuda").to(dt)
            ref = x.clone()
            comm.all_reduce(x)
            comm.all_reduce(x, MAX)
            comm.all_reduce(x, AVG)
            torch.cuda.synchronize()
            assert torch.equal(x, ref)
        y = torch.arange(17, dtype=torch.float32, device="cuda")
        comm.broadcast(y, 0)
        torch.cuda.synchronize()
        assert torch.equal(y, torch.arange(17, dtype=torch.float32, device="cuda"))
    finally:
        comm.close()


@pytest.mark.parametrize("comm_dtype", [torch.float32, torch.bfloat16])
def test_bucketed_allreduce_in_hipgraph(pg, comm_dtype):
    dev = torch.device("cuda", 0)
    comm = RcclComm(dev)
    n = 3 << 20
    src = torch.randn(n, device=dev)
    grad = torch.zeros(n, device=dev)
    out = torch.zeros(n, device=dev)
    buckets = [(2 << 20, n), (1 << 20, 2 << 20), (0, 1 << 20)]
    ar = BucketAllReduce(grad, buckets, comm=comm, comm_dtype=comm_dtype)

    def step():
        # "backward": gradients become final back to front, the all-reduce of each bucket
        # is forked onto the side stream while the remaining producers still run
        grad[2 << 20:].copy_(src[2 << 20:] * 2)
        ar.ready(2 << 20)
        grad[:2 << 20].copy_(src[:2 << 20] * 2)
        ar.ready(0)
        ar.flush()
        ar.wait()
        red = ar.grad16 if ar.grad16 is not None else grad
        out.copy_(red.float() + 1)   # consumer of the reduced gradients (the optimizer's slot)

    runner = StepGraph(step, warmup=2, enabled=True, capture_error_mode="thread_local")
    try:
        for i in range(5):
            src.normal_()
            runner()
            torch.cuda.synchronize()
            exp = (src * 2).to(comm_dtype).float() + 1
            assert torch.equal(out, exp), i
        assert runner.graph is not None, runner.capture_error
    finally:
        comm.close()


def test_mnist_cnn_step_with_rccl_bucket_graph(pg):
    """The bench's world>1 step shape at world 1: fused CNN step + in-graph bucketed RCCL
    all-reduce (bf16 wire) + Adam on the reduced bf16 gradients, one hipGraph."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    dev = torch.device("cuda", 0)
    comm = RcclComm(dev)
    try:
        tr = MnistCnnTrainer(256, dev, seed=0)
        ar = BucketAllReduce(tr.P.grad, tr.buckets, comm=comm, comm_dtype=torch.bfloat16)
        tr.allreduce = ar

        def step():
            tr.forward_backward()
            tr.opt.step(grad16=ar.grad16, gscale=1.0)

        runner = StepGraph(step, warmup=2, enabled=True, capture_error_mode="thread_local")
        losses = []
        for _ in range(30):
            runner()
            losses.append(float(tr.loss_sum.item()) / tr.B)
        assert runner.graph is not None, runner.capture_error
        assert int(tr.global_step.item()) == 30
        assert all(l == l for l in losses)
        assert ops.available()
    finally:
        comm.close()


@pytest.mark.parametrize("mode", ["auto", "rccl", "ipc"])
def test_make_comm_routes(pg, mode):
    from dtfe.parallel.comm import make_comm

    dev = torch.device("cuda", 0)
    sizes = [6 << 20, 1 << 16]
    comm = make_comm(dev, None, sizes, torch.bfloat16, mode=mode)
    try:
        for b in sizes:
            x = torch.randn(b // 2, device=dev).to(torch.bfloat16)
            ref = x.clone()
            comm.all_reduce(x)
            torch.cuda.synchronize()
            assert torch.equal(x, ref)
        d = comm.describe()
        assert isinstance(d, str) and d
        if mode == "ipc":
            assert "rccl" not in d
    finally:
        comm.close()


@pytest.mark.parametrize("split", ["1", "0"])
def test_cnn_late_split_apply_with_allreduce(pg, split):
    """With an all-reduce attached, step() applies the fc/head bucket while the conv bucket is
    still being reduced (split optimizers, per-bucket completion events); the trajectory must
    equal the whole-model apply."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    dev = torch.device("cuda", 0)
    comm = RcclComm(dev)
    try:
        tr = MnistCnnTrainer(256, dev, seed=4)
        tr.late_split = split == "1"
        ar = BucketAllReduce(tr.P.grad, tr.buckets, comm=comm, comm_dtype=torch.bfloat16)
        tr.allreduce = ar
        runner = StepGraph(lambda: tr.step(grad16=ar.grad16, gscale=1.0), warmup=2, enabled=True,
                           capture_error_mode="thread_local")
        for _ in range(6):
            runner()
        torch.cuda.synchronize()
        assert runner.graph is not None, runner.capture_error
        assert (tr.opt_fc is not None) == (split == "1")
        assert int(tr.global_step.item()) == 6
        _LATE[split] = tr.P.master.clone()
        if len(_LATE) == 2:
            assert torch.allclose(_LATE["1"], _LATE["0"], rtol=1e-4, atol=1e-6)
    finally:
        comm.close()


_LATE = {}
