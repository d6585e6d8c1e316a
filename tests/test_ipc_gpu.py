"""hipIpc two-shot all-reduce (csrc/kernels/ipc_allreduce.hip, parallel/ipc.py).

Two processes on the one GPU of a test box: hipIpcOpenMemHandle maps the other process's
uncached exchange buffer exactly as it maps a peer GPU's, so the staging, the per-workgroup
cross-process barriers (release/acquire at system scope), the reduce and the gather all run
for real; only the xGMI hop itself needs the driver's multi-GPU node.  Results are compared
with the fp32 sum of both ranks' inputs (computed in the same order the kernel adds)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dtfe  # noqa: F401

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(rank, n, dt, seed):
    g = torch.Generator().manual_seed(seed * 100 + rank)
    return torch.randn(n, generator=g).to(dt)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dtfe.parallel.ipc import IpcComm
        from dtfe.utils.graphs import StepGraph

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        comm = IpcComm(dev, cap_bytes=8 << 20, timeout_s=20.0)   # runs its own self-check
        errs = []
        for case, (n, off, dt) in enumerate([(7, 0, torch.float32), (1000, 1, torch.bfloat16),
                                             (3 << 20, 0, torch.bfloat16), (777777, 3, torch.float32)]):
            base = torch.zeros(n + 8, device=dev, dtype=dt)
            x = base[off:off + n]
            x.copy_(_inputs(rank, n, dt, case).to(dev))
            comm.all_reduce(x)
            torch.cuda.synchronize()
            exp = sum(_inputs(r, n, dt, case).float() for r in range(world)).to(dt)
            if not torch.equal(x.cpu(), exp):
                errs.append((case, int((x.cpu() != exp).sum())))
            if not (torch.equal(base[:off].cpu(), torch.zeros(off, dtype=dt))
                    and torch.equal(base[off + n:].cpu(), torch.zeros(8 - off, dtype=dt))):
                errs.append((case, "wrote outside the tensor"))
        # captured into a hipGraph and replayed with fresh inputs
        n = 1 << 20
        src = torch.zeros(n, device=dev, dtype=torch.bfloat16)
        buf = torch.zeros_like(src)

        def step():
            buf.copy_(src)
            comm.all_reduce(buf)

        runner = StepGraph(step, warmup=1, enabled=True)
        for it in range(5):
            src.copy_(_inputs(rank, n, torch.bfloat16, 100 + it).to(dev))
            runner()
            torch.cuda.synchronize()
            exp = sum(_inputs(r, n, torch.bfloat16, 100 + it).float() for r in range(world)).to(torch.bfloat16)
            if not torch.equal(buf.cpu(), exp):
                errs.append(("graph", it))
        errs.append(("graph_captured", runner.graph is not None))
        # alternating bucket sizes (different block counts per launch), as the CNN step issues
        # its fc bucket then its conv bucket: staging parity must flip per launch on every block
        big = torch.zeros(3 << 20, device=dev, dtype=torch.bfloat16)
        small = torch.zeros(53000, device=dev, dtype=torch.bfloat16)
        for it in range(6):
            for j, t in enumerate((big, small)):
                t.copy_(_inputs(rank, t.numel(), torch.bfloat16, 200 + 2 * it + j).to(dev))
                comm.all_reduce(t)
            torch.cuda.synchronize()
            for j, t in enumerate((big, small)):
                exp = sum(_inputs(r, t.numel(), torch.bfloat16, 200 + 2 * it + j).float()
                          for r in range(world)).to(torch.bfloat16)
                if not torch.equal(t.cpu(), exp):
                    errs.append(("mixed", it, j))
        st = comm.status()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, st, None))
    except Exception as e:  # noqa: BLE001 - report to the parent
        q.put((rank, None, None, repr(e)))


def test_ipc_allreduce_two_processes_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, errs, st, exc in res:
        assert exc is None, (rank, exc)
        assert st == 0, rank
        assert errs == [("graph_captured", True)], (rank, errs)


def test_ipc_allreduce_single_rank():
    from dtfe.parallel.ipc import IpcComm

    comm = IpcComm(torch.device("cuda", 0), cap_bytes=1 << 20, timeout_s=5.0)
    try:
        x = torch.randn(12345, device="cuda")
        ref = x.clone()
        comm.all_reduce(x)
        assert comm.status() == 0
        assert torch.equal(x, ref)
        with pytest.raises(ValueError):
            comm.all_reduce(torch.zeros(1 << 20, device="cuda"))   # 4 MB > 1 MB staging, no fallback
    finally:
        comm.close()
