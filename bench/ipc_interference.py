#!/usr/bin/env python
"""How much does the in-graph IPC all-reduce slow the backward kernels it overlaps?

Two ranks share cuda:0 (gloo control, hipIpc exchange buffers).  Rank 0 times the MNIST CNN's
conv backward pair - conv2 data gradient (main stream) and conv2 weight gradient (side stream),
the kernels the fc bucket's all-reduce overlaps at world > 1 (models/mnist_cnn.py) - alone and
with the 6.5 MB bf16 fc-bucket all-reduce launched concurrently on a third stream; rank 1 only
takes part in the all-reduce.  The IPC kernel's workgroups spin on their barriers while the
peer's half has not arrived, so they hold CUs the conv kernels could use.

    python bench/ipc_interference.py [--batch 1024] [--reps 50] [--caps 128,64,32,16]

Sweeps the all-reduce kernel's grid cap (IpcComm.set_max_blocks).  Caveat: both ranks run on the
same GPU here, so the all-reduce's kernels of BOTH ranks share the conv kernels' CUs and every
peer read is a local HBM read; on a node each GPU hosts one rank and the peer reads cross xGMI -
the interference and the all-reduce time both differ there.

(self-launches its two ranks; one GPU)
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(rank, port, args):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import dtfe  # noqa: F401
    from dtfe import ops
    from dtfe.models.mnist_cnn import MnistCnnTrainer
    from dtfe.parallel.ipc import IpcComm

    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = MnistCnnTrainer(args.batch, dev, keep_prob=1.0, seed=1)
    tr.forward_backward()          # fills dp2 / p1 / the workspaces
    lo, hi = tr.buckets[0]
    bucket = torch.zeros(hi - lo, dtype=torch.bfloat16, device=dev)
    comm = IpcComm(dev, None, cap_bytes=bucket.numel() * 2 + 4096)
    main, side, cs = torch.cuda.current_stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def convs():
        side.wait_stream(main)
        tr._conv2_dgrad()
        with torch.cuda.stream(side):
            ops.imgwgrad(tr.p1, tr.gw["wc2"], tr.gw["bc2"], dy_pooled=tr.dp2, dy_argmax=tr.a2, workspace=tr.ws_c2,
                         max_blocks=tr.c2_blocks, **tr.ic2)
        main.wait_stream(side)

    def allreduce():
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            comm.all_reduce(bucket)
        main.wait_stream(cs)

    def timed(fn, reps):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000 / reps

    caps = [int(c) for c in args.caps.split(",")]
    for rnd in range(2):
        for cap in caps:
            comm.set_max_blocks(cap)
            if rank == 0:
                t_conv = timed(convs, args.reps)
            else:
                dist.barrier()
            t_ar = timed(allreduce, args.reps)
            if rank == 0:
                t_both = timed(lambda: (allreduce(), convs()), args.reps)
            else:
                t_both = timed(allreduce, args.reps)
            if rank == 0:
                print("grid cap %3d | conv2 dgrad+wgrad alone %.1f us | fc-bucket IPC all-reduce alone %.1f us | "
                      "both concurrent (span) %.1f us | serial sum %.1f us | interference on the convs %+.1f %%"
                      % (cap, t_conv, t_ar, t_both, t_conv + t_ar, 100.0 * (t_both - t_conv) / t_conv), flush=True)
    comm.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--caps", default="128,64,32,16", help="all-reduce grid caps to sweep")
    ap.add_argument("--child", type=int, default=-1)
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    if a.child >= 0:
        child(a.child, a.port, a)
        return
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", str(r), "--port", str(port),
                               "--batch", str(a.batch), "--reps", str(a.reps), "--caps", a.caps]) for r in range(2)]
    codes = [p.wait() for p in procs]
    sys.exit(max(codes))


if __name__ == "__main__":
    main()
