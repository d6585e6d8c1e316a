"""Multi-process cluster roles on the GPU (one MI355X box): the MNIST CNN through the
parameter-server path with the ps and both workers on cuda:0 (BASELINE.json config 4 in
miniature).  Every task drives a GPU of this host, so PUSH / PULL take the native data plane
(parallel/ps_native.py: hipIpc mailboxes written by the workers' GPUs, a C++ service thread on
the ps applying them) and only control messages use gloo; compute and the apply are HIP kernels."""
import os
import re
import sys

import pytest

from dtfe import ckpt

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "launch"))
import local_cluster  # noqa: E402

pytestmark = pytest.mark.gpu


def _gs(lines):
    return [int(m.group(1)) for l in lines for m in [re.match(r"Global step (\d+) Local step", l)] if m]


@pytest.mark.parametrize("n_ps,sync", [(1, False), (1, True), (2, False), (2, True)])
def test_cnn_ps_on_gpu(tmp_path, n_ps, sync):
    """n_ps = 2: the variables are sharded round-robin over two ps tasks; every
    exchange carries ONE request number to both shards and each shard's own version tag."""
    md = str(tmp_path / "ck")
    extra = ["--device=cuda", "--synthetic", "--num_steps=8", "--workers=2", "--batch_size=64", "--seed=3",
             "--model_dir=" + md, "--save_model_secs=0.2"] + (["--sync"] if sync else [])
    codes, out, _ = local_cluster.launch("cnn", n_ps, 2, extra, timeout=600, stream=False, gpus=1)
    assert all(c == 0 for c in codes.values()), "%s\n%s" % (codes, "\n".join(
        "---- %s\n%s" % (k, "\n".join(v[-40:])) for k, v in out.items()))
    for k in range(n_ps):
        assert "ps %d: quitting" % k in out[("ps", k)]
        # every worker task is on this host's GPU: PUSH / PULL take the native hipIpc data plane
        assert any(l.startswith("ps %d: native data plane:" % k) for l in out[("ps", k)]), out[("ps", k)][-10:]
    for w in (0, 1):  # a missed reply would stall 60 s and then raise from the device error word
        assert not any("no reply" in l for l in out[("worker", w)])
    gs = _gs(out[("worker", 0)]) + _gs(out[("worker", 1)])
    assert max(gs) >= 8
    t = ckpt.load_bundle(ckpt.latest_checkpoint(md))
    assert tuple(t["Variable_1"].shape) == (5, 5, 32, 64) and "Variable_1/Adam" in t


def test_cnn_allreduce_two_workers_ipc_in_graph(tmp_path):
    """--mode=allreduce with the reference CLI, 2 workers sharing cuda:0: the IPC all-reduce
    engine inside the captured step graph (gloo only carries the control traffic)."""
    md = str(tmp_path / "ck")
    extra = ["--mode=allreduce", "--device=cuda", "--backend=gloo", "--comm=ipc", "--comm_dtype=bf16",
             "--synthetic", "--num_steps=12", "--batch_size=128", "--model_dir=" + md, "--save_model_secs=0.2",
             "--check_pull"]
    codes, out, _ = local_cluster.launch("cnn", 0, 2, extra, timeout=600, stream=False, gpus=1)
    assert all(c == 0 for c in codes.values()), "%s\n%s" % (codes, "\n".join(
        "---- %s\n%s" % (k, "\n".join(v[-40:])) for k, v in out.items()))
    for w in (0, 1):
        assert any(l.startswith("Total Time: ") for l in out[("worker", w)])
        assert max(_gs(out[("worker", w)])) == 12
    sums = [[l for l in out[("worker", w)] if l.startswith("params checksum")] for w in (0, 1)]
    assert sums[0] and sums[0] == sums[1], sums
    # the CLI runs the benchmarked schedule: the fc bucket's all-reduce is launched right after the
    # grouped fc backward, before conv2's data gradient, the conv bucket after the conv backward
    sched = [l for l in out[("worker", 0)] if l.startswith("schedule: ")]
    assert sched == ["schedule: allreduce:0 < conv2_dgrad < allreduce:1"], sched
    for w in (0, 1):  # the CNN prints the reference's Test-Accuracy line (LSTM:134-138)
        assert any(l.startswith("Test-Accuracy: ") for l in out[("worker", w)])
    t = ckpt.load_bundle(ckpt.latest_checkpoint(md))
    assert "Variable_1/Adam" in t and "beta1_power" in t


def test_allreduce_rank_crash_ends_every_rank(tmp_path):
    """--mode=allreduce, 2 workers sharing cuda:0 (gloo + in-graph IPC all-reduce), worker 1 crashes
    at step 5 (DTFE_FAULT): worker 0's step graph would wait on the dead peer; its comm watchdog
    sees the silent heartbeat, aborts the collectives and exits non-zero - no rank hangs.  No
    --heartbeat_secs: failure detection is on by default in --mode=allreduce."""
    import time

    extra = ["--mode=allreduce", "--device=cuda", "--backend=gloo", "--comm=ipc", "--comm_dtype=bf16",
             "--synthetic", "--num_steps=400", "--batch_size=128", "--model_dir=" + str(tmp_path / "ck"),
             "--save_model_secs=0", "--heartbeat_timeout=6"]
    env = dict(os.environ, DTFE_FAULT="crash@worker:1:step=5")
    t0 = time.time()
    codes, out, _ = local_cluster.launch("cnn", 0, 2, extra, env=env, timeout=240, stream=False, gpus=1)
    assert time.time() - t0 < 200
    assert codes[("worker", 1)] == 17, codes
    assert codes[("worker", 0)] not in (0, None), (codes, out[("worker", 0)][-20:])
    # worker 0 ends either through its comm watchdog (peer silent / store gone / engine error) or
    # because the host-side collective (gloo) raised on the dead peer first - never a hang
    w0 = out[("worker", 0)]
    assert any("silent for" in l or "store unreachable" in l or "engine failure" in l or "Traceback" in l
               for l in w0), "\n".join(w0[-30:])


@pytest.mark.parametrize("hogwild", [False, True])
def test_bench_ps_native_plane(hogwild):
    """bench.py --mode ps: 1 ps + 2 workers sharing cuda:0 over the native hipIpc data plane; every
    pushed gradient is applied exactly once and the JSON line reports the whole job's images/sec.
    hogwild=False forces the bucket announcements (--ps_overlap on) that a ps on another GPU gets;
    hogwild=True keeps the shared-GPU default (whole push applied at the request)."""
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--mode", "ps", "--gpus", "2", "--steps", "30",
           "--warmup", "4", "--batch_size", "256"] + (["--hogwild"] if hogwild else ["--ps_overlap", "on"])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    rec = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    c = rec["config"]
    n = 34 + c["prewarm"]["steps"]   # timed + warmup + pre-warm steps per worker
    assert c["prewarm"]["steps"] >= 10
    assert c["ps_applies"] == c["pushes_issued"] == 2 * n
    # the CNN pushes two buckets per step; the first is announced and applied as it lands (during
    # backward - or with the request, if the ps noticed it only then); the last is never announced:
    # the request applies it in the launch that advances the step scalars and writes the reply
    assert c["ps_bucket_applies"] == (0 if hogwild else 2 * 1 * n)
    assert c["ps_global_step"] == 2 * n and 0 < c["global_step"] <= 2 * n
    assert 0.0 < c["last_loss"] < 10.0
    # with announced buckets, the other worker's bucket applies land between a worker's own bucket
    # apply and its request: those ranges are re-copied into its reply (the pull is current)
    if not hogwild:
        assert c["ps_refreshed_ranges"] > 0


def _ps_verify(extra):
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--mode", "ps", "--gpus", "1", "--ps_verify", "6",
           "--batch_size", "256", "--prewarm_ms", "0"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith('{"ps_verify"')][-1])


def test_ps_replies_bitwise_across_data_plane_variants():
    """1 ps + 1 worker (async, one GPU): after every exchange the worker's pulled bf16 copies
    (natural + transposed) and fp32 variables equal, bit for bit, the ps shard's variables (fetched
    over the control channel); and the fused-reply path (the apply writes the reply buffer, default),
    the snapshot-copy path, and the bucket announcements on / off all give the same pulled
    parameters, step by step."""
    variants = [[], ["--ps_overlap", "on"], ["--ps_fused_reply", "off"],
                ["--ps_fused_reply", "off", "--ps_overlap", "on"]]
    recs = [_ps_verify(v) for v in variants]
    for v, r in zip(variants, recs):
        assert r["n_mismatch"] == 0, (v, r["mismatches"])
    for v, r in zip(variants[1:], recs[1:]):
        assert r["ps_verify"] == recs[0]["ps_verify"], (v, r["ps_verify"], recs[0]["ps_verify"])
    assert len(set(recs[0]["ps_verify"])) == len(recs[0]["ps_verify"])  # the parameters do move


def test_ps_replies_bitwise_two_partitioned_ps():
    """2 ps tasks with the fc1 weight in 4 partitions dealt over both (--ps_partition_mb 4): after every
    exchange the worker's pulled copies equal both shards' variables bit for bit (partitions compared
    through the worker's alias views), and the fused-reply / snapshot / announced-bucket data-plane
    variants give the same pulled parameters step by step.  (The partitioned model trains the same
    function as the unpartitioned one but its applies split into different launches, so only
    variants of the partitioned layout are compared with each other.)"""
    part = ["--num_ps", "2", "--ps_partition_mb", "4"]
    variants = [part, part + ["--ps_overlap", "on"], part + ["--ps_fused_reply", "off"]]
    recs = [_ps_verify(v) for v in variants]
    for v, r in zip(variants, recs):
        assert r["n_mismatch"] == 0, (v, r["mismatches"])
    for v, r in zip(variants[1:], recs[1:]):
        assert r["ps_verify"] == recs[0]["ps_verify"], (v, r["ps_verify"], recs[0]["ps_verify"])
    assert len(set(recs[0]["ps_verify"])) == len(recs[0]["ps_verify"])


def test_bench_ps_two_partitioned_ps():
    """bench.py --mode ps --num_ps 2 --ps_partition_mb 4: 2 ps + 2 workers (all sharing cuda:0 here;
    ps k sits on GPU k * ndev / 2 on a node), each ps holding half the fc1 partitions - every push
    applied once on each shard, the params split near evenly."""
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--mode", "ps", "--gpus", "2", "--steps", "20",
           "--warmup", "3", "--batch_size", "256", "--num_ps", "2", "--ps_partition_mb", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    rec = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    c = rec["config"]
    assert c["num_ps"] == 2 and c["parallelism"] == "ps2+w2" and rec["value"] > 0
    n = 23 + c["prewarm"]["steps"]
    shards = c["ps_shards"]
    assert [s_["applies"] for s_ in shards] == [2 * n, 2 * n]
    big = max(s_["params"] for s_ in shards)
    assert big < 0.6 * sum(s_["params"] for s_ in shards)  # fc1 split, not on one ps
