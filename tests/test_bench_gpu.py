"""bench.py contract on one GPU: the self-launcher (``--gpus N`` without torchrun) starts N
ranks before any GPU call, every rank takes part in the gradient collective, and rank 0
prints ONE JSON line whose n_gpus / ranks_seen_by_comm / replicas_identical come from the
real N-rank run.  With one GPU the ranks share it (gloo process group + the hipIpc in-graph
all-reduce), which is the rehearsal of the driver's 8-GPU scaling run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(*args, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    r = _bench("--gpus", "2", "--backend", "gloo", "--comm", "ipc", "--steps", "6", "--warmup", "3",
               "--batch_size", "256")
    assert r["n_gpus"] == 2 and r["steps"] == 6 and r["warmup"] == 3
    cfg = r["config"]
    assert cfg["ranks_seen_by_comm"] == 2
    assert cfg["replicas_identical"] is True   # (also: both ranks ran the same pre-warm steps)
    assert cfg["prewarm"]["steps"] >= 10
    assert cfg["global_batch"] == 512 and cfg["parallelism"] == "dp2"
    assert "ipc" in cfg["grad_allreduce"] and cfg["hip_graph"] is True
    assert len(r["window_ms_per_step"]) >= 1 and r["value"] > 0


def test_bench_resnet20_two_ranks():
    r = _bench("--model", "resnet20", "--gpus", "2", "--backend", "gloo", "--comm", "ipc", "--steps", "4",
               "--warmup", "3", "--batch_size", "64")
    assert r["n_gpus"] == 2 and r["config"]["replicas_identical"] is True
    assert r["config"]["ranks_seen_by_comm"] == 2


def test_bench_resnet50_two_ranks():
    """ResNet-50 at world 2: seven ~8 MB bf16 buckets launched from the backward progress hook, the
    bottleneck weight gradients on their own stream (the all-reduce fork waits on an event of that
    stream, the compute stream never joins it mid-backward), one hipGraph per step."""
    r = _bench("--model", "resnet50", "--gpus", "2", "--backend", "gloo", "--comm", "ipc", "--steps", "4",
               "--warmup", "3", "--batch_size", "32", timeout=400)
    cfg = r["config"]
    assert r["n_gpus"] == 2 and cfg["replicas_identical"] is True and cfg["ranks_seen_by_comm"] == 2
    assert cfg["hip_graph"] is True and "ipc" in cfg["grad_allreduce"]


@pytest.mark.parametrize("model,batch", [("mnist_cnn", 256), ("resnet20", 64)])
def test_bench_eight_ranks(model, batch):
    """The W = 8 template of the IPC all-reduce kernel (the driver's 8-GPU node): eight ranks share
    the one GPU here, every one of them in every bucket's collective."""
    r = _bench("--model", model, "--gpus", "8", "--backend", "gloo", "--comm", "ipc", "--steps", "4", "--warmup", "3",
               "--batch_size", str(batch), timeout=400)
    cfg = r["config"]
    assert r["n_gpus"] == 8 and cfg["replicas_identical"] is True and cfg["ranks_seen_by_comm"] == 8
    assert cfg["global_batch"] == 8 * batch and cfg["parallelism"] == "dp8"


def test_bench_single_rank_json_contract():
    r = _bench("--steps", "10", "--warmup", "3")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r
    assert r["n_gpus"] == 1 and r["dtype"] == "bf16" and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 1024
