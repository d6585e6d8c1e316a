"""Multi-process cluster roles on the GPU (one MI355X box): the MNIST CNN through the
parameter-server path with the ps and both workers on cuda:0 (BASELINE.json config 4 in
miniature).  Every (ps, worker) pair shares the GPU, so the pairs exchange payloads through
host memory (Server.pair_comm_device); compute and the optimizer apply run on the GPU kernels."""
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


@pytest.mark.parametrize("sync", [False, True])
def test_cnn_ps_on_gpu(tmp_path, sync):
    md = str(tmp_path / "ck")
    extra = ["--device=cuda", "--synthetic", "--num_steps=8", "--workers=2", "--batch_size=64", "--seed=3",
             "--model_dir=" + md, "--save_model_secs=0.2"] + (["--sync"] if sync else [])
    codes, out, _ = local_cluster.launch("cnn", 1, 2, extra, timeout=600, stream=False, gpus=1)
    assert all(c == 0 for c in codes.values()), "%s\n%s" % (codes, "\n".join(
        "---- %s\n%s" % (k, "\n".join(v[-40:])) for k, v in out.items()))
    assert out[("ps", 0)][-1] == "ps 0: quitting"
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
    t = ckpt.load_bundle(ckpt.latest_checkpoint(md))
    assert "Variable_1/Adam" in t
