"""MNIST CNN program on CPU (the fp32 PyTorch reference path of every op): the --dtype fp32 step
against fp32 autograd, evaluation (the Test-Accuracy line), the data-parallel launch order, and
the --dtype / --bucket_mb flag routing."""
import pytest
import torch
import torch.nn.functional as F

from dtfe import ops, train
from dtfe.models.mnist_cnn import MnistCnnModel
from dtfe.utils import flags as flagmod


def _batch(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, 784, generator=g)
    y = F.one_hot(torch.randint(0, 10, (n,), generator=g), 10).float()
    return x, y


def autograd_f32(core):
    """fp32 autograd of the CNN on the program's own parameters and staged batch (dropout off)."""
    P, n = core.P, core.names

    def v(k):
        return P.view(n[k]).detach().float().clone().requires_grad_(True)

    wc1, wc2, wd1, wo, bc1, bc2, bd1, bo = (v(k) for k in ("wc1", "wc2", "wd1", "out", "bc1", "bc2", "bd1", "bout"))
    x = core.x.float().permute(0, 3, 1, 2)
    z = F.max_pool2d(F.relu(F.conv2d(x, wc1.permute(0, 3, 1, 2), bc1, padding=2)), 2)
    z = F.max_pool2d(F.relu(F.conv2d(z, wc2.permute(0, 3, 1, 2), bc2, padding=2)), 2)
    h = F.relu(z.permute(0, 2, 3, 1).reshape(x.shape[0], -1) @ wd1.t() + bd1)
    logits = h @ wo.t() + bo
    loss = F.cross_entropy(logits, core.labels.long())
    loss.backward()
    return loss.item(), {"wc1": wc1.grad, "wc2": wc2.grad, "wd1": wd1.grad, "out": wo.grad, "bc1": bc1.grad,
                         "bc2": bc2.grad, "bd1": bd1.grad, "bout": bo.grad}, logits.detach()


def test_fp32_cnn_step_matches_autograd():
    m = MnistCnnModel()
    m.set_dtype("fp32")
    prog = m.program(torch.device("cpu"), 16, seed=3)
    prog.core.keep = 1.0
    prog.load_batch(_batch(16))
    met = prog.compute_grads()
    loss_ref, grads, _ = autograd_f32(prog.core)
    assert abs(met["loss"].item() - loss_ref) <= 1e-5 * abs(loss_ref)
    for k, g in grads.items():
        got = prog.core.gw[k]
        err = ((got - g).norm() / (g.norm() + 1e-12)).item()
        assert err < 1e-4, (k, err)


def test_cnn_evaluate_counts_real_rows_only():
    """bf16 program (CPU reference ops): evaluate pads the last chunk by repeating rows and counts
    only the real ones; it equals the argmax agreement of the program's own no-dropout forward."""
    m = MnistCnnModel()
    prog = m.program(torch.device("cpu"), 8, seed=4)
    x, y = _batch(13, seed=5)
    acc = prog.evaluate(x, y)
    c = prog.core
    assert c.loss_sum.item() == 0.0 and int(c.correct.item()) == 0
    c.logits = torch.empty(8, 10)
    hits = 0
    for lo in (0, 8):
        mrows = min(8, 13 - lo)
        idx = torch.arange(lo, lo + 8).clamp_max(12)
        prog.load_batch((x[idx], y[idx]))
        c.forward(keep=1.0, logits=c.logits)
        hits += int((c.logits[:mrows].argmax(1) == y[lo:lo + mrows].argmax(1)).sum())
    assert acc == hits / 13


def test_fp32_evaluate_matches_autograd_argmax():
    m = MnistCnnModel()
    m.set_dtype("fp32")
    prog = m.program(torch.device("cpu"), 16, seed=6)
    x, y = _batch(16, seed=7)
    acc = prog.evaluate(x, y)
    prog.load_batch((x, y))
    _, _, logits = autograd_f32(prog.core)
    assert acc == float((logits.argmax(1) == y.argmax(1)).float().mean())


class _RecordingAllReduce:
    def __init__(self, log):
        self.log = log

    def launch(self, i, after=None):
        self.log.append("launch:%d" % i)

    def wait_bucket(self, i):
        self.log.append("wait:%d" % i)

    def wait(self):
        self.log.append("wait")


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_cnn_fc_bucket_launches_before_conv_backward(dtype):
    """The data-parallel schedule: bucket 0 (head + fc1, 98 % of the bytes) is handed to the
    all-reduce right after the fc backward, before conv2's data gradient; bucket 1 after the conv
    backward; the step waits for both before applying."""
    m = MnistCnnModel()
    m.set_dtype(dtype)
    prog = m.program(torch.device("cpu"), 4, seed=1)
    log = []
    prog.core.allreduce = _RecordingAllReduce(log)
    prog.load_batch(_batch(4))
    prog.compute_grads()
    assert prog.core.schedule == ["allreduce:0", "conv2_dgrad", "allreduce:1"]
    assert log[:2] == ["launch:0", "launch:1"] and log[-1] == "wait"


def test_dtype_flag_routing():
    assert flagmod.parse(["--dtype=fp32"]).dtype == "fp32"
    with pytest.raises(SystemExit):
        flagmod.parse(["--dtype=fp16"])
    m = MnistCnnModel()
    m.set_dtype("auto")
    assert m.dtype == "bf16"
    m.set_dtype("fp32")
    assert m.dtype == "fp32"
    for name, bad in (("resnet50", "fp32"), ("gan", "bf16"), ("lstm", "bf16")):
        cls, lr = train.MODELS[name]
        with pytest.raises(ValueError):
            cls(lr=lr).set_dtype(bad)
        cls(lr=lr).set_dtype("auto")


def test_bucket_mb_boundaries():
    class _P:
        total = 1000000

    b = train._buckets(_P(), 1)          # 1 MB of fp32 = 262144 elements per bucket, back to front
    assert b[0] == (1000000 - 262144, 1000000)
    assert b[-1][0] == 0
    assert all(hi - lo <= 262144 for lo, hi in b)
    assert sum(hi - lo for lo, hi in b) == 1000000
    assert all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))
    assert len(train._buckets(_P())) >= 1
    for bad in (0, -2):
        with pytest.raises(ValueError):
            train._buckets(_P(), bad)


def test_head_loss_partials_cpu_semantics():
    """CPU path of head_xent(parts=) + head_wgrad(parts=): 4-row workgroup sums, folded into the
    accumulators by the weight-gradient call - the same totals as the direct accumulation."""
    torch.manual_seed(3)
    B, K, NC = 30, 64, 10
    h = torch.relu(torch.randn(B, K))
    w = torch.randn(NC, K) * 0.1
    labels = torch.randint(0, NC, (B,), dtype=torch.int32)
    args = lambda: (torch.empty(B, K), torch.empty(B, 16))  # noqa: E731
    loss_a, corr_a = torch.zeros(1), torch.zeros(1, dtype=torch.int32)
    ops.head_xent(h, w, None, labels, *args(), loss_a, corr_a, scale=1.0 / B)
    parts = torch.zeros(2 * ((B + 3) // 4))
    loss, corr = torch.ones(1), torch.ones(1, dtype=torch.int32)
    dz, dl = args()
    ops.head_xent(h, w, None, labels, dz, dl, loss, corr, scale=1.0 / B, parts=parts)
    assert float(loss) == 1.0 and int(corr) == 1
    ops.head_wgrad(dl, h, torch.empty(NC, K), torch.empty(NC), NC, parts=parts, loss_sum=loss, correct=corr)
    assert abs(float(loss) - 1.0 - float(loss_a)) < 1e-5 and int(corr) - 1 == int(corr_a)
