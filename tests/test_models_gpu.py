"""Reference-model step programs on the HIP kernels vs the same programs on the CPU fp32 path."""
import pytest
import torch
import torch.nn.functional as F

from dtfe.models.autoencoder import AutoencoderModel
from dtfe.models.gan import GanModel
from dtfe.models.lstm import LstmModel
from dtfe.models.softmax_reg import SoftmaxRegressionModel

pytestmark = pytest.mark.gpu


def _pair(model, B, seed=7):
    cpu = model.program("cpu", B, seed=seed)
    gpu = model.program("cuda", B, seed=seed)
    assert torch.equal(cpu.P.master, gpu.P.master.cpu())
    return cpu, gpu


def _cmp(cpu, gpu, tol):
    torch.cuda.synchronize()
    for s in cpu.model.specs:
        a, b = gpu.P.gview(s.name).cpu(), cpu.P.gview(s.name)
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < tol, (s.name, rel)


def _poison(*progs):
    """NaN-fill the gradient buffers: compute_grads must store every element (it does not zero)."""
    for p in progs:
        p.P.grad.fill_(float("nan"))


@pytest.mark.parametrize("B", [32, 256])
@pytest.mark.parametrize("name", ["softmax", "encoder", "lstm"])
def test_supervised_models_gpu_match_cpu(name, B):
    torch.manual_seed(0)
    model = {"softmax": SoftmaxRegressionModel, "encoder": AutoencoderModel, "lstm": LstmModel}[name]()
    cpu, gpu = _pair(model, B)
    _poison(cpu, gpu)
    x = torch.rand(B, 784)
    y = F.one_hot(torch.randint(0, 10, (B,)), 10).float()
    batch = x if name == "encoder" else (x, y)
    cpu.load_batch(batch)
    gpu.load_batch(tuple(t.cuda() for t in batch) if isinstance(batch, tuple) else batch.cuda())
    mc = cpu.compute_grads()
    mg = gpu.compute_grads()
    _cmp(cpu, gpu, 1e-4)
    assert abs(float(mc["loss"]) - float(mg["loss"])) < 1e-4 * max(1.0, abs(float(mc["loss"])))


@pytest.mark.parametrize("B", [64, 128])
def test_gan_gpu_matches_cpu(B):
    torch.manual_seed(1)
    model = GanModel()
    cpu, gpu = _pair(model, B)
    _poison(cpu, gpu)
    x = torch.rand(B, 784)
    gpu.load_batch(x.cuda())
    cpu.load_batch(x)
    cpu.z.copy_(gpu.z.cpu())  # same noise (device RNG vs host RNG)
    mc = cpu.compute_grads()
    mg = gpu.compute_grads()
    _cmp(cpu, gpu, 1e-4)
    for k in ("gen_loss", "disc_loss"):
        assert abs(float(mc[k]) - float(mg[k])) < 1e-4


def test_lstm_trains_on_gpu_with_graph():
    from dtfe.data.mnist import synthetic_arrays
    from dtfe.optim import Optimizer
    from dtfe.utils.graphs import StepGraph

    model = LstmModel(lr=0.5)
    prog = model.program("cuda", 128, seed=0)
    opt = Optimizer(model.opt_groups[0][0], prog.P)
    (xs, ys), _ = synthetic_arrays(4096, 10)
    xs = xs.copy()
    for k in range(10):  # class k also lights a vertical band: visible at every timestep
        xs[ys == k, :, 2 + 2 * k:4 + 2 * k] = 255
    X = torch.from_numpy(xs.reshape(4096, 784)).float().cuda() / 255
    Y = F.one_hot(torch.from_numpy(ys).long(), 10).float().cuda()

    def step():
        prog.compute_grads()
        opt.step()

    run = StepGraph(step, warmup=2)
    first = None
    for it in range(150):
        i0 = (it * 128) % 3968
        prog.load_batch((X[i0:i0 + 128], Y[i0:i0 + 128]))
        run()
        if first is None:
            first = float(prog.loss.item()) / 128
    last = float(prog.loss.item()) / 128
    assert run.graph is not None, run.capture_error
    assert last < 0.5 * first, (first, last)


@pytest.mark.parametrize("split", ["1", "4", "0"])
@pytest.mark.parametrize("batch", [128, 48, 1024])
def test_lstm_persistent_matches_per_step(batch, split, monkeypatch):
    """Persistent whole-sequence kernels (lstm_seq.hip; split=1: each row group over 8 CUs (B <= 512) or
    4 CUs with a per-step flag exchange, split=4: forced 4, split=0: one CU per row group) vs the
    per-step cell kernels + GEMMs:
    forward activations, cell states, logits, and every gradient."""
    model = LstmModel()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(batch, 784, generator=g)
    y = F.one_hot(torch.randint(0, 10, (batch,), generator=g), 10).float()
    out = {}
    monkeypatch.setenv("DTFE_LSTM_SPLIT", split)
    for mode in ("1", "0"):
        monkeypatch.setenv("DTFE_LSTM_PERSIST", mode)
        prog = model.program("cuda", batch, seed=11)
        prog.load_batch((x.cuda(), y.cuda()))
        prog.compute_grads()
        torch.cuda.synchronize()
        out[mode] = {k: v.detach().cpu().clone() for k, v in
                     dict(act=prog.act, c=prog.c, xh=prog.xh, logits=prog.logits, dg=prog.dg, grad=prog.P.grad).items()}
    for k in out["0"]:
        a, b = out["1"][k], out["0"][k]
        err = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err < 1e-5, (k, err)


def test_lstm_split_kernels_replay_in_a_graph(monkeypatch):
    """The split kernels' step flags are epoch-stamped: replaying a captured step many times
    (fwd and bwd share the flag words) must keep giving the eager result."""
    from dtfe.utils.graphs import StepGraph
    monkeypatch.setenv("DTFE_LSTM_SPLIT", "1")
    model = LstmModel()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(256, 784, generator=g).cuda()
    y = F.one_hot(torch.randint(0, 10, (256,), generator=g), 10).float().cuda()
    prog = model.program("cuda", 256, seed=2)
    prog.load_batch((x, y))
    prog.compute_grads()
    ref = prog.P.grad.clone()
    run = StepGraph(prog.compute_grads, warmup=1)
    for _ in range(40):
        run()
    torch.cuda.synchronize()
    assert run.graph is not None, run.capture_error
    assert torch.equal(prog.P.grad, ref)
    prog.check_health()  # the split kernels' exchange error word stayed clear
    assert int(torch.ops.dtfe.lstm_status(False)) == 0


@pytest.mark.parametrize("split", ["1", "0"])
def test_lstm_stage_folded_into_captured_forward(split, monkeypatch):
    """load_batch captured together with the step (bench/ref_models.py): the forward launch stages the batch
    itself (lstm_seq_fwd xsrc - x_t read from the images, xh / labels / accumulator clears in its prologue;
    split=0: the launcher stages first).  Replays over a refilled input buffer give the eager seq_stage
    path's gradients, xh and hit count bitwise."""
    from dtfe.utils.graphs import StepGraph
    monkeypatch.setenv("DTFE_LSTM_SPLIT", split)
    model = LstmModel()
    B = 128
    g = torch.Generator().manual_seed(7)
    xs = [torch.rand(B, 784, generator=g).cuda() for _ in range(3)]
    ys = [F.one_hot(torch.randint(0, 10, (B,), generator=g), 10).float().cuda() for _ in range(3)]
    eager = model.program("cuda", B, seed=4)
    refs = []
    for x, y in zip(xs, ys):
        eager.load_batch((x, y))
        eager.compute_grads()
        torch.cuda.synchronize()
        refs.append((eager.P.grad.clone(), eager.xh.clone(), eager.loss.clone(), eager.correct.clone()))
    prog = model.program("cuda", B, seed=4)
    xb, yb = xs[0].clone(), ys[0].clone()

    def step():
        prog.load_batch((xb, yb))
        prog.compute_grads()

    run = StepGraph(step, warmup=1)
    for i in (0, 1, 2, 1, 0):
        xb.copy_(xs[i])
        yb.copy_(ys[i])
        run()
        torch.cuda.synchronize()
        for name, got, want in zip(("grad", "xh", "correct"), (prog.P.grad, prog.xh, prog.correct),
                                   (refs[i][0], refs[i][1], refs[i][3])):
            assert torch.equal(got, want), (i, name)
        assert torch.allclose(prog.loss, refs[i][2], rtol=1e-6, atol=0), i  # (loss: an atomic sum)
    assert run.graph is not None, run.capture_error
    assert prog._stage is None
    assert int(torch.ops.dtfe.lstm_status(False)) == 0


def test_encoder_captured_load_reads_batch_in_place():
    """Autoencoder step with load_batch captured in the graph (bench/ref_models.py): the layers read the
    caller's batch tensor in place (no staging copy) and the MSE loss is stored by the kernel's last
    workgroup (no memset).  Replays over a refilled input buffer give the eager gradients and loss
    bitwise (the ticketed loss sum is order-fixed)."""
    from dtfe.utils.graphs import StepGraph
    model = AutoencoderModel()
    B = 256
    g = torch.Generator().manual_seed(9)
    xs = [torch.rand(B, 784, generator=g).cuda() for _ in range(3)]
    eager = model.program("cuda", B, seed=6)
    refs = []
    for x in xs:
        eager.load_batch(x)
        eager.compute_grads()
        torch.cuda.synchronize()
        refs.append((eager.P.grad.clone(), eager.loss.clone()))
    prog = model.program("cuda", B, seed=6)
    xb = xs[0].clone()

    def step():
        prog.load_batch(xb)
        prog.compute_grads()

    run = StepGraph(step, warmup=1)
    for i in (0, 1, 2, 1):
        xb.copy_(xs[i])
        run()
        torch.cuda.synchronize()
        assert torch.equal(prog.P.grad, refs[i][0]), i
        assert torch.equal(prog.loss, refs[i][1]), i
    assert run.graph is not None, run.capture_error
    assert prog.xin.data_ptr() == xb.data_ptr()


@pytest.mark.parametrize("B,DH", [(128, 256), (37, 128), (5, 60)])
def test_gan_disc_head_matches_fp32_chain(B, DH):
    """ops.gan_disc_head (one launch: output layer, both GAN losses, dWd2 / dbd2, dd1, ddf) vs its CPU fp32
    oracle (the N = 1 GEMM, gan_loss and the three gradient GEMMs it replaces); two launches bitwise equal
    (ticketed fixed-order partial sums)."""
    from dtfe import ops
    g = torch.Generator().manual_seed(B + DH)
    d1 = torch.relu(torch.randn(2 * B, DH, generator=g))
    w = torch.randn(DH, 1, generator=g) / DH ** 0.5
    b = torch.randn(1, generator=g)

    def outs(dev):
        z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
        return dict(p=z(2 * B, 1), dlog=z(2 * B, 1), dlog_g=z(B, 1), gw=z(DH, 1), gb=z(1), dd1=z(2 * B, DH),
                    ddf=z(B, DH), gen=z(1), disc=z(1))

    ref = outs("cpu")
    assert ops.gan_disc_head(d1, w, b, ref["p"], ref["dlog"], ref["dlog_g"], ref["gw"], ref["gb"], ref["dd1"],
                             ref["ddf"], ref["gen"], ref["disc"])
    ws = torch.zeros(ops.gan_head_ws_floats(B, DH), device="cuda")
    assert ops.gan_head_ws_floats(B, DH) == int(torch.ops.dtfe.gan_head_ws_floats(B, DH))
    runs = []
    for _ in range(2):
        o = outs("cuda")
        assert ops.gan_disc_head(d1.cuda(), w.cuda(), b.cuda(), o["p"], o["dlog"], o["dlog_g"], o["gw"], o["gb"],
                                 o["dd1"], o["ddf"], o["gen"], o["disc"], ws)
        torch.cuda.synchronize()
        runs.append({k: v.cpu() for k, v in o.items()})
    for k in ref:
        assert torch.equal(runs[0][k], runs[1][k]), k
        r, got = ref[k], runs[0][k]
        err = ((got - r).norm() / (r.norm() + 1e-12)).item()
        assert err < 2e-5, (k, err)
