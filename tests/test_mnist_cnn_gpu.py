"""End-to-end numerics of the fused MNIST-CNN step program vs torch autograd (fp32)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


class _Bf16Point(torch.autograd.Function):
    """Round to bf16 in forward AND backward: mirrors where the kernels store bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


q = _Bf16Point.apply


def _reference_grads(trainer):
    P, n = trainer.P, trainer.names
    x = trainer.x.float().permute(0, 3, 1, 2).cpu()            # what the kernels consumed
    y = trainer.labels.long().cpu()

    def w(k):
        return P.view(n[k]).detach().cpu().to(torch.bfloat16).float().requires_grad_(True)

    def b(k):
        return P.view(n[k]).detach().cpu().float().requires_grad_(True)

    wc1, wc2, wd1, wo = w("wc1"), w("wc2"), w("wd1"), w("out")
    bc1, bc2, bd1, bo = b("bc1"), b("bc2"), b("bd1"), b("bout")
    # the kernels pool the fp32 accumulators and round the pooled value (argmax on exact values)
    z = F.conv2d(x, wc1.permute(0, 3, 1, 2), bc1, padding=2)
    z = q(F.max_pool2d(F.relu(z), 2))
    z = F.conv2d(z, wc2.permute(0, 3, 1, 2), bc2, padding=2)
    z = q(F.max_pool2d(F.relu(z), 2))
    z = z.permute(0, 2, 3, 1).reshape(x.shape[0], -1)           # NHWC flatten, as the kernels
    h = F.relu(q(z @ wd1.t() + bd1))
    logits = h @ wo.t() + bo
    loss = F.cross_entropy(logits, y)
    loss.backward()
    return loss.item(), {"wc1": wc1.grad, "wc2": wc2.grad, "wd1": wd1.grad, "out": wo.grad,
                         "bc1": bc1.grad, "bc2": bc2.grad, "bd1": bd1.grad, "bout": bo.grad}


def test_cnn_step_matches_autograd():
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    torch.manual_seed(0)
    tr = MnistCnnTrainer(64, "cuda", keep_prob=1.0, seed=3)
    tr.forward_backward()
    torch.cuda.synchronize()
    loss_ref, grads = _reference_grads(tr)
    loss = tr.loss_sum.item() / tr.B
    assert abs(loss - loss_ref) < 2e-2 * max(1.0, abs(loss_ref))
    errs = {}
    for k, gref in grads.items():
        got = tr.gw[k].detach().cpu()
        errs[k] = ((got - gref).norm() / (gref.norm() + 1e-12)).item()
    assert all(e < 3e-2 for e in errs.values()), sorted(errs.items(), key=lambda kv: -kv[1])


def test_cnn_trains_and_graph_replays():
    from dtfe.models.mnist_cnn import MnistCnnTrainer, SyntheticMnist
    from dtfe.utils.graphs import StepGraph

    # a learnable synthetic task: label = brightest of 10 pixel bands
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 64, (4096, 784), generator=g, dtype=torch.uint8)
    lab = torch.randint(0, 10, (4096,), generator=g, dtype=torch.int32)
    for i in range(4096):
        band = int(lab[i])
        imgs[i, band * 78:(band + 1) * 78] = 255
    data = SyntheticMnist(0, "cuda", images=imgs, labels=lab)
    tr = MnistCnnTrainer(128, "cuda", data=data, lr=1e-3)
    run = StepGraph(tr.step, warmup=2)
    losses = []
    for _ in range(60):
        run()
        losses.append(tr.loss_sum.item() / tr.B)
    assert run.graph is not None, run.capture_error
    assert losses[-1] < 0.5 * losses[0]
    assert int(tr.global_step.item()) == 60


def test_cnn_repeated_step_grads_do_not_accumulate():
    """Only the atomically-accumulated grads are cleared per step (fused into the batch gather);
    every other gradient must be fully overwritten: the same batch twice -> the same grads,
    and the result matches autograd after a previous step left garbage behind."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    tr = MnistCnnTrainer(64, "cuda", keep_prob=1.0, seed=5)
    tr.P.grad.fill_(7.0)            # stale values everywhere
    tr.loss_sum.fill_(3.0)
    ctr0 = int(tr.data_ctr.item())
    tr.forward_backward()
    g1 = tr.P.grad.clone()
    l1 = tr.loss_sum.clone()
    tr.data_ctr.fill_(ctr0)         # same batch again
    tr.forward_backward()
    torch.cuda.synchronize()
    assert torch.allclose(tr.P.grad, g1, rtol=1e-4, atol=1e-6)
    assert torch.allclose(tr.loss_sum, l1, rtol=1e-5)
    loss_ref, grads = _reference_grads(tr)
    assert abs(tr.loss_sum.item() / tr.B - loss_ref) < 2e-2 * max(1.0, abs(loss_ref))
    for k, gref in grads.items():
        got = tr.gw[k].detach().cpu()
        assert ((got - gref).norm() / (gref.norm() + 1e-12)).item() < 3e-2, k


def test_cnn_fused_sampling_conv1_matches_separate_gather():
    """B >= 256: batch sampling + accumulator clearing fused into conv1's forward launch must
    give the same batch, labels, activations and gradients as gather kernel + conv1."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    res = {}
    for fused in ("1", "0"):
        tr = MnistCnnTrainer(256, "cuda", keep_prob=1.0, seed=7)
        tr.fused_gather = fused == "1"
        tr.P.grad.fill_(5.0)
        for _ in range(2):            # second step: counter advanced once, stale accumulators cleared
            tr.forward_backward()
        torch.cuda.synchronize()
        res[fused] = dict(x=tr.x.clone(), lab=tr.labels.clone(), p1=tr.p1.clone(), g=tr.P.grad.clone(),
                          ctr=int(tr.data_ctr.item()), loss=tr.loss_sum.clone())
    a, b = res["1"], res["0"]
    assert a["ctr"] == b["ctr"] == 2
    assert torch.equal(a["x"], b["x"]) and torch.equal(a["lab"], b["lab"]) and torch.equal(a["p1"], b["p1"])
    assert torch.allclose(a["g"], b["g"], rtol=1e-4, atol=1e-6)
    assert abs(a["loss"].item() - b["loss"].item()) <= 1e-5 * abs(b["loss"].item())


def _reference_grads_on(trainer, device):
    """_reference_grads with the fp32 oracle on ``device`` (the bench-sized batches)."""
    P, n = trainer.P, trainer.names
    x = trainer.x.float().permute(0, 3, 1, 2).to(device)
    y = trainer.labels.long().to(device)

    def w(k):
        return P.view(n[k]).detach().to(device).to(torch.bfloat16).float().requires_grad_(True)

    def b(k):
        return P.view(n[k]).detach().to(device).float().requires_grad_(True)

    wc1, wc2, wd1, wo = w("wc1"), w("wc2"), w("wd1"), w("out")
    bc1, bc2, bd1, bo = b("bc1"), b("bc2"), b("bd1"), b("bout")
    with torch.backends.cudnn.flags(enabled=True, allow_tf32=False):
        z = F.conv2d(x, wc1.permute(0, 3, 1, 2), bc1, padding=2)
        z = q(F.max_pool2d(F.relu(z), 2))
        z = F.conv2d(z, wc2.permute(0, 3, 1, 2), bc2, padding=2)
        z = q(F.max_pool2d(F.relu(z), 2))
        z = z.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
        h = F.relu(q(z @ wd1.t() + bd1))
        logits = h @ wo.t() + bo
        loss = F.cross_entropy(logits, y)
        loss.backward()
    return loss.item(), {"wc1": wc1.grad, "wc2": wc2.grad, "wd1": wd1.grad, "out": wo.grad,
                         "bc1": bc1.grad, "bc2": bc2.grad, "bd1": bd1.grad, "bout": bo.grad}


@pytest.mark.parametrize("B", [512, 1024])
def test_cnn_bench_shaped_step_matches_autograd(B):
    """The headline configuration itself (bench.py: B=1024 per GPU, fused gather+conv1 launch,
    split-K head wgrad with splits=8, conv2 blocks=128 on the side branch), dropout off, against
    fp32 autograd of the same bf16-rounded network."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    tr = MnistCnnTrainer(B, "cuda", keep_prob=1.0, seed=11)
    assert tr.fused_gather and tr.par
    tr.P.grad.fill_(3.0)               # stale values: every gradient must be overwritten / cleared
    tr.forward_backward()
    torch.cuda.synchronize()
    loss_ref, grads = _reference_grads_on(tr, "cuda")
    loss = tr.loss_sum.item() / tr.B
    assert abs(loss - loss_ref) < 2e-2 * max(1.0, abs(loss_ref)), (loss, loss_ref)
    errs = {k: ((tr.gw[k].detach().float() - g).norm() / (g.norm() + 1e-12)).item() for k, g in grads.items()}
    assert all(e < 3e-2 for e in errs.values()), sorted(errs.items(), key=lambda kv: -kv[1])


def test_cnn_adam_step_matches_torch_adam_tf1_form():
    """One fused apply_gradients launch over all 3.27 M parameters (master, Adam slots, bf16 and
    transposed bf16 copies) against torch.optim.Adam on the same gradients.  TF1 Adam
    (lr_t = lr*sqrt(1-b2^t)/(1-b1^t), v -= lr_t*m/(sqrt(v)+eps)) is torch's Adam with
    eps_torch = eps / sqrt(1 - b2^t)."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    tr = MnistCnnTrainer(1024, "cuda", keep_prob=0.75, seed=13)
    tr.forward_backward()
    torch.cuda.synchronize()
    p0 = tr.P.master.detach().clone()
    g = tr.P.grad.detach().clone()
    tr.opt.step(gscale=1.0)
    torch.cuda.synchronize()
    ref = p0.clone().requires_grad_(True)
    ref.grad = g.clone()
    b1, b2, eps = 0.9, 0.999, 1e-8
    opt = torch.optim.Adam([ref], lr=1e-3, betas=(b1, b2), eps=eps / (1 - b2) ** 0.5)
    opt.step()
    got = tr.P.master.detach()
    mask = g != 0   # padding between variables stays untouched
    err = (got - ref.detach())[mask].abs().max().item()
    assert err < 2e-6, err
    assert torch.equal(got[~mask], p0[~mask])
    # beta powers and global step advanced once
    assert torch.allclose(tr.opt.beta_pow.cpu(), torch.tensor([b1 * b1, b2 * b2]))
    assert int(tr.global_step.item()) == 1
    # bf16 working copies written by the same launch
    P, n = tr.P, tr.names
    for k in ("wc1", "wc2", "wd1", "out"):
        assert torch.equal(P.w16[n[k]], P.view(n[k]).to(torch.bfloat16)), k
    R, T, C = P.spec(n["wc2"]).transpose
    wt = P.view(n["wc2"]).reshape(R, T, C).permute(2, 1, 0).reshape(-1).to(torch.bfloat16)
    assert torch.equal(P.wt16[n["wc2"]], wt)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [256, 1024])
def test_cnn_training_is_bitwise_reproducible(B):
    """Two trainers with the same seed follow the same trajectory bit for bit: every reduction of
    the step (split-K combines, conv weight-gradient partial sums) runs in a fixed order, no
    float atomics - the property the data-parallel replicas_identical check builds on."""
    from dtfe.models.mnist_cnn import MnistCnnTrainer

    outs = []
    for _ in range(2):
        tr = MnistCnnTrainer(B, "cuda", seed=5)
        for _ in range(5):
            tr.step()
        torch.cuda.synchronize()
        outs.append(tr.P.master.clone())
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())


def test_cnn_evaluate_matches_argmax_agreement():
    """CnnProgram.evaluate (the Test-Accuracy line) = argmax agreement of the no-dropout forward
    with fp32 autograd's logits on a fixed batch, including a padded last chunk."""
    from dtfe.models.mnist_cnn import MnistCnnModel

    model = MnistCnnModel()
    prog = model.program(torch.device("cuda"), 64, seed=2)
    g = torch.Generator().manual_seed(1)
    n = 100
    imgs = torch.rand(n, 784, generator=g).cuda()
    lab = torch.nn.functional.one_hot(torch.randint(0, 10, (n,), generator=g), 10).float().cuda()
    acc = prog.evaluate(imgs, lab)
    c = prog.core
    assert c.loss_sum.item() == 0.0 and int(c.correct.item()) == 0
    hits = 0
    for lo in range(0, n, 64):
        m = min(64, n - lo)
        idx = torch.arange(lo, lo + 64).clamp_max(n - 1)
        prog.load_batch((imgs[idx.cuda()], lab[idx.cuda()]))
        c.forward(keep=1.0, logits=c.logits)
        torch.cuda.synchronize()
        _, logits_ref = _reference_forward(c)
        hits += int((logits_ref[:m].argmax(1).cuda() == lab[lo:lo + m].argmax(1)).sum())
    # the bf16 forward can flip a near-tie: allow one row of slack in 100
    assert abs(acc * n - hits) <= 1, (acc, hits / n)


def _reference_forward(trainer):
    P, n = trainer.P, trainer.names
    x = trainer.x.float().permute(0, 3, 1, 2).cpu()

    def w(k):
        return P.view(n[k]).detach().cpu().to(torch.bfloat16).float()

    def b(k):
        return P.view(n[k]).detach().cpu().float()

    z = F.conv2d(x, w("wc1").permute(0, 3, 1, 2), b("bc1"), padding=2)
    z = q(F.max_pool2d(F.relu(z), 2))
    z = F.conv2d(z, w("wc2").permute(0, 3, 1, 2), b("bc2"), padding=2)
    z = q(F.max_pool2d(F.relu(z), 2))
    z = z.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    h = q(F.relu(z @ w("wd1").t() + b("bd1")))
    return h, h @ w("out").t() + b("bout")


def test_cnn_fp32_step_matches_fp32_autograd():
    """--dtype fp32: the exact-fp32 MFMA step (conv_f32.hip convs, fp32 dense GEMMs, softmax-xent)
    against fp32 autograd of the same network on the CPU, dropout off: <= 1e-4 relative."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_cnn_cpu import _batch, autograd_f32
    from dtfe.models.mnist_cnn import MnistCnnModel

    m = MnistCnnModel()
    m.set_dtype("fp32")
    prog = m.program(torch.device("cuda"), 128, seed=3)
    prog.core.keep = 1.0
    x, y = _batch(128, seed=2)
    prog.load_batch((x.cuda(), y.cuda()))
    prog.P.grad.fill_(9.0)             # stale values: stored gradients overwritten, accumulated ones cleared
    met = prog.compute_grads()
    torch.cuda.synchronize()
    core = prog.core
    cpu = type("C", (), {})()
    cpu.P = type("P", (), {"view": staticmethod(lambda k: core.P.view(k).cpu())})()
    cpu.names, cpu.x, cpu.labels = core.names, core.x.cpu(), core.labels.cpu()
    loss_ref, grads, _ = autograd_f32(cpu)
    assert abs(met["loss"].item() - loss_ref) <= 1e-5 * abs(loss_ref), (met["loss"].item(), loss_ref)
    errs = {k: ((core.gw[k].cpu() - g).norm() / (g.norm() + 1e-12)).item() for k, g in grads.items()}
    assert all(e <= 1e-4 for e in errs.values()), sorted(errs.items(), key=lambda kv: -kv[1])


def test_cnn_fp32_local_run_trains(capsys, tmp_path):
    """train.run with --dtype fp32 on the GPU (local mode, hipGraph-captured step): loss lines and
    the Test-Accuracy line print, the global step advances."""
    from dtfe import train

    rc = train.run("cnn", ["--mode=local", "--device=cuda", "--synthetic", "--num_steps=4", "--dtype=fp32",
                           "--batch_size=64", "--save_model_secs=0", "--model_dir=" + str(tmp_path / "ck")])
    out = capsys.readouterr().out
    assert rc == 0
    assert "Global step 4 Local step 3" in out and "Test-Accuracy: " in out, out[-2000:]
