"""The explicit step programs' hand-written backward passes vs torch autograd (CPU, fp32).

Each model's compute_grads() (ops reference path on CPU) must equal the
gradient of the reference loss built with plain torch ops on the same
parameters and batch - this pins the math the HIP kernels implement.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dtfe.models.autoencoder import AutoencoderModel
from dtfe.models.gan import GanModel
from dtfe.models.lstm import LstmModel
from dtfe.models.softmax_reg import SoftmaxRegressionModel


def _params(prog, names):
    return {n: prog.P.view(n).detach().clone().requires_grad_(True) for n in names}


def _check(prog, p, atol=1e-5, rtol=1e-4):
    for n, t in p.items():
        got = prog.P.gview(n)
        assert t.grad is not None, n
        assert torch.allclose(got, t.grad, atol=atol, rtol=rtol), (n, (got - t.grad).abs().max().item())


def test_softmax_regression_grads():
    torch.manual_seed(0)
    m = SoftmaxRegressionModel()
    prog = m.program("cpu", 16)
    prog.P.view("Variable").normal_()
    x = torch.rand(16, 784)
    y = F.one_hot(torch.randint(0, 10, (16,)), 10).float()
    prog.load_batch((x, y))
    prog.compute_grads()
    p = _params(prog, ["Variable", "Variable_1"])
    loss = F.cross_entropy(x @ p["Variable"] + p["Variable_1"], y.argmax(1))
    loss.backward()
    _check(prog, p)


def test_autoencoder_grads():
    torch.manual_seed(1)
    m = AutoencoderModel()
    prog = m.program("cpu", 8, seed=3)
    x = torch.rand(8, 784)
    prog.load_batch(x)
    out = prog.compute_grads()
    names = [s.name for s in m.specs]
    p = _params(prog, names)
    a = x
    for i in range(4):
        a = torch.sigmoid(a @ p[names[i]] + p[names[4 + i]])
    loss = ((x - a) ** 2).mean()
    loss.backward()
    assert abs(float(out["loss"]) - loss.item()) < 1e-5
    _check(prog, p)


def test_gan_grads_both_losses_same_snapshot():
    torch.manual_seed(2)
    m = GanModel()
    prog = m.program("cpu", 8, seed=4)
    x = torch.rand(8, 784)
    prog.load_batch(x)
    z = prog.z.clone()
    out = prog.compute_grads()
    n = m.names
    p = _params(prog, [s.name for s in m.specs])

    def G(zz):
        h = F.relu(zz @ p[n["Wg1"]] + p[n["bg1"]])
        return torch.sigmoid(h @ p[n["Wg2"]] + p[n["bg2"]])

    def D(xx):
        h = F.relu(xx @ p[n["Wd1"]] + p[n["bd1"]])
        return torch.sigmoid(h @ p[n["Wd2"]] + p[n["bd2"]])

    fake = G(z)
    gen_loss = -torch.log(D(fake)).mean()
    disc_loss = -(torch.log(D(x)) + torch.log(1.0 - D(fake))).mean()
    gen_vars = [n[k] for k in ("Wg1", "Wg2", "bg1", "bg2")]
    disc_vars = [n[k] for k in ("Wd1", "Wd2", "bd1", "bd2")]
    gg = torch.autograd.grad(gen_loss, [p[v] for v in gen_vars], retain_graph=True)
    gd = torch.autograd.grad(disc_loss, [p[v] for v in disc_vars])
    for v, g in list(zip(gen_vars, gg)) + list(zip(disc_vars, gd)):
        got = prog.P.gview(v)
        assert torch.allclose(got, g, atol=1e-5, rtol=1e-4), (v, (got - g).abs().max().item())
    assert abs(float(out["gen_loss"]) - gen_loss.item()) < 1e-5
    assert abs(float(out["disc_loss"]) - disc_loss.item()) < 1e-5


def _tf_basic_lstm(x, K, b, H, forget_bias=1.0):
    B, T, _ = x.shape
    h = torch.zeros(B, H)
    c = torch.zeros(B, H)
    for t in range(T):
        g = torch.cat([x[:, t], h], 1) @ K + b
        i, j, f, o = g.split(H, 1)
        c = c * torch.sigmoid(f + forget_bias) + torch.sigmoid(i) * torch.tanh(j)
        h = torch.tanh(c) * torch.sigmoid(o)
    return h


def test_lstm_grads_and_eval():
    torch.manual_seed(3)
    m = LstmModel()
    prog = m.program("cpu", 4, seed=5)
    x = torch.rand(4, 784)
    lab = torch.tensor([1, 7, 3, 3])
    y = F.one_hot(lab, 10).float()
    prog.load_batch((x, y))
    out = prog.compute_grads()
    p = _params(prog, [s.name for s in m.specs])
    h = _tf_basic_lstm(x.view(4, 28, 28), p[m.kname], p[m.bname], 128)
    logits = h @ p["Variable"] + p["Variable_1"]
    loss = F.cross_entropy(logits, lab)
    loss.backward()
    assert abs(float(out["loss"]) - loss.item()) < 1e-5
    _check(prog, p, atol=1e-5, rtol=1e-3)
    acc = prog.evaluate(x, y)
    assert acc == pytest.approx(float((logits.argmax(1) == lab).float().mean()))


def test_var_order_and_names_match_survey():
    # SURVEY §2.9 tables
    g = GanModel()
    assert g.var_order == ["Variable"] + ["Variable_%d" % i for i in range(1, 9)]
    assert g.gs_name == "Variable_8"
    shapes = {s.name: s.shape for s in g.specs}
    assert shapes["Variable"] == (100, 256) and shapes["Variable_3"] == (256, 1) and shapes["Variable_7"] == (1,)
    e = AutoencoderModel()
    assert {s.name: s.shape for s in e.specs}["Variable_3"] == (256, 784)
    lm = LstmModel()
    assert lm.var_order == ["Variable", "Variable_1", "rnn/basic_lstm_cell/kernel", "rnn/basic_lstm_cell/bias",
                            "Variable_2"]
    assert {s.name: s.shape for s in lm.specs}["rnn/basic_lstm_cell/kernel"] == (156, 512)
    assert sum(s.numel for s in g.specs) == 428561
    assert sum(s.numel for s in e.specs) == 468368
    assert sum(s.numel for s in lm.specs) == 81674


def test_glorot_init_is_he_normal_like_reference():
    # glorot_init = random_normal(stddev = 1/sqrt(shape[0]/2)) (GAN:72-73)
    from dtfe.models.gan import glorot_init

    w = glorot_init((784, 256), torch.Generator().manual_seed(0))
    assert abs(w.std().item() - np.sqrt(2 / 784)) < 2e-3


def test_gan_disc_head_oracle_matches_autograd():
    """ops.gan_disc_head's CPU path (the oracle its GPU kernel is checked against) vs torch autograd of the
    reference losses (GAN:128-143): p = sigmoid(d1 Wd2 + bd2); gen_loss = -mean(log p_fake); disc_loss =
    -mean(log p_real + log(1 - p_fake)); gradients w.r.t. Wd2, bd2 and d1 (split into the disc / gen parts)."""
    from dtfe import ops
    B, DH = 6, 12
    g = torch.Generator().manual_seed(2)
    d1 = torch.relu(torch.randn(2 * B, DH, generator=g, dtype=torch.float64))
    w = torch.randn(DH, 1, generator=g, dtype=torch.float64)
    b = torch.randn(1, generator=g, dtype=torch.float64)
    z = lambda *s: torch.zeros(*s, dtype=torch.float64)  # noqa: E731
    o = dict(p=z(2 * B, 1), dlog=z(2 * B, 1), dlog_g=z(B, 1), gw=z(DH, 1), gb=z(1), dd1=z(2 * B, DH), ddf=z(B, DH),
             gen=z(1), disc=z(1))
    assert ops.gan_disc_head(d1, w, b, o["p"], o["dlog"], o["dlog_g"], o["gw"], o["gb"], o["dd1"], o["ddf"], o["gen"],
                             o["disc"])
    x, wv, bv = d1.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    p = torch.sigmoid(x @ wv + bv).view(-1)
    disc = -(torch.log(p[:B]) + torch.log(1 - p[B:])).mean()
    gw, gb, gx = torch.autograd.grad(disc, (wv, bv, x), retain_graph=True)
    gen = -torch.log(p[B:]).mean()
    gxg, = torch.autograd.grad(gen, (x,))
    mask = (d1 > 0).double()  # relu'(d1) as the backward through the hidden ReLU sees it
    torch.testing.assert_close(o["p"].view(-1), p.detach())
    torch.testing.assert_close(o["disc"], disc.detach().view(1))
    torch.testing.assert_close(o["gen"], gen.detach().view(1))
    torch.testing.assert_close(o["gw"], gw)
    torch.testing.assert_close(o["gb"], gb)
    torch.testing.assert_close(o["dd1"], gx * mask)
    torch.testing.assert_close(o["ddf"], gxg[B:] * mask[B:])
