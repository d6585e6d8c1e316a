"""MNIST GAN (reference ``gan/distributed_gan.py``).

G: z[B,100] -> Dense 256 ReLU -> Dense 784 sigmoid
D: x[B,784] -> Dense 256 ReLU -> Dense 1 sigmoid   (applied to real and fake)
gen_loss  = -mean(log D(G(z)))                         (GAN:142)
disc_loss = -mean(log D(x) + log(1 - D(G(z))))         (GAN:143)
Two TF1 Adams (lr 2e-4) over disjoint var_lists, both advancing global_step
(so it moves by 2 per iteration, GAN:158-159).

MI355X step program (fp32, exact-fp32 MFMA GEMMs):
  noise (device hash RNG) -> G (2 fused GEMM+bias+act) -> D's hidden layer on
  the stacked [real; fake] batch (one 2B-row GEMM) -> ONE discriminator-head
  kernel (output layer, both losses, dWd2 and the gradients at d1) ->
  backward of both losses from the SAME parameter snapshot.  The reference
  runs train_gen / train_disc unordered in one sess.run (a race);
  here both gradients come from one snapshot and the ps applies them in a
  fixed order (disc then gen), deterministically.
"""
from __future__ import annotations

import torch

from .. import ops
from ..optim import OptimizerConfig, VarSpec
from .base import ModelDef, StepProgram, tf_auto_names, zeros_init

NOISE, GH, IMG, DH = 100, 256, 784, 256
LR = 0.0002


def glorot_init(shape, g):
    # reference glorot_init: random_normal(stddev = 1/sqrt(shape[0]/2)) (GAN:72-73)
    return torch.randn(*shape, generator=g) / (shape[0] / 2.0) ** 0.5


class GanModel(ModelDef):
    name = "gan"
    default_batch = 128
    default_steps = 100000
    gs_increments = 2
    needs_labels = False

    def __init__(self, lr: float = LR):
        keys = ["Wg1", "Wg2", "Wd1", "Wd2", "bg1", "bg2", "bd1", "bd2", "global_step"]
        self.names = tf_auto_names(keys)
        shapes = {"Wg1": (NOISE, GH), "Wg2": (GH, IMG), "Wd1": (IMG, DH), "Wd2": (DH, 1),
                  "bg1": (GH,), "bg2": (IMG,), "bd1": (DH,), "bd2": (1,)}
        self.specs = [VarSpec(self.names[k], shapes[k], glorot_init if k.startswith("W") else zeros_init)
                      for k in keys[:-1]]
        self.var_order = [self.names[k] for k in keys]
        self.gs_name = self.names["global_step"]
        n = self.names
        gen_vars = [n["Wg1"], n["Wg2"], n["bg1"], n["bg2"]]
        disc_vars = [n["Wd1"], n["Wd2"], n["bd1"], n["bd2"]]
        # TF names the second Adam's non-slot variables beta1_power_1 / beta2_power_1
        self.opt_groups = [
            (OptimizerConfig(kind="adam", lr=lr), disc_vars, ("beta1_power_1", "beta2_power_1")),
            (OptimizerConfig(kind="adam", lr=lr), gen_vars, ("beta1_power", "beta2_power")),
        ]

    def program(self, device, batch_size=None, seed: int = 0):
        return GanProgram(self, device, batch_size or self.default_batch, seed)


class GanProgram(StepProgram):
    def __init__(self, model: GanModel, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        B, d = batch_size, self.device
        f = dict(device=d, dtype=torch.float32)
        self.z = torch.empty(B, NOISE, **f)
        self.xx = torch.empty(2 * B, IMG, **f)        # [real; fake]
        self.h1 = torch.empty(B, GH, **f)
        self.d1 = torch.empty(2 * B, DH, **f)
        self.p = torch.empty(2 * B, 1, **f)
        self.dlog = torch.empty(2 * B, 1, **f)          # d disc_loss / d logit for [real; fake]
        self.dlog_g = torch.empty(B, 1, **f)            # d gen_loss / d logit_fake
        self.dd1 = torch.empty(2 * B, DH, **f)
        self.ddf = torch.empty(B, DH, **f)
        self.dg = torch.empty(B, IMG, **f)
        self.dh1 = torch.empty(B, GH, **f)
        self.gen_loss = torch.zeros(1, **f)
        self.disc_loss = torch.zeros(1, **f)
        self.noise_ctr = torch.zeros(1, dtype=torch.int64, device=d)
        self.noise_done = torch.zeros(1, dtype=torch.int32, device=d)
        self.seed = seed
        # the discriminator's output layer, both losses and their gradients down to d1 in one launch
        # (ops.gan_disc_head: 5 launches -> 1); GPU only
        self.head_ws = (torch.zeros(ops.gan_head_ws_floats(B, DH), **f) if self.device.type == "cuda" else None)
        n = model.names
        self.W = {k: self.P.view(n[k]) for k in ("Wg1", "Wg2", "Wd1", "Wd2", "bg1", "bg2", "bd1", "bd2")}
        self.G = {k: self.P.gview(n[k]) for k in self.W}

    def load_batch(self, batch):
        x = batch[0] if isinstance(batch, (tuple, list)) else batch
        x = x.reshape(self.batch_size, IMG)
        real = self.xx[: self.batch_size]
        # z ~ U(-1, 1) (GAN:189); device hash RNG on GPU, torch RNG on CPU.  On the GPU the real batch
        # is staged into the stacked [real; fake] buffer by the same launch.
        fused = x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.data_ptr() % 16 == 0
        if not fused:
            real.copy_(x)
        ops.uniform_fill(self.z, -1.0, 1.0, seed=self.seed, counter=self.noise_ctr, done=self.noise_done,
                         copy=(x, real) if fused else None)

    def forward(self, d2=True):
        """``d2=False``: stop at d1 (the fused discriminator head forms p itself)."""
        B, W = self.batch_size, self.W
        R = ops.RMAJ
        ops.gemm(self.z, W["Wg1"], self.h1, M=B, N=GH, K=NOISE, bmode=R, ldb=GH, bias=W["bg1"], act=ops.ACT_RELU)
        fake = self.xx[B:]
        ops.gemm(self.h1, W["Wg2"], fake, M=B, N=IMG, K=GH, bmode=R, ldb=IMG, bias=W["bg2"], act=ops.ACT_SIGMOID)
        ops.gemm(self.xx, W["Wd1"], self.d1, M=2 * B, N=DH, K=IMG, bmode=R, ldb=DH, bias=W["bd1"],
                 act=ops.ACT_RELU)
        if d2:
            ops.gemm(self.d1, W["Wd2"], self.p, M=2 * B, N=1, K=DH, bmode=R, ldb=1, bias=W["bd2"],
                     act=ops.ACT_SIGMOID)

    def compute_grads(self):
        B, W, G = self.batch_size, self.W, self.G
        R, K = ops.RMAJ, ops.KMAJ
        # no P.grad.zero_(): every gradient element is stored (not accumulated) by this step's kernels
        fused = self.head_ws is not None
        self.forward(d2=not fused)
        if fused and ops.gan_disc_head(self.d1, W["Wd2"], W["bd2"], self.p, self.dlog, self.dlog_g, G["Wd2"],
                                       G["bd2"], self.dd1, self.ddf, self.gen_loss, self.disc_loss, self.head_ws):
            pass  # p, both losses, dWd2 / dbd2, dd1 and ddf from one launch
        else:
            if fused:
                ops.gemm(self.d1, W["Wd2"], self.p, M=2 * B, N=1, K=DH, bmode=R, ldb=1, bias=W["bd2"],
                         act=ops.ACT_SIGMOID)
            ops.gan_loss(self.p[:B], self.p[B:], self.gen_loss, self.disc_loss, self.dlog[:B], self.dlog[B:],
                         self.dlog_g)
            # ---- discriminator: d disc_loss over the stacked batch
            # weight grads carry their bias grads in a ones row of A (no separate column-sum launches)
            ops.gemm(self.d1, self.dlog, G["Wd2"], M=DH + 1, N=1, K=2 * B, amode=R, lda=DH, bmode=R, ldb=1,
                     a_ones_row=DH, bias_out=G["bd2"])
            ops.gemm(self.dlog, W["Wd2"], self.dd1, M=2 * B, N=DH, K=1, amode=K, lda=1, bmode=K, ldb=1,
                     aux=self.d1, aux_act=ops.ACT_RELU)
            # (generator side: d gen_loss through D, same parameter snapshot)
            ops.gemm(self.dlog_g, W["Wd2"], self.ddf, M=B, N=DH, K=1, amode=K, lda=1, bmode=K, ldb=1,
                     aux=self.d1[B:], aux_act=ops.ACT_RELU)
        # each (weight gradient, data gradient) pair below is independent: one paired launch (ops.gemm_group)
        with ops.gemm_group(self.d1):
            ops.gemm(self.xx, self.dd1, G["Wd1"], M=IMG + 1, N=DH, K=2 * B, amode=R, lda=IMG, bmode=R, ldb=DH,
                     a_ones_row=IMG, bias_out=G["bd1"])
            # ---- generator: d gen_loss through D (same parameter snapshot)
            ops.gemm(self.ddf, W["Wd1"], self.dg, M=B, N=IMG, K=DH, amode=K, lda=DH, bmode=K, ldb=DH,
                     aux=self.xx[B:], aux_act=ops.ACT_SIGMOID)
        with ops.gemm_group(self.d1):
            ops.gemm(self.h1, self.dg, G["Wg2"], M=GH + 1, N=IMG, K=B, amode=R, lda=GH, bmode=R, ldb=IMG,
                     a_ones_row=GH, bias_out=G["bg2"])
            ops.gemm(self.dg, W["Wg2"], self.dh1, M=B, N=GH, K=IMG, amode=K, lda=IMG, bmode=K, ldb=IMG,
                     aux=self.h1, aux_act=ops.ACT_RELU)
        ops.gemm(self.z, self.dh1, G["Wg1"], M=NOISE + 1, N=GH, K=B, amode=R, lda=NOISE, bmode=R, ldb=GH,
                 a_ones_row=NOISE, bias_out=G["bg1"])
        return {"gen_loss": self.gen_loss, "disc_loss": self.disc_loss}
