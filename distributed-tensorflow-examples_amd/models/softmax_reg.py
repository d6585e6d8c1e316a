"""MNIST softmax (logistic) regression - BASELINE.json config 1 ([NS]).

784 -> 10 linear + softmax cross-entropy, GradientDescent(0.01), batch 100,
zero-initialised W/b (TensorFlow-Examples ``logistic_regression``).
Runs on CPU/gloo as the plumbing configuration and on the GPU kernels alike.
"""
from __future__ import annotations

import torch

from .. import ops
from ..optim import OptimizerConfig, VarSpec
from .base import ModelDef, ScaledScalar, StepProgram, zeros_init

IMG, NC = 784, 10


class SoftmaxRegressionModel(ModelDef):
    name = "softmax"
    default_batch = 100
    default_steps = 10000

    def __init__(self, lr: float = 0.01):
        self.specs = [VarSpec("Variable", (IMG, NC), zeros_init), VarSpec("Variable_1", (NC,), zeros_init)]
        self.var_order = ["Variable", "Variable_1", "Variable_2"]
        self.gs_name = "Variable_2"
        self.opt_groups = [(OptimizerConfig(kind="sgd", lr=lr), ["Variable", "Variable_1"],
                            ("beta1_power", "beta2_power"))]

    def program(self, device, batch_size=None, seed: int = 0):
        return SoftmaxProgram(self, device, batch_size or self.default_batch, seed)


class SoftmaxProgram(StepProgram):
    def __init__(self, model, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        B = batch_size
        f = dict(device=self.device, dtype=torch.float32)
        self.x = torch.empty(B, IMG, **f)
        self.y = torch.empty(B, NC, **f)
        self.logits = torch.empty(B, NC, **f)
        self.dlogits = torch.empty(B, NC, **f)
        self.loss = torch.zeros(1, **f)
        self.correct = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.W, self.b = self.P.view("Variable"), self.P.view("Variable_1")
        self.gW, self.gb = self.P.gview("Variable"), self.P.gview("Variable_1")

    def load_batch(self, batch):
        x, y = batch
        self.x.copy_(x.reshape(self.batch_size, IMG))
        self.y.copy_(y.reshape(self.batch_size, NC))

    def compute_grads(self):
        B = self.batch_size
        # no P.grad.zero_(): every gradient element is stored (not accumulated) by this step's kernels
        self.loss.zero_()
        self.correct.zero_()
        ops.gemm(self.x, self.W, self.logits, M=B, N=NC, K=IMG, bmode=ops.RMAJ, ldb=NC, bias=self.b)
        ops.softmax_xent(self.logits, labels_oh=self.y, scale=1.0 / B, dlogits=self.dlogits, loss_sum=self.loss,
                         correct=self.correct)
        ops.gemm(self.x, self.dlogits, self.gW, M=IMG + 1, N=NC, K=B, amode=ops.RMAJ, lda=IMG, bmode=ops.RMAJ,
                 ldb=NC, a_ones_row=IMG, bias_out=self.gb)
        return {"loss": ScaledScalar(self.loss, 1.0 / B)}

    def evaluate(self, images, labels) -> float:
        n = images.shape[0]
        x = images.to(self.device).reshape(n, IMG).float()
        logits = torch.empty(n, NC, device=self.device)
        ops.gemm(x, self.W, logits, M=n, N=NC, K=IMG, bmode=ops.RMAJ, ldb=NC, bias=self.b)
        corr = torch.zeros(1, dtype=torch.int32, device=self.device)
        ops.softmax_xent(logits, labels_oh=labels.to(self.device).float().reshape(n, NC), correct=corr)
        return int(corr.item()) / n
