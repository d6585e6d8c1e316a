"""MNIST autoencoder (reference ``encoder/distributed_encoder.py``).

784 -> 256 -> 128 -> 256 -> 784, sigmoid after every layer (ENC:67-85);
weights AND biases ~ N(0, 1); loss = mean((x - y)^2) (ENC:135);
TF1 RMSProp(0.01): decay 0.9, momentum 0, eps 1e-10, ms slot initialised to 1.

MI355X step program (fp32, exact-fp32 MFMA): 4 fused GEMM+bias+sigmoid
forward kernels, a fused MSE+sigmoid-grad kernel (one launch, the last workgroup stores
the loss), and per layer one wgrad
GEMM (bias gradient through a ones row) + one dgrad GEMM whose epilogue applies
sigmoid'(a) of the layer below (TF's SigmoidGrad fused away), the pair as ONE
launch.
"""
from __future__ import annotations

import torch

from .. import ops
from ..optim import OptimizerConfig, VarSpec
from .base import ModelDef, StepProgram, normal_init, tf_auto_names

DIMS = [784, 256, 128, 256, 784]
LR = 0.01


class AutoencoderModel(ModelDef):
    name = "encoder"
    default_batch = 256
    default_steps = 100000
    needs_labels = False

    def __init__(self, lr: float = LR):
        keys = ["encoder_h1", "encoder_h2", "decoder_h1", "decoder_h2",
                "encoder_b1", "encoder_b2", "decoder_b1", "decoder_b2", "global_step"]
        self.names = tf_auto_names(keys)
        shapes = {}
        for i, k in enumerate(keys[:4]):
            shapes[k] = (DIMS[i], DIMS[i + 1])
        for i, k in enumerate(keys[4:8]):
            shapes[k] = (DIMS[i + 1],)
        self.specs = [VarSpec(self.names[k], shapes[k], normal_init(1.0)) for k in keys[:-1]]
        self.var_order = [self.names[k] for k in keys]
        self.gs_name = self.names["global_step"]
        self.opt_groups = [(OptimizerConfig(kind="rmsprop", lr=lr, rho=0.9, momentum=0.0),
                            [s.name for s in self.specs], ("beta1_power", "beta2_power"))]
        self.w_keys = keys[:4]
        self.b_keys = keys[4:8]

    def program(self, device, batch_size=None, seed: int = 0):
        return AutoencoderProgram(self, device, batch_size or self.default_batch, seed)


class AutoencoderProgram(StepProgram):
    def __init__(self, model: AutoencoderModel, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        B = batch_size
        f = dict(device=self.device, dtype=torch.float32)
        self.x = torch.empty(B, DIMS[0], **f)
        self.a = [torch.empty(B, d, **f) for d in DIMS[1:]]
        self.dz = [torch.empty(B, d, **f) for d in DIMS[1:]]
        self.loss = torch.zeros(1, **f)
        self.mse_ws = torch.zeros(ops.MSE_WS_FLOATS, **f) if self.device.type == "cuda" else None
        self.xin = self.x  # the batch the layers read: self.x, or the caller's tensor in a captured step
        n = model.names
        self.W = [self.P.view(n[k]) for k in model.w_keys]
        self.b = [self.P.view(n[k]) for k in model.b_keys]
        self.gW = [self.P.gview(n[k]) for k in model.w_keys]
        self.gb = [self.P.gview(n[k]) for k in model.b_keys]

    def load_batch(self, batch):
        x = batch[0] if isinstance(batch, (tuple, list)) else batch
        x = x.reshape(self.batch_size, DIMS[0])
        if (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.data_ptr() % 16 == 0
                and torch.cuda.is_current_stream_capturing()):
            # batch load captured with the step (bench/ref_models.py): the layers read the caller's tensor
            # in place - no staging copy node.  An eager load before a graph replay (train.py) must copy.
            self.xin = x
            return
        self.x.copy_(x)
        self.xin = self.x

    def forward(self):
        B = self.batch_size
        inp = self.xin
        for i in range(4):
            ops.gemm(inp, self.W[i], self.a[i], M=B, N=DIMS[i + 1], K=DIMS[i], bmode=ops.RMAJ, ldb=DIMS[i + 1],
                     bias=self.b[i], act=ops.ACT_SIGMOID)
            inp = self.a[i]
        return self.a[3]

    def compute_grads(self):
        B = self.batch_size
        # no P.grad.zero_(): every gradient element is stored (not accumulated) by this step's kernels
        y = self.forward()
        ops.mse_sigmoid(y, self.xin, self.loss, self.dz[3], ws=self.mse_ws)
        for i in range(3, -1, -1):
            inp = self.xin if i == 0 else self.a[i - 1]
            # a layer's weight and data gradients are independent: one paired launch (ops.gemm_group)
            with ops.gemm_group(self.loss):
                # dW_i[K][N] = inp^T . dz_i ; db_i = sum_b dz_i through the GEMM's ones row (no colsum launch)
                ops.gemm(inp, self.dz[i], self.gW[i], M=DIMS[i] + 1, N=DIMS[i + 1], K=B, amode=ops.RMAJ,
                         lda=DIMS[i], bmode=ops.RMAJ, ldb=DIMS[i + 1], a_ones_row=DIMS[i], bias_out=self.gb[i])
                if i > 0:
                    # dz_{i-1} = (dz_i . W_i^T) * sigmoid'(a_{i-1})
                    ops.gemm(self.dz[i], self.W[i], self.dz[i - 1], M=B, N=DIMS[i], K=DIMS[i + 1],
                             bmode=ops.KMAJ, ldb=DIMS[i + 1], aux=self.a[i - 1], aux_act=ops.ACT_SIGMOID)
        return {"loss": self.loss}
