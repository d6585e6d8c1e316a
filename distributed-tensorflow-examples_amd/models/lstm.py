"""MNIST row-sequence LSTM classifier (reference ``lstm/distributed_lstm.py``).

x[B,28,28] -> 28 steps of BasicLSTMCell(128, forget_bias=1.0) -> h_T . W_out + b_out
-> softmax cross-entropy; GradientDescent(0.001); accuracy on 128 test images.
Variables in creation order: Variable (W_out [128,10]), Variable_1 (b_out [10]),
rnn/basic_lstm_cell/kernel [156,512] (glorot-uniform), rnn/basic_lstm_cell/bias
[512] (zeros), Variable_2 (global_step).

MI355X step program (fp32): the per-step gate GEMM reads one [x_t, h_{t-1}]
row buffer (h_{t-1} is written straight into it by the previous cell kernel),
so each timestep is one exact-fp32 MFMA GEMM + one fused cell kernel; BPTT is
one fused cell-backward kernel + one dgrad GEMM per step, and the kernel
gradient is a single [156 x 512] GEMM reducing over all T*B rows at the end
(TF accumulates 28 separate MatMul grads).  On the GPU the whole forward
recurrence and the whole BPTT recurrence are each ONE persistent kernel
(csrc/kernels/lstm_seq.hip); the per-step path remains for the
CPU reference and unsupported shapes (DTFE_LSTM_PERSIST=0 forces it).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..optim import OptimizerConfig, VarSpec
from .base import ModelDef, ScaledScalar, StepProgram, glorot_uniform_init, normal_init, zeros_init

T, I, H, NC = 28, 28, 128, 10
LR = 0.001


class LstmModel(ModelDef):
    name = "lstm"
    default_batch = 128
    default_steps = 10000

    def __init__(self, lr: float = LR):
        self.kname, self.bname = "rnn/basic_lstm_cell/kernel", "rnn/basic_lstm_cell/bias"
        self.specs = [
            VarSpec("Variable", (H, NC), normal_init(1.0)),
            VarSpec("Variable_1", (NC,), normal_init(1.0)),
            VarSpec(self.kname, (I + H, 4 * H), glorot_uniform_init),
            VarSpec(self.bname, (4 * H,), zeros_init),
        ]
        self.var_order = ["Variable", "Variable_1", self.kname, self.bname, "Variable_2"]
        self.gs_name = "Variable_2"
        self.opt_groups = [(OptimizerConfig(kind="sgd", lr=lr), [s.name for s in self.specs],
                            ("beta1_power", "beta2_power"))]

    def program(self, device, batch_size=None, seed: int = 0):
        return LstmProgram(self, device, batch_size or self.default_batch, seed)


class LstmProgram(StepProgram):
    def __init__(self, model: LstmModel, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        B = batch_size
        f = dict(device=self.device, dtype=torch.float32)
        self.xh = torch.zeros(T, B, I + H, **f)      # [x_t, h_{t-1}] rows
        self.gates = torch.empty(T, B, 4 * H, **f)
        self.act = torch.empty(T, B, 4 * H, **f)
        self.c = torch.empty(T, B, H, **f)
        self.hT = torch.empty(B, H, **f)
        self.logits = torch.empty(B, NC, **f)
        self.y = torch.empty(B, NC, **f)
        self.dlogits = torch.empty(B, NC, **f)
        self.dh = torch.empty(B, H, **f)
        self.dc = torch.empty(B, H, **f)
        self.dg = torch.empty(T, B, 4 * H, **f)
        self.loss = torch.zeros(1, **f)
        self.correct = torch.zeros(1, dtype=torch.int32, device=self.device)
        m = model
        self.Wo, self.bo = self.P.view("Variable"), self.P.view("Variable_1")
        self.K, self.b = self.P.view(m.kname), self.P.view(m.bname)
        self.gWo, self.gbo = self.P.gview("Variable"), self.P.gview("Variable_1")
        self.gK, self.gb = self.P.gview(m.kname), self.P.gview(m.bname)
        # the kernel gradient's own split-K workspace (DTFE_LSTM_TALLK=0: the generic GEMM instead)
        self.k_splits = 32  # tall-K kernel-gradient splits (profiles/r2_lstm_wgrad_sweep.txt)
        self.ws_k = None
        if self.device.type == "cuda" and os.environ.get("DTFE_LSTM_TALLK", "1") != "0":
            self.ws_k = torch.empty(ops.tallk_ws_floats(I + H, 4 * H, self.k_splits), **f)
        self._stage = None  # (x, y) of a batch the next forward launch stages (load_batch, GPU)

    def load_batch(self, batch):
        x, y = batch
        B = self.batch_size
        # batch_x.reshape((B, timesteps, num_input)) (LSTM:127): row t of the image is step t.
        # One launch stages x, zeroes h_{-1}, copies the labels and clears the step's loss / hit
        # accumulators (compute_grads then skips its own clearing) - on the GPU the forward launch itself
        # (the split recurrence reads x_t from the images and writes xh in its prologue) when the load is
        # captured together with the step.
        if x.dtype == torch.float32 and y.dtype == torch.float32 and x.numel() == B * T * I and y.numel() == B * NC:
            if (self._persistent() and x.is_contiguous() and y.is_contiguous()
                    and torch.cuda.is_current_stream_capturing()):
                # batch load captured with the step (bench/ref_models.py): staged by the forward launch itself
                # (lstm_seq_fwd xsrc: seq_stage folded in).  An eager load_batch before a graph replay
                # (train.py) must stage now - the replayed forward would not see a later batch.
                self._stage = (x, y)
            else:
                ops.seq_stage(x, self.xh, T, I, y, self.y, zero=(self.loss, self.correct))
            self._acc_cleared = True
            return
        self.xh[:, :, :I].copy_(x.reshape(B, T, I).transpose(0, 1))
        self.xh[0, :, I:].zero_()
        self.y.copy_(y.reshape(B, NC))

    def _persistent(self):
        return self.device.type == "cuda" and os.environ.get("DTFE_LSTM_PERSIST", "1") != "0"

    def forward(self, head=False):
        """``head`` (compute_grads, GPU): the classifier head forward + backward as ONE single-workgroup
        launch (ops.dense_head: logits, softmax-xent, dW_out / db_out stored, dh) instead of the head
        GEMM, softmax_xent and two gradient GEMMs; returns whether it ran."""
        B = self.batch_size
        st, self._stage = self._stage, None
        if st is not None:  # the batch load_batch left for this launch to stage
            xs, ys, ydst, z0, z1 = st[0], st[1], self.y, self.loss, self.correct
        else:
            xs = ys = ydst = z0 = z1 = None
        if self._persistent() and ops.require().lstm_seq_fwd(self.xh, self.K, self.b, 1.0, self.act, self.c,
                                                               self.hT, xs, ys, ydst, z0, z1):
            # (dfeat = dh_T is formed by the BPTT kernel from these dlogits: lstm_seq_bwd(dl=...))
            if head and ops.dense_head(self.hT, self.Wo, self.bo, self.y, self.logits, self.loss, self.correct,
                                       self.gWo, self.gbo, None, 1.0 / B, w_fmajor=True, store=True,
                                       dl_out=self.dlogits):
                return True
            ops.gemm(self.hT, self.Wo, self.logits, M=B, N=NC, K=H, bmode=ops.RMAJ, ldb=NC, bias=self.bo)
            return False
        if st is not None:
            ops.seq_stage(st[0], self.xh, T, I, st[1], self.y, zero=(self.loss, self.correct))
        for t in range(T):
            ops.gemm(self.xh[t], self.K, self.gates[t], M=B, N=4 * H, K=I + H, bmode=ops.RMAJ, ldb=4 * H,
                     bias=self.b)
            if t + 1 < T:
                h_out, ld = self.xh[t + 1, :, I:], I + H
            else:
                h_out, ld = self.hT, H
            ops.lstm_cell_fwd(self.gates[t], self.act[t], self.c[t - 1] if t > 0 else None, self.c[t], h_out, ld,
                              1.0)
        ops.gemm(self.hT, self.Wo, self.logits, M=B, N=NC, K=H, bmode=ops.RMAJ, ldb=NC, bias=self.bo)

    def compute_grads(self):
        B = self.batch_size
        # no P.grad.zero_(): every gradient element is stored (not accumulated) by this step's kernels
        if not getattr(self, "_acc_cleared", False):
            self.loss.zero_()
            self.correct.zero_()
        self._acc_cleared = False
        fused = self.forward(head=True)
        if not fused:
            ops.softmax_xent(self.logits, labels_oh=self.y, scale=1.0 / B, dlogits=self.dlogits, loss_sum=self.loss,
                             correct=self.correct)
            ops.gemm(self.hT, self.dlogits, self.gWo, M=H + 1, N=NC, K=B, amode=ops.RMAJ, lda=H, bmode=ops.RMAJ,
                     ldb=NC, a_ones_row=H, bias_out=self.gbo)
            ops.gemm(self.dlogits, self.Wo, self.dh, M=B, N=H, K=NC, bmode=ops.KMAJ, ldb=NC)
        if fused:
            # the fused head left dlogits (not dh_T): the persistent BPTT forms dh_T = dlogits . W_out^T
            if not ops.require().lstm_seq_bwd(self.K, self.act, self.c, self.dh, self.dg, I, dl=self.dlogits,
                                              wo=self.Wo):
                ops.gemm(self.dlogits, self.Wo, self.dh, M=B, N=H, K=NC, bmode=ops.KMAJ, ldb=NC)
                self._bptt_steps()
        elif self._persistent() and ops.require().lstm_seq_bwd(self.K, self.act, self.c, self.dh, self.dg, I):
            pass  # whole BPTT recurrence in one launch (dc / dh stay on chip)
        else:
            self._bptt_steps()
        if self.ws_k is not None:  # kernel + bias gradient over all T*B rows: split-K slabs (wgrad_tallk.hip)
            ops.wgrad_tallk(self.xh, I + H, self.dg, 4 * H, I + H, 4 * H, T * B, self.gK, bias=self.gb,
                            splits=self.k_splits, workspace=self.ws_k)
        else:
            ops.gemm(self.xh, self.dg, self.gK, M=I + H + 1, N=4 * H, K=T * B, amode=ops.RMAJ, lda=I + H,
                     bmode=ops.RMAJ, ldb=4 * H, a_ones_row=I + H, bias_out=self.gb)
        return {"loss": ScaledScalar(self.loss, 1.0 / B)}

    def _bptt_steps(self):
        """Per-step BPTT: fused cell-backward kernel + dgrad GEMM per timestep (CPU reference /
        shapes the persistent kernel does not cover)."""
        B = self.batch_size
        self.dc.zero_()
        Kh = self.K[I:]  # recurrent rows [H][4H]
        for t in range(T - 1, -1, -1):
            ops.lstm_cell_bwd(self.act[t], self.c[t - 1] if t > 0 else None, self.c[t], self.dh, None, self.dc,
                              self.dg[t], self.dc)
            if t > 0:
                ops.gemm(self.dg[t], Kh, self.dh, M=B, N=H, K=4 * H, bmode=ops.KMAJ, ldb=4 * H)

    def check_health(self):
        """The split persistent kernels (4 CUs per row group) exchange h / dh through memory; a
        peer workgroup that never ran makes the poll time out and set an error word, after which
        that launch's outputs are wrong.  Raise instead of training on them."""
        if self.device.type == "cuda" and int(ops.require().lstm_status(True)) != 0:
            raise RuntimeError("LSTM split kernel: a cross-workgroup h exchange timed out (a peer workgroup "
                               "was not co-resident); that step's activations / gradients are invalid")

    def evaluate(self, images, labels) -> float:
        """accuracy = mean(argmax(softmax(logits)) == argmax(Y)) (LSTM:98-100, 134-138).  Any number
        of images: evaluated in program-batch chunks, the last one padded by repeating rows (only
        the real rows are counted)."""
        n, B = images.shape[0], self.batch_size
        if n == B:
            self.load_batch((images, labels))
            self._acc_cleared = False
            self.forward()
            self.correct.zero_()
            ops.softmax_xent(self.logits, labels_oh=self.y, correct=self.correct)
            return int(self.correct.item()) / n
        hits = 0
        for lo in range(0, n, B):
            m = min(B, n - lo)
            idx = torch.arange(lo, lo + B, device=images.device).clamp_max(n - 1)
            xb, yb = images[idx], labels[idx]
            self.load_batch((xb, yb))
            self._acc_cleared = False
            self.forward()
            hits += int((self.logits[:m].argmax(1) == self.y[:m].argmax(1)).sum().item())
        return hits / n
