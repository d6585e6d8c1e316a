"""TF1-exact optimizers over a flat fp32 master buffer.

``FlatParams`` owns every trainable variable of a model as one contiguous fp32
buffer (plus the matching fp32 gradient buffer and optional bf16 working
copies for the MFMA kernels).  ``Optimizer`` applies TF1 ``GradientDescent``,
``Momentum``, ``Adam`` or ``RMSProp`` to a *subset* of those variables (the
reference's ``var_list``) in one fused HIP launch, advancing ``global_step``
(and Adam's ``beta1_power``/``beta2_power``) on device.  CPU tensors take an
exact PyTorch path with the same formulas.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from .. import ops


# fused apply: the transposed-tile work items ahead of the flat ranges (test hook / A/B switch)
TILES_FIRST = True


@dataclass
class VarSpec:
    """One trainable variable.

    name:  TF checkpoint key (e.g. "Variable_3", "rnn/basic_lstm_cell/kernel")
    shape: shape in *this framework's* storage layout
    init:  callable(shape, generator) -> fp32 CPU tensor
    bf16:  keep a natural-layout bf16 working copy
    transpose: (R, T, C) view -> also keep a [C][T][R] bf16 copy (backward GEMM operand)
    tf_shape / to_tf / from_tf: layout conversion for TF-compatible checkpoints
    """
    name: str
    shape: tuple
    init: object
    bf16: bool = False
    transpose: tuple | None = None
    tf_shape: tuple | None = None
    to_tf: object = None
    from_tf: object = None

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape)) if self.shape else 1


class FlatParams:
    """Contiguous fp32 master weights + grads (+ bf16 copies) for a list of VarSpecs."""

    ALIGN = 64  # elements: keep every variable 256-byte aligned for 16 B vector loads

    def __init__(self, specs, device, seed: int = 0, init: bool = True):
        self.specs = list(specs)
        self.device = torch.device(device)
        self.offsets = {}
        off = 0
        for s in self.specs:
            self.offsets[s.name] = off
            off += (s.numel + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.total = off
        self.master = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.w16 = {}
        self.wt16 = {}
        for s in self.specs:
            if s.bf16:
                self.w16[s.name] = torch.zeros(s.shape, dtype=torch.bfloat16, device=self.device)
            if s.transpose is not None:
                self.wt16[s.name] = torch.zeros(s.numel, dtype=torch.bfloat16, device=self.device)
        if init:
            self.initialize(seed)

    # views ------------------------------------------------------------
    def view(self, name):
        s = self.spec(name)
        o = self.offsets[name]
        return self.master[o:o + s.numel].view(s.shape)

    def gview(self, name):
        s = self.spec(name)
        o = self.offsets[name]
        return self.grad[o:o + s.numel].view(s.shape)

    def spec(self, name) -> VarSpec:
        for s in self.specs:
            if s.name == name:
                return s
        a = getattr(self, "aliases", {}).get(name)
        if a is not None:
            return a
        raise KeyError(name)

    def add_alias(self, spec: VarSpec, parent: str, elem_off: int):
        """Register ``spec`` as a view of elements [elem_off, elem_off + numel) of variable ``parent``
        (a partition of it, parallel/partition.py): ``offsets`` / ``view`` / ``gview`` / ``w16`` then
        address it like a variable; layout, initialisation and copies stay the parent's."""
        ps = self.spec(parent)
        assert spec.transpose is None and elem_off + spec.numel <= ps.numel, spec.name
        if not hasattr(self, "aliases"):
            self.aliases = {}
        self.aliases[spec.name] = spec
        self.offsets[spec.name] = self.offsets[parent] + elem_off
        if parent in self.w16:
            self.w16[spec.name] = self.w16[parent].view(-1)[elem_off:elem_off + spec.numel].view(spec.shape)

    def range_of(self, names):
        """[lo, hi) element range covering the given variables (must be contiguous)."""
        los = [self.offsets[n] for n in names]
        his = [self.offsets[n] + self.spec(n).numel for n in names]
        return min(los), max(his)

    # init / copies -------------------------------------------------------
    def initialize(self, seed: int):
        g = torch.Generator().manual_seed(seed)
        for s in self.specs:
            v = s.init(s.shape, g).to(torch.float32)
            self.view(s.name).copy_(v.view(s.shape).to(self.device))
        self.refresh_copies()

    def refresh_copies(self):
        """Recompute bf16 working copies from the masters (after init/restore)."""
        for s in self.specs:
            if s.name in self.w16:
                self.w16[s.name].copy_(self.view(s.name).to(torch.bfloat16))
            if s.name in self.wt16:
                R, T, C = s.transpose
                self.wt16[s.name].copy_(self.view(s.name).reshape(R, T, C).permute(2, 1, 0).reshape(-1)
                                        .to(torch.bfloat16))

    def state_dict(self):
        return {s.name: self.view(s.name).detach().cpu().clone() for s in self.specs}

    def load_state_dict(self, sd):
        for s in self.specs:
            self.view(s.name).copy_(sd[s.name].view(s.shape).to(self.device))
        self.refresh_copies()


KINDS = {"sgd": ops.OPT_SGD, "momentum": ops.OPT_MOMENTUM, "adam": ops.OPT_ADAM, "rmsprop": ops.OPT_RMSPROP}


@dataclass
class OptimizerConfig:
    kind: str = "sgd"
    lr: float = 0.01
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = None  # default per kind: adam 1e-8, rmsprop 1e-10 (TF1 defaults)
    momentum: float = 0.0
    rho: float = 0.9
    name: str = field(default="")

    def resolved_eps(self):
        if self.eps is not None:
            return self.eps
        return 1e-10 if self.kind == "rmsprop" else 1e-8


class Optimizer:
    """Fused TF1 optimizer over a subset (var_list) of a FlatParams.

    Slot variables follow TF1 naming: ``<var>/Adam``, ``<var>/Adam_1``;
    ``<var>/RMSProp`` (initialised to ones), ``<var>/RMSProp_1``;
    ``<var>/Momentum``.  Adam's non-slot ``beta1_power``/``beta2_power`` are a
    2-element device tensor advanced by the kernel itself.
    """

    SLOT_NAMES = {"adam": ("Adam", "Adam_1"), "rmsprop": ("RMSProp", "RMSProp_1"), "momentum": ("Momentum",),
                  "sgd": ()}

    def __init__(self, cfg: OptimizerConfig, params: FlatParams, var_list=None, global_step=None,
                 beta_power_names=("beta1_power", "beta2_power")):
        self.cfg = cfg
        self.P = params
        self.kind = KINDS[cfg.kind]
        self.var_list = [s.name for s in params.specs] if var_list is None else list(var_list)
        self.device = params.device
        self.global_step = global_step  # int32 [1] device tensor or None
        self.beta_power_names = beta_power_names
        nslots = len(self.SLOT_NAMES[cfg.kind])
        # slots live in full-size flat buffers (same offsets as the masters)
        self.s1 = self.s2 = None
        if nslots >= 1:
            fill = 1.0 if cfg.kind == "rmsprop" else 0.0
            self.s1 = torch.full((params.total,), fill, dtype=torch.float32, device=self.device)
        if nslots >= 2:
            self.s2 = torch.zeros(params.total, dtype=torch.float32, device=self.device)
        self.beta_pow = torch.tensor([cfg.beta1, cfg.beta2], dtype=torch.float32, device=self.device) \
            if cfg.kind == "adam" else None
        self.done = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._blob = None
        if self.device.type == "cuda":
            self._build_plan()

    # ---- plan of work items for the fused kernel
    def _build_plan(self, chunk: int = 0):
        # flat work items of `chunk` elements (DTFE_OPT_CHUNK; multiple of 1024): one workgroup
        # each, up to 2048 workgroups per launch.  Default 8192; 2048 for var lists under 2 M elements
        # (the GAN's two Adams over 0.43 M params: 52 workgroups -> 209, 0.0736 -> 0.0702 ms/step; the
        # autoencoder -1 %, LSTM / ResNet-20 neutral - profiles/r6_ref_models_fused.txt)
        if not chunk:
            env = os.environ.get("DTFE_OPT_CHUNK")
            total = sum(self.P.spec(name).numel for name in self.var_list)
            chunk = int(env) if env else (2048 if total < 2_000_000 else 8192)
        segs, work = [], []
        for si, name in enumerate(self.var_list):
            s = self.P.spec(name)
            w16 = self.P.w16.get(name)
            wt16 = self.P.wt16.get(name)
            if s.transpose is not None:
                R, T, C = s.transpose
            else:
                R, T, C = s.numel, 1, 1
            segs.append([self.P.offsets[name], R, T, C, w16.data_ptr() if w16 is not None else 0,
                         wt16.data_ptr() if wt16 is not None else 0])
            if wt16 is not None:
                for t in range(T):
                    for r0 in range(0, R, 64):
                        for c0 in range(0, C, 64):
                            work.append([1, si, t, r0, c0, 0, 0])
            else:
                n = s.numel
                for st in range(0, n, chunk):
                    work.append([0, si, 0, 0, 0, st, min(chunk, n - st)])
        if TILES_FIRST:
            # transposed-copy tiles first: they are short latency chains (16 dependent-free loads, an
            # LDS transpose, scattered stores); dispatched last they were the launch's tail
            work.sort(key=lambda w: -w[0])
        self.nseg, self.nwork = len(segs), len(work)
        self._blob = ops.opt_pack(torch.tensor(segs, dtype=torch.int64), torch.tensor(work, dtype=torch.int64),
                                  self.P.master)

    def step(self, grad=None, grad16=None, gscale: float = 1.0, gs_inc: int = 1, group: int = 0):
        """Apply gradients (default: the FlatParams grad buffer) to var_list.  ``group`` (GPU):
        1 queues this apply, 2 queues it and launches every queued one together (``step_all``)."""
        c = self.cfg
        if grad is None and grad16 is None:
            grad = self.P.grad
        if self.device.type == "cuda":
            ops.apply_gradients(self.kind, self.P.master, grad, grad16, gscale, self.s1, self.s2, c.lr, c.beta1,
                                c.beta2, c.resolved_eps(), c.momentum, c.rho, self.beta_pow, self.global_step, gs_inc,
                                self.done, self._blob, self.nseg, self.nwork, group)
            return
        self._step_cpu(grad if grad is not None else grad16.float(), gscale, gs_inc)

    @staticmethod
    def step_all(opts, gs_incs, grad=None, grad16=None, gscale: float = 1.0):
        """Apply several optimizers over disjoint var lists of one FlatParams (the reference's
        several ``minimize`` calls per step).  On the GPU, optimizers of one kind share ONE grouped
        launch (each keeps its own beta powers / global-step increment); the math equals
        calling ``step`` on each in order."""
        kinds = {o.kind for o in opts}
        if len(opts) > 1 and len(opts) <= 4 and len(kinds) == 1 and all(o.device.type == "cuda" for o in opts):
            for i, (o, inc) in enumerate(zip(opts, gs_incs)):
                o.step(grad=grad, grad16=grad16, gscale=gscale, gs_inc=inc, group=2 if i == len(opts) - 1 else 1)
            return
        for o, inc in zip(opts, gs_incs):
            o.step(grad=grad, grad16=grad16, gscale=gscale, gs_inc=inc)

    @torch.no_grad()
    def _step_cpu(self, grad, gscale, gs_inc):
        c = self.cfg
        lr_t = c.lr
        if c.kind == "adam":
            b1p, b2p = self.beta_pow.tolist()
            lr_t = c.lr * math.sqrt(1 - b2p) / (1 - b1p)
        eps = c.resolved_eps()
        for name in self.var_list:
            s = self.P.spec(name)
            o, n = self.P.offsets[name], s.numel
            v, g = self.P.master[o:o + n], grad[o:o + n] * gscale
            if c.kind == "sgd":
                v -= c.lr * g
            elif c.kind == "momentum":
                a = self.s1[o:o + n]
                a.mul_(c.momentum).add_(g)
                v -= c.lr * a
            elif c.kind == "adam":
                m, v2 = self.s1[o:o + n], self.s2[o:o + n]
                m.mul_(c.beta1).add_((1 - c.beta1) * g)
                v2.mul_(c.beta2).add_((1 - c.beta2) * g * g)
                v -= lr_t * m / (v2.sqrt() + eps)
            else:
                ms, mom = self.s1[o:o + n], self.s2[o:o + n]
                ms.mul_(c.rho).add_((1 - c.rho) * g * g)
                mom.mul_(c.momentum).add_(c.lr * g / (ms + eps).sqrt())
                v -= mom
        if c.kind == "adam":
            self.beta_pow[0] *= c.beta1
            self.beta_pow[1] *= c.beta2
        if self.global_step is not None and gs_inc:
            self.global_step += gs_inc

    # ---- checkpoint naming (TF1 slot conventions)
    def slot_tensors(self):
        """{checkpoint key: fp32 CPU tensor} for this optimizer's slots and non-slot variables."""
        out = {}
        names = self.SLOT_NAMES[self.cfg.kind]
        for var in self.var_list:
            s = self.P.spec(var)
            o, n = self.P.offsets[var], s.numel
            for i, sn in enumerate(names):
                buf = self.s1 if i == 0 else self.s2
                out[f"{var}/{sn}"] = buf[o:o + n].detach().cpu().view(s.shape).clone()
        if self.beta_pow is not None:
            bp = self.beta_pow.detach().cpu()
            out[self.beta_power_names[0]] = bp[0].clone()
            out[self.beta_power_names[1]] = bp[1].clone()
        return out

    def load_slot_tensors(self, tensors):
        names = self.SLOT_NAMES[self.cfg.kind]
        for var in self.var_list:
            s = self.P.spec(var)
            o, n = self.P.offsets[var], s.numel
            for i, sn in enumerate(names):
                key = f"{var}/{sn}"
                if key in tensors:
                    buf = self.s1 if i == 0 else self.s2
                    buf[o:o + n].copy_(tensors[key].reshape(-1).to(self.device))
        if self.beta_pow is not None and self.beta_power_names[0] in tensors:
            self.beta_pow[0] = float(tensors[self.beta_power_names[0]])
            self.beta_pow[1] = float(tensors[self.beta_power_names[1]])
