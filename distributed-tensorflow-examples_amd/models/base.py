"""Model-definition protocol shared by every workload.

A ``ModelDef`` is the static description the cluster roles need:

* ``var_order``   - TF variable creation order (checkpoint keys / ps placement),
                    *including* the global step at its creation ordinal;
* ``specs``       - trainable ``VarSpec``s in flat-buffer order;
* ``opt_groups``  - ``(OptimizerConfig, var_list, beta_power_names)`` per
                    ``optimizer.minimize`` call (the GAN has two);
* ``gs_increments`` - how many ``minimize(global_step=...)`` calls run per
                    step (GAN: 2);
* ``program(...)``  - builds the per-worker step program.

A ``StepProgram`` owns a ``FlatParams`` (the worker's copy of the variables)
and pre-allocated activation buffers; ``load_batch`` stages the next batch,
``compute_grads`` fills ``P.grad`` (zeroed first) with d(loss)/d(var) and
returns lazily-evaluated metrics.  All math goes through ``dtfe.ops`` - HIP
kernels on the GPU, the PyTorch reference path on CPU.
"""
from __future__ import annotations

import torch

from ..optim import FlatParams



class ScaledScalar:
    """A step metric kept as (device scalar, host scale): ``.item()`` reads and scales it on the
    host, so a captured step issues no extra kernel just to divide a loss sum by the batch."""

    def __init__(self, t, scale: float):
        self.t, self.scale = t, float(scale)

    def item(self) -> float:
        return float(self.t.item()) * self.scale

    __float__ = item

class StepProgram:
    batch_size: int

    def __init__(self, model, device, batch_size: int, seed: int = 0):
        self.model = model
        self.device = torch.device(device)
        self.batch_size = batch_size
        self.P = FlatParams(model.specs, self.device, seed=seed)

    def load_batch(self, batch):  # pragma: no cover - interface
        raise NotImplementedError

    def compute_grads(self) -> dict:  # pragma: no cover - interface
        raise NotImplementedError

    def evaluate(self, images, labels) -> float:
        raise NotImplementedError("this model has no evaluation metric")

    def check_health(self):
        """Raise if a kernel of this program reported a failure it could not surface itself (e.g.
        a cross-workgroup exchange timeout).  Synchronises; callers do it every log step."""


class ModelDef:
    name = "model"
    var_order: list = []
    gs_name: str = ""
    specs: list = []
    opt_groups: list = []
    gs_increments: int = 1
    default_batch: int = 128
    default_steps: int = 1000
    needs_labels: bool = True
    # compute dtypes the model's step program implements (--dtype); the first is the default
    dtypes: tuple = ("fp32",)
    dtype: str | None = None

    def set_dtype(self, dt):
        """--dtype routing: ``auto`` keeps the model's default; anything the program does not
        implement is an error (never a silent fallback)."""
        if dt in (None, "auto"):
            self.dtype = self.dtypes[0]
            return
        if dt not in self.dtypes:
            raise ValueError("--dtype=%s: model %r computes in %s" % (dt, self.name, "/".join(self.dtypes)))
        self.dtype = dt

    def program(self, device, batch_size=None, seed: int = 0) -> StepProgram:  # pragma: no cover
        raise NotImplementedError

    def tf_shapes(self):
        """{name: shape in TF layout} for every trainable var."""
        return {s.name: (s.tf_shape if s.tf_shape is not None else s.shape) for s in self.specs}

    def to_tf(self, name, t: torch.Tensor) -> torch.Tensor:
        s = next(x for x in self.specs if x.name == name)
        return s.to_tf(t) if s.to_tf is not None else t

    def from_tf(self, name, t: torch.Tensor) -> torch.Tensor:
        s = next(x for x in self.specs if x.name == name)
        return s.from_tf(t) if s.from_tf is not None else t


def tf_auto_names(keys):
    """TF names unnamed tf.Variable()s Variable, Variable_1, ... in creation order."""
    return {k: ("Variable" if i == 0 else "Variable_%d" % i) for i, k in enumerate(keys)}


def normal_init(std):
    return lambda shape, g: torch.randn(*shape, generator=g) * std


def zeros_init(shape, g):
    return torch.zeros(*shape)


def glorot_uniform_init(shape, g):
    fan_in, fan_out = shape[0], shape[-1]
    lim = (6.0 / (fan_in + fan_out)) ** 0.5
    return (torch.rand(*shape, generator=g) * 2 - 1) * lim
