"""ResNet family: CIFAR-10 ResNet-20 and ImageNet-shape ResNet-50 (BASELINE.json configs 3 and 5).

Neither model exists in the reference; they are the
north-star workloads of the conv2d MFMA path.  Both are ResNet v1 in the
TensorFlow layer conventions so checkpoints use ``tf.layers`` names
(``conv2d_3/kernel``, ``batch_normalization_3/{gamma,beta,moving_mean,
moving_variance}``, ``dense/{kernel,bias}``, ``global_step``) and TF layouts.

* ResNet-20 (He et al. 2016, CIFAR): 3x3 conv 16 -> 3 stages x 3 basic blocks
  (16/32/64 channels, stride 2 at stages 2 and 3) -> global average pool -> fc 10.
  Shortcuts are the paper's parameter-free "option A" (identity, stride-2
  subsample, zero-padded channels): 0.27 M parameters.
* ResNet-50 (v1.5: stride on the 3x3 conv): 7x7/2 conv 64 + 3x3/2 max pool ->
  bottleneck stages [3, 4, 6, 3] (64/128/256/512 x 4) with projection
  shortcuts -> global average pool -> fc 1000: 25.6 M parameters.

Execution: NHWC bf16 activations in pre-allocated buffers, fp32 master weights /
grads / Momentum slots in one flat buffer, BatchNorm in training mode (batch
statistics; TF defaults momentum 0.99, epsilon 1e-3), every op a HIP kernel:

  conv fwd     whole-image LDS conv (persistent, weights in LDS) when the image
               and weights fit (all of ResNet-20), else the implicit-GEMM conv
  conv dgrad   stride 1: the same kernel over dY with flipped taps; else implicit GEMM
  conv wgrad   persistent register-accumulating kernel, else implicit GEMM
  BN           channel statistics (one atomic per channel and workgroup),
               apply + ReLU + residual add fused, backward stats + apply fused
               with the ReLU mask and the shortcut-gradient copy
  head         global average pool, fp32 fc + softmax-xent (exact fp32 MFMA GEMMs)

BatchNorm moving statistics live in the flat buffer (so checkpoints and the
all-reduce broadcast carry them) but outside every optimizer var_list; in
--mode=ps they stay worker-local.  No weight decay (not part of the reference
contract).
"""
from __future__ import annotations

import math
import os

import torch

from .. import ops
from ..optim import OptimizerConfig, VarSpec
from .base import ModelDef, ScaledScalar, StepProgram

BN_EPS, BN_MOMENTUM = 1e-3, 0.99
# Schedule switches below are module constants - test hooks that tests/test_resnet.py monkeypatches
# to compare a fused path against its unfused oracle, not environment knobs.
# bottleneck input gradient: shortcut share written into dx, conv1's data gradient accumulated on
# top (False: separate buffer + add pass; profiles/r2_resnet50_shortcut_fuse_ab.txt)
_SHORTCUT_FUSE = True
# (test hook, not a knob: tests/test_resnet.py compares against the stored-dres path)
_PROJ_FROM_BITS = True
# activation / activation-gradient storage dtype: bf16 on the GPU kernels; the CPU reference
# path also runs with fp32 storage (exactness tests of the program logic)
ACT_DTYPE = torch.bfloat16


def _conv_to_tf(t):    # ours [Cout][KH][KW][Cin] -> TF [KH][KW][Cin][Cout]
    return t.permute(1, 2, 3, 0).contiguous()


def _conv_from_tf(t):
    return t.permute(3, 0, 1, 2).contiguous()


def _fc_to_tf(t):      # ours [out][in] -> TF [in][out]
    return t.t().contiguous()


def _he_normal(fan_in):
    std = math.sqrt(2.0 / fan_in)
    return lambda shape, g: torch.randn(*shape, generator=g) * std


def _const(v):
    return lambda shape, g: torch.full(shape, float(v))


def _glorot(fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return lambda shape, g: (torch.rand(*shape, generator=g) * 2 - 1) * lim


class Registry:
    """tf.layers-style auto names (conv2d, conv2d_1, ...) and the VarSpecs in creation order."""

    def __init__(self):
        self.specs = []
        self._count = {}

    def scope(self, base):
        i = self._count.get(base, 0)
        self._count[base] = i + 1
        return base if i == 0 else "%s_%d" % (base, i)

    def add(self, spec):
        self.specs.append(spec)
        return spec.name


# ------------------------------------------------------------------ layers
class Conv:
    """NHWC conv without bias (ResNet convs are followed by BatchNorm)."""

    def __init__(self, reg, cin, cout, k, stride, H, W):
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.pad = (k - 1) // 2
        self.H, self.W = H, W
        self.OH = (H + 2 * self.pad - k) // stride + 1
        self.OW = (W + 2 * self.pad - k) // stride + 1
        self.name = reg.add(VarSpec(reg.scope("conv2d") + "/kernel", (cout, k, k, cin), _he_normal(k * k * cin),
                                    bf16=True, transpose=(cout, k * k, cin), tf_shape=(k, k, cin, cout),
                                    to_tf=_conv_to_tf, from_tf=_conv_from_tf))

    def bind(self, P, B, dev):
        self.B = B
        self.w, self.wt, self.gw = P.w16[self.name], P.wt16[self.name], P.gview(self.name)
        self.y = torch.empty(B, self.OH, self.OW, self.cout, device=dev, dtype=ACT_DTYPE)
        self.g = dict(B=B, H=self.H, W=self.W, C=self.cin, Cout=self.cout, OH=self.OH, OW=self.OW, KH=self.k,
                      KW=self.k, stride=self.stride, pad=self.pad)
        self.ic = dict(B=B, SH=self.H, SW=self.W, CS=self.cin, OH=self.OH, OW=self.OW, N=self.cout, KH=self.k,
                       KW=self.k, stride=self.stride, pad=self.pad)
        LH = (self.OH - 1) * self.stride + self.k
        LW = (self.OW - 1) * self.stride + self.k
        few = self.cin <= 4 and self.k * self.k * self.cin <= 32  # tap-packed network-input kernels
        self.img_fwd = (self.cin % 8 == 0 or few) and self.cout <= 64 and LH * LW * self.cin * 2 <= 150 * 1024
        # data gradient as a stride-1 flipped-tap conv over dY, dilated by the stride (persistent kernel: B >= 64)
        self.dil = self.stride if (self.H == self.OH * self.stride and self.W == self.OW * self.stride) else 0
        self.img_dgrad = (self.dil > 0 and (self.stride == 1 or B >= 64) and self.cout % 8 == 0 and self.cin <= 64
                          and (self.H + self.k - 1) * (self.W + self.k - 1) * self.cout * 2 <= 150 * 1024)
        self.img_wgrad = (self.cin % 8 == 0 or few) and self.cout <= 64 and self.OW <= 32 and self.cout % 8 == 0
        # the implicit-GEMM data gradient can accumulate into dx (a block's input gradient gets its
        # shortcut share first, then the conv's on top: no separate add pass)
        self.can_accum = not self.img_dgrad and self.cin % 64 == 0 and self.cout % 64 == 0

    def fwd(self, x, stats=None, bn_src=None):
        """Forward; ``stats``: the following BatchNorm's [2][C] accumulators, filled by the conv
        launch itself where it can (returns True then; the BN skips its statistics pass).
        ``bn_src``: the preceding BatchNorm + ReLU (BN.src_fold) for the whole-image kernel, which
        forms it while staging the raw input x and saves the BN's statistics / moving averages."""
        if self.img_fwd:
            # (no output statistics: the BN runs its bn_stats pass - in the staged epilogue with a
            # last-arriver fold they cost 11-12 us per conv against a 4.5-6.7 us pass,
            # profiles/r6_resnet20_ostats_ab.txt)
            if bn_src is not None:
                ops.imgconv(self.w, self.y, src=x, bn_src=bn_src.src_args(), bn_eps=BN_EPS,
                            bn_momentum=BN_MOMENTUM, bn_save=True, **self.ic)
            else:
                ops.imgconv(self.w, self.y, src=x, **self.ic)
            return self.y, False
        assert bn_src is None
        ops.conv_fwd(x, self.w, None, self.y, None, self.g, act=ops.ACT_NONE, stats=stats)
        return self.y, stats is not None

    def wgrad(self, dy, x, after=None, bn_src=None):
        """``after``: the side stream's fork point (SideStream.fork_point, taken when dy was final).
        ``bn_src``: as in fwd (x is then the BN's raw input)."""
        dws = getattr(self, "defer_ws", None)
        if bn_src is not None:
            assert self.img_wgrad
            ops.imgwgrad(x, self.gw, None, dy=dy, bn_src=bn_src.src_args(), bn_eps=BN_EPS, workspace=dws,
                         defer=dws is not None, **self.ic)
            return
        if dws is not None and self.img_wgrad:
            ops.imgwgrad(x, self.gw, None, dy=dy, workspace=dws, defer=True, **self.ic)
            return
        side = getattr(self, "side", None)
        if side is not None and not self.img_wgrad and self.cin % 64 == 0 and self.cout % 64 == 0:
            side.run(lambda: ops.conv_wgrad(dy, x, self.gw, None, self.g), after)
            return
        if self.img_wgrad:
            ops.imgwgrad(x, self.gw, None, dy=dy, **self.ic)
        else:
            ops.conv_wgrad(dy, x, self.gw, None, self.g)

    def dgrad_fuses_bn(self, accumulate=False):
        """Whether conv_dgrad produces the consuming BatchNorm's backward statistics with dx (every
        stride-1 implicit-GEMM data gradient: the statistics pass is launched inside conv_dgrad right
        after the GEMM; the per-tile kernel's LDS epilogue for them measured slower,
        profiles/r2_resnet50_bn_bwd_fuse_ab.txt)."""
        return not self.img_dgrad and self.cin % 64 == 0 and self.cout % 64 == 0 and self.stride == 1

    def dgrad(self, dy, dx, accumulate=False, bn_bwd=None, acc_src=None, shortcut=None):
        """``bn_bwd``: BN.bwd_stats_args of the BatchNorm that consumes dx; returns True when its
        backward statistics were produced with dx (the BN then skips its statistics pass).
        ``acc_src``: (src, relu bits) - dx = dgrad + src * bit (ops.conv_dgrad).  ``shortcut``:
        (g, stride) of an option-A shortcut whose gradient the whole-image kernel adds to dx in its
        epilogue (ops.imgconv_shortcut; returns True when it did)."""
        if self.img_dgrad:
            assert not accumulate
            geom = dict(B=self.B, SH=self.OH, SW=self.OW, CS=self.cout, OH=self.H, OW=self.W, N=self.cin, KH=self.k,
                        KW=self.k, stride=1, pad=self.k - 1 - self.pad, dil=self.dil)
            if shortcut is not None:
                return ops.imgconv_shortcut(self.wt, dx, shortcut[0], shortcut[1], src=dy, **geom)
            ops.imgconv(self.wt, dx, src=dy, flip_taps=True, **geom)
            return False
        fuse = bn_bwd is not None and self.dgrad_fuses_bn(accumulate)
        ops.conv_dgrad(dy, self.wt, dx, self.g, accumulate=accumulate, bn_bwd=bn_bwd if fuse else None,
                       acc_src=acc_src)
        return fuse


class SideStream:
    """Weight gradients of the implicit-GEMM convs on a second HIP stream.

    A conv's weight gradient needs only its output gradient and its (forward) input, and nothing
    downstream in the backward reads it, so it runs concurrently with the data-gradient and
    BatchNorm-backward chain on the main stream: compute-bound implicit GEMMs overlap the
    HBM-bound BatchNorm passes.  ``run`` forks after the producer of ``dy`` (an event on the
    current stream), ``join`` makes the current stream wait for every launch so far; inside a
    hipGraph capture this becomes a parallel branch.  The weight-gradient split partials have
    their own workspace (igemm.hip ``g_wg``), so the two streams never share scratch memory."""

    def __init__(self, device):
        # high-priority queue: the weight gradients are the step's tail once the data-gradient chain
        # no longer waits on them (11,260 vs 11,234-11,251 img/s, profiles/r4_resnet50_graph_order.txt)
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self.pending = False

    @staticmethod
    def fork_point():
        """An event on the current stream now: a later ``run(fn, after=...)`` depends on exactly the
        work before this point, though it is launched after the main stream's next kernels."""
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def run(self, fn, after=None):
        if after is None:
            after = self.fork_point()
        self.stream.wait_event(after)
        with torch.cuda.stream(self.stream):
            fn()
        self.pending = True

    def mark(self):
        """An event covering every launch on the side stream so far (the stream stays forked)."""
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def join(self):
        if self.pending:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            torch.cuda.current_stream().wait_event(ev)
            self.pending = False


_WGRAD_STREAM = os.environ.get("DTFE_WGRAD_STREAM", "1") != "0"
# ResNet-20: bn1's apply formed by conv2's whole-image kernels (BN.src_fold; profiles/r5_resnet20_kernels.txt)
_R20_SRC_FOLD = True
# classifier head forward + backward in one launch (ops.dense_head)
_HEAD_FUSE = True
# ResNet-20 weight-gradient reduces deferred to grouped launches (ops.wgrad_flush)
_WGRAD_DEFER = True


class BN:
    infer = False  # set by ResNetProgram.evaluate

    def __init__(self, reg, C):
        self.C = C
        s = reg.scope("batch_normalization")
        self.gamma = reg.add(VarSpec(s + "/gamma", (C,), _const(1.0)))
        self.beta = reg.add(VarSpec(s + "/beta", (C,), _const(0.0)))
        self.mm = reg.add(VarSpec(s + "/moving_mean", (C,), _const(0.0)))
        self.mv = reg.add(VarSpec(s + "/moving_variance", (C,), _const(1.0)))

    def bind(self, P, shape, dev, arena):
        self.P = P
        self.y = torch.empty(*shape, device=dev, dtype=ACT_DTYPE)
        # 1-bit ReLU mask of y (a ReLU after a residual add): what the backward reads instead of y
        self.ybits = torch.empty(math.prod(shape) // 8, device=dev, dtype=torch.uint8) \
            if torch.device(dev).type == "cuda" else None
        self.use_bits = False
        self.stats, self.dstats, self.mean, self.invstd = arena.take(2 * self.C), arena.take(2 * self.C), \
            arena.take(self.C), arena.take(self.C)

    def src_fold(self, x):
        """BN + ReLU whose output only whole-image convs read (ResNet-20's bn1 -> conv2 forward and
        weight gradient): no apply pass - the consumers form it from the raw input x while staging
        it (Conv.fwd / wgrad ``bn_src=self``; the forward's kernel saves mean / invstd and updates the
        moving averages).  The backward recomputes the ReLU mask from x.  Returns x."""
        x, have_stats = x if isinstance(x, tuple) else (x, False)
        if not have_stats:
            ops.bn_stats(x, self.stats)
        self.mask_from_x, self.use_bits = True, False
        return x

    def src_args(self):
        P = self.P
        return [self.stats, P.view(self.gamma), P.view(self.beta), self.mean, self.invstd, P.view(self.mm),
                P.view(self.mv)]

    def stats_only(self, x):
        """A projection shortcut's BN (no activation) whose apply is folded into the residual add of
        the block's last BN (``fwd(..., res_bn=self)``): only the statistics here.  Returns the raw
        conv output."""
        x, have_stats = x if isinstance(x, tuple) else (x, False)
        if not have_stats:
            ops.bn_stats(x, self.stats)
        self.mask_from_x, self.use_bits = False, False
        return x

    def res_bn_args(self):
        P = self.P
        return [self.stats, P.view(self.gamma), P.view(self.beta), self.mean, self.invstd, P.view(self.mm),
                P.view(self.mv)]

    def fwd(self, x, act=ops.ACT_RELU, res=None, rstride=1, res_bn=None):
        """``x``: the conv output, or (conv output, statistics already accumulated by the conv).
        ``res_bn``: the BN of a projection shortcut whose raw output ``res`` is (see stats_only)."""
        P = self.P
        x, have_stats = x if isinstance(x, tuple) else (x, False)
        if self.infer:  # evaluation: moving averages, nothing updated (TF training=False)
            ops.bn_infer(x, P.view(self.gamma), P.view(self.beta), P.view(self.mm), P.view(self.mv), self.y,
                         eps=BN_EPS, act=act, res=res, rstride=rstride)
            return self.y
        # backward recomputes the ReLU mask from x unless a shortcut was added before the ReLU; then
        # it reads the 1-bit mask this apply writes beside y (1 byte per 8 channels instead of 16:
        # the block-output BN's two backward passes read dy, x and the mask, not dy, x and y)
        self.mask_from_x = act == ops.ACT_RELU and res is None
        self.use_bits = act == ops.ACT_RELU and res is not None and self.ybits is not None
        if not have_stats:
            ops.bn_stats(x, self.stats)
        ops.bn_apply(x, self.stats, P.view(self.gamma), P.view(self.beta), self.y, mean=self.mean,
                     invstd=self.invstd, moving_mean=P.view(self.mm), moving_var=P.view(self.mv), eps=BN_EPS,
                     momentum=BN_MOMENTUM, act=act, res=res, rstride=rstride,
                     mask_out=self.ybits if self.use_bits else None,
                     res_bn=res_bn.res_bn_args() if res_bn is not None else None)
        return self.y

    def fwd_pool3(self, x, pool, am):
        """BN + ReLU + the 3x3 / stride-2 max pool of the ResNet-50 stem.  Training on the GPU: ONE
        pass (ops.bn_relu_pool3) that never stores the normalised 112x112 map - the backward
        recomputes this BN's ReLU mask from x and the pool's from ``am`` (bn_apply + maxpool3_fwd
        wrote 411 MB and read it back at B=256: 22.64-22.69 vs 22.74-22.77 ms per ResNet-50 step,
        profiles/r4_resnet50_stem_pool_ab.txt).  Returns ``pool``."""
        xx = x[0] if isinstance(x, tuple) else x
        if self.infer or not xx.is_cuda:
            ops.maxpool3_fwd(self.fwd(x), pool, am)
            return pool
        P = self.P
        x, have_stats = x if isinstance(x, tuple) else (x, False)
        self.mask_from_x, self.use_bits = True, False
        if not have_stats:
            ops.bn_stats(x, self.stats)
        ops.bn_relu_pool3(x, self.stats, P.view(self.gamma), P.view(self.beta), pool, am, mean=self.mean,
                          invstd=self.invstd, moving_mean=P.view(self.mm), moving_var=P.view(self.mv), eps=BN_EPS,
                          momentum=BN_MOMENTUM)
        return pool

    def bwd_pool3(self, dp, am, x, dx, tmp):
        """Backward of fwd_pool3: max-pool backward + this BN's backward.  On the GPU one statistics
        and one apply pass straight from the pooled gradient ``dp`` and argmax ``am``
        (ops.pool3_bn_bwd: the unpooled 112x112 gradient is not stored); elsewhere maxpool3_bwd into
        ``tmp`` and the plain backward.  22.54-22.59 vs 22.66-22.70 ms per ResNet-50 step
        (profiles/r4_resnet50_stem_pool_ab.txt)."""
        if dx.is_cuda and getattr(self, "mask_from_x", False):
            P = self.P
            ops.pool3_bn_bwd(dp, am, x, self.mean, self.invstd, P.view(self.gamma), P.view(self.beta), self.dstats,
                             dx, dgamma=P.gview(self.gamma), dbeta=P.gview(self.beta))
            return
        ops.maxpool3_bwd(dp, am, tmp)
        self.bwd(tmp, x, dx)

    def _mask_src(self, act):
        """(y argument, beta) of the backward ops: the bit mask, y, or nothing (mask from x)."""
        from_x = act == ops.ACT_RELU and getattr(self, "mask_from_x", False)
        if act == ops.ACT_NONE or from_x:
            return None, (self.P.view(self.beta) if from_x else None)
        return (self.ybits if self.use_bits and act == ops.ACT_RELU else self.y), None

    def bwd_stats_args(self, x, act=ops.ACT_RELU):
        """(x, y, mean, invstd, gamma, beta, stats, act) of this BN's backward statistics, for the
        launch that produces its output gradient (ops.conv_dgrad(bn_bwd=...))."""
        P = self.P
        y, beta = self._mask_src(act)
        return (x, y, self.mean, self.invstd, P.view(self.gamma), beta, self.dstats, act)

    def bwd(self, dy, x, dx, act=ops.ACT_RELU, dres=None, stats_done=False, mask=None, res_bn=None):
        """``mask``: a uint8 ReLU bit mask to take act' from instead of this BN's own (a projection
        shortcut's BN differentiated straight from the block's output gradient and bn3's mask).
        ``res_bn`` = (that shortcut BN, its x): its backward statistics ride along in this BN's
        statistics pass (same g)."""
        P = self.P
        y, beta = (mask, None) if mask is not None else self._mask_src(act)
        if not stats_done:
            ops.bn_bwd_stats(dy, y, x, self.mean, self.invstd, self.dstats, act, gamma=P.view(self.gamma), beta=beta,
                             res_bn=None if res_bn is None else [res_bn[1], res_bn[0].mean, res_bn[0].invstd,
                                                                 res_bn[0].dstats])
        ops.bn_bwd_apply(dy, y, x, self.mean, self.invstd, P.view(self.gamma), self.dstats, dx, act=act, dres=dres,
                         dgamma=P.gview(self.gamma), dbeta=P.gview(self.beta), beta=beta)


class Arena:
    """One zero-per-step fp32 buffer holding every BN layer's statistics accumulators."""

    def __init__(self, n, dev):
        self.buf = torch.zeros(n, device=dev)
        self.off = 0

    def take(self, n):
        t = self.buf[self.off:self.off + n]
        self.off += (n + 15) // 16 * 16
        return t


class BasicBlock:
    """ResNet v1 basic block with the option-A shortcut (identity / subsample + zero channels)."""

    def __init__(self, reg, cin, cout, stride, H, W):
        self.cin, self.cout, self.stride = cin, cout, stride
        self.conv1 = Conv(reg, cin, cout, 3, stride, H, W)
        self.bn1 = BN(reg, cout)
        self.conv2 = Conv(reg, cout, cout, 3, 1, self.conv1.OH, self.conv1.OW)
        self.bn2 = BN(reg, cout)
        self.OH, self.OW = self.conv2.OH, self.conv2.OW
        self.stats_len = 6 * cout * 2 + 64
        self.src_fold = False

    def bind(self, P, B, dev, arena):
        for c in (self.conv1, self.conv2):
            c.bind(P, B, dev)
        shp = (B, self.OH, self.OW, self.cout)
        self.bn1.bind(P, shp, dev, arena)
        self.bn2.bind(P, shp, dev, arena)
        bf = dict(device=dev, dtype=ACT_DTYPE)
        self.dc2, self.dh1, self.dc1, self.dres = (torch.empty(*shp, **bf) for _ in range(4))

    def fwd(self, x):
        self.x = x
        # bn1's apply formed by conv2's whole-image kernels while they stage its input (forward and
        # weight gradient): no bn_apply pass (profiles/r5_resnet20_kernels.txt)
        # (instance flag: ResNetProgram.evaluate sets it on every BN; evaluation takes the plain path)
        self.src_fold = (_R20_SRC_FOLD and not self.bn1.infer and x.is_cuda and self.conv2.img_fwd
                         and self.conv2.img_wgrad and self.conv2.B >= 128)
        if self.src_fold:
            r1 = self.bn1.src_fold(self.conv1.fwd(x, self.bn1.stats))
            return self.bn2.fwd(self.conv2.fwd(r1, self.bn2.stats, bn_src=self.bn1), res=x, rstride=self.stride)
        h1 = self.bn1.fwd(self.conv1.fwd(x, self.bn1.stats))
        return self.bn2.fwd(self.conv2.fwd(h1, self.bn2.stats), res=x, rstride=self.stride)

    def bwd(self, dout, dx):
        self.bn2.bwd(dout, self.conv2.y, self.dc2, dres=self.dres)
        if self.src_fold:
            self.conv2.wgrad(self.dc2, self.conv1.y, bn_src=self.bn1)
        else:
            self.conv2.wgrad(self.dc2, self.bn1.y)
        self.conv2.dgrad(self.dc2, self.dh1)
        self.bn1.bwd(self.dh1, self.conv1.y, self.dc1)
        self.conv1.wgrad(self.dc1, self.x)
        if dx is not None:
            # the shortcut's gradient rides in the data gradient's epilogue where the kernel allows
            # (profiles/r5_resnet20_kernels.txt); else its own pass
            if not self.conv1.dgrad(self.dc1, dx, shortcut=(self.dres, self.stride)):
                ops.shortcut_grad_add(self.dres, dx, self.stride)


class Bottleneck:
    """ResNet v1.5 bottleneck: 1x1 -> 3x3 (stride) -> 1x1 (x4), projection shortcut when the shape changes."""

    def __init__(self, reg, cin, width, stride, H, W):
        cout = 4 * width
        self.cin, self.cout, self.stride = cin, cout, stride
        self.proj = stride != 1 or cin != cout
        if self.proj:  # tf.layers creation order: shortcut conv first (as in the TF official model)
            self.convs = Conv(reg, cin, cout, 1, stride, H, W)
            self.bns = BN(reg, cout)
        self.conv1 = Conv(reg, cin, width, 1, 1, H, W)
        self.bn1 = BN(reg, width)
        self.conv2 = Conv(reg, width, width, 3, stride, H, W)
        self.bn2 = BN(reg, width)
        self.conv3 = Conv(reg, width, cout, 1, 1, self.conv2.OH, self.conv2.OW)
        self.bn3 = BN(reg, cout)
        self.OH, self.OW = self.conv3.OH, self.conv3.OW

    def bind(self, P, B, dev, arena):
        bf = dict(device=dev, dtype=ACT_DTYPE)
        w = self.conv1.cout
        convs = [self.conv1, self.conv2, self.conv3] + ([self.convs] if self.proj else [])
        for c in convs:
            c.bind(P, B, dev)
        self.bn1.bind(P, (B, self.conv1.OH, self.conv1.OW, w), dev, arena)
        self.bn2.bind(P, (B, self.OH, self.OW, w), dev, arena)
        self.bn3.bind(P, (B, self.OH, self.OW, self.cout), dev, arena)
        if self.proj:
            self.bns.bind(P, (B, self.OH, self.OW, self.cout), dev, arena)
            self.dsc = torch.empty(B, self.OH, self.OW, self.cout, **bf)
            self.dxs = torch.empty(B, self.conv1.H, self.conv1.W, self.cin, **bf)
        self.dc3 = torch.empty(B, self.OH, self.OW, self.cout, **bf)
        self.dres = torch.empty(B, self.OH, self.OW, self.cout, **bf)
        self.dh2 = torch.empty(B, self.OH, self.OW, w, **bf)
        self.dc2 = torch.empty(B, self.OH, self.OW, w, **bf)
        self.dh1 = torch.empty(B, self.conv1.OH, self.conv1.OW, w, **bf)
        self.dc1 = torch.empty(B, self.conv1.OH, self.conv1.OW, w, **bf)

    def fwd(self, x):
        self.x = x
        res, res_bn = x, None
        if self.proj:
            zs = self.convs.fwd(x, self.bns.stats)
            if x.is_cuda and not self.bns.infer:
                # the shortcut BN is applied inside bn3's residual apply (bn_apply res_bn): its output
                # (411 MB at the first stage, B=256) is neither written nor read back: 22.47-22.49 vs
                # 22.66-22.69 ms per step (profiles/r4_resnet50_residual_bn_fold_ab.txt)
                res, res_bn = self.bns.stats_only(zs), self.bns
            else:
                res = self.bns.fwd(zs, act=ops.ACT_NONE)
        # (bn1 / bn2 formed on conv2 / conv3's operand loads instead of stored - bit-identical, 10 %
        # slower end to end: measured in round 5 and removed, profiles/r5_resnet50_bn_fold_ab.txt)
        h1 = self.bn1.fwd(self.conv1.fwd(x, self.bn1.stats))
        h2 = self.bn2.fwd(self.conv2.fwd(h1, self.bn2.stats))
        return self.bn3.fwd(self.conv3.fwd(h2, self.bn3.stats), res=res, rstride=1, res_bn=res_bn)

    def bwd(self, dout, dx, dout_stats_done=False, next_bn=None):
        """``next_bn``: (BN, its x) of the layer that consumes dx (the previous block's bn3): its
        backward statistics come out of the launch that finishes dx; returns True if they did.
        ``dout_stats_done``: bn3's statistics of dout were produced that way by the next block."""
        # shortcut gradient straight into dx, the conv1 data gradient accumulated on top
        fuse = (dx is not None and self.conv1.can_accum and (not self.proj or self.convs.can_accum)
                and _SHORTCUT_FUSE)
        # identity shortcut: its gradient dout * ReLU'(block output) is added by conv1's data-gradient
        # epilogue from dout and bn3's bit mask - bn3's backward does not store it at all
        masked = fuse and not self.proj and self.bn3.use_bits and self.conv1.stride == 1
        # projection shortcut: its BN's backward reads dout and bn3's bit mask directly - bn3's backward
        # does not store the masked gradient (dres) for it to read back twice: 22.32-22.34 vs 22.43-22.46
        # ms per step (profiles/r4_resnet50_residual_bn_fold_ab.txt)
        proj_bits = self.proj and self.bn3.use_bits and _PROJ_FROM_BITS
        dres = None if (masked or proj_bits) else (dx if (fuse and not self.proj) else self.dres)
        # Capture order: each data gradient BEFORE the weight gradient forked at the same point (the
        # fork event is taken when dy is final).  The hipGraph executor keeps a node's first-captured
        # child on its queue; with the weight gradient captured first, the data-gradient chain kept
        # landing on the side queue behind the weight gradients - 13 stalls, ~1.5 ms per step
        # (profiles/r4_resnet50_graph_order.txt)
        fork = SideStream.fork_point
        # (projection block: the shortcut BN's backward statistics come out of bn3's statistics pass)
        dual = proj_bits and not dout_stats_done  # 22.19-22.30 vs 22.30-22.41 ms (r4_resnet50_residual_bn_fold_ab)
        self.bn3.bwd(dout, self.conv3.y, self.dc3, dres=dres, stats_done=dout_stats_done,
                     res_bn=(self.bns, self.convs.y) if dual else None)
        ev = fork()
        done = self.conv3.dgrad(self.dc3, self.dh2, bn_bwd=self.bn2.bwd_stats_args(self.conv2.y))
        self.conv3.wgrad(self.dc3, self.bn2.y, after=ev)
        self.bn2.bwd(self.dh2, self.conv2.y, self.dc2, stats_done=done)
        ev = fork()
        done = self.conv2.dgrad(self.dc2, self.dh1, bn_bwd=self.bn1.bwd_stats_args(self.conv1.y))
        self.conv2.wgrad(self.dc2, self.bn1.y, after=ev)
        self.bn1.bwd(self.dh1, self.conv1.y, self.dc1, stats_done=done)
        ev1 = fork()
        evs = None
        if self.proj:
            if proj_bits:  # g = dout * ReLU'(block output) = what dres held, bit for bit
                self.bns.bwd(dout, self.convs.y, self.dsc, act=ops.ACT_RELU, mask=self.bn3.ybits, stats_done=dual)
            else:
                self.bns.bwd(self.dres, self.convs.y, self.dsc, act=ops.ACT_NONE)
            evs = fork()
        nb = next_bn[0].bwd_stats_args(next_bn[1]) if next_bn is not None else None
        ret = None
        if dx is not None:
            if fuse:
                if self.proj:
                    # the strided shortcut's data gradient first (it covers every pixel, zeros on the
                    # parity phases no tap reaches), conv1's (stride 1, all pixels) accumulated on top:
                    # the LAST producer of dx covers every pixel, so it can fold the previous block's
                    # bn3 backward statistics into its epilogue
                    self.convs.dgrad(self.dsc, dx)
                    ret = self.conv1.dgrad(self.dc1, dx, accumulate=True, bn_bwd=nb)
                else:
                    ret = self.conv1.dgrad(self.dc1, dx, accumulate=True, bn_bwd=nb,
                                           acc_src=(dout, self.bn3.ybits) if masked else None)
            else:
                self.conv1.dgrad(self.dc1, dx)
                if self.proj:
                    self.convs.dgrad(self.dsc, self.dxs)
                    ops.shortcut_grad_add(self.dxs, dx, 1)
                else:
                    ops.shortcut_grad_add(self.dres, dx, 1)
        self.conv1.wgrad(self.dc1, self.x, after=ev1)
        if self.proj:
            self.convs.wgrad(self.dsc, self.x, after=evs)
        return ret


class Dense:
    """fp32 classifier layer (exact-fp32 MFMA GEMMs; tiny next to the convs)."""

    def __init__(self, reg, cin, cout):
        self.cin, self.cout = cin, cout
        s = reg.scope("dense")
        self.kernel = reg.add(VarSpec(s + "/kernel", (cout, cin), _glorot(cin, cout), tf_shape=(cin, cout),
                                      to_tf=_fc_to_tf, from_tf=_fc_to_tf))
        self.bias = reg.add(VarSpec(s + "/bias", (cout,), _const(0.0)))


# ------------------------------------------------------------------- model
ARCHS = {
    # name: (image, channels, classes, builder)
    "resnet20": (32, 3, 10),
    "resnet50": (224, 3, 1000),
}


def build(arch, reg):
    """Create the layers (and their VarSpecs, in TF creation order) of an architecture."""
    img, ch, ncls = ARCHS[arch]
    L = {}
    if arch == "resnet20":
        L["stem"] = Conv(reg, ch, 16, 3, 1, img, img)
        L["stem_bn"] = BN(reg, 16)
        blocks, H, cin = [], img, 16
        for stage, cout in enumerate((16, 32, 64)):
            for i in range(3):
                stride = 2 if (stage > 0 and i == 0) else 1
                n0 = len(reg.specs)
                b = BasicBlock(reg, cin, cout, stride, H, H)
                b.var_names = [sp.name for sp in reg.specs[n0:]]
                blocks.append(b)
                H, cin = b.OH, cout
        L["blocks"], L["feat"], L["HW"] = blocks, cin, H
    else:
        L["stem"] = Conv(reg, ch, 64, 7, 2, img, img)
        L["stem_bn"] = BN(reg, 64)
        H = L["stem"].OH
        L["pool_hw"] = ((H + 2 - 3) // 2 + 1)
        H, cin = L["pool_hw"], 64
        blocks = []
        for stage, (width, n) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
            for i in range(n):
                stride = 2 if (stage > 0 and i == 0) else 1
                n0 = len(reg.specs)
                b = Bottleneck(reg, cin, width, stride, H, H)
                b.var_names = [sp.name for sp in reg.specs[n0:]]
                blocks.append(b)
                H, cin = b.OH, b.cout
        L["blocks"], L["feat"], L["HW"] = blocks, cin, H
    L["dense"] = Dense(reg, L["feat"], ncls)
    return L


class ResNetModel(ModelDef):
    default_steps = 1000
    dtypes = ("bf16",)

    def __init__(self, lr: float = 0.1, arch: str = "resnet20"):
        self.name = arch
        self.arch = arch
        self.default_batch = 128 if arch == "resnet20" else 64
        reg = Registry()
        self.layers = build(arch, reg)
        creation = [s.name for s in reg.specs]
        self.var_order = creation + ["global_step"]
        self.gs_name = "global_step"
        # flat (gradient bucket) order = backward completion order: head first, stem last
        self.specs = list(reversed(reg.specs))
        trainable = [n for n in creation if not n.endswith(("/moving_mean", "/moving_variance"))]
        self.opt_groups = [(OptimizerConfig(kind="momentum", lr=lr, momentum=0.9), trainable,
                            ("beta1_power", "beta2_power"))]
        self.image, self.channels, self.num_classes = ARCHS[arch]

    def num_params(self, trainable_only=True):
        names = set(self.opt_groups[0][1]) if trainable_only else None
        return sum(s.numel for s in self.specs if names is None or s.name in names)

    def flops_per_image(self) -> float:
        """fwd+bwd conv/fc FLOPs per image (3x the forward MACs*2; the stem has no dgrad)."""
        L = self.layers
        convs = [L["stem"]]
        for b in L["blocks"]:
            convs += [c for c in (getattr(b, "convs", None), b.conv1, b.conv2, getattr(b, "conv3", None)) if c]
        f = 0.0
        for i, c in enumerate(convs):
            fwd = 2.0 * c.OH * c.OW * c.cout * c.k * c.k * c.cin
            f += fwd * (2 if i == 0 else 3)
        d = L["dense"]
        return f + 3 * 2.0 * d.cin * d.cout

    def program(self, device, batch_size=None, seed: int = 0):
        return ResNetProgram(self, device, batch_size or self.default_batch, seed)


class ResNetProgram(StepProgram):
    def __init__(self, model, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        if self.device.type == "cuda":
            ops.require()
        reg = Registry()
        self.L = L = build(model.arch, reg)  # same names as the ModelDef (deterministic)
        B, dev, P = batch_size, self.device, self.P
        img, ch = model.image, model.channels
        n_bn = sum(1 for s in reg.specs if s.name.endswith("/gamma"))
        max_c = max(s.shape[0] for s in reg.specs if s.name.endswith("/gamma"))
        self.arena = Arena(n_bn * (6 * max_c + 64), dev)
        bf = dict(device=dev, dtype=ACT_DTYPE)
        self.x = torch.empty(B, img, img, ch, **bf)
        self.y = torch.empty(B, model.num_classes, device=dev)
        L["stem"].bind(P, B, dev)
        st = L["stem"]
        L["stem_bn"].bind(P, (B, st.OH, st.OW, st.cout), dev, self.arena)
        self.d_stem = torch.empty(B, st.OH, st.OW, st.cout, **bf)
        self.dc_stem = torch.empty(B, st.OH, st.OW, st.cout, **bf)
        if "pool_hw" in L:
            ph = L["pool_hw"]
            self.pool = torch.empty(B, ph, ph, st.cout, **bf)
            self.pool_am = torch.empty(B, ph, ph, st.cout, device=dev, dtype=torch.uint8)
            self.d_pool = torch.empty(B, ph, ph, st.cout, **bf)
        for b in L["blocks"]:
            b.bind(P, B, dev, self.arena)
        # block input-gradient buffers: d_in[i] is the gradient w.r.t. block i's input
        self.d_in = [torch.empty(B, b.conv1.H, b.conv1.W, b.cin, **bf) for b in L["blocks"]]
        self.d_last = torch.empty(B, L["HW"], L["HW"], L["feat"], **bf)
        d = L["dense"]
        self.feat16 = torch.empty(B, d.cin, **bf)
        self.feat = torch.empty(B, d.cin, device=dev)
        self.logits = torch.empty(B, d.cout, device=dev)
        self.dlogits = torch.empty(B, d.cout, device=dev)
        self.dfeat = torch.empty(B, d.cin, device=dev)
        self.dfeat16 = torch.empty(B, d.cin, **bf)
        self.loss = torch.zeros(1, device=dev)
        self.correct = torch.zeros(1, dtype=torch.int32, device=dev)
        # lowest flat offset of each block's variables: after block i's backward every gradient
        # at or above it is final (variables are laid out in creation = forward order)
        self.block_lo = [min(P.offsets[n] for n in b.var_names) for b in L["blocks"]]
        self.dense_lo = min(P.offsets[d.kernel], P.offsets[d.bias])
        self.grad_ready = None  # optional backward-progress hook (BucketAllReduce.ready)
        self.training = True    # False inside evaluate(): no fused head (it writes gradients), no BN folds
        self._defer_convs = [c for b in L["blocks"] for c in (b.conv1, b.conv2, getattr(b, "conv3", None))
                             if c is not None and c.img_wgrad and c.cin % 16 == 0 and B >= 128]
        self._defer_ok = self.device.type == "cuda" and _WGRAD_DEFER and 0 < len(self._defer_convs) <= 32
        self._defer_ws = {c: torch.empty(ops.wgrad_ws_floats(c.cout, c.k * c.k * c.cin), device=dev)
                          for c in self._defer_convs} if self._defer_ok else {}
        self.defer_wgrad = False
        # ResNet-50 (bottleneck) weight gradients on a side stream (SideStream; DTFE_WGRAD_STREAM=0 off)
        self.side = None
        if self.device.type == "cuda" and _WGRAD_STREAM and model.arch == "resnet50":
            self.side = SideStream(self.device)
            for b in L["blocks"]:
                for c in (b.conv1, b.conv2, b.conv3, getattr(b, "convs", None)):
                    if c is not None:
                        c.side = self.side

    def _ready(self, lo):
        """Backward progress: every gradient at flat offset >= lo has been launched.  The bucket's
        weight gradients may still run on the wgrad side stream: the all-reduce fork waits on an
        event recorded there, the compute stream does not (no per-block join serialising the
        data-gradient chain behind the weight gradients).

        Deferred weight-gradient reduces: the ones queued so far are flushed as ONE grouped launch
        just before the hook launches a bucket (only when a bucket boundary is crossed, so the
        multi-rank schedules keep most of the 18 -> 1 saving; profiles/r6_resnet20_bucket_flush.txt)."""
        if self.grad_ready is not None:
            if self.defer_wgrad and self._bucket_completes(lo):
                ops.wgrad_flush()
            after = None
            if self.side is not None and self.side.pending:
                after = [self.side.mark()]
            self.grad_ready(lo, after)

    def _bucket_completes(self, lo):
        """Whether the progress hook launches a bucket at ``lo`` (some bucket starts at or above lo
        and was not reached before).  Hooks without a bucket list: every call counts."""
        bks = getattr(getattr(self.grad_ready, "__self__", None), "buckets", None)
        if bks is None:
            return True
        fire = any(self._ready_lo > b[0] >= lo for b in bks)
        self._ready_lo = min(self._ready_lo, lo)
        return fire

    def load_batch(self, batch):
        x, y = batch
        self.x.copy_(x.reshape(self.x.shape).to(self.x.dtype))
        yy = y.reshape(self.batch_size, -1)
        if yy.shape[1] == 1:
            self.y.zero_()
            self.y.scatter_(1, yy.long(), 1.0)
        else:
            self.y.copy_(yy)

    def forward(self):
        L = self.L
        z = L["stem"].fwd(self.x, L["stem_bn"].stats)
        if "pool_hw" in L:
            h = L["stem_bn"].fwd_pool3(z, self.pool, self.pool_am)
        else:
            h = L["stem_bn"].fwd(z)
        for b in L["blocks"]:
            h = b.fwd(h)
        ops.gap_fwd(h, self.feat16)
        d, P, B = L["dense"], self.P, self.batch_size
        # the classifier head's forward and backward as one launch where it fits one workgroup
        # (ResNet-20: 7 launches fewer, profiles/r5_resnet20_kernels.txt); not in evaluation (it
        # writes the dense gradients: only while training, never from evaluate())
        self.head_fused = False
        if self.device.type == "cuda" and self.training and _HEAD_FUSE:
            self.head_fused = ops.dense_head(self.feat16, P.view(d.kernel), P.view(d.bias), self.y, self.logits,
                                             self.loss, self.correct, P.gview(d.kernel), P.gview(d.bias),
                                             self.dfeat16, 1.0 / B)
            if self.head_fused:
                return
        ops.cast_(self.feat16, self.feat)
        ops.gemm(self.feat, P.view(d.kernel), self.logits, M=B, N=d.cout, K=d.cin, bias=P.view(d.bias))
        ops.softmax_xent(self.logits, labels_oh=self.y, scale=1.0 / B, dlogits=self.dlogits, loss_sum=self.loss,
                         correct=self.correct)

    def backward(self):
        # the deferred weight-gradient queue (a thread-local list of device pointers in the kernel
        # library) must be empty here: a stale entry would reduce into freed or foreign buffers
        if self._defer_ok:
            stale = ops.wgrad_pending()
            if stale:
                ops.wgrad_discard()
                raise RuntimeError(f"ResNetProgram.backward: {stale} deferred weight-gradient reduce(s) left "
                                   "queued by an earlier interrupted backward or a stray imgwgrad(defer=True); "
                                   "discarded - rerun the step")
        try:
            self._backward()
        except BaseException:
            if self._defer_ok:
                ops.wgrad_discard()  # nothing queued by this backward may leak into the next one
            raise

    def _backward(self):
        L, P, B = self.L, self.P, self.batch_size
        # the whole-image weight gradients queue their partial-slab reduces (own workspaces); ONE
        # grouped launch sums them: at the end of the backward with one replica
        # (profiles/r5_resnet20_kernels.txt), before each bucket's launch when a progress hook (all-reduce
        # / ps push) waits on per-block gradients (_ready)
        self.defer_wgrad = self._defer_ok
        self._ready_lo = 1 << 62
        for c in self._defer_convs:
            c.defer_ws = self._defer_ws[c] if self.defer_wgrad else None
        d = L["dense"]
        fused = getattr(self, "head_fused", False)
        if not fused:
            ops.gemm(self.dlogits, self.feat, P.gview(d.kernel), M=d.cout, N=d.cin, K=B, amode=ops.RMAJ,
                     lda=d.cout, bmode=ops.RMAJ, ldb=d.cin)
            ops.colsum(self.dlogits, B, d.cout, d.cout, P.gview(d.bias))
        self._ready(self.dense_lo)
        if not fused:
            ops.gemm(self.dlogits, P.view(d.kernel), self.dfeat, M=B, N=d.cin, K=d.cout, bmode=ops.RMAJ, ldb=d.cin)
            ops.cast_(self.dfeat, self.dfeat16)
        ops.gap_bwd(self.dfeat16, self.d_last)
        dout = self.d_last
        blocks = L["blocks"]
        done = False
        for i in range(len(blocks) - 1, -1, -1):
            if isinstance(blocks[i], Bottleneck):
                # (a projection block's bn3 statistics stay with that block: its statistics pass also
                # produces the shortcut BN's, Bottleneck.bwd)
                nb = (blocks[i - 1].bn3, blocks[i - 1].conv3.y) if i > 0 and not (
                    _PROJ_FROM_BITS and blocks[i - 1].proj and blocks[i - 1].bn3.use_bits) else None
                done = bool(blocks[i].bwd(dout, self.d_in[i], dout_stats_done=done, next_bn=nb))
            else:
                blocks[i].bwd(dout, self.d_in[i])
            self._ready(self.block_lo[i])
            dout = self.d_in[i]
        st = L["stem"]
        if "pool_hw" in L:
            L["stem_bn"].bwd_pool3(dout, self.pool_am, st.y, self.dc_stem, self.d_stem)
        else:
            L["stem_bn"].bwd(dout, st.y, self.dc_stem)
        st.wgrad(self.dc_stem, self.x)
        if self.defer_wgrad:
            ops.wgrad_flush()  # every (remaining) deferred weight-gradient reduce in one launch
        if self.side is not None:
            self.side.join()
        self._ready(0)

    def step_accumulators(self):
        """The buffers a step accumulates into (cleared at its start): gradients, BN statistics,
        loss and hit counters.  ``ops.gather_rows(zero=...)`` clears them inside the batch gather."""
        return [self.P.grad, self.arena.buf, self.loss, self.correct]

    def compute_grads(self, zeroed: bool = False):
        """Forward + backward.  ``zeroed``: the caller already cleared ``step_accumulators()``
        (bench.py does it in the fused gather launch, so no fill kernel runs per step)."""
        if not zeroed:
            for t in self.step_accumulators():
                t.zero_()
        self.forward()
        self.backward()
        return {"loss": ScaledScalar(self.loss, 1.0 / self.batch_size), "correct": self.correct}

    def batchnorms(self):
        L = self.L
        out = [L["stem_bn"]]
        for b in L["blocks"]:
            out += [bn for bn in (getattr(b, "bns", None), b.bn1, b.bn2, getattr(b, "bn3", None)) if bn is not None]
        return out

    def evaluate(self, images, labels) -> float:
        """Top-1 accuracy with inference-mode BatchNorm (the moving averages; TF ``training=False``),
        the evaluation analog of LSTM:134-138.  Any number of images, in program-batch chunks (the
        last one padded by repeating rows; only the real rows are counted).  Parameters and moving
        averages are left untouched; the step accumulators the forward touched are cleared."""
        n, B = images.shape[0], self.batch_size
        bns = self.batchnorms()
        for bn in bns:
            bn.infer = True
        self.training = False
        hits = 0
        try:
            for lo in range(0, n, B):
                m = min(B, n - lo)
                idx = torch.arange(lo, lo + B, device=images.device).clamp_max(n - 1)
                self.load_batch((images[idx], labels[idx]))
                self.forward()
                hits += int((self.logits[:m].argmax(1) == self.y[:m].argmax(1)).sum().item())
        finally:
            self.training = True
            for bn in bns:
                bn.infer = False
            for t in self.step_accumulators()[1:]:
                t.zero_()
        return hits / n
