"""MNIST 2-layer CNN - the north-star headline workload (BASELINE.json config 2/4).

Architecture (TensorFlow-Examples ``convolutional_network``, the notebook
family the reference scripts come from, ENC:14):

    x[B,28,28,1] -> conv5x5 1->32 SAME + ReLU -> maxpool 2x2
                 -> conv5x5 32->64 SAME + ReLU -> maxpool 2x2
                 -> fc 3136->1024 + ReLU -> dropout(keep 0.75) -> fc 1024->10
                 -> softmax cross-entropy                     (3,274,634 params)

MI355X design: the step is an explicit program of 10 fused HIP kernels over
pre-allocated NHWC bf16 buffers (fp32 master weights / grads / Adam slots in
one flat buffer), captured into one hipGraph:

  gather      batch from the HBM-resident dataset (device RNG, no host feed)
  conv1/pool  1-channel LDS image, tap-packed MFMA (k = 25 taps in one step),
              bias+ReLU+2x2 max-pool+argmax in registers
  conv2/pool  whole-image LDS conv (A fragments = ds_read_b128 of the staged image),
              same fused pool epilogue (rows in pool-window order)
  fc1         MFMA GEMM, bias+ReLU+dropout epilogue
  head        fc2 + softmax-xent + dlogit rows + dropout/ReLU grad (one wave per row)
  head wgrad  split-K MFMA GEMM dlogit^T . H, bias grad through a ones column
  fc1 dgrad   MFMA GEMM (W1 read through ds_read_b64_tr_b16), ReLU'(P2) epilogue
              -> pooled-res dP2 (never un-pooled in memory)
  fc1 wgrad   MFMA GEMM (both operands via the transposing LDS read), fc1 bias
              grad as its ones column
  conv2 dgrad whole-image LDS conv over un-pool(dP2) (argmax routing while staging),
              flipped taps, ReLU'(P1) epilogue -> pooled-res dP1
  conv2 wgrad whole-image LDS wgrad, both operands by ds_read_b64_tr_b16, bias grad
  conv1 wgrad tap-packed (dW^T = shifted image^T . un-pool(dP1)), un-pooling while staging
  Adam        one fused TF1 Adam launch, writes the bf16 (+ transposed) copies

In data-parallel mode the fc/head gradient bucket (98% of the bytes) is
all-reduced over RCCL while the conv backward kernels still run.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from .. import ops
from ..optim import FlatParams, Optimizer, OptimizerConfig, VarSpec
from .base import ModelDef, ScaledScalar, StepProgram

IMG, C1, C2, FC, NCLS = 28, 32, 64, 1024, 10
KS = 5


def _normal(std):
    return lambda shape, g: torch.randn(*shape, generator=g) * std


def _zeros(shape, g):
    return torch.zeros(*shape)


def _conv_to_tf(t):   # ours [Cout][KH][KW][Cin] -> TF [KH][KW][Cin][Cout]
    return t.permute(1, 2, 3, 0).contiguous()


def _conv_from_tf(t):
    return t.permute(3, 0, 1, 2).contiguous()


def _fc_to_tf(t):     # ours [out][in] -> TF [in][out]
    return t.t().contiguous()


def _fc_from_tf(t):
    return t.t().contiguous()


def var_specs():
    """Variables in TF creation order (weights dict then biases dict, as in the
    TensorFlow-Examples notebook) -> TF auto names Variable, Variable_1, ...

    Flat-buffer order is the backward-completion order (head first, conv1
    last) so gradient buckets fill front to back.
    """
    tf_order = [
        ("wc1", (C1, KS, KS, 1), _normal(0.1), "conv"),
        ("wc2", (C2, KS, KS, C1), _normal(0.05), "conv"),
        ("wd1", (FC, 7 * 7 * C2), _normal(0.02), "fc"),
        ("out", (NCLS, FC), _normal(0.05), "fc"),
        ("bc1", (C1,), _zeros, None),
        ("bc2", (C2,), _zeros, None),
        ("bd1", (FC,), _zeros, None),
        ("bout", (NCLS,), _zeros, None),
    ]
    names = {}
    for i, (k, *_rest) in enumerate(tf_order):
        names[k] = "Variable" if i == 0 else f"Variable_{i}"
    spec = {}
    for k, shape, init, kind in tf_order:
        kw = dict(name=names[k], shape=shape, init=init)
        if kind == "conv":
            kw.update(bf16=True, to_tf=_conv_to_tf, from_tf=_conv_from_tf,
                      tf_shape=(shape[1], shape[2], shape[3], shape[0]))
        elif kind == "fc":
            kw.update(bf16=True, to_tf=_fc_to_tf, from_tf=_fc_from_tf, tf_shape=(shape[1], shape[0]))
        spec[k] = VarSpec(**kw)
    # transposed bf16 copies needed by the backward GEMMs
    spec["wc2"].transpose = (C2, KS * KS, C1)    # -> Wt[C1][25][C2] for conv2 dgrad
    # fc1 dgrad reads W1 [1024][3136] itself through the transposing LDS read (RMAJ operand)
    flat_order = ["out", "bout", "bd1", "wd1", "wc2", "bc2", "wc1", "bc1"]
    return [spec[k] for k in flat_order], names


def num_params():
    specs, _ = var_specs()
    return sum(s.numel for s in specs)


class SyntheticMnist:
    """HBM-resident MNIST-shaped dataset (uint8 pixels + int32 labels)."""

    def __init__(self, n: int, device, seed: int = 1234, images=None, labels=None):
        if images is None:
            g = torch.Generator().manual_seed(seed)
            images = torch.randint(0, 256, (n, IMG * IMG), generator=g, dtype=torch.uint8)
            labels = torch.randint(0, NCLS, (n,), generator=g, dtype=torch.int32)
        self.images = images.to(device).contiguous()
        self.labels = labels.to(device=device, dtype=torch.int32).contiguous()
        self.n = self.images.shape[0]


class MnistCnnTrainer:
    """Per-rank training-step program for the MNIST CNN."""

    def __init__(self, batch: int, device, lr: float = 1e-3, keep_prob: float = 0.75, seed: int = 0,
                 data: SyntheticMnist | None = None, allreduce=None, world_size: int = 1, P: FlatParams | None = None,
                 standalone: bool = True, rank: int = 0):
        """standalone: own optimizer + HBM dataset (bench / smoke).  With standalone=False the
        caller supplies P and the batches (``CnnProgram``: ps / all-reduce roles of train.py)."""
        self.B = batch
        self.device = torch.device(device)
        if self.device.type == "cuda":
            ops.require()  # GPU buffers always take the HIP kernels; fail loudly without them
        self.keep = keep_prob
        # weights come from `seed` (identical on every replica); batch sampling and dropout
        # streams are offset by `rank` so data-parallel replicas train on different data
        self.seed = seed + 7919 * rank
        self.world = world_size
        self.allreduce = allreduce
        specs, self.names = var_specs()
        self.P = P if P is not None else FlatParams(specs, self.device, seed=seed)
        self.global_step = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.opt = self.data = None
        if standalone:
            self.opt = Optimizer(OptimizerConfig(kind="adam", lr=lr), self.P, global_step=self.global_step)
            self.data = data or SyntheticMnist(60000, self.device, seed=self.seed + 17)
        d = self.device
        B = batch
        bf = torch.bfloat16
        self.x = torch.empty(B, IMG, IMG, 1, device=d, dtype=bf)
        self.labels = torch.empty(B, dtype=torch.int32, device=d)
        self.p1 = torch.empty(B, 14, 14, C1, device=d, dtype=bf)
        self.a1 = torch.empty(B, 14, 14, C1, device=d, dtype=torch.uint8)
        self.p2 = torch.empty(B, 7, 7, C2, device=d, dtype=bf)
        self.a2 = torch.empty(B, 7, 7, C2, device=d, dtype=torch.uint8)
        self.h = torch.empty(B, FC, device=d, dtype=bf)
        self.dzf = torch.empty(B, FC, device=d, dtype=bf)
        self.dl = torch.empty(B, 16, device=d, dtype=bf)      # dlogit rows (10 classes, padded to 16)
        self.dp2 = torch.empty(B, 7, 7, C2, device=d, dtype=bf)    # pooled-res conv2 grad (ReLU-masked)
        self.dp1 = torch.empty(B, 14, 14, C1, device=d, dtype=bf)  # pooled-res conv1 grad (ReLU-masked)
        self.loss_sum = torch.zeros(1, device=d)
        self.correct = torch.zeros(1, dtype=torch.int32, device=d)
        self.data_ctr = torch.zeros(1, dtype=torch.int64, device=d)
        self.data_done = torch.zeros(1, dtype=torch.int32, device=d)
        self.no_done = torch.zeros(0, dtype=torch.int32, device=d)
        self.g1 = dict(B=B, H=IMG, W=IMG, C=1, Cout=C1, OH=IMG, OW=IMG, KH=KS, KW=KS, stride=1, pad=2)
        self.g2 = dict(B=B, H=14, W=14, C=C1, Cout=C2, OH=14, OW=14, KH=KS, KW=KS, stride=1, pad=2)
        # whole-image LDS conv geometry: conv1 (1-channel tap-packed kernels), conv2 (forward /
        # weight-grad) and conv2's data-grad
        self.ic1 = dict(B=B, SH=IMG, SW=IMG, CS=1, OH=IMG, OW=IMG, N=C1, KH=KS, KW=KS, stride=1, pad=2)
        self.ic2 = dict(B=B, SH=14, SW=14, CS=C1, OH=14, OW=14, N=C2, KH=KS, KW=KS, stride=1, pad=2)
        self.ic2_dgrad = dict(B=B, SH=14, SW=14, CS=C2, OH=14, OW=14, N=C1, KH=KS, KW=KS, stride=1, pad=KS - 1 - 2)
        n = self.names
        P = self.P
        self.w = {k: P.w16[n[k]] for k in ("wc1", "wc2", "wd1", "out")}
        self.wt = {"wc2": P.wt16[n["wc2"]]}
        self.b = {k: P.view(n[k]) for k in ("bc1", "bc2", "bd1", "bout")}
        self.gw = {k: P.gview(n[k]) for k in ("wc1", "wc2", "wd1", "out", "bc1", "bc2", "bd1", "bout")}
        # gradient buckets in flat order: [head + fc1] then [conv2 + conv1]
        lo1, hi1 = P.range_of([n["out"], n["bout"], n["bd1"], n["wd1"]])
        lo2, hi2 = P.range_of([n["wc2"], n["bc2"], n["wc1"], n["bc1"]])
        self.buckets = [(lo1, hi1), (lo2, hi2)]
        # the only step state that is accumulated into (atomics) rather than stored: the head
        # weight grad (split-K atomics), the conv weight grads (partial-sum reduce), the loss /
        # hit counters.  fc1's weight + bias grads (98% of P.grad) are plain stores.
        ra = P.range_of([n["out"], n["bout"]])
        rc = P.range_of([n["wc2"], n["bc2"], n["wc1"], n["bc1"]])
        self.accum = [P.grad[ra[0]:ra[1]], P.grad[rc[0]:rc[1]], self.loss_sum, self.correct]
        # backward branches that do not feed the critical path (head/fc1 weight grads, conv2
        # weight grad) run on their own streams: inside the captured hipGraph they become
        # parallel branches that fill the CUs the dgrad chain leaves idle.  conv2's weight
        # grad gets its own partial-sum workspace (conv1's runs concurrently on the main stream).
        # DTFE_CNN_BRANCHES (A/B only): "fc,c2" (default), "fc", "c2" or "none".  Measured-slower
        # schedules were removed in round 3: the head weight gradient inside the fc1 dgrad launch
        # (profiles/r2_cnn_head_fuse_ab.txt), one combined weight-gradient branch, the critical
        # chain captured first (profiles/r2_cnn_branch_orders.txt), and the fc/head Adam as its own
        # launch on the fc branch (313-325 vs 293 us; superseded by the fc1 GEMM Adam epilogue).
        self.fused_gather = os.environ.get("DTFE_CNN_FUSED_GATHER", "1") != "0"
        br = os.environ.get("DTFE_CNN_BRANCHES", "fc,c2").split(",")
        self.par = self.device.type == "cuda" and bool(set(br) & {"fc", "c2"})
        self.br_fc = self.par and "fc" in br
        self.br_c2 = self.par and "c2" in br
        # conv2's data gradient is captured before its weight gradient (same fork point): the graph
        # runs the data gradient -> conv1 weight-gradient chain on the launch queue, first on the
        # CUs, and the weight gradient (192 workgroups) fills in beside it - 0.2103-0.2126 vs
        # 0.2159-0.2181 ms/step (profiles/r3_cnn_kernel_tuning.txt, r3y / r3z)
        self.dgrad_first = os.environ.get("DTFE_CNN_DGRAD_FIRST", "1") == "1"
        self.c2_blocks = int(os.environ.get("DTFE_CNN_C2_BLOCKS", "192" if self.dgrad_first else "128"))
        # Data-parallel "late split" (default whenever an all-reduce is attached): the fc/head Adam
        # (bucket 0, already reduced during the conv backward) runs while the small conv bucket's
        # all-reduce is still in flight, so that collective's latency hides behind ~20 us of Adam.
        self.opt_fc = self.opt_conv = None
        self._apply = None
        # (Adam for fc1 applied in the fc1 weight-gradient GEMM epilogue on one replica measured
        # ~45 us/step slower - its traffic contends with the persistent conv2 backward kernels -
        # and was removed: profiles/r3_cnn_fused_adam_ab.txt)
        self.late_split = os.environ.get("DTFE_CNN_SPLIT_APPLY", "1") != "0"
        # One replica, DTFE_CNN_FC_APPLY (where the fc/head Adam runs; its gradients are final once
        # the grouped fc backward launch is done and that launch is its weights' last reader):
        #   "join" - the whole-model Adam after the conv2 weight-gradient branch joins;
        #   "main" - on the main chain after conv1's weight gradient, before the join (its ~18 us
        #            hide the join's cross-queue wait), the conv Adam after the join;
        #   "c2"   - at the end of the conv2 weight-gradient branch, the conv Adam after the join.
        # (conv2's Adam can not move onto the branch: conv2's data gradient still reads its weights)
        self.fc_apply = os.environ.get("DTFE_CNN_FC_APPLY", "join")
        # fc1 GEMMs on the global_load_lds tiles (gemm_glds.h) where the shapes allow: the
        # forward streams 3 k-tiles deep (one 64x64 tile per CU), data / weight gradient take the
        # 2-stage variant (784 / 800 tiles, several workgroups per CU)
        self.glds = self.device.type == "cuda" and os.environ.get("DTFE_CNN_GLDS", "1") != "0"
        # DTFE_CNN_FC_GROUP=0: the fc backward as a forked side branch instead of one grouped launch
        self.fc_group = self.par and os.environ.get("DTFE_CNN_FC_GROUP", "1") != "0"
        # the head weight gradient as the grouped launch's first piece (4-column body, 84 VGPRs: the
        # GEMM pieces keep 5 workgroups per CU) - 0.2033-0.2071 vs 0.2105-0.2124 ms/step as its own
        # launch before the group (DTFE_CNN_HEAD_IN_GROUP=0; profiles/r3_cnn_kernel_tuning.txt r3ze)
        self.head_in_group = self.fc_group and os.environ.get("DTFE_CNN_HEAD_IN_GROUP", "1") == "1"
        K1 = 7 * 7 * C2
        # DTFE_CNN_TILES=fwd,dgrad,wgrad overrides the glds tile ids (A/B sweeps)
        tiles = [int(t) for t in os.environ.get("DTFE_CNN_TILES", "8,12,12").split(",")]
        self.t_fwd = self._glds_tile(self.p2, P.w16[n["wd1"]], B, FC, K1, K1, K1, tiles[0])
        self.t_dgrad = self._glds_tile(self.dzf, P.w16[n["wd1"]], B, K1, FC, FC, K1, tiles[1])
        self.t_wgrad = self._glds_tile(self.dzf, self.p2, FC, K1 + 1, B, FC, K1, tiles[2], b_ones_row=K1)
        # fc1 forward split-K (deterministic last-arriver combine, write-through slabs): A/B only -
        # 2 and 3 splits measured 1-2 % slower per step (profiles/r3_cnn_kernel_tuning.txt)
        self.fwd_splits = int(os.environ.get("DTFE_CNN_FWD_SPLITS", "1"))
        self.ws_fwd = None
        if self.fwd_splits > 1 and self.t_fwd is not None:
            self.ws_fwd = ops.split_workspace(d, self.fwd_splits, B, FC, self.t_fwd, private=True)
        # head weight gradient: split-K over the batch with the deterministic last-arriver combine
        # (fixed split order - no float atomics, so the step is bitwise reproducible); its own
        # workspace, since it runs on the fc branch beside other GEMMs
        self.head_gemm = os.environ.get("DTFE_CNN_HEAD_GEMM", "0") == "1" or batch > 1024
        self.head_splits = max(1, min(16, B // 128))
        bm, bn = ops.TILE_DIMS[4]
        ntiles = -(-NCLS // bm) * -(-(FC + 1) // bn)
        self.ws_head = (torch.empty(self.head_splits * ntiles * bm * bn, device=d, dtype=torch.float32),
                        torch.zeros(ntiles, device=d, dtype=torch.int32)) if self.head_splits > 1 else None
        if self.par:
            self.s_fc = torch.cuda.Stream(device=d)
            self.s_c2 = torch.cuda.Stream(device=d)
            self.ws_c2 = torch.empty(ops.wgrad_ws_floats(C2, KS * KS * C1), device=d, dtype=torch.float32)

    def _glds_tile(self, A, Bm, M, N, K, lda, ldb, tile, b_ones_row=-1):
        if self.glds and ops.glds_ok(A, Bm, M, N, K, tile, lda, ldb, b_ones_row=b_ones_row):
            return tile
        return None

    # ------------------------------------------------------------------
    def forward_backward(self):
        B = self.B
        fused = False
        if self.data is not None and self.device.type == "cuda" and B >= 256 and self.fused_gather:
            # standalone: batch sampling (advances data_ctr), accumulator clearing and conv1 in ONE launch
            # (the sampling counter is advanced by head_xent, after its last reader: fc1's dropout -
            # a grid-wide last-arriver atomic here serialised ~10 us of the launch)
            ops.require().conv1_gather_fwd(self.data.images, self.data.labels, self.seed + 1, self.data_ctr,
                                           self.no_done, self.labels, self.x, self.w["wc1"], self.b["bc1"],
                                           self.p1, self.a1, self.accum)
            fused = True
        else:
            if self.data is not None:  # sample the batch on device (advances data_ctr) and clear
                ops.gather_rows(self.data.images, self.x.view(B, -1), None, self.data.labels, self.labels,
                                seed=self.seed + 1, counter=self.data_ctr, done=self.data_done, zero=self.accum)
            else:
                for t in self.accum:
                    t.zero_()
            ops.imgconv(self.w["wc1"], self.p1, src=self.x, bias=self.b["bc1"], argmax=self.a1, act=ops.ACT_RELU,
                        pool=True, **self.ic1)
        ops.imgconv(self.w["wc2"], self.p2, src=self.p1, bias=self.b["bc2"], argmax=self.a2, act=ops.ACT_RELU,
                    pool=True, **self.ic2)
        K1 = 7 * 7 * C2
        ops.gemm(self.p2, self.w["wd1"], self.h, M=B, N=FC, K=K1, bias=self.b["bd1"], act=ops.ACT_RELU,
                 keep=self.keep, seed=self.seed + 2, counter=self.data_ctr, tile=self.t_fwd, splits=self.fwd_splits,
                 workspace=self.ws_fwd)
        ops.head_xent(self.h, self.w["out"], self.b["bout"], self.labels, self.dzf, self.dl, self.loss_sum,
                      self.correct, None, scale=1.0 / B, inv_keep=1.0 / self.keep,
                      step_counter=self.data_ctr if fused else None)
        main = torch.cuda.current_stream(self.device) if self.par else None
        if self.fc_group:
            # fc1 data gradient + fc1 weight gradient as ONE launch on the main
            # stream (ops.gemm_group): no fork / join of an fc side branch, whose cross-queue edges
            # cost 5-11 us of idle time each in the captured graph; the dispatcher starts the head and
            # data-gradient workgroups first (lower grid ranges)
            # (the head piece stays its own launch: its 10x8 accumulators per thread would set the
            # grouped kernel's register allocation to 148 VGPRs, 3 workgroups per CU instead of 7)
            if not self.head_in_group:
                self._head_wgrad()
            with ops.gemm_group(self.dzf):
                if self.head_in_group:
                    self._head_wgrad()   # recorded as the grouped launch's first piece
                self._fc1_dgrad(B, K1)
                self._fc1_wgrad(B, K1)
            if self.allreduce is not None:
                self.allreduce.launch(0)  # bucket 0 (head + fc1, 98% of the bytes)
        else:
            # weight-gradient branch of the fc layers (forked after head_xent), then the dgrad chain
            with self._branch(self.s_fc, main) if self.br_fc else contextlib.nullcontext():
                self._head_wgrad()
                self._fc1_wgrad(B, K1)
                if self.allreduce is not None:
                    self.allreduce.launch(0)  # bucket 0 (head + fc1, 98% of the bytes) forks off this branch
            self._fc1_dgrad(B, K1)
        def conv2_wgrad(forked=False):
            ctx = contextlib.nullcontext()
            if self.br_c2:
                ctx = torch.cuda.stream(self.s_c2) if forked else self._branch(self.s_c2, main)
            with ctx:
                # conv2 wgrad: dW = sum_p un-pool(dP2)[p] (x) P1[p + tap] ; bias grad alongside
                ops.imgwgrad(self.p1, self.gw["wc2"], self.gw["bc2"], dy_pooled=self.dp2, dy_argmax=self.a2,
                             workspace=self.ws_c2 if self.br_c2 else None,
                             max_blocks=self.c2_blocks if self.br_c2 else 0, **self.ic2)
                if self._apply is not None and self._apply[0] == "c2":
                    self.opt_fc.step(grad16=self._apply[1], gscale=self._apply[2], gs_inc=0)

        # (forking conv2's weight gradient after its data gradient, beside conv1's weight gradient,
        # measured 0.242 vs 0.233 ms/step: profiles/r3_cnn_c2_after_ab.txt)
        if self.dgrad_first and self.br_c2:
            # fork point unchanged (after the fc backward); the data gradient's graph node is
            # captured before the weight gradient's
            self.s_c2.wait_stream(main)
            self._conv2_dgrad()
            conv2_wgrad(forked=True)
        else:
            conv2_wgrad()
            self._conv2_dgrad()
        ops.imgwgrad(self.x, self.gw["wc1"], self.gw["bc1"], dy_pooled=self.dp1, dy_argmax=self.a1, **self.ic1)
        if self._apply is not None and self._apply[0] == "main":
            self.opt_fc.step(grad16=self._apply[1], gscale=self._apply[2], gs_inc=0)
        if self.br_fc and not self.fc_group:  # join the weight-grad branches
            main.wait_stream(self.s_fc)
        if self.br_c2:
            main.wait_stream(self.s_c2)
        if self.allreduce is not None:
            self.allreduce.launch(1)
            if self._apply is not None and self._apply[0] == "late":
                self.allreduce.wait_bucket(0)   # fc/head Adam overlaps the conv bucket's all-reduce
                self.opt_fc.step(grad16=self._apply[1], gscale=self._apply[2], gs_inc=0)
            self.allreduce.wait()
        if self._apply is not None:
            self.opt_conv.step(grad16=self._apply[1], gscale=self._apply[2], gs_inc=1)

    def _head_wgrad(self):
        """head wgrad: dW[10][1024] = dlogit^T . H, db = sum dlogit (dedicated whole-batch kernel; the
        split-K GEMM path is kept behind DTFE_CNN_HEAD_GEMM=1)"""
        if self.head_gemm:
            ops.gemm(self.dl, self.h, self.gw["out"], M=NCLS, N=FC + 1, K=self.B, amode=ops.RMAJ,
                     lda=self.dl.shape[1], bmode=ops.RMAJ, ldb=FC, ldc=FC, b_ones_row=FC, bias_out=self.gw["bout"],
                     splits=self.head_splits, tile=4, workspace=self.ws_head)
        else:
            ops.head_wgrad(self.dl, self.h, self.gw["out"], self.gw["bout"], NCLS)  # B <= 1024

    def _fc1_wgrad(self, B, K1):
        """fc1 wgrad: dW[1024][3136] = dZf^T . P2 ; bias grad = sum dZf via the ones column."""
        ops.gemm(self.dzf, self.p2, self.gw["wd1"], M=FC, N=K1 + 1, K=B, amode=ops.RMAJ, lda=FC,
                 bmode=ops.RMAJ, ldb=K1, ldc=K1, b_ones_row=K1, bias_out=self.gw["bd1"], tile=self.t_wgrad)

    def _fc1_dgrad(self, B, K1):
        """fc1 dgrad -> dP2 at pooled resolution, ReLU'(P2)-masked (consumers un-pool on load)."""
        ops.gemm(self.dzf, self.w["wd1"], self.dp2, M=B, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=self.p2,
                 aux_act=ops.ACT_RELU, tile=self.t_dgrad)

    def _conv2_dgrad(self):
        """conv2 dgrad: whole-image LDS conv over un-pool(dP2) with flipped taps -> dP1 (ReLU'(P1)-masked)."""
        ops.imgconv(self.wt["wc2"], self.dp1, src_pooled=self.dp2, src_argmax=self.a2, relu_mask=self.p1,
                    flip_taps=True, **self.ic2_dgrad)

    def _ensure_split(self):
        """fc/head and conv optimizers over disjoint var lists, sharing one set of slot buffers."""
        if self.opt_fc is None:
            n_, cfg = self.names, self.opt.cfg
            self.opt_fc = Optimizer(cfg, self.P, var_list=[n_[k] for k in ("out", "bout", "bd1", "wd1")],
                                    global_step=self.global_step)
            self.opt_conv = Optimizer(cfg, self.P, var_list=[n_[k] for k in ("wc2", "bc2", "wc1", "bc1")],
                                      global_step=self.global_step)
            self.opt_conv.s1, self.opt_conv.s2 = self.opt_fc.s1, self.opt_fc.s2

    @staticmethod
    def _branch(stream, main):
        """Run the enclosed launches on ``stream`` forked from ``main`` (no-op without one)."""
        if stream is None:
            return contextlib.nullcontext()
        stream.wait_stream(main)
        return torch.cuda.stream(stream)

    def apply(self):
        self.opt.step(gscale=1.0 / self.world)

    def step(self, grad16=None, gscale=None):
        """One training step: forward, backward (+ all-reduce), Adam.  ``grad16``: the all-reduced
        bf16 gradients to apply instead of P.grad; ``gscale`` defaults to 1/world."""
        gscale = 1.0 / self.world if gscale is None else gscale
        mode = None
        if self.par and self.br_fc and self.late_split and self.allreduce is not None:
            mode = "late"
        elif self.br_c2 and self.fc_group and self.fc_apply in ("main", "c2") and self.allreduce is None:
            mode = self.fc_apply
        if mode is None or (self.opt_fc is None and self.global_step_started()):
            self.forward_backward()
            self.opt.step(grad16=grad16, gscale=gscale)
            self._whole_steps = getattr(self, "_whole_steps", 0) + 1
            return
        self._ensure_split()
        self._apply = (mode, grad16, gscale)
        try:
            self.forward_backward()
        finally:
            self._apply = None

    def global_step_started(self) -> bool:
        """True once the whole-model optimizer has applied a step (its slots then hold the state,
        so the schedule must not switch to the split optimizers)."""
        return getattr(self, "_whole_steps", 0) > 0

    def flops_per_image(self) -> float:
        """Training FLOPs per image (fwd + dgrad + wgrad of every GEMM-shaped op)."""
        c1 = 2 * IMG * IMG * C1 * KS * KS
        c2 = 2 * 14 * 14 * C2 * KS * KS * C1
        f1 = 2 * 7 * 7 * C2 * FC
        f2 = 2 * FC * NCLS
        return c1 * 2 + c2 * 3 + f1 * 3 + f2 * 3  # conv1 has no dgrad


# ----------------------------------------------------------------------------
# ModelDef for the cluster roles of train.py (ps / sync ps / all-reduce / local):
# BASELINE.json config 4 "MNIST CNN parameter-server async SGD, 1 ps + 8 workers".
def tf_var_order():
    """TF creation order: weights dict, biases dict (Variable..Variable_7), then global_step."""
    return ["Variable"] + ["Variable_%d" % i for i in range(1, 9)]


class MnistCnnModel(ModelDef):
    """``ModelDef`` of the CNN (TensorFlow-Examples convolutional_network hyper-parameters:
    batch 128, Adam 1e-3, dropout keep 0.75)."""
    name = "cnn"
    default_batch = 128
    default_steps = 500
    gs_increments = 1
    needs_labels = True

    def __init__(self, lr: float = 1e-3):
        self.specs, self.names = var_specs()
        self.var_order = tf_var_order()
        self.gs_name = "Variable_8"
        self.opt_groups = [(OptimizerConfig(kind="adam", lr=lr), [s.name for s in self.specs],
                            ("beta1_power", "beta2_power"))]

    def program(self, device, batch_size=None, seed: int = 0):
        return CnnProgram(self, device, batch_size or self.default_batch, seed)


class CnnProgram(StepProgram):
    """StepProgram over MnistCnnTrainer's fused kernels (batches fed by the caller)."""

    def __init__(self, model, device, batch_size: int, seed: int = 0):
        super().__init__(model, device, batch_size, seed)
        self.core = MnistCnnTrainer(batch_size, self.device, seed=seed, P=self.P, standalone=False)

    def load_batch(self, batch):
        x, y = batch
        B = self.batch_size
        c = self.core
        c.x.copy_(x.reshape(B, IMG, IMG, 1).to(c.x.dtype))
        lab = y.reshape(B, -1)
        c.labels.copy_((lab.argmax(1) if lab.shape[1] > 1 else lab[:, 0]).to(c.labels.dtype))
        c.data_ctr += 1  # dropout stream position (the HBM gather advances it in standalone mode)

    def compute_grads(self):
        self.core.forward_backward()
        return {"loss": ScaledScalar(self.core.loss_sum, 1.0 / self.batch_size), "correct": self.core.correct}

    def evaluate(self, images, labels) -> float:
        raise NotImplementedError("the CNN example has no evaluation step")

