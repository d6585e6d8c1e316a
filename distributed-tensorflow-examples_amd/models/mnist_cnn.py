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
        # ONE schedule per world size (every measured-slower alternative was removed in round 4;
        # their A/B tables stay in profiles/r2_cnn_branch_orders.txt, r2_cnn_head_fuse_ab.txt,
        # r3_cnn_kernel_tuning.txt, r3_cnn_c2_after_ab.txt, r3_cnn_fused_adam_ab.txt):
        #   * batch sampling + accumulator clearing + conv1 in one launch (standalone, B >= 256);
        #   * the fc backward (head weight gradient, fc1 data + weight gradients) as ONE grouped
        #     launch on the main stream;
        #   * conv2's data gradient on the main stream, its weight gradient (192 workgroups, own
        #     partial-sum workspace) on a forked branch captured after it, conv1's weight gradient
        #     on the main stream beside it, then the join;
        #   * one replica: the whole-model Adam after the join.  Data parallel: the fc/head bucket's
        #     all-reduce is launched right after the grouped fc backward (before conv2's data
        #     gradient), and the fc/head Adam runs while the small conv bucket is still in flight
        #     ("late split"), then the conv Adam.
        self.par = self.device.type == "cuda"
        self.c2_blocks = 192
        # (test hooks, not knobs: the separate gather launch and the whole-model apply with an
        # all-reduce attached are the oracles the fused / split schedule is checked against)
        self.fused_gather = True
        self.late_split = True
        # fc1 GEMMs on the global_load_lds tiles (gemm_glds.h) where the shapes allow: the forward
        # (one 64x64 tile per CU, 49 k-tiles) with two 4-wave k-groups per workgroup, 3 stages each
        # (tile 19: 15.6 us vs 19.9 for one group, torch.mm 21.3 - profiles/r4_fc1_kgroups.txt);
        # data / weight gradient: the 8-wave 256x128 tile (gemm_fc.hip: 100 tiles each, 154 MB of
        # L2 -> LDS traffic for the pair instead of 410 MB on 64x64 tiles, profiles/r6_fc1_tile22.txt),
        # else the 64x64 2-stage tile
        K1 = 7 * 7 * C2
        self.t_fwd = self._glds_tile(self.p2, P.w16[n["wd1"]], B, FC, K1, K1, K1, 19)
        self.t_dgrad = (self._glds_tile(self.dzf, P.w16[n["wd1"]], B, K1, FC, FC, K1, ops.FC_TILE, bmode=ops.RMAJ)
                        or self._glds_tile(self.dzf, P.w16[n["wd1"]], B, K1, FC, FC, K1, 12))
        self.t_wgrad = (self._glds_tile(self.dzf, self.p2, FC, K1 + 1, B, FC, K1, ops.FC_TILE, b_ones_row=K1,
                                        bmode=ops.RMAJ)
                        or self._glds_tile(self.dzf, self.p2, FC, K1 + 1, B, FC, K1, 12, b_ones_row=K1))
        if (self.t_dgrad == ops.FC_TILE) != (self.t_wgrad == ops.FC_TILE):  # one grouped launch: same tile
            self.t_dgrad = self._glds_tile(self.dzf, P.w16[n["wd1"]], B, K1, FC, FC, K1, 12)
            self.t_wgrad = self._glds_tile(self.dzf, self.p2, FC, K1 + 1, B, FC, K1, 12, b_ones_row=K1)
        # head weight gradient: the dedicated whole-batch kernel up to B = 1024, above that a split-K
        # GEMM with the deterministic last-arriver combine (own workspace: it runs in the group)
        self.head_gemm = batch > 1024
        # head_xent's per-workgroup loss / hit partials, folded by the head weight gradient's bias
        # workgroup instead of 256 same-address atomics (0.1943-0.1961 vs 0.1952-0.1985 ms/step,
        # profiles/r4_cnn_head_parts_ab.txt)
        self.head_parts = None if self.head_gemm else torch.zeros(2 * ((B + 3) // 4), device=d, dtype=torch.float32)
        self.head_splits = max(1, min(16, B // 128))
        bm, bn = ops.TILE_DIMS[4]
        ntiles = -(-NCLS // bm) * -(-(FC + 1) // bn)
        self.ws_head = (torch.empty(self.head_splits * ntiles * bm * bn, device=d, dtype=torch.float32),
                        torch.zeros(ntiles, device=d, dtype=torch.int32)) if self.head_gemm else None
        self.opt_fc = self.opt_conv = None
        self._late = None        # (grad16, gscale) while a data-parallel step runs its split Adam
        self.schedule = []       # launch order of the last step's milestones (host side = graph order)
        self.logits = None
        # (one replica runs the whole-model Adam after the backward: the fc/head Adam on a side
        # stream beside the conv backward measured 0.204 -> 0.234-0.241 ms/step,
        # profiles/r4_comm_rehearsal.txt)
        if self.par:
            self.s_c2 = torch.cuda.Stream(device=d)
            self.ws_c2 = torch.empty(ops.wgrad_ws_floats(C2, KS * KS * C1), device=d, dtype=torch.float32)
            # deferred join (opt-in, one replica, no all-reduce: bench.py with several steps per hipGraph
            # replay): the conv2 weight-gradient branch signals a device counter instead of a stream join
            # before Adam - Adam's wc2 / bc2 items wait on it (OptArgs::wait_done) - and the branch rejoins
            # the launch stream only in join_side(), once per replay.  The join is a cross-queue barrier
            # that idled the GPU ~11 us per step (profiles/r6_steps_per_graph.txt).
            self.c2_done = torch.zeros(1, device=d, dtype=torch.int32)
            self.c2_seen = torch.zeros(1, device=d, dtype=torch.int32)
        self.defer_join = False
        self._signalled = False
        # (the conv weight-gradient partial reduces stay their own launches: summing the partial slabs
        # inside the Adam launch measured 0.2033-0.2042 vs 0.1989-0.1997 ms/step,
        # profiles/r4_cnn_step_b1024.txt)

    def _glds_tile(self, A, Bm, M, N, K, lda, ldb, tile, b_ones_row=-1, bmode=ops.KMAJ):
        if self.device.type == "cuda" and ops.glds_ok(A, Bm, M, N, K, tile, lda, ldb, b_ones_row=b_ones_row,
                                                      bmode=bmode):
            return tile
        return None

    # ------------------------------------------------------------------
    def forward(self, keep=None, logits=None):
        """conv1 (+ the fused batch sampling in standalone mode), conv2, fc1 (+dropout), head.
        ``keep=1.0`` and a ``logits`` buffer: the evaluation forward (no dropout)."""
        B = self.B
        keep = self.keep if keep is None else keep
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
                 keep=keep, seed=self.seed + 2, counter=self.data_ctr, tile=self.t_fwd)
        ops.head_xent(self.h, self.w["out"], self.b["bout"], self.labels, self.dzf, self.dl, self.loss_sum,
                      self.correct, logits, scale=1.0 / B, inv_keep=1.0 / keep,
                      step_counter=self.data_ctr if fused else None,
                      parts=self.head_parts)

    def forward_backward(self):
        B = self.B
        K1 = 7 * 7 * C2
        self.schedule = []
        self.forward()
        main = torch.cuda.current_stream(self.device) if self.par else None
        # fc backward: head weight gradient, fc1 data gradient, fc1 weight gradient - ONE grouped
        # launch on the GPU (ops.gemm_group; no fork / join of an fc side branch, whose cross-queue
        # edges cost 5-11 us of idle time each in the captured graph)
        with ops.gemm_group(self.dzf):
            self._head_wgrad()
            self._fc1_dgrad(B, K1)
            self._fc1_wgrad(B, K1)
        if self.allreduce is not None:
            self.allreduce.launch(0)  # bucket 0 (head + fc1, 98% of the bytes) overlaps the conv backward
            self.schedule.append("allreduce:0")
        # conv2's data gradient is captured before its weight gradient (same fork point): the graph
        # runs the data gradient -> conv1 weight-gradient chain on the launch queue, first on the
        # CUs, and the weight gradient (192 workgroups) fills in beside it - 0.2103-0.2126 vs
        # 0.2159-0.2181 ms/step (profiles/r3_cnn_kernel_tuning.txt, r3y / r3z)
        if self.par:
            self.s_c2.wait_stream(main)
        self._conv2_dgrad()
        self.schedule.append("conv2_dgrad")
        signal = self.par and self.defer_join and self.allreduce is None
        with torch.cuda.stream(self.s_c2) if self.par else contextlib.nullcontext():
            # conv2 wgrad: dW = sum_p un-pool(dP2)[p] (x) P1[p + tap] ; bias grad alongside
            ops.imgwgrad(self.p1, self.gw["wc2"], self.gw["bc2"], dy_pooled=self.dp2, dy_argmax=self.a2,
                         workspace=self.ws_c2 if self.par else None,
                         max_blocks=self.c2_blocks if self.par else 0, **self.ic2)
            if signal:
                ops.epoch_signal(self.c2_done)
        ops.imgwgrad(self.x, self.gw["wc1"], self.gw["bc1"], dy_pooled=self.dp1, dy_argmax=self.a1, **self.ic1)
        self._signalled = signal
        if signal:
            self._pending_join = True
        elif self.par:
            main.wait_stream(self.s_c2)
        if self.allreduce is not None:
            self.allreduce.launch(1)
            self.schedule.append("allreduce:1")
            if self._late is not None:
                self.allreduce.wait_bucket(0)   # fc/head Adam overlaps the conv bucket's all-reduce
                self.opt_fc.step(grad16=self._late[0], gscale=self._late[1], gs_inc=0)
            self.allreduce.wait()
        if self._late is not None:
            self.opt_conv.step(grad16=self._late[0], gscale=self._late[1], gs_inc=1)

    def _head_wgrad(self):
        """head wgrad: dW[10][1024] = dlogit^T . H, db = sum dlogit (dedicated whole-batch kernel; the
        split-K GEMM path takes B > 1024)"""
        if self.head_gemm:
            ops.gemm(self.dl, self.h, self.gw["out"], M=NCLS, N=FC + 1, K=self.B, amode=ops.RMAJ,
                     lda=self.dl.shape[1], bmode=ops.RMAJ, ldb=FC, ldc=FC, b_ones_row=FC, bias_out=self.gw["bout"],
                     splits=self.head_splits, tile=4, workspace=self.ws_head)
        else:
            # B <= 1024; its bias workgroup also folds head_xent's loss / hit partials into
            # loss_sum / correct (256 same-address atomics cost ~2.5 us of head_xent's 7.8)
            ops.head_wgrad(self.dl, self.h, self.gw["out"], self.gw["bout"], NCLS, parts=self.head_parts,
                           loss_sum=self.loss_sum, correct=self.correct)

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
        """fc/head and conv optimizers over disjoint var lists (the data-parallel "late split"),
        sharing the whole-model optimizer's slot buffers and global step.  The conv optimizer
        advances the whole-model optimizer's beta powers (what a checkpoint saves); the fc one
        keeps an equal copy, advanced by itself - both apply once per step."""
        if self.opt_fc is None:
            n_, o = self.names, self.opt
            lists = ([n_[k] for k in ("out", "bout", "bd1", "wd1")], [n_[k] for k in ("wc2", "bc2", "wc1", "bc1")])
            self.opt_fc, self.opt_conv = (Optimizer(o.cfg, self.P, var_list=v, global_step=o.global_step)
                                          for v in lists)
            for s in (self.opt_fc, self.opt_conv):
                s.s1, s.s2 = o.s1, o.s2
            if o.beta_pow is not None:
                self.opt_fc.beta_pow.copy_(o.beta_pow)
                self.opt_conv.beta_pow = o.beta_pow

    def apply(self):
        self.opt.step(gscale=1.0 / self.world)

    def step(self, grad16=None, gscale=None):
        """One training step: forward, backward (+ all-reduce), Adam.  ``grad16``: the all-reduced
        bf16 gradients to apply instead of P.grad; ``gscale`` defaults to 1/world."""
        gscale = 1.0 / self.world if gscale is None else gscale
        if not self.par or not (self.late_split and self.allreduce is not None):
            self.forward_backward()
            if getattr(self, "_signalled", False):  # Adam's conv2 items wait for the branch's device-side signal
                vl = self.opt.var_list
                mask = sum(1 << vl.index(self.names[k]) for k in ("wc2", "bc2"))
                ops.apply_wait_next(self.c2_done, self.c2_seen, mask)
            self.opt.step(grad16=grad16, gscale=gscale)
            return
        self._ensure_split()
        self._late = (grad16, gscale)
        try:
            self.forward_backward()
        finally:
            self._late = None

    def join_side(self):
        """Rejoin the conv2 weight-gradient branch to the launch stream (after the last step of a replay when
        ``defer_join`` is on; a no-op otherwise)."""
        if getattr(self, "_pending_join", False):
            torch.cuda.current_stream(self.device).wait_stream(self.s_c2)
            self._pending_join = False

    def flops_per_image(self) -> float:
        """Training FLOPs per image (fwd + dgrad + wgrad of every GEMM-shaped op)."""
        c1 = 2 * IMG * IMG * C1 * KS * KS
        c2 = 2 * 14 * 14 * C2 * KS * KS * C1
        f1 = 2 * 7 * 7 * C2 * FC
        f2 = 2 * FC * NCLS
        return c1 * 2 + c2 * 3 + f1 * 3 + f2 * 3  # conv1 has no dgrad


class MnistCnnF32Trainer(MnistCnnTrainer):
    """The same CNN step at the reference's precision (``--dtype fp32``): fp32 activations and
    gradients, every product in exact fp32 (v_mfma_f32_16x16x4_f32 or VALU fmaf: an fmaf chain per
    dot product), fp32 weights read straight from the masters, the same fused TF1 Adam.

      conv1           conv_f32.hip 1-channel VALU kernel (LDS image, packed fp32 FMA), bias + ReLU +
                      2x2 max-pool + argmax
      conv2           conv_f32.hip implicit GEMM, bias + ReLU + 2x2 max-pool + argmax epilogue
      fc1             dense fp32 GEMM, bias + ReLU + dropout epilogue
      head            one fused fp32 kernel: logits, softmax-xent (loss, hits), dlogits, dH (below)
      head / fc1 dW   fp32 GEMMs, bias gradient through a ones column
      dH, dP2         1/keep * ReLU'(h) in the head kernel; fp32 GEMM with the ReLU'(p2) epilogue
      un-pool         argmax routing kernel (dP2 -> dY2)
      conv2 dX / dW   conv_f32.hip (ReLU'(p1) epilogue; weight grad + bias grad atomics)
      conv1 dW        conv_f32.hip from the pooled dP1 + argmax (only the argmax pixels: a quarter of
                      the dense products), fixed-order partial reduce
    A parity path, not the benchmarked one: no fused sampling, no hipGraph-specific scheduling,
    one stream."""

    def __init__(self, batch, device, lr: float = 1e-3, keep_prob: float = 0.75, seed: int = 0, data=None,
                 allreduce=None, world_size: int = 1, P: FlatParams | None = None, standalone: bool = True,
                 rank: int = 0):
        self.B = batch
        self.device = torch.device(device)
        if self.device.type == "cuda":
            ops.require()
        self.keep = keep_prob
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
        d, B, f = self.device, batch, torch.float32
        self.x = torch.empty(B, IMG, IMG, 1, device=d, dtype=f)
        self.labels = torch.empty(B, dtype=torch.int32, device=d)
        self.p1 = torch.empty(B, 14, 14, C1, device=d, dtype=f)
        self.a1 = torch.empty(B, 14, 14, C1, device=d, dtype=torch.uint8)
        self.p2 = torch.empty(B, 7, 7, C2, device=d, dtype=f)
        self.a2 = torch.empty(B, 7, 7, C2, device=d, dtype=torch.uint8)
        self.h = torch.empty(B, FC, device=d, dtype=f)
        self.logits = torch.empty(B, NCLS, device=d, dtype=f)
        self.dlogits = torch.empty(B, NCLS, device=d, dtype=f)
        self.dzf = torch.empty(B, FC, device=d, dtype=f)
        self.dp2 = torch.empty(B, 7, 7, C2, device=d, dtype=f)
        self.dy2 = torch.empty(B, 14, 14, C2, device=d, dtype=f)
        self.dp1 = torch.empty(B, 14, 14, C1, device=d, dtype=f)
        self.dy1 = torch.empty(B, IMG, IMG, C1, device=d, dtype=f)
        self.wt2 = torch.empty(C1, KS * KS, C2, device=d, dtype=f)
        self.loss_sum = torch.zeros(1, device=d)
        self.correct = torch.zeros(1, dtype=torch.int32, device=d)
        self.data_ctr = torch.zeros(1, dtype=torch.int64, device=d)
        self.data_done = torch.zeros(1, dtype=torch.int32, device=d)
        self.g1 = dict(B=B, H=IMG, W=IMG, C=1, Cout=C1, OH=IMG, OW=IMG, KH=KS, KW=KS, stride=1, pad=2)
        self.g2 = dict(B=B, H=14, W=14, C=C1, Cout=C2, OH=14, OW=14, KH=KS, KW=KS, stride=1, pad=2)
        n = self.names
        self.w = {k: self.P.view(n[k]) for k in ("wc1", "wc2", "wd1", "out")}
        self.b = {k: self.P.view(n[k]) for k in ("bc1", "bc2", "bd1", "bout")}
        self.gw = {k: self.P.gview(n[k]) for k in ("wc1", "wc2", "wd1", "out", "bc1", "bc2", "bd1", "bout")}
        lo1, hi1 = self.P.range_of([n["out"], n["bout"], n["bd1"], n["wd1"]])
        lo2, hi2 = self.P.range_of([n["wc2"], n["bc2"], n["wc1"], n["bc1"]])
        self.buckets = [(lo1, hi1), (lo2, hi2)]
        rc = self.P.range_of([n["wc2"], n["bc2"], n["wc1"], n["bc1"]])
        self.accum = [self.P.grad[rc[0]:rc[1]], self.loss_sum, self.correct]  # atomically accumulated
        self.par = False
        self.late_split = False
        self.opt_fc = self.opt_conv = None
        self._late = None
        self.schedule = []

    def forward(self, keep=None, logits=None, advance=False):
        """``advance``: the training step's forward - the fused head also advances the dropout /
        sampling counter (forward_backward's call)."""
        B, K1 = self.B, 7 * 7 * C2
        keep = self.keep if keep is None else keep
        if self.data is not None:
            ops.gather_rows(self.data.images, self.x.view(B, -1), None, self.data.labels, self.labels,
                            seed=self.seed + 1, counter=self.data_ctr, done=self.data_done, zero=self.accum)
        else:
            for t in self.accum:
                t.zero_()
        ops.conv_fwd(self.x, self.w["wc1"], self.b["bc1"], self.p1, self.a1, self.g1, pool=True, act=ops.ACT_RELU)
        ops.conv_fwd(self.p1, self.w["wc2"], self.b["bc2"], self.p2, self.a2, self.g2, pool=True, act=ops.ACT_RELU)
        ops.gemm(self.p2, self.w["wd1"], self.h, M=B, N=FC, K=K1, bias=self.b["bd1"], act=ops.ACT_RELU, keep=keep,
                 seed=self.seed + 2, counter=self.data_ctr)
        # head: logits, softmax-xent, dlogits, dZ = dlogits . W * 1/keep * ReLU'(h) (+ the counter) in
        # one launch on the GPU; the GEMM + softmax_xent (+ GEMM in forward_backward) chain otherwise
        ctr = self.data_ctr if (advance and self.data is not None) else None
        self._fused_head = ops.head_xent_f32(self.h, self.w["out"], self.b["bout"], self.labels, self.dzf,
                                             self.dlogits, self.loss_sum, self.correct, logits=self.logits,
                                             scale=1.0 / B, inv_keep=1.0 / keep, step_counter=ctr)
        if not self._fused_head:
            ops.gemm(self.h, self.w["out"], self.logits, M=B, N=NCLS, K=FC, bias=self.b["bout"])
            ops.softmax_xent(self.logits, labels_i=self.labels, scale=1.0 / B, dlogits=self.dlogits,
                             loss_sum=self.loss_sum, correct=self.correct)
        if logits is not None and logits is not self.logits:
            logits.copy_(self.logits)
        self._keep_used = keep

    def forward_backward(self):
        B, K1 = self.B, 7 * 7 * C2
        self.schedule = []
        self.forward(advance=True)
        if self.data is not None and not self._fused_head:
            self.data_ctr += 1  # next step's batch / dropout stream (the fused head advances it)
        inv_keep = 1.0 / self._keep_used
        # head: dW = dlogits^T . h (+ bias column), dh = dlogits . W * 1/keep * ReLU'(h)
        ops.gemm(self.dlogits, self.h, self.gw["out"], M=NCLS, N=FC + 1, K=B, amode=ops.RMAJ, lda=NCLS,
                 bmode=ops.RMAJ, ldb=FC, ldc=FC, b_ones_row=FC, bias_out=self.gw["bout"])
        if not self._fused_head:
            ops.gemm(self.dlogits, self.w["out"], self.dzf, M=B, N=FC, K=NCLS, bmode=ops.RMAJ, ldb=FC,
                     alpha=inv_keep, aux=self.h, aux_act=ops.ACT_RELU)
        # fc1: dW = dz^T . p2 (+ bias column), dP2 = dz . W1 * ReLU'(p2)
        ops.gemm(self.dzf, self.p2, self.gw["wd1"], M=FC, N=K1 + 1, K=B, amode=ops.RMAJ, lda=FC, bmode=ops.RMAJ,
                 ldb=K1, ldc=K1, b_ones_row=K1, bias_out=self.gw["bd1"])
        ops.gemm(self.dzf, self.w["wd1"], self.dp2, M=B, N=K1, K=FC, bmode=ops.RMAJ, ldb=K1, aux=self.p2,
                 aux_act=ops.ACT_RELU)
        if self.allreduce is not None:
            self.allreduce.launch(0)
            self.schedule.append("allreduce:0")
        # conv2: un-pool, data gradient (ReLU'(p1) epilogue), weight + bias gradient
        ops.unpool_f32(self.dp2, self.a2, self.dy2)
        ops.transpose_taps_f32(self.w["wc2"], self.wt2, C2, KS * KS, C1)
        ops.conv_dgrad(self.dy2, self.wt2, self.dp1, self.g2, relu_mask=self.p1)
        self.schedule.append("conv2_dgrad")
        ops.conv_wgrad(self.dy2, self.p1, self.gw["wc2"], self.gw["bc2"], self.g2)
        # conv1: weight + bias gradient straight from the pooled gradient (argmax pixels only; the
        # un-pooled tensor is formed only by the oracle / fallback path)
        ops.conv1_wgrad_pooled_f32(self.dp1, self.a1, self.x, self.gw["wc1"], self.gw["bc1"], self.g1, dy=self.dy1)
        if self.allreduce is not None:
            self.allreduce.launch(1)
            self.schedule.append("allreduce:1")
            self.allreduce.wait()


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
    dtypes = ("bf16", "fp32")

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
        cls = MnistCnnF32Trainer if getattr(model, "dtype", None) == "fp32" else MnistCnnTrainer
        self.core = cls(batch_size, self.device, seed=seed, P=self.P, standalone=False)

    def load_batch(self, batch):
        x, y = batch
        B = self.batch_size
        c = self.core
        c.x.copy_(x.reshape(B, IMG, IMG, 1).to(c.x.dtype))  # bf16 or fp32 (--dtype)
        lab = y.reshape(B, -1)
        c.labels.copy_((lab.argmax(1) if lab.shape[1] > 1 else lab[:, 0]).to(c.labels.dtype))
        c.data_ctr += 1  # dropout stream position (the HBM gather advances it in standalone mode)

    def compute_grads(self):
        self.core.forward_backward()
        return {"loss": ScaledScalar(self.core.loss_sum, 1.0 / self.batch_size), "correct": self.core.correct}

    def attach_data_parallel(self, allreduce, opt):
        """--mode=allreduce on the GPU: the trainer runs the benchmarked schedule (fc bucket's
        all-reduce launched right after the fc backward, before conv2's data gradient; split Adam
        overlapping the conv bucket) with ``opt`` - train.py's whole-model optimizer, whose slots
        and beta powers the Supervisor checkpoints - as the owner of the optimizer state."""
        self.core.allreduce = allreduce
        self.core.opt = opt

    def train_step(self, grad16=None, gscale=1.0):
        """Forward, backward, all-reduce (when attached) and Adam in the trainer's own order."""
        self.core.step(grad16=grad16, gscale=gscale)
        return {"loss": ScaledScalar(self.core.loss_sum, 1.0 / self.batch_size), "correct": self.core.correct}

    @torch.no_grad()
    def evaluate(self, images, labels) -> float:
        """Top-1 accuracy of the current weights (the CNN analog of LSTM:134-138): the training
        forward without dropout (keep 1.0), logits out of the fused head, argmax against the
        labels.  Any number of images, in program-batch chunks (the last one padded by repeating
        rows; only the real rows count).  Parameters are untouched; the loss / hit accumulators
        and the dropout stream position are restored."""
        c, B, n = self.core, self.batch_size, images.shape[0]
        if c.logits is None:
            c.logits = torch.empty(B, NCLS, device=self.device, dtype=torch.float32)
        ctr = c.data_ctr.clone()
        hits = 0
        for lo in range(0, n, B):
            m = min(B, n - lo)
            idx = torch.arange(lo, lo + B, device=images.device).clamp_max(n - 1)
            self.load_batch((images[idx], labels[idx]))
            c.forward(keep=1.0, logits=c.logits)
            hits += int((c.logits[:m].argmax(1) == c.labels[:m].long()).sum().item())
        c.data_ctr.copy_(ctr)
        c.loss_sum.zero_()
        c.correct.zero_()
        return hits / n
