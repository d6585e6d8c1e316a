"""dtfe — MI355X-native distributed training examples.

A re-design, for AMD Instinct MI355X (gfx950 / CDNA4), of the capabilities of
Xingskcs/Distributed-TensorFlow-Examples: the MNIST GAN / autoencoder / LSTM
examples with the ``--ps_hosts/--worker_hosts/--job_name/--task_index``
cluster-spec CLI, between-graph parameter-server training (async, plus sync
with a chief), a Supervisor lifecycle with TF-layout checkpoints, and - beyond
the reference - ring all-reduce data parallelism, MNIST CNN / ResNet workloads
and hand-written CDNA4 HIP kernels for every per-step op.

Layout:
  ops/       torch.ops.dtfe.* wrappers (HIP kernels; CPU reference paths)
  models/    model definitions as explicit fwd/bwd step programs
  parallel/  cluster spec, rendezvous, PS service, all-reduce engine
  optim/     TF1-exact optimizers over flat fp32 master buffers
  ckpt/      TF tensor-bundle checkpoints + events files (native runtime)
  data/      MNIST idx reader, synthetic datasets, device batchers
  utils/     flags, timing, HIP-graph capture, logging
"""
import os as _os

__version__ = "0.1.0"
PKG_DIR = _os.path.dirname(_os.path.abspath(__file__))
REPO_ROOT = _os.path.dirname(PKG_DIR)
