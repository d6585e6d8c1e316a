"""MNIST conv1 forward (batch sampling fused) at B=1024, for the DTFE_DIAG=c1=<bits> ablations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtfe  # noqa: E402,F401
from dtfe import ops  # noqa: E402
from dtfe.models.mnist_cnn import MnistCnnTrainer  # noqa: E402
from conv2_scale import timeit  # noqa: E402

t = MnistCnnTrainer(1024, "cuda")
t.step()
torch.cuda.synchronize()
f = lambda: ops.require().conv1_gather_fwd(t.data.images, t.data.labels, t.seed + 1, t.data_ctr, t.data_done, t.labels,  # noqa: E731
                                            t.x, t.w["wc1"], t.b["bc1"], t.p1, t.a1, t.accum)
g = lambda: ops.imgconv(t.w["wc1"], t.p1, src=t.x, bias=t.b["bc1"], argmax=t.a1, act=ops.ACT_RELU, pool=True, **t.ic1)  # noqa: E731
print("DIAG=%s fused-gather conv1 %.1f us   plain conv1 %.1f us" % (os.environ.get("DTFE_DIAG", ""), timeit(f, 50),
                                                                   timeit(g, 50)), flush=True)
