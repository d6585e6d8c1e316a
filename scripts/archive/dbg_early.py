import os, sys
sys.path.insert(0, os.getcwd())
import torch
import dtfe
from dtfe.models.mnist_cnn import MnistCnnTrainer
out = {}
for tag, early in (("e1", "1"), ("e0", "0"), ("e0b", "0"), ("e1b", "1")):
    os.environ["DTFE_CNN_EARLY_APPLY"] = early
    tr = MnistCnnTrainer(256, "cuda", seed=9)
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    out[tag] = tr.P.master.clone()
for a, b in (("e1", "e0"), ("e0", "e0b"), ("e1", "e1b")):
    d = (out[a] - out[b]).abs()
    i = int(d.argmax())
    print(a, b, "maxdiff %.3e at %d (%.5f vs %.5f)" % (float(d.max()), i, float(out[a][i]), float(out[b][i])),
          "n>1e-6:", int((d > 1e-6).sum()))
