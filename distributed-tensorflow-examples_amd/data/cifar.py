"""CIFAR-10 input pipeline for the ResNet-20 configuration (BASELINE.json config 3).

``read_data_sets(data_dir)`` reads the CIFAR-10 binary distribution
(``data_batch_1.bin`` .. ``data_batch_5.bin``, ``test_batch.bin``: records of
1 label byte + 3072 bytes of CHW pixels) and stores images HWC-flattened
(NHWC rows of 3072 uint8, the layout of the conv kernels), labels one-hot [10].
Batching reuses the MNIST ``DataSet`` (TF ``next_batch`` epoch semantics) and
``DeviceBatcher`` (HBM-resident gather).  No network here: without the files a
deterministic synthetic CIFAR-shaped set is generated and that is logged.
"""
from __future__ import annotations

import os

import numpy as np

from .mnist import DataSet, DataSets

IMG, CH, NCLS = 32, 3, 10
TRAIN_FILES = ["data_batch_%d.bin" % i for i in range(1, 6)]
TEST_FILE = "test_batch.bin"


def _read_bin(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 1 + CH * IMG * IMG)
    y = raw[:, 0].astype(np.int64)
    x = raw[:, 1:].reshape(-1, CH, IMG, IMG).transpose(0, 2, 3, 1)  # CHW -> HWC
    return np.ascontiguousarray(x).reshape(len(y), -1), y


def _find_dir(data_dir):
    for d in (data_dir, os.path.join(data_dir, "cifar-10-batches-bin")):
        if d and all(os.path.exists(os.path.join(d, f)) for f in TRAIN_FILES + [TEST_FILE]):
            return d
    return None


def synthetic_arrays(n_train=50000, n_test=10000, seed=4321):
    """CIFAR-shaped uint8 images with a learnable cue: class k brightens channel k%3 in row band k."""
    rng = np.random.RandomState(seed)

    def make(n):
        y = rng.randint(0, NCLS, size=n)
        x = rng.randint(0, 120, size=(n, IMG, IMG, CH)).astype(np.uint8)
        for k in range(NCLS):
            sel = y == k
            x[sel, 3 * k: 3 * k + 2, :, k % CH] = 255
        return x.reshape(n, -1), y

    return make(n_train), make(n_test)


def read_data_sets(data_dir: str, one_hot: bool = True, validation_size: int = 0, seed: int = 0,
                   allow_synthetic: bool = True, log=print) -> DataSets:
    d = _find_dir(data_dir) if data_dir else None
    if d:
        parts = [_read_bin(os.path.join(d, f)) for f in TRAIN_FILES]
        tr_x = np.concatenate([p[0] for p in parts])
        tr_y = np.concatenate([p[1] for p in parts])
        te_x, te_y = _read_bin(os.path.join(d, TEST_FILE))
        synthetic = False
    else:
        if not allow_synthetic:
            raise FileNotFoundError("CIFAR-10 binary batches not found in %r" % data_dir)
        log("CIFAR-10 binary batches not found in %r (no network): using synthetic CIFAR-shaped data" % data_dir)
        (tr_x, tr_y), (te_x, te_y) = synthetic_arrays()
        synthetic = True
    val = DataSet(tr_x[:validation_size], tr_y[:validation_size], one_hot, seed + 1) if validation_size else None
    train = DataSet(tr_x[validation_size:], tr_y[validation_size:], one_hot, seed)
    test = DataSet(te_x, te_y, one_hot, seed + 2)
    return DataSets(train, val, test, synthetic)
