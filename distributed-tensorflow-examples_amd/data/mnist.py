"""MNIST input pipeline.

``read_data_sets(data_dir, one_hot=True)`` mirrors
``tensorflow.examples.tutorials.mnist.input_data`` (GAN:177): the four idx
files (``train-images-idx3-ubyte.gz`` ...) are parsed by the native runtime,
images become float32 in [0, 1] flattened to 784, 5000 training images are
split off as validation, labels are one-hot [10].  ``next_batch(B)`` has TF's
semantics (shuffle on first use, stitch epoch boundaries) via the native
``EpochBatcher``.  Each worker holds its own full copy and shuffle - the
reference does not shard data across workers.

There is no network here: when the idx files are absent a deterministic
synthetic MNIST-shaped dataset is generated instead and that fact is logged
(``DataSets.synthetic``).

For GPU workers ``DeviceBatcher`` stages the images once in HBM and gathers
each batch on device from host-computed indices (4 bytes/row over PCIe
instead of 3 KB/row).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils import native

FILES = {
    "train_images": "train-images-idx3-ubyte",
    "train_labels": "train-labels-idx1-ubyte",
    "test_images": "t10k-images-idx3-ubyte",
    "test_labels": "t10k-labels-idx1-ubyte",
}


def _find(data_dir, stem):
    for cand in (stem + ".gz", stem, stem.replace("-idx", ".idx")):
        p = os.path.join(data_dir, cand)
        if os.path.exists(p):
            return p
    return None


class DataSet:
    def __init__(self, images_u8: np.ndarray, labels: np.ndarray, one_hot: bool, seed: int, num_classes: int = 10):
        self.images_u8 = images_u8.reshape(images_u8.shape[0], -1)
        self.labels_int = labels.astype(np.int64)
        self.one_hot = one_hot
        self.num_classes = num_classes
        self._batcher = native.rt().EpochBatcher(self.num_examples, seed)

    @property
    def num_examples(self):
        return self.images_u8.shape[0]

    @property
    def images(self):
        return self.images_u8.astype(np.float32) / 255.0

    @property
    def labels(self):
        if self.one_hot:
            out = np.zeros((len(self.labels_int), self.num_classes), dtype=np.float32)
            out[np.arange(len(self.labels_int)), self.labels_int] = 1.0
            return out
        return self.labels_int

    @property
    def epochs_completed(self):
        return self._batcher.epochs_completed

    def next_batch_indices(self, batch_size: int) -> np.ndarray:
        return self._batcher.next(batch_size)

    def next_batch(self, batch_size: int):
        idx = self.next_batch_indices(batch_size)
        x = self.images_u8[idx].astype(np.float32) / 255.0
        if self.one_hot:
            y = np.zeros((batch_size, self.num_classes), dtype=np.float32)
            y[np.arange(batch_size), self.labels_int[idx]] = 1.0
        else:
            y = self.labels_int[idx]
        return x, y


class DataSets:
    def __init__(self, train, validation, test, synthetic: bool):
        self.train, self.validation, self.test = train, validation, test
        self.synthetic = synthetic


def synthetic_arrays(n_train=60000, n_test=10000, seed=1234):
    """Deterministic MNIST-shaped data with learnable structure: class k lights band k."""
    rng = np.random.RandomState(seed)

    def make(n):
        y = rng.randint(0, 10, size=n)
        x = rng.randint(0, 80, size=(n, 28, 28)).astype(np.uint8)
        for k in range(10):
            sel = y == k
            x[sel, 2 + 2 * k: 4 + 2 * k, 4:24] = 255
        return x, y

    return make(n_train), make(n_test)


def read_data_sets(data_dir: str, one_hot: bool = True, validation_size: int = 5000, seed: int = 0,
                   allow_synthetic: bool = True, log=print) -> DataSets:
    paths = {k: _find(data_dir, v) if data_dir else None for k, v in FILES.items()}
    rt = native.rt()
    if all(paths.values()):
        tr_x = rt.idx_read(paths["train_images"])
        tr_y = rt.idx_read(paths["train_labels"])
        te_x = rt.idx_read(paths["test_images"])
        te_y = rt.idx_read(paths["test_labels"])
        synthetic = False
    else:
        if not allow_synthetic:
            raise FileNotFoundError("MNIST idx files not found in %r (no network to download them)" % data_dir)
        log("Extracting MNIST: idx files not found in %r (no network): using synthetic MNIST-shaped data"
            % data_dir)
        (tr_x, tr_y), (te_x, te_y) = synthetic_arrays()
        synthetic = True
    tr_x, tr_y = np.asarray(tr_x), np.asarray(tr_y)
    val = DataSet(tr_x[:validation_size], tr_y[:validation_size], one_hot, seed + 1)
    train = DataSet(tr_x[validation_size:], tr_y[validation_size:], one_hot, seed)
    test = DataSet(np.asarray(te_x), np.asarray(te_y), one_hot, seed + 2)
    return DataSets(train, val, test, synthetic)


class DeviceBatcher:
    """HBM-resident copy of a DataSet; batches gathered on device (K14)."""

    def __init__(self, ds: DataSet, device, batch_size: int, one_hot: bool = True):
        from .. import ops

        self.ops = ops
        self.ds = ds
        self.B = batch_size
        self.device = torch.device(device)
        self.images = torch.from_numpy(ds.images_u8).to(self.device)
        self.labels = torch.from_numpy(ds.labels_int.astype(np.int32)).to(self.device)
        self.idx = torch.empty(batch_size, dtype=torch.int32, device=self.device)
        self.x = torch.empty(batch_size, ds.images_u8.shape[1], dtype=torch.float32, device=self.device)
        self.y_int = torch.empty(batch_size, dtype=torch.int32, device=self.device)
        self.y = torch.empty(batch_size, ds.num_classes, dtype=torch.float32, device=self.device)
        self.one_hot = one_hot
        self._host_idx = torch.empty(batch_size, dtype=torch.int32).pin_memory() \
            if self.device.type == "cuda" else torch.empty(batch_size, dtype=torch.int32)

    def next_batch(self):
        self._host_idx.copy_(torch.from_numpy(self.ds.next_batch_indices(self.B)))
        self.idx.copy_(self._host_idx, non_blocking=True)
        self.ops.gather_rows(self.images, self.x, self.idx, self.labels, self.y_int)
        if self.one_hot:
            self.y.zero_()
            self.y.scatter_(1, self.y_int.long().unsqueeze(1), 1.0)
            return self.x, self.y
        return self.x, self.y_int
