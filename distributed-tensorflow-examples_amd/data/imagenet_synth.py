"""Synthetic ImageNet-shape data for the ResNet-50 scaling configuration (BASELINE.json
config 5: "ImageNet-shape synthetic ResNet-50").  224x224x3 uint8 NHWC images and
1000-class labels, deterministic; a small pool (default 512 images, 77 MB) is enough
because the benchmark measures throughput, and DeviceBatcher keeps it in HBM."""
from __future__ import annotations

import numpy as np

from .mnist import DataSet, DataSets

IMG, CH, NCLS = 224, 3, 1000


def read_data_sets(n_train: int = 512, n_test: int = 64, one_hot: bool = True, seed: int = 0, log=print) -> DataSets:
    log("ImageNet-shape synthetic data: %d train images 224x224x3, 1000 classes (no dataset on this host)" % n_train)
    rng = np.random.RandomState(7 + seed)

    def make(n):
        return rng.randint(0, 256, size=(n, IMG * IMG * CH), dtype=np.uint8), rng.randint(0, NCLS, size=n)

    tr, te = make(n_train), make(n_test)
    return DataSets(DataSet(tr[0], tr[1], one_hot, seed, NCLS), None, DataSet(te[0], te[1], one_hot, seed + 2, NCLS),
                    synthetic=True)
