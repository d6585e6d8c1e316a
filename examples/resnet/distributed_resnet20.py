#!/usr/bin/env python
"""Distributed resnet20 (BASELINE.json configs 3 (CIFAR-10)) - the reference's command line.

    python distributed_resnet20.py --worker_hosts=h0:2222,h1:2222 --job_name=worker --task_index=0 \
        --mode=allreduce [--data_dir=... --model_dir=/tmp/checkpoints --batch_size=...]

Sync all-reduce data parallelism (bucketed RCCL all-reduce launched during the backward pass)
or the reference's parameter-server modes; all logic lives in dtfe.train.  Without data files
in --data_dir the example trains on synthetic data of the same shape.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import dtfe  # noqa: E402,F401
from dtfe.train import main  # noqa: E402

if __name__ == "__main__":
    main("resnet20")
