#!/usr/bin/env python
"""Distributed MNIST CNN (BASELINE.json configs 2 and 4) - same command line as the reference's distributed_cnn.py.

    python distributed_cnn.py --ps_hosts=h0:2222 --worker_hosts=h1:2222,h2:2222 \
        --job_name=worker --task_index=0 [--data_dir=/data_dir --model_dir=/tmp/checkpoints --workers=2]

All logic lives in dtfe.train (shared by every example); see README.md for the
north-star flags (--sync, --mode=allreduce, --device, ...).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import dtfe  # noqa: E402,F401
from dtfe.train import main  # noqa: E402

if __name__ == "__main__":
    main("cnn")
