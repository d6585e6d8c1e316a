"""TF-compatible checkpoints and events.

Layout written by the chief (same names as ``tf.train.Saver`` under
``tf.train.Supervisor`` in TF 1.11):

    <model_dir>/checkpoint                              text CheckpointState
    <model_dir>/model.ckpt-<gs>.index                   tensor-bundle SSTable
    <model_dir>/model.ckpt-<gs>.data-00000-of-00001     raw tensor bytes
    <model_dir>/model.ckpt-<gs>.meta                    minimal MetaGraphDef
    <model_dir>/graph.pbtxt                             text GraphDef of the variables
    <model_dir>/events.out.tfevents.<ts>.<host>         TFRecord Event stream

The binary formats (SSTable, BundleEntryProto, crc32c, TFRecord framing) are
produced by the native runtime ``_dtfe_rt`` (csrc/runtime/tf_formats.cpp).
"""
from __future__ import annotations

import os
import re
import socket
import threading
import time

import numpy as np
import torch

from ..utils import native

DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT64, DT_BFLOAT16 = 1, 2, 3, 4, 9, 14
_TORCH_TO_TF = {torch.float32: DT_FLOAT, torch.float64: DT_DOUBLE, torch.int32: DT_INT32, torch.uint8: DT_UINT8,
                torch.int64: DT_INT64, torch.bfloat16: DT_BFLOAT16}
_TF_TO_NP = {DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32, DT_UINT8: np.uint8,
             DT_INT64: np.int64}


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


class Sliced:
    """A partitioned variable's full value (TF layout) and its partitions along ``axis``:
    ``bounds`` = [(start, length), ...].  ``save_bundle`` writes it the way tf.train.Saver writes a
    PartitionedVariable: one full-tensor entry listing the slices (BundleEntryProto.slices), each
    slice's data under its ``EncodeTensorNameSlice`` key; ``load_bundle`` reassembles the full tensor."""

    def __init__(self, full: torch.Tensor, axis: int, bounds):
        self.full, self.axis, self.bounds = full, axis, [(int(a), int(b)) for a, b in bounds]

    def slice_specs(self):
        for start, length in self.bounds:
            yield [(start, length) if d == self.axis else (0, -1) for d in range(self.full.dim())], \
                self.full.narrow(self.axis, start, length)


def save_bundle(prefix: str, tensors: dict, write_meta: bool = True):
    """Write ``prefix.index`` + ``prefix.data-00000-of-00001`` (+ ``prefix.meta``)."""
    rt = native.rt()
    w = rt.BundleWriter()
    meta_vars = []
    for name, t in tensors.items():
        if isinstance(t, Sliced):
            dt = _TORCH_TO_TF[t.full.dtype]
            for spec, part in t.slice_specs():
                w.add_slice(name, dt, list(t.full.shape), spec, _tensor_bytes(part))
            meta_vars.append((name, dt, list(t.full.shape)))
            continue
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(t)
        dt = _TORCH_TO_TF[t.dtype]
        w.add(name, dt, list(t.shape), _tensor_bytes(t))
        meta_vars.append((name, dt, list(t.shape)))
    w.finish(prefix)
    if write_meta:
        gd = rt.graph_def_for_variables(meta_vars)
        with open(prefix + ".meta.tempstate", "wb") as f:
            f.write(rt.meta_graph_def(gd, "1.11.0 (dtfe-mi355x)"))
        os.replace(prefix + ".meta.tempstate", prefix + ".meta")


def load_bundle(prefix: str) -> dict:
    """Read every tensor of a bundle into CPU tensors (crc32c verified)."""
    rt = native.rt()
    out = {}

    def decode(raw, dt, shape):
        if dt == DT_BFLOAT16:
            return torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16).reshape(shape)
        return torch.from_numpy(np.frombuffer(raw, dtype=_TF_TO_NP[dt]).copy()).reshape(shape)

    for name, (dt, shape, _off, _size, _crc, slices) in rt.read_bundle_index(prefix).items():
        if not slices:
            out[name] = decode(rt.read_bundle_tensor(prefix, name), dt, shape)
            continue
        # a partitioned variable: every slice read from its own key and placed into the full tensor
        full = None
        for spec in slices:
            sshape = [shape[d] if ln == -1 else ln for d, (_st, ln) in enumerate(spec)]
            part = decode(rt.read_bundle_slice(prefix, name, spec), dt, sshape)
            if full is None:
                full = torch.zeros(shape, dtype=part.dtype)
            idx = tuple(slice(None) if ln == -1 else slice(st, st + ln) for st, ln in spec)
            full[idx] = part
        out[name] = full
    return out


# ---------------------------------------------------------------- state file
def write_checkpoint_state(model_dir: str, latest: str, all_paths: list):
    """``checkpoint`` text proto, as tf.train.update_checkpoint_state writes it."""
    lines = ['model_checkpoint_path: "%s"' % latest]
    lines += ['all_model_checkpoint_paths: "%s"' % p for p in all_paths]
    tmp = os.path.join(model_dir, "checkpoint.tmp%d" % os.getpid())
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(model_dir, "checkpoint"))


def read_checkpoint_state(model_dir: str):
    p = os.path.join(model_dir, "checkpoint")
    if not os.path.exists(p):
        return None, []
    latest, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
        if not m:
            continue
        if m.group(1) == "model_checkpoint_path":
            latest = m.group(2)
        else:
            allp.append(m.group(2))
    return latest, allp


def latest_checkpoint(model_dir: str):
    latest, _ = read_checkpoint_state(model_dir)
    if latest is None:
        return None
    path = latest if os.path.isabs(latest) else os.path.join(model_dir, latest)
    return path if os.path.exists(path + ".index") else None


class Saver:
    """tf.train.Saver equivalent: ``save(tensors, global_step)`` with max_to_keep retention."""

    def __init__(self, model_dir: str, max_to_keep: int = 5, basename: str = "model.ckpt"):
        self.model_dir = model_dir
        self.max_to_keep = max_to_keep
        self.basename = basename
        os.makedirs(model_dir, exist_ok=True)
        _, self._kept = read_checkpoint_state(model_dir)
        self._lock = threading.Lock()

    def save(self, tensors: dict, global_step: int) -> str:
        with self._lock:
            prefix = os.path.join(os.path.abspath(self.model_dir), "%s-%d" % (self.basename, int(global_step)))
            save_bundle(prefix, tensors)
            self._kept = [p for p in self._kept if p != prefix] + [prefix]
            while self.max_to_keep and len(self._kept) > self.max_to_keep:
                old = self._kept.pop(0)
                for suf in (".index", ".data-00000-of-00001", ".meta"):
                    try:
                        os.remove(old + suf)
                    except OSError:
                        pass
            write_checkpoint_state(self.model_dir, prefix, self._kept)
            return prefix

    def restore(self, path: str | None = None) -> dict | None:
        path = path or latest_checkpoint(self.model_dir)
        return load_bundle(path) if path else None


# -------------------------------------------------------------------- events
class EventWriter:
    """events.out.tfevents.<ts>.<host> writer (TFRecord-framed Event protos)."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "events.out.tfevents.%d.%s%s" % (int(time.time()), socket.gethostname(),
                                                                          filename_suffix))
        self._rt = native.rt()
        self._f = open(self.path, "ab")
        self._lock = threading.Lock()
        self._write(self._rt.event_file_version(time.time()))

    def _write(self, event: bytes):
        with self._lock:
            self._f.write(self._rt.tfrecord_frame(event))
            self._f.flush()

    def add_scalars(self, step: int, scalars: dict):
        self._write(self._rt.event_scalars(time.time(), int(step), [(k, float(v)) for k, v in scalars.items()]))

    def add_graph_of_variables(self, vars_: list):
        self._write(self._rt.event_graph(time.time(), self._rt.graph_def_for_variables(vars_)))

    def close(self):
        with self._lock:
            if not self._f.closed:
                self._f.close()


def write_graph_pbtxt(model_dir: str, vars_: list):
    """graph.pbtxt: text-format GraphDef listing the variables (Supervisor writes this on the chief)."""
    names = {DT_FLOAT: "DT_FLOAT", DT_INT32: "DT_INT32", DT_INT64: "DT_INT64", DT_BFLOAT16: "DT_BFLOAT16",
             DT_DOUBLE: "DT_DOUBLE", DT_UINT8: "DT_UINT8"}
    out = []
    for name, dt, shape in vars_:
        dims = "".join("\n        dim {\n          size: %d\n        }" % d for d in shape)
        out.append('node {\n  name: "%s"\n  op: "VariableV2"\n  attr {\n    key: "dtype"\n    value {\n'
                   '      type: %s\n    }\n  }\n  attr {\n    key: "shape"\n    value {\n      shape {%s\n      }\n'
                   '    }\n  }\n}' % (name, names[dt], dims))
    out.append("versions {\n  producer: 26\n}")
    with open(os.path.join(model_dir, "graph.pbtxt"), "w") as f:
        f.write("\n".join(out) + "\n")
