"""Partitioned variables for the parameter-server mode (``--ps_partition_mb``).

The reference places whole variables round-robin over the ps tasks (``replica_device_setter``,
gan/distributed_gan.py:64-69,119-121), so the MNIST CNN's fc1 weight - 3.21 M of its 3.27 M
parameters - always lands on ONE ps task: that task's HBM and links carry 98 % of every pull and
every apply.  TF's answer is a partitioner on the variable scope; this module is the equivalent of
``tf.variable_axis_size_partitioner(max_shard_bytes)``:

* a variable of more than ``max_bytes`` (fp32) is split into ``n = ceil(rows / rows_per_shard)``
  partitions along the TF axis that is this framework's leading storage dimension (rows of our
  layout, so every partition is a contiguous range of the worker's flat buffer);
  ``rows_per_shard = max(1, max_bytes // bytes_per_row)``; sizes as TF's ``_iter_slices``
  (the first ``rows % n`` partitions one row longer);
* partitions are variables of their own, named ``<var>/part_<i>`` and created consecutively in
  place of the variable, so the round-robin placement deals them to consecutive ps tasks (as
  ``replica_device_setter`` does with a PartitionedVariable's parts);
* the optimizer slots follow their partition (``<var>/part_<i>/Adam``);
* checkpoints keep TF's PartitionedVariable layout: one entry per full variable (and full slot)
  listing its slices, each slice's data under its ``EncodeTensorNameSlice`` key (``ckpt.Sliced``),
  so a restore reads the full variable whatever the partitioning was.  (Parity unpinned: no TF in
  this image and no checkpoint fixtures in the reference.)

Variables with a transposed bf16 working copy (``VarSpec.transpose``: conv kernels read by a data
gradient) are never partitioned - their transposed copy is not a row range.
"""
from __future__ import annotations

import math
from dataclasses import replace

import torch

from ..ckpt import Sliced


def split_rows(rows: int, n: int):
    """TF ``_iter_slices``: [(start, length)] of n partitions of `rows` rows."""
    q, r = divmod(rows, n)
    out, off = [], 0
    for i in range(n):
        ln = q + (1 if i < r else 0)
        out.append((off, ln))
        off += ln
    return out


def num_partitions(spec, max_bytes: int) -> int:
    """variable_axis_size_partitioner: partitions of `spec` along its leading storage dimension."""
    if max_bytes <= 0 or spec.transpose is not None or len(spec.shape) < 1 or spec.shape[0] < 2:
        return 1
    if spec.numel * 4 <= max_bytes:
        return 1
    row_bytes = spec.numel // spec.shape[0] * 4
    per_shard = max(1, max_bytes // row_bytes)
    return min(spec.shape[0], math.ceil(spec.shape[0] / per_shard))


def tf_axis_of_rows(spec) -> int:
    """The TF-layout axis along which this framework's storage rows (dim 0) run (the layout
    conversions are axis permutations: follow element 0 and the first element of row 1)."""
    if spec.to_tf is None:
        return 0
    tf = spec.to_tf(torch.arange(spec.numel, dtype=torch.float64).view(spec.shape))
    p0 = (tf == 0).nonzero()[0]
    p1 = (tf == spec.numel // spec.shape[0]).nonzero()[0]
    diff = (p0 != p1).nonzero().flatten()
    if len(diff) != 1:
        raise ValueError("no single TF axis carries the storage rows of %s" % spec.name)
    return int(diff[0])


class PartitionedModel:
    """A ModelDef seen through the partitioner: the ps shards' variables (parts in place of the
    partitioned variables), their optimizer var lists, and the TF-name conversions between the two
    views for checkpoints.  Everything else is delegated to the wrapped model."""

    def __init__(self, model, max_bytes: int):
        self.base = model
        self.max_bytes = int(max_bytes)
        self.parts = {}     # var -> [(part name, first row, rows)]
        self.part_of = {}   # part name -> (var, first row, rows)
        self.axis = {}      # var -> TF axis of the partitions
        self._spec = {}
        specs = []
        for s in model.specs:
            n = num_partitions(s, self.max_bytes)
            if n == 1:
                specs.append(s)
                self._spec[s.name] = s
                continue
            self.axis[s.name] = tf_axis_of_rows(s)
            plist = []
            for i, (r0, ln) in enumerate(split_rows(s.shape[0], n)):
                name = "%s/part_%d" % (s.name, i)
                shape = (ln,) + tuple(s.shape[1:])
                tf_shape = None
                if s.tf_shape is not None:
                    tf_shape = list(s.tf_shape)
                    tf_shape[self.axis[s.name]] = ln
                    tf_shape = tuple(tf_shape)
                ps = replace(s, name=name, shape=shape, tf_shape=tf_shape)
                ps.init = None
                specs.append(ps)
                self._spec[name] = ps
                plist.append((name, r0, ln))
                self.part_of[name] = (s.name, r0, ln)
            self.parts[s.name] = plist
        self.specs = specs
        self.var_order = []
        for n_ in model.var_order:
            self.var_order += [p for p, _, _ in self.parts[n_]] if n_ in self.parts else [n_]
        self.opt_groups = []
        for cfg, var_list, bp in model.opt_groups:
            vl = []
            for v in var_list:
                vl += [p for p, _, _ in self.parts[v]] if v in self.parts else [v]
            self.opt_groups.append((cfg, vl, bp))

    def __getattr__(self, item):  # name, gs_name, gs_increments, ...
        return getattr(self.base, item)

    # ---- TF layout of a part: the partitioned variable's conversion applies to any row count
    def _owner(self, name):
        return self.part_of[name][0] if name in self.part_of else name

    def to_tf(self, name, t):
        return self.base.to_tf(self._owner(name), t)

    def from_tf(self, name, t):
        return self.base.from_tf(self._owner(name), t)

    def tf_shapes(self):
        return {s.name: (s.tf_shape if s.tf_shape is not None else s.shape) for s in self.specs}

    # ---- worker side
    def add_aliases(self, P):
        """Register every part as an alias view of its variable in the worker's full FlatParams
        (offsets / views / bf16 working copies), so the ps data planes address parts directly."""
        for var, plist in self.parts.items():
            row = P.spec(var).numel // P.spec(var).shape[0]
            for name, r0, _ln in plist:
                P.add_alias(self._spec[name], var, r0 * row)

    # ---- checkpoints: part-named shard tensors <-> full TF variables
    def _split_key(self, key):
        """(var, part index, suffix) of a part-named key 'var/part_i[/slot]', or None."""
        for var, plist in self.parts.items():
            for i, (name, _r0, _ln) in enumerate(plist):
                if key == name or key.startswith(name + "/"):
                    return var, i, key[len(name):]
        return None

    def merge_tf(self, tensors: dict) -> dict:
        """Shard tensors (TF layout, part names) -> full variables and slots as ``ckpt.Sliced``."""
        out, groups = {}, {}
        for k, t in tensors.items():
            hit = self._split_key(k)
            if hit is None:
                out[k] = t
                continue
            var, i, suffix = hit
            groups.setdefault(var + suffix, (var, {}))[1][i] = t
        for full_name, (var, pieces) in groups.items():
            plist = self.parts[var]
            if len(pieces) != len(plist):
                raise KeyError("checkpoint of %s is missing partitions" % full_name)
            ax = self.axis[var]
            full = torch.cat([pieces[i] for i in range(len(plist))], dim=ax)
            out[full_name] = Sliced(full, ax, [(r0, ln) for _n, r0, ln in plist])
        return out

    def split_tf(self, tensors: dict) -> dict:
        """Full TF variables / slots (as ``ckpt.load_bundle`` returns them) -> part-named tensors."""
        out = {}
        for k, t in tensors.items():
            var = next((v for v in self.parts if k == v or k.startswith(v + "/")), None)
            if var is None:
                out[k] = t
                continue
            suffix = k[len(var):]
            if isinstance(t, Sliced):
                t = t.full
            for name, r0, ln in self.parts[var]:
                out[name + suffix] = t.narrow(self.axis[var], r0, ln).contiguous()
        return out
